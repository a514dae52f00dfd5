#!/usr/bin/env python3
"""Per-frame timeline from a rocprofv3 kernel trace (run_kernel_trace.csv):
the last --frames renders, and for each the preparation kernels dispatched
since the previous render (k_prep count / fill passes, k_size_lists), with
start/end relative to the previous render's start, in microseconds, and the
steady-state means: render-to-render step, render duration, prep-chain span,
idle gaps between a frame's last preparation kernel and its render's start.

  python tools/trace_timeline.py DIR_OR_CSV [--frames 8]
"""
import argparse
import csv
import glob
import os
import statistics


def short(name):
    for k in ("k_prep", "k_size_lists", "k_scatter_pairs", "k_render_binned_hits", "k_render_binned", "k_render_tiled", "k_render_brute",
              "k_reduce_stats", "k_tile_plan", "k_band_model", "k_hole_fill"):
        if k in name:
            return k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--frames", type=int, default=8)
    args = ap.parse_args()
    f = args.path
    if os.path.isdir(f):
        f = sorted(glob.glob(os.path.join(f, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = []
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        if k:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, int(r["Queue_Id"])))
    rows.sort()
    renders = [i for i, r in enumerate(rows) if r[2].startswith("k_render")]
    steps, durs, preps, gaps = [], [], [], []
    lines = []
    for j in range(1, len(renders)):
        a, b = renders[j - 1], renders[j]
        r0, r1 = rows[a], rows[b]
        prep = [rows[i] for i in range(a + 1, b) if rows[i][2] in ("k_prep", "k_size_lists", "k_scatter_pairs")]
        steps.append((r1[0] - r0[0]) / 1e3)
        durs.append((r1[1] - r1[0]) / 1e3)
        if prep:
            preps.append((max(p[1] for p in prep) - min(p[0] for p in prep)) / 1e3)
        if j >= len(renders) - args.frames:
            parts = " ".join(f"{p[2]}[q{p[3]}] {(p[0] - r0[0]) / 1e3:.1f}..{(p[1] - r0[0]) / 1e3:.1f}" for p in prep)
            lines.append(f"render[q{r1[3]}] {(r1[0] - r0[0]) / 1e3:7.1f}..{(r1[1] - r0[0]) / 1e3:7.1f} | {parts}")
    n = max(1, len(steps) // 2)            # the steady second half
    print(f"{len(renders)} renders; second half means: step {statistics.mean(steps[-n:]):.1f} us, render "
          f"{statistics.mean(durs[-n:]):.1f} us, prep chain {statistics.mean(preps[-n:]) if preps else 0:.1f} us")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
