#!/usr/bin/env python3
"""The render / k_prep dispatches of a rocprofv3 kernel-trace CSV: one line per
render (start, duration, gap after the previous render's end, the k_prep
dispatches that ran since) and a summary over the steady frames (the last
`n` renders before the untimed end-to-end context: median duration, median
start-to-start period and gap)."""
import csv
import statistics
import sys

path = sys.argv[1]
rows = sorted((r for r in csv.DictReader(open(path)) if "xrt::k_" in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
renders = [r for r in rows if "k_render" in r["Kernel_Name"]]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = prev_start = None
lines, durs, periods, gaps = [], [], [], []
for r in renders:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else float("nan")
    per = (s - prev_start) / 1e3 if prev_start is not None else float("nan")
    lines.append((s, e, gap, per))
    prev_end, prev_start = e, s
# steady frames: skip the first 3 and the end-to-end context's frame (the last)
steady = lines[3:-1] if len(lines) > 5 else lines
for s, e, gap, per in lines:
    print(f"render {(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  period {per:8.1f}")
durs = [(e - s) / 1e3 for s, e, _, _ in steady]
periods = [p for _, _, _, p in steady]
gaps = [g for _, _, g, _ in steady]
preps = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_prep" in r["Kernel_Name"]]
print(f"steady renders {len(steady)}: median dur {statistics.median(durs):.1f} us, mean dur "
      f"{statistics.mean(durs):.1f} us, median period {statistics.median(periods):.1f} us, median gap "
      f"{statistics.median(gaps):.1f} us, min gap {min(gaps):.1f} us")
print(f"k_prep dispatches {len(preps)}: median {statistics.median(preps):.1f} us")
