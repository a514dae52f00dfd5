#!/usr/bin/env python3
"""Per-wave timeline of one binned render (steady state): the waves' in-kernel
s_memrealtime records (xrt_debug_wave_times) with their statistics records.

    python tools/wave_timeline.py [--size W H] [--tile-mesh n] [--frames K]

Prints the kernel span, waves alive per 1-us bin, per-wave duration
percentiles, the tail (time after 90 / 99 % of the waves ended), and the
duration by the wave's survivor tests (tile_tests)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import simpleraytracing_amd as xrt                      # noqa: E402
from simpleraytracing_amd.scenes import tiled_mesh     # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, nargs=2, default=[2048, 2048])
ap.add_argument("--tile-mesh", type=int, default=1)
ap.add_argument("--frames", type=int, default=20)
ap.add_argument("--inflight", type=int, default=1,
                help="frame k on stream k %% N into its own planes (bench.py --inflight); the last four "
                     "frames' start/end then show how consecutive renders overlap")
a = ap.parse_args()
import torch                                             # noqa: E402

W, H = a.size
tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
if a.tile_mesh > 1:
    tris = tiled_mesh(tris, a.tile_mesh)
cam = xrt.camera_for_mesh(tris, W, H)
dev = torch.device("cuda", 0)
sets = [(torch.empty(W * H, dtype=torch.float32, device=dev), torch.empty(W * H, dtype=torch.float32, device=dev),
         torch.empty(W * H, dtype=torch.uint8, device=dev),
         torch.cuda.current_stream(dev) if f == 0 else torch.cuda.Stream(dev)) for f in range(max(1, a.inflight))]
with xrt.Context(0) as ctx:
    ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
    ctx.upload_mesh(tris)
    for k in range(a.frames):
        img, lb, u8, stream = sets[k % len(sets)]
        ctx.render_rows_device(cam, 0, H, img.data_ptr(), lb.data_ptr(), u8.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    frames = [ctx.wave_times(k).astype(np.int64) for k in (3, 2, 1, 0)]   # oldest first
    t = frames[-1]
    rec = ctx.block_records()
    st = ctx.read_stats()
# consecutive frames: start / end of each (us, from the oldest frame's first start)
ref0 = frames[0][:, 0].min()
seq = []
for f in frames:
    fs = ((f[:, 0] - ref0 + 2**31) % 2**32) - 2**31
    fe = ((f[:, 1] - ref0 + 2**31) % 2**32) - 2**31
    seq.append((fs.min() / 100.0, fe.max() / 100.0))
ref = t[0, 0]
s = ((t[:, 0] - ref + 2**31) % 2**32) - 2**31
e = ((t[:, 1] - ref + 2**31) % 2**32) - 2**31
live = rec[:, 0] > 0                     # records of waves that rendered rays (fill copies included)
s0 = s.min()
s, e = (s - s0) / 100.0, (e - s0) / 100.0   # us
span = e.max()
dur = e - s
tests = rec[:, 5]
out = {"span_us": float(span), "kernel_ms_read_stats": st.kernel_ms, "records": int(len(t)),
       "last_frames_start_end_us": [[round(a, 2), round(b, 2)] for a, b in seq],
       "next_start_minus_end_us": [round(seq[i + 1][0] - seq[i][1], 2) for i in range(len(seq) - 1)],
       "dur_us_pctl": {p: float(np.percentile(dur[live], p)) for p in (10, 50, 90, 99, 100)},
       "end_pctl_us": {p: float(np.percentile(e[live], p)) for p in (50, 90, 99, 100)},
       "start_pctl_us": {p: float(np.percentile(s[live], p)) for p in (50, 90, 99, 100)}}
bins = np.arange(0.0, span + 1.0, 1.0)
alive = [int(((s <= b + 0.5) & (e > b + 0.5) & live).sum()) for b in bins]
out["alive_per_us"] = alive
groups = {}
for lo, hi in ((0, 1), (1, 5), (5, 20), (20, 60), (60, 10**9)):
    m = live & (tests >= lo) & (tests < hi)
    if m.any():
        groups[f"tests {lo}-{hi}"] = {"waves": int(m.sum()), "dur_us_median": float(np.median(dur[m])),
                                      "dur_us_max": float(dur[m].max())}
out["by_tests"] = groups
slow = np.argsort(-np.where(live, dur, -1.0))[:12]
out["slowest"] = [{"record": int(k), "start_us": round(float(s[k]), 2), "dur_us": round(float(dur[k]), 2),
                   "rays": int(rec[k, 0]), "hit_rays": int(rec[k, 1]), "overflow_rays": int(rec[k, 3]),
                   "hits": int(rec[k, 4]), "tile_tests": int(rec[k, 5]), "candidates": int(rec[k, 6]),
                   "max_hits": int(rec[k, 7])} for k in slow]
# tile workgroups (4 tile waves each, ahead of the fill plan's records): how
# many have no survivor in any of their tiles, and what their waves cost
tile = rec[:, 0] <= 64
n_tile = int(np.argmin(tile)) if not tile.all() else len(rec)
n_wg = n_tile // 4
tt = rec[:n_wg * 4, 5].reshape(n_wg, 4)
dd = dur[:n_wg * 4].reshape(n_wg, 4)
dead_wg = (tt == 0).all(axis=1)
part_wg = (tt == 0).any(axis=1) & ~dead_wg
out["tile_workgroups"] = {"n": n_wg, "all_tiles_without_survivor": int(dead_wg.sum()),
                          "some_tiles_without_survivor": int(part_wg.sum()),
                          "dead_wg_wave_us": float(dd[dead_wg].sum()),
                          "dead_waves_in_mixed_wg_us": float(dd[part_wg][tt[part_wg] == 0].sum()),
                          "all_tile_wave_us": float(dd.sum())}
ov = live & (rec[:, 3] > 0)
out["overflow_waves"] = {"n": int(ov.sum()), "dur_us_median": float(np.median(dur[ov])) if ov.any() else None,
                         "dur_us_sum": float(dur[ov].sum()) if ov.any() else 0.0}
print(json.dumps(out))
