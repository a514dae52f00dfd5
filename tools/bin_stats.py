#!/usr/bin/env python3
"""Diagnostics: binning statistics of the conservative footprints (dragon, W x W)
-- region count distribution, small/big split, and how well the wave-run
aggregation of k_prep / k_bin_fill merges same-region atomics."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import simpleraytracing_amd as xrt  # noqa: E402

W = H = int(os.environ.get("SIZE", "2048"))
tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
cam = xrt.camera_for_mesh(tris, W, H)
with xrt.Context(0) as ctx:
    ctx.upload_mesh(tris)
    rec, fp = ctx.probe_prep(cam, len(tris))
T = len(tris)
bb = fp[:, :4].astype(np.float64)
E = [fp[:, 4 * k:4 * k + 4].astype(np.float32) for k in (1, 2, 3)]
RX, RY = (W + 31) // 32, (H + 31) // 32
ok = (bb[:, 0] <= bb[:, 1]) & (bb[:, 2] <= bb[:, 3])
xmin = np.maximum(bb[:, 0], -64); xmax = np.minimum(bb[:, 1], W + 64)
ymin = np.maximum(bb[:, 2], -64); ymax = np.minimum(bb[:, 3], H + 64)
ok &= ~((xmax < 0) | (ymax < 0) | (xmin > W) | (ymin > H))
ix0 = np.maximum(np.floor((xmin - 31) / 32), 0); ix1 = np.minimum(np.floor(xmax / 32), RX - 1)
iy0 = np.maximum(np.floor((ymin - 31) / 32), 0); iy1 = np.minimum(np.floor(ymax / 32), RY - 1)
ok &= (ix0 <= ix1) & (iy0 <= iy1)
area = np.where(ok, (ix1 - ix0 + 1) * (iy1 - iy0 + 1), 0)
print("T", T, "no region", int((~ok).sum()), "area pct 50/90/99/max", np.percentile(area[ok], [50, 90, 99, 100]))
print("big (>16 regions)", int((area > 16).sum()), "sum big area", int(area[area > 16].sum()))


def edge_pass(j, xc, yc, h):
    for e in E:
        a, b, c = e[j, 0], e[j, 1], e[j, 2]
        if (a * np.float32(xc) + b * np.float32(yc)) + (c + (abs(a) * np.float32(h) + abs(b) * np.float32(h))) < 0:
            return False
    return True


counts = np.zeros(RX * RY, np.int64)
small = [[] for _ in range(T)]
for j in np.nonzero(ok)[0]:
    for ry in range(int(iy0[j]), int(iy1[j]) + 1):
        for rx in range(int(ix0[j]), int(ix1[j]) + 1):
            if edge_pass(j, rx * 32 + 15.5, ry * 32 + 15.5, 15.5):
                counts[ry * RX + rx] += 1
                if area[j] <= 16:
                    small[j].append(ry * RX + rx)
print("pairs", int(counts.sum()), "regions nonempty", int((counts > 0).sum()), "of", RX * RY,
      "count pct 50/90/99/max", np.percentile(counts[counts > 0], [50, 90, 99, 100]))
# run aggregation: per wave (64 consecutive triangles) and slot k
atoms = 0
runs_per_region = np.zeros(RX * RY, np.int64)
for w0 in range(0, T, 64):
    for k in range(16):
        prev = None
        for j in range(w0, min(T, w0 + 64)):
            r = small[j][k] if k < len(small[j]) else None
            if r is not None and r != prev:
                atoms += 1
                runs_per_region[r] += 1
            prev = r
print("small pairs", sum(len(s) for s in small), "atomics after run aggregation", atoms,
      "max atomics on one region", int(runs_per_region.max()))
