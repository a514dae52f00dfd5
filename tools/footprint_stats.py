#!/usr/bin/env python3
"""Diagnostics: distribution of conservative footprint sizes (dragon, W x W)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import simpleraytracing_amd as xrt
W = H = int(os.environ.get("SIZE", "2048"))
tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
cam = xrt.camera_for_mesh(tris, W, H)
with xrt.Context(0) as ctx:
    ctx.upload_mesh(tris)
    rec, fp = ctx.probe_prep(cam, len(tris))
bb = fp[:, :4]
w = bb[:, 1] - bb[:, 0]
h = bb[:, 3] - bb[:, 2]
fin = np.isfinite(w) & np.isfinite(h) & (w >= 0)
print("T", len(tris), "finite boxes", fin.sum(), "empty", int((w < 0).sum()), "infinite", int((~np.isfinite(w)).sum()))
print("width pct 50/90/99/99.9/max", np.percentile(w[fin], [50, 90, 99, 99.9, 100]))
print("height pct", np.percentile(h[fin], [50, 90, 99, 99.9, 100]))
nreg = (np.floor(bb[:, 1] / 32) - np.floor((bb[:, 0] - 31) / 32) + 1) * (np.floor(bb[:, 3] / 32) - np.floor((bb[:, 2] - 31) / 32) + 1)
big = np.nonzero(fin & (nreg > 64))[0]
print("footprints over > 64 regions:", len(big))
for j in big[:12]:
    print(" tri", j, "box", bb[j], "edges", fp[j, 4:7], fp[j, 8:11], fp[j, 12:15], "tnum", rec[j, 12])
