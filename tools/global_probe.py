#!/usr/bin/env python3
"""Which triangles go to the BINNED global list (DESIGN.md "Tile cull" step 5)
and why: their conservative footprints (xrt_probe_prep) -- box, relaxed edges,
the loosened triangle's reach (e2.w; inf for an unbounded footprint) -- and the
region rectangle the box spans.

    python tools/global_probe.py [--size W H] [--tile-mesh n]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, nargs=2, default=[8192, 8192])
    ap.add_argument("--tile-mesh", type=int, default=7)
    ap.add_argument("--global-regions", type=int, default=4096)
    a = ap.parse_args()
    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.scenes import tiled_mesh
    W, H = a.size
    tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    if a.tile_mesh > 1:
        tris = tiled_mesh(tris, a.tile_mesh)
    cam = xrt.camera_for_mesh(tris, W, H)
    with xrt.Context(0) as c:
        c.upload_mesh(tris)
        _, fp = c.probe_prep(cam, len(tris))
    bb = fp[:, 0:4]
    reach = fp[:, 15]                       # e2.w (plane 3 = edge 2)
    rx, ry = -(-W // 32), -(-H // 32)
    xmin = np.clip(bb[:, 0], -64, W + 64)
    xmax = np.clip(bb[:, 1], -64, W + 64)
    ymin = np.clip(bb[:, 2], -64, H + 64)
    ymax = np.clip(bb[:, 3], -64, H + 64)
    ix0 = np.maximum(np.floor((xmin - 31) / 32), 0)
    ix1 = np.minimum(np.floor(xmax / 32), rx - 1)
    iy0 = np.maximum(np.floor((ymin - 31) / 32), 0)
    iy1 = np.minimum(np.floor(ymax / 32), ry - 1)
    ok = (bb[:, 0] <= bb[:, 1]) & (bb[:, 2] <= bb[:, 3]) & (ix0 <= ix1) & (iy0 <= iy1)
    cells = np.where(ok, (ix1 - ix0 + 1) * (iy1 - iy0 + 1), 0)
    big = cells > a.global_regions
    glob = big & ~(reach <= a.global_regions)
    out = {"triangles": len(tris), "regions": rx * ry, "box_over_limit": int(big.sum()), "global": int(glob.sum()),
           "global_unbounded_reach": int((glob & ~np.isfinite(reach)).sum()),
           "walked_slivers": int((big & ~glob).sum()),
           "examples": []}
    for i in np.nonzero(glob)[0][:12]:
        out["examples"].append({"tri": int(i), "box": [round(float(v), 1) for v in bb[i]], "cells": int(cells[i]),
                                "reach": float(reach[i]), "edges": [[float(v) for v in fp[i, 4 + 4 * k:7 + 4 * k]]
                                                                    for k in range(3)],
                                "verts": [float(v) for v in tris[i]]})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
