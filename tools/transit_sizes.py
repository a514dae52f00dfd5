#!/usr/bin/env python3
"""Bytes a frame's row strips send to rank 0 under packed transit (bench.py
--transit packed) against dense L-buffer strips, for an N-way split.

    python tools/transit_sizes.py [--size W H] [--ranks 2 4 8]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, nargs=2, default=[4096, 4096])
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    args = ap.parse_args()
    import torch
    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.strips import strip_bounds
    W, H = args.size
    tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    cam = xrt.camera_for_mesh(tris, W, H)
    dev = torch.device("cuda", 0)
    out = {}
    with xrt.Context(0) as ctx:
        ctx.upload_mesh(tris)
        ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
        ctx.set_miss_code(xrt.XRT_MISS_TRANSIT)
        for n in args.ranks:
            dense = packed = 0
            for g in range(1, n):
                r0, r1 = strip_bounds(H, n, g)
                lb = torch.empty((r1 - r0) * W, device=dev)
                ctx.render_rows_device(cam, r0, r1, 0, lb.data_ptr(), 0, 0)
                _, n_packed = ctx.plan_region_map(W, r1 - r0)
                dense += 4 * (r1 - r0) * W
                packed += 4096 * n_packed
            torch.cuda.synchronize()
            out[n] = {"dense_bytes": dense, "packed_bytes": packed, "ratio": round(dense / max(packed, 1), 2)}
    print(json.dumps({"image": [W, H], "strips": out}))


if __name__ == "__main__":
    main()
