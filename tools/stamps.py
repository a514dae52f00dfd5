#!/usr/bin/env python3
"""Workgroup timeline of one culled render (diagnostics).

    tools/build_variants.sh stamps "-DXRT_STAMPS=1"
    python tools/stamps.py --lib simpleraytracing_amd/lib/ab/libxrt_stamps.so --kernel binned

The XRT_STAMPS build stores each workgroup's s_memrealtime start/end (100 MHz),
XCC id and HW_ID in its BlockStats record; this renders a few frames, reads the
last frame's records (xrt_debug_block_records) and prints the span, the
duration distribution, the concurrency profile and the tail.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REC = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("hits", "<u4"), ("tile_tests", "<u4"),
                ("hwid", "<u4"), ("xcc", "<u4")])
TICK_US = 0.01   # s_memrealtime runs at 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--kernel", default="binned")
    ap.add_argument("--size", type=int, nargs=2, default=[2048, 2048])
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--out", default=None, help="write the raw records (.npy)")
    args = ap.parse_args()

    import torch

    import simpleraytracing_amd as xrt
    from simpleraytracing_amd import _abi

    L = _abi._bind(ctypes.CDLL(os.path.abspath(args.lib), mode=ctypes.RTLD_LOCAL), _abi.XRT_SYMBOLS)
    ctx = _abi._CtxP()
    assert L.xrt_create(0, ctypes.byref(ctx)) == 0
    W, H = args.size
    tris = np.ascontiguousarray(xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply")))
    cam = xrt.camera_for_mesh(tris, W, H)
    assert L.xrt_upload_mesh(ctx, tris.ctypes.data_as(_abi._fp), tris.shape[0]) == 0
    kid = {"brute": 1, "tiled": 2, "binned": 3}[args.kernel]
    assert L.xrt_set_kernel(ctx, kid) == 0
    dev = torch.device("cuda", 0)
    img = torch.empty(W * H, dtype=torch.float32, device=dev)
    lb = torch.empty(W * H, dtype=torch.float32, device=dev)
    u8 = torch.empty(W * H, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    for _ in range(args.frames):
        rc = L.xrt_render_rows_device(ctx, ctypes.byref(cam), 0, H, ctypes.c_void_p(img.data_ptr()),
                                      ctypes.c_void_p(lb.data_ptr()), ctypes.c_void_p(u8.data_ptr()),
                                      ctypes.c_void_p(stream.cuda_stream))
        assert rc == 0, L.xrt_last_error(ctx)
    torch.cuda.synchronize()
    n = _abi._u64()
    L.xrt_debug_block_records(ctx, None, 0, ctypes.byref(n))
    recs = np.zeros(n.value, dtype=REC)
    assert L.xrt_debug_block_records(ctx, recs.ctypes.data_as(ctypes.c_void_p), recs.nbytes,
                                     ctypes.byref(n)) == 0
    L.xrt_destroy(ctx)
    if args.out:
        np.save(args.out, recs)

    recs = recs[recs["t0"] != 0]        # the fill plan's padding records (no wave behind them)
    t0 = recs["t0"].astype(np.int64)
    t1 = recs["t1"].astype(np.int64)
    base = t0.min()
    s = (t0 - base) * TICK_US
    e = (t1 - base) * TICK_US
    d = e - s
    work = recs["tile_tests"].astype(np.int64)
    hw = recs["hwid"]
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    xcc = recs["xcc"] & 15
    span = e.max()
    order = np.argsort(e)
    res = {
        "blocks": int(len(recs)),
        "span_us": round(float(span), 2),
        "start_last_us": round(float(s.max()), 2),
        "end_p50_us": round(float(np.percentile(e, 50)), 2),
        "end_p90_us": round(float(np.percentile(e, 90)), 2),
        "end_p99_us": round(float(np.percentile(e, 99)), 2),
        "dur_us_p50_p90_p99_max": [round(float(np.percentile(d, q)), 2) for q in (50, 90, 99, 100)],
        "dur_us_zero_work_p50": round(float(np.median(d[work == 0])), 2) if (work == 0).any() else None,
        "dur_us_top_work": [[int(work[i]), round(float(d[i]), 2), round(float(s[i]), 2)]
                            for i in np.argsort(-work)[:8]],
        "work_total": int(work.sum()),
        "work_max": int(work.max()),
        "blocks_with_work": int((work > 0).sum()),
        "last_blocks": [[int(i), int(work[i]), round(float(s[i]), 2), round(float(e[i]), 2)]
                        for i in order[-8:]],
        "per_xcc_span_us": {int(x): round(float(e[xcc == x].max() - s[xcc == x].min()), 2)
                            for x in np.unique(xcc)},
        "distinct_cus": int(len(np.unique(xcc.astype(np.int64) * 1024 + se * 64 + cu))),
    }
    grid = np.linspace(0, span, 41)
    res["concurrent_blocks"] = [int(((s <= g) & (e > g)).sum()) for g in grid[:-1]]
    # busy fraction: sum of block durations / (span x average resident slots)
    res["sum_block_us"] = round(float(d.sum()), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
