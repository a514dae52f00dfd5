#!/usr/bin/env python3
"""Phase timeline of the binning kernels (diagnostics).

    tools/build_variants.sh stamps "-DXRT_STAMPS=1"
    python tools/prep_stamps.py --lib simpleraytracing_amd/lib/ab/libxrt_stamps.so [--size W H]

k_prep stamps per workgroup: 0 start, 1 footprint done, 2 rectangles + scan
done, 3 cell expansion done, 4 pairs copied out (workgroups with pairs).
Times in us relative to the first k_prep
start; per phase: median / max duration over workgroups and the last end.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
TICK_US = 0.01


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--size", type=int, nargs=2, default=[2048, 2048])
    ap.add_argument("--tile-mesh", type=int, default=1)
    args = ap.parse_args()
    import torch

    import simpleraytracing_amd as xrt
    from simpleraytracing_amd import _abi
    from simpleraytracing_amd.scenes import tiled_mesh

    L = _abi._bind(ctypes.CDLL(os.path.abspath(args.lib), mode=ctypes.RTLD_LOCAL), _abi.XRT_SYMBOLS)
    ctx = _abi._CtxP()
    assert L.xrt_create(0, ctypes.byref(ctx)) == 0
    W, H = args.size
    tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    if args.tile_mesh > 1:
        tris = tiled_mesh(tris, args.tile_mesh)
    tris = np.ascontiguousarray(tris)
    cam = xrt.camera_for_mesh(tris, W, H)
    assert L.xrt_upload_mesh(ctx, tris.ctypes.data_as(_abi._fp), tris.shape[0]) == 0
    assert L.xrt_set_kernel(ctx, 3) == 0
    dev = torch.device("cuda", 0)
    img = torch.empty(W * H, dtype=torch.float32, device=dev)
    lb = torch.empty(W * H, dtype=torch.float32, device=dev)
    u8 = torch.empty(W * H, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    for _ in range(5):
        assert L.xrt_render_rows_device(ctx, ctypes.byref(cam), 0, H, ctypes.c_void_p(img.data_ptr()),
                                        ctypes.c_void_p(lb.data_ptr()), ctypes.c_void_p(u8.data_ptr()),
                                        ctypes.c_void_p(stream.cuda_stream)) == 0
    torch.cuda.synchronize()
    n = 1 << 16
    st = np.zeros(n, np.uint64)
    assert L.xrt_debug_stamps(ctx, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n) == 0
    L.xrt_destroy(ctx)
    prep_threads = int(os.environ.get("XRT_PREP_THREADS", "64"))
    prep_tris = int(os.environ.get("XRT_PREP_TRIS", "32"))      # the stamps build's -DXRT_PREP_TRIS
    nwg = max((len(tris) + prep_tris - 1) // prep_tris, (W + H + prep_threads - 1) // prep_threads)
    prep = st[:8 * nwg].reshape(nwg, 8).astype(np.int64)
    t0 = prep[:, 0].min()
    rel = lambda x: (x - t0) * TICK_US  # noqa: E731
    res = {"prep_workgroups": nwg, "prep_start_spread_us": float(rel(prep[:, 0].max()))}
    for k in range(1, 6):
        have = prep[:, k] > 0
        if not have.any():
            continue
        d = (prep[have, k] - prep[have, k - 1 if k != 5 else 4]) * TICK_US
        res[f"phase{k}"] = {"n": int(have.sum()), "med_us": round(float(np.median(d)), 2),
                            "max_us": round(float(d.max()), 2), "last_end_us": round(float(rel(prep[have, k].max())), 2)}
    if (prep[:, 6] > 0).any():          # stamp 6: before the final commit (inside phase 3)
        have = prep[:, 6] > 0
        for name, a, b in (("phase3_expand", 2, 6), ("phase3_commit", 6, 3)):
            d = (prep[have, b] - prep[have, a]) * TICK_US
            res[name] = {"med_us": round(float(np.median(d)), 2), "max_us": round(float(d.max()), 2)}
    scan = st[60000:60004].astype(np.int64)
    res["scan_us"] = [round(float(rel(x)), 2) for x in scan]
    fill = st[32768:32768 + 2 * 4096].reshape(4096, 2).astype(np.int64)
    fill = fill[fill[:, 0] > 0]
    if len(fill):
        res["fill"] = {"blocks": len(fill), "first_start_us": round(float(rel(fill[:, 0].min())), 2),
                       "last_end_us": round(float(rel(fill[:, 1].max())), 2),
                       "dur_med_us": round(float(np.median(fill[:, 1] - fill[:, 0]) * TICK_US), 2),
                       "dur_max_us": round(float((fill[:, 1] - fill[:, 0]).max() * TICK_US), 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
