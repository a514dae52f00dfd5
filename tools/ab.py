#!/usr/bin/env python3
"""A/B timing of libxrt.so variants, interleaved in one process on one GPU.

    python tools/ab.py --variants name1=path/libxrt.so name2=... [--kernel tiled]
                       [--size 2048 2048] [--rounds 7] [--frames 10]

Each round renders `frames` frames with every variant in turn (device buffers,
HIP-event kernel time via xrt_timing_begin/end); prints the median and min
kernel time per variant.  Variants are separate builds of the same ABI
(tools/build_variants.sh), loaded side by side with RTLD_LOCAL.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--kernel", default="tiled")
    ap.add_argument("--size", type=int, nargs=2, default=[2048, 2048])
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--tile-mesh", type=int, default=1)
    args = ap.parse_args()

    import numpy as np
    import torch

    import simpleraytracing_amd as xrt
    from simpleraytracing_amd import _abi
    from simpleraytracing_amd.scenes import tiled_mesh

    kid = {"auto": 0, "brute": 1, "tiled": 2, "binned": 3}[args.kernel]
    W, H = args.size
    tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    if args.tile_mesh > 1:
        tris = tiled_mesh(tris, args.tile_mesh)
    cam = xrt.camera_for_mesh(tris, W, H)
    dev = torch.device("cuda", 0)
    img = torch.empty(W * H, dtype=torch.float32, device=dev)
    lb = torch.empty(W * H, dtype=torch.float32, device=dev)
    u8 = torch.empty(W * H, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    libs = []
    for spec in args.variants:
        name, path = spec.split("=", 1)
        need = ["xrt_create", "xrt_last_error", "xrt_upload_mesh", "xrt_set_kernel",
                "xrt_render_rows_device", "xrt_timing_begin", "xrt_timing_end"]
        L = _abi._bind(ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL),
                       {k: _abi.XRT_SYMBOLS[k] for k in need})
        ctx = _abi._CtxP()
        assert L.xrt_create(0, ctypes.byref(ctx)) == 0, L.xrt_last_error(None)
        t = np.ascontiguousarray(tris)
        assert L.xrt_upload_mesh(ctx, t.ctypes.data_as(_abi._fp), len(t)) == 0
        assert L.xrt_set_kernel(ctx, kid) == 0
        libs.append((name, L, ctx))

    ref = None
    times = {name: [] for name, _, _ in libs}
    for r in range(args.rounds + 1):
        for name, L, ctx in libs:
            L.xrt_timing_begin(ctx)
            for _ in range(args.frames):
                rc = L.xrt_render_rows_device(ctx, ctypes.byref(cam), 0, H, img.data_ptr(), lb.data_ptr(),
                                              u8.data_ptr(), stream.cuda_stream)
                assert rc == 0, L.xrt_last_error(ctx)
            ms = ctypes.c_double()
            n = ctypes.c_uint64()
            L.xrt_timing_end(ctx, ctypes.byref(ms), ctypes.byref(n))
            torch.cuda.synchronize(dev)
            if r > 0:   # round 0 is warm-up
                times[name].append(ms.value / n.value)
            out = img.cpu().numpy().view(np.uint32)
            csum = int(out.astype(np.uint64).sum())
            if r == 0:
                pass                       # warm-up round: not timed, not compared
            elif ref is None:
                ref = csum
            elif csum != ref:
                print(f"WARNING: round {r} variant {name} checksum {csum} != {ref}", file=sys.stderr)
            img.fill_(-1.0)
    res = {name: {"median_ms": statistics.median(v), "min_ms": min(v)} for name, v in times.items()}
    print(json.dumps({"kernel": args.kernel, "size": [W, H], "results": res}))


if __name__ == "__main__":
    main()
