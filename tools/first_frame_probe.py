#!/usr/bin/env python3
"""A fresh context's first frame (the reference's whole workload is one frame):
per repetition a new context, the mesh uploaded, one device-plane render
synchronised (or, --host, one host-buffer call of the L-buffer) -- its host
call and wall time -- then a second and a third frame
of the same camera.  HIP and the kernels are warmed first by a throwaway
context's 64x64 frame.  Run with XRT_SIZING_PROFILE=1 for the sizing path's
steps (each synchronised).

  python tools/first_frame_probe.py [--size 2048] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tile-mesh", type=int, default=1)
    ap.add_argument("--host", action="store_true", help="host-buffer calls (xrt_render_rows, the L-buffer only)")
    args = ap.parse_args()
    import torch
    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.scenes import tiled_mesh
    W = H = args.size
    dev = torch.device("cuda", 0)
    tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    if args.tile_mesh > 1:
        tris = tiled_mesh(tris, args.tile_mesh)
    cam = xrt.camera_for_mesh(tris, W, H)
    planes = (torch.empty(W * H, device=dev), torch.empty(W * H, device=dev),
              torch.empty(W * H, dtype=torch.uint8, device=dev))
    ptrs = [t.data_ptr() for t in planes]
    s = torch.cuda.current_stream(dev).cuda_stream
    with xrt.Context(0) as w:                      # warm HIP and the kernels
        w.set_kernel(xrt.XRT_KERNEL_BINNED)
        w.upload_mesh(tris)
        w.render_rows(xrt.camera_for_mesh(tris, 64, 64))
    out = []
    for rep in range(args.reps):
        with xrt.Context(0) as c:
            c.set_kernel(xrt.XRT_KERNEL_BINNED)
            c.upload_mesh(tris)
            torch.cuda.synchronize(dev)
            times = []
            for k in range(3):
                t0 = time.perf_counter()
                if args.host:
                    c.render_rows(cam, image=False, lbuffer=True, u8=False)
                else:
                    c.render_rows_device(cam, 0, H, *ptrs, s)
                t1 = time.perf_counter()
                torch.cuda.synchronize(dev)
                t2 = time.perf_counter()
                times.append({"call_ms": round((t1 - t0) * 1e3, 3), "wall_ms": round((t2 - t0) * 1e3, 3),
                              "host_call": c.host_call_ms() if args.host else None})
            g = c.geometry_counters()
            ff = c.first_frames()
        r = {"rep": rep, "frames": times, "sizings": g["sizings"], "first_frames": ff}
        out.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
