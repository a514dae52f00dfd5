#!/usr/bin/env python3
"""Diagnostics: a fresh context's first host-buffer render right after a
frames-in-flight loop (DESIGN.md "Measurement", round 4's in-process stall).

    python tools/stall_probe.py [--streams 1|2] [--null] [--frames 400] [--size 2048]

Renders --frames frames of dragon.ply alternating --streams torch streams
(--null: the first is the null stream, as the bench's frame 0), synchronises,
then creates two fresh contexts one after the other and prints the host-call
breakdown of each one's first xrt_render_rows (XRT_SIZING_PROFILE=1 adds the
sizing path's steps, each synchronised, on stderr)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--null", action="store_true")
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="sleep between the loop and the fresh contexts")
    args = ap.parse_args()
    import torch

    import simpleraytracing_amd as xrt
    W = H = args.size
    dev = torch.device("cuda", 0)
    tris = xrt.load_ply(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data",
                                     "dragon.ply"))
    cam = xrt.camera_for_mesh(tris, W, H)
    streams = [torch.cuda.current_stream(dev) if (args.null and i == 0) else torch.cuda.Stream(dev)
               for i in range(args.streams)]
    sets = [(torch.empty(W * H, device=dev), torch.empty(W * H, device=dev),
             torch.empty(W * H, dtype=torch.uint8, device=dev)) for _ in streams]
    out = {"streams": args.streams, "null": args.null, "frames": args.frames,
           "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
    with xrt.Context(0) as c:
        c.upload_mesh(tris)
        t0 = time.perf_counter()
        for k in range(args.frames):
            a, b, u = sets[k % len(sets)]
            c.render_rows_device(cam, 0, H, a.data_ptr(), b.data_ptr(), u.data_ptr(),
                                 streams[k % len(streams)].cuda_stream)
        torch.cuda.synchronize(dev)
        out["loop_ms_per_frame"] = (time.perf_counter() - t0) / max(args.frames, 1) * 1e3
        if args.idle_ms:
            time.sleep(args.idle_ms / 1e3)
        for name in ("first", "second"):
            t_c = time.perf_counter()
            with xrt.Context(0) as f:
                create = (time.perf_counter() - t_c) * 1e3
                f.upload_mesh(tris)
                t1 = time.perf_counter()
                f.render_rows(cam)
                out[name] = {"create_ms": round(create, 3), "render_rows_ms": round((time.perf_counter() - t1) * 1e3, 3),
                             "breakdown": {k: round(v, 3) for k, v in f.host_call_ms().items()}}
            print(f"--- {name} fresh context done", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
