#!/usr/bin/env python3
"""Which path a still camera takes after a moving sweep (device-pointer frames
in flight): per frame, the geometry and pipeline counter deltas, and the
per-frame time of blocks of still frames.

  python tools/still_after_moving.py [--size 2048] [--moving 30] [--still 60]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--moving", type=int, default=30)
    ap.add_argument("--still", type=int, default=60)
    ap.add_argument("--bench-leg", action="store_true")
    ap.add_argument("--extra-contexts", type=int, default=0)
    ap.add_argument("--busy-extra", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch
    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.scenes import orbit_camera
    W = H = args.size
    dev = torch.device("cuda", 0)
    tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    cam = xrt.camera_for_mesh(tris, W, H)
    lo, hi = xrt.mesh_bbox(tris)
    centre = 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64))
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    planes = [(torch.empty(W * H, device=dev), torch.empty(W * H, device=dev),
               torch.empty(W * H, dtype=torch.uint8, device=dev)) for _ in streams]
    extra = []
    for _ in range(args.extra_contexts):   # idle contexts alive beside the probe's (their streams)
        e = xrt.Context(0)
        e.set_kernel(xrt.XRT_KERNEL_BINNED)
        e.upload_mesh(tris)
        if args.busy_extra:                  # as bench.py's main context: a frames-in-flight run, then idle
            sets = [(p_[0].data_ptr(), p_[1].data_ptr(), p_[2].data_ptr(), s_.cuda_stream)
                    for p_, s_ in zip(planes, streams)]
            e.render_frames_device(cam, 0, H, 300, sets)
            torch.cuda.synchronize(dev)
        else:
            e.render_rows(xrt.camera_for_mesh(tris, 64, 64))
        extra.append(e)
    with xrt.Context(0) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(tris)

        def frame(k, cm):
            a, b, u = planes[k % 2]
            c.render_rows_device(cm, 0, H, a.data_ptr(), b.data_ptr(), u.data_ptr(), streams[k % 2].cuda_stream)

        def run(cams, label, per_frame):
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for k, cm in enumerate(cams):
                g0, q0 = c.geometry_counters(), c.pipeline_counters()
                frame(k, cm)
                if per_frame:
                    g1, q1 = c.geometry_counters(), c.pipeline_counters()
                    d = {kk: g1[kk] - g0[kk] for kk in g1 if g1[kk] != g0[kk]}
                    d.update({kk: q1[kk] - q0[kk] for kk in q1 if q1[kk] != q0[kk]})
                    print(f"{label} frame {k}: {d} fill_regions {c.fill_regions()}", flush=True)
            torch.cuda.synchronize(dev)
            print(f"{label}: {(time.perf_counter() - t) / len(cams) * 1e6:.1f} us per frame", flush=True)

        if args.bench_leg:                     # bench.py's orbit leg sequence
            n_ramp = 420
            cams = [orbit_camera(cam, centre, (k - n_ramp) * 1.0) for k in range(n_ramp + 4 + 60)]
            run(cams[:n_ramp + 4], "ramp (moving)", False)
            run(cams[n_ramp + 4:], "timed moving", False)
            run([cams[-1]] * 8, "still, untimed", True)
            run([cams[-1]] * 60, "still, timed", False)
            run([cams[-1]] * 60, "still, timed again", False)
            return
        run([cam] * args.still, "still (fresh)", False)
        run([cam] * args.still, "still (fresh, again)", False)
        run([orbit_camera(cam, centre, k * 1.0) for k in range(args.moving)], "moving", False)
        last = orbit_camera(cam, centre, (args.moving - 1) * 1.0)
        run([last] * 12, "still after moving", True)
        run([last] * args.still, "still after moving, steady", False)
        run([cam] * args.still, "back to the first camera", False)
        run([cam] * args.still, "first camera, steady", False)


if __name__ == "__main__":
    main()
