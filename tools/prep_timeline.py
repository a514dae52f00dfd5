"""k_prep's wave timeline (xrt_debug_prep_times): where its time goes.

Per wave k_prep records s_memrealtime (100 MHz) at its start, after its
records and footprints, after its cell tests (binning phase 1) and at its end.
This prints, for k_prep running alone (a host-buffer frame: nothing beside it)
and beside the renders of a frames-in-flight loop (the bench's pipeline): the
span, when its waves start (launch ramp: waiting for wave slots) and how long
each phase of a wave takes, as percentiles in microseconds, and the renders'
spans on the same clock.

  python tools/prep_timeline.py [--size W H] [--tile-mesh n] [--frames N] [--inflight F]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(x):
    return {f"p{q}": round(float(np.percentile(x, q)), 2) for q in (0, 10, 50, 90, 100)} if len(x) else {}


PHASES = ["load_record", "footprint", "stage_scan", "union", "cells_small", "cells_large", "commit_stores"]


def summary(t, label):
    t = t.astype(np.int64)
    ref = t[:, 0].min()
    rel = (t - ref) % 2**32 / 100.0                       # us from the first wave's start
    start, end = rel[:, 0], rel[:, 7]
    out = {"what": label, "waves": int(len(t)), "span_us": round(float(end.max()), 2),
           "start_us": pct(start), "wave_us": pct(end - start)}
    valid = (t[:, 1:7] != 0).all(axis=1)
    for k, name in enumerate(PHASES):
        if valid.any():
            out[name + "_us"] = pct((rel[:, k + 1] - rel[:, k])[valid])
    return out, ref


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, nargs=2, default=(2048, 2048))
    ap.add_argument("--tile-mesh", type=int, default=1)
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--inflight", type=int, default=None)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.scenes import tiled_mesh

    W, H = args.size
    dev = torch.device("cuda", 0)
    tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    if args.tile_mesh > 1:
        tris = tiled_mesh(tris, args.tile_mesh)
    cam = xrt.camera_for_mesh(tris, W, H)
    inflight = args.inflight or (2 if W * H <= 2048 * 2048 else 1)
    res = {"size": [W, H], "triangles": int(len(tris)), "inflight": inflight}
    with xrt.Context(0) as ctx:
        ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
        ctx.upload_mesh(tris)
        ctx.render_rows(cam)                             # sizing
        ctx.prep_times(True)
        for rep in range(3):                             # alone: a host-buffer frame's k_prep, nothing beside it
            torch.cuda.synchronize(dev)
            ctx.render_rows(cam)
            s, _ = summary(ctx.prep_times(), f"alone (host-buffer frame), rep {rep}")
            res.setdefault("alone", []).append(s)
        planes = [(torch.zeros(W * H, device=dev), torch.zeros(W * H, device=dev),
                   torch.zeros(W * H, dtype=torch.uint8, device=dev),
                   torch.cuda.current_stream(dev) if f == 0 else torch.cuda.Stream(dev)) for f in range(inflight)]
        sets = [(a.data_ptr(), b.data_ptr(), c.data_ptr(), s.cuda_stream) for a, b, c, s in planes]
        ctx.render_frames_device(cam, 0, H, args.frames, sets)
        torch.cuda.synchronize(dev)
        s, ref = summary(ctx.prep_times(), f"beside the renders ({inflight} in flight, last k_prep of "
                                           f"{args.frames} frames)")
        renders = []
        for back in range(4):
            wt = ctx.wave_times(back).astype(np.int64)
            renders.append({"frames_back": back, "start_us": round(float(((wt[:, 0] - ref) % 2**32).min()) / 100 if
                                                               ((wt[:, 0] - ref) % 2**32).min() < 2**31 else
                                                               -float(((ref - wt[:, 0]) % 2**32).min()) / 100, 2),
                            "span_us": round(float(((wt[:, 1] - wt[:, 0].min()) % 2**32).max()) / 100, 2)})
        s["renders_relative_to_prep_start"] = renders
        res["beside"] = s
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
