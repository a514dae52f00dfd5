#!/usr/bin/env python3
"""Multi-GPU model inputs for bench.py's strips mode, measured on one GPU:
for an N-way split of the frame (the root-weighted split bench.py uses by
default, strips.root_share, and the reference's equal H/N split), each strip's
render time (its own context, steady frames, in-kernel spans) and the bytes its
strip sends to rank 0 -- packed L-buffer blocks, or the hit layout (a 64-bit
mask per tile of the packed regions and 4 B per hit ray, xrt_set_transit_hits,
with the strip's render into that layout timed as well) -- against dense
strips.  --transit picks the bytes the balanced split and the predicted step
use.  The predicted
step per link rate is max(root strip render + unpack, slowest sender render,
largest sender transfer) -- the gather of frame k overlaps the render of frame
k+1, each sender has its own link into rank 0 (DESIGN.md "Multi-GPU").

    python tools/transit_sizes.py [--size W H] [--tile-mesh n] [--ranks 1 2 4 8] [--link-gbs 64 128]
                                  [--splits weighted equal balanced capi] [--ramp-ms 50]
                                  [--transit packed|hits]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def strip_time_ms(xrt, torch, tris, cam, r0, r1, W, frames, miss_code, ramp_ms=0.0):
    """(render ms, packed regions, hit rays, hit-layout words, render ms into the
    hit layout or None) of strip [r0, r1)."""
    dev = torch.device("cuda", 0)
    with xrt.Context(0) as ctx:
        ctx.upload_mesh(tris)
        ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
        if miss_code:
            ctx.set_miss_code(xrt.XRT_MISS_TRANSIT)
        lb = torch.empty((r1 - r0) * W, device=dev)
        img = torch.empty((r1 - r0) * W, device=dev) if not miss_code else None
        u8 = torch.empty((r1 - r0) * W, dtype=torch.uint8, device=dev) if not miss_code else None
        args = (img.data_ptr() if img is not None else 0, lb.data_ptr(), u8.data_ptr() if u8 is not None else 0)
        for _ in range(5):
            ctx.render_rows_device(cam, r0, r1, *args, 0)
        torch.cuda.synchronize()
        if ramp_ms > 0:                     # loaded clocks (DESIGN.md "Measurement"): keep the GPU busy first
            t0 = time.perf_counter()
            while (time.perf_counter() - t0) * 1e3 < ramp_ms:
                for _ in range(20):
                    ctx.render_rows_device(cam, r0, r1, *args, 0)
                torch.cuda.synchronize()
        ctx.timing_begin()
        for _ in range(frames):
            ctx.render_rows_device(cam, r0, r1, *args, 0)
        torch.cuda.synchronize()
        ms, n = ctx.timing_end()
        _, n_packed = ctx.plan_region_map(W, r1 - r0)
        hit_rays = ctx.read_stats().hit_rays
        words, ms_hits = None, None
        if miss_code:                       # a sender: its hit plan, then frames into the hit layout
            try:
                _, words = ctx.plan_hit_layout()
            except RuntimeError:
                words = None
        if words is not None:
            msg = torch.empty(max(words, 4) + 64, device=dev)
            ctx.set_transit_hits(msg.numel())
            for _ in range(3):
                ctx.render_rows_device(cam, r0, r1, 0, msg.data_ptr(), 0, 0)
            torch.cuda.synchronize()
            ctx.timing_begin()
            for _ in range(frames):
                ctx.render_rows_device(cam, r0, r1, 0, msg.data_ptr(), 0, 0)
            torch.cuda.synchronize()
            mh, nh = ctx.timing_end()
            ms_hits = mh / max(nh, 1)
            ctx.set_transit_hits(0)
    return ms / max(n, 1), n_packed, hit_rays, words, ms_hits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, nargs=2, default=[4096, 4096])
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--link-gbs", type=float, nargs="+", default=[64.0, 128.0])
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--tile-mesh", type=int, default=1, help="n x n tiled copies (7 = BASELINE configs[4])")
    ap.add_argument("--splits", nargs="+", default=["weighted", "equal", "balanced", "capi"],
                    help="balanced: bench.py's band model through strips.balanced_bounds; capi: the strips the C "
                         "ABI's xrt_multi_plan picks itself (its own frame model), both per --link-gbs")
    ap.add_argument("--ramp-ms", type=float, default=50.0, help="GPU kept busy with the strip before timing it")
    ap.add_argument("--transit", choices=["packed", "hits"], default="hits",
                    help="the bytes behind the balanced split and the predicted step")
    args = ap.parse_args()
    import torch
    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.strips import root_share, strip_bounds, weighted_bounds
    W, H = args.size
    tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    if args.tile_mesh > 1:
        from simpleraytracing_amd.scenes import tiled_mesh
        tris = tiled_mesh(tris, args.tile_mesh)
    cam = xrt.camera_for_mesh(tris, W, H)
    import bench
    from simpleraytracing_amd.strips import balanced_bounds
    band_cost, band_bytes, _ = bench.band_model(xrt, torch, tris, cam, W, H, 0, transit=args.transit)
    out = {}
    splits = [s for s in ("weighted", "equal") if s in args.splits]
    if "balanced" in args.splits:
        splits += [f"balanced@{g:g}" for g in args.link_gbs]
    if "capi" in args.splits:
        splits += [f"capi@{g:g}" for g in args.link_gbs]
    for split in splits:
        for n in args.ranks:
            if split != "weighted" and n == 1:
                continue
            share0 = root_share(n)
            plan = None
            if split.startswith("balanced@"):
                link = float(split.split("@")[1]) * 1e3           # GB/s -> bytes/us
                bounds = balanced_bounds(band_cost, band_bytes, n, link, H)
            elif split.startswith("capi@"):                       # the product path's own plan
                link = float(split.split("@")[1]) * 1e3
                with xrt.MultiContext([0] * n) as m:
                    m.set_kernel(xrt.XRT_KERNEL_BINNED)
                    m.upload_mesh(tris)
                    m.set_split(xrt.XRT_SPLIT_BALANCED, link)
                    m.set_transit(xrt.XRT_TRANSIT_HITS if args.transit == "hits" else xrt.XRT_TRANSIT_PACKED)
                    bounds, plan = m.plan(cam)
            else:
                bounds = [weighted_bounds(H, n, g, share0) if split == "weighted" else strip_bounds(H, n, g)
                          for g in range(n)]
            ranks = []
            for g, (r0, r1) in enumerate(bounds):
                ms, n_packed, hit_rays, words, ms_hits = strip_time_ms(xrt, torch, tris, cam, r0, r1, W, args.frames,
                                                                       miss_code=g > 0, ramp_ms=args.ramp_ms)
                # hit_bytes: the hit layout's message as built (xrt_plan_hit_layout's words, at least 4)
                ranks.append({"rows": r1 - r0, "render_us": round(ms * 1e3, 2),
                              "render_us_hit_layout": round(ms_hits * 1e3, 2) if ms_hits is not None else None,
                              "packed_bytes": 4096 * n_packed if g else 0, "dense_bytes": 4 * (r1 - r0) * W if g else 0,
                              "hit_rays": hit_rays,
                              "hit_bytes": 4 * max(words, 4) if g and words is not None else 0})
            senders = ranks[1:]
            unpack_us = 0.0 if n == 1 else 5.0       # one unpack launch (measured ~5 us at 4096^2)
            key = "hit_bytes" if args.transit == "hits" else "packed_bytes"
            rkey = "render_us_hit_layout" if args.transit == "hits" else "render_us"
            pred = {"bytes_into_root": sum(s[key] for s in senders),
                    "packed_bytes_into_root": sum(s["packed_bytes"] for s in senders),
                    "hit_bytes_into_root": sum(s["hit_bytes"] for s in senders)}
            for gbs in args.link_gbs:
                transfer = max((s[key] / (gbs * 1e3) for s in senders), default=0.0)
                step = max(ranks[0]["render_us"] + unpack_us,
                           max((s[rkey] or s["render_us"] for s in senders), default=0.0), transfer)
                pred[f"{gbs:g}GBs"] = {"step_us": round(step, 1), "transfer_us": round(transfer, 1),
                                       "mrays_s": round(W * H / step, 0) if step else None}
            out[f"{split}_{n}"] = {"ranks": ranks, "bounds": bounds, "predicted": pred, "plan": plan}
    print(json.dumps({"image": [W, H], "triangles": len(tris), "ramp_ms": args.ramp_ms, "transit": args.transit,
                      "splits": out}))


if __name__ == "__main__":
    main()
