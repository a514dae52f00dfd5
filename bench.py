#!/usr/bin/env python3
"""bench.py -- Mrays/s of the X-ray render path (BASELINE.json metric).

A step renders one frame (default dragon.ply; outputs f32 image + f32
L-buffer + u8 image, every ray against the mesh through the exact
Moller-Trumbore test of its culled candidates).  The mesh is resident in HBM
before the timed region; the per-frame triangle preparation (binning) and the
render are inside it.

  one GPU (default): dragon.ply 2048x2048 frames (BASELINE configs[2]), two
                 frames in flight for frames up to 2048x2048 (--inflight:
                 frame k on stream k % 2 into its own output planes; both
                 checked bit for bit after timing).  Before the timed
                 region: W untimed steps (the first frame, with its list
                 sizing, and W - 1 warm-up steps), nothing else unless
                 --ramp-ms asks for it.  After it, --loaded-ms of untimed
                 steps and K more timed steps give the rate at the GPU's
                 loaded clocks (at_loaded_clocks, reported beside `value`).
  --gpus N > 1 (default --mode strips, 4096x4096: BASELINE configs[3]):
                 strong scaling -- one frame per step split into row strips
                 (--root-share balanced: from the frame's per-band render cost
                 and transit bytes, strips.balanced_bounds; 'equal': H/N, as
                 main-pthreads-rows.cxx:311-334); every rank but 0 sends its
                 strip to rank 0 over RCCL (--transit hits: per 8x8 tile a hit
                 mask and the hit rays' L values; packed / dense as named),
                 which expands it into its frame's three planes; frame k's
                 gather overlaps frame k+1's render.  The gathered frame is
                 checked bit for bit against rank 0's own single-device render
                 after timing.
  --mode frames  weak scaling: every rank renders whole frames, no exchange.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size W H]
                    [--kernel auto|binned|tiled|brute] [--mode frames|strips]
                    [--tile-mesh n] [--no-cpu-baseline] [--dist-backend nccl|gloo]

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import datetime
import gc
import json
import traceback
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
BYTES_PER_TEST = 36            # 9 f32 vertex operands per ray-triangle test
BYTES_OUT_PER_RAY = 9          # L f32 + image f32 + u8
VALU_PEAK_WAVE_INSTR_S = 256 * 4 * 2.4e9 / 2   # CUs x SIMDs x clock / 2 cycles per wave64 VALU op


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--size", type=int, nargs=2, default=None, metavar=("W", "H"),
                    help="default 2048 2048; 4096 4096 for strips over N > 1 GPUs (BASELINE configs[3])")
    ap.add_argument("--kernel", choices=["auto", "binned", "tiled", "brute"], default="auto")
    ap.add_argument("--model", choices=["attenuation", "signed"], default="attenuation",
                    help="signed: the L-buffer fork (main-pthreads-lbuffer.cxx) -- signed L-buffer render "
                         "+ hole fill per step (frames mode; not the headline metric)")
    ap.add_argument("--mode", choices=["frames", "strips"], default=None,
                    help="default: frames on one GPU, strips over N > 1")
    ap.add_argument("--mesh", default=os.path.join(ROOT, "data", "dragon.ply"))
    ap.add_argument("--tile-mesh", type=int, default=1,
                    help="n x n tiled copies of the mesh (7 = the 1M-triangle config)")
    ap.add_argument("--orbit", type=float, default=0.0, metavar="DEG",
                    help="frames mode: frame k's camera is the default one turned k*DEG degrees about the "
                         "detector's up axis through the mesh centre (a projection sweep: every frame a "
                         "new geometry for the region lists); 0 = one camera")
    ap.add_argument("--orbit-legs", type=float, nargs="*", default=[0.25, 1.0], metavar="DEG",
                    help="after the timed region (one GPU, frames mode): a moving-camera leg per value, the camera "
                         "turning DEG degrees per frame (reported under `orbit`, never `value`); none: no legs")
    ap.add_argument("--no-tile-plan-leg", action="store_true",
                    help="skip the opt-in tile plan's leg after the timed region (counter runs: its renders differ)")
    ap.add_argument("--orbit-ramp-ms", type=float, default=30.0,
                    help="untimed moving frames before each orbit leg's timed ones, ms of sustained load")
    ap.add_argument("--orbit-frames", type=int, default=60,
                    help="timed frames per orbit leg (after 4 untimed ones)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL over xGMI (production); gloo = CPU-staged, for rehearsing "
                         "N ranks on fewer GPUs")
    ap.add_argument("--transit", choices=["hits", "packed", "dense"], default="hits",
                    help="strips mode: send per tile of the strip's fill plan a hit mask and the hit rays' L "
                         "values (hits), the regions the fill plan did not fill (packed) or the whole L-buffer "
                         "strip (dense)")
    ap.add_argument("--root-share", default="balanced",
                    help="strips mode: 'balanced' (default): strips from the frame's measured per-band render "
                         "cost and packed bytes and the measured link rate (strips.balanced_bounds); or the "
                         "fraction of the rows rank 0 renders first ('auto': strips.root_share, "
                         "'equal': H/N each as the reference's row partition)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank uses device 0 (with --dist-backend gloo)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU time of the bounded cpu_baseline sample")
    ap.add_argument("--inflight", type=int, default=None, metavar="F",
                    help="frames mode: frame k renders on stream k %% F into output planes k %% F, so a "
                         "frame's render can start while the previous frame's last waves run (default 2 "
                         "for frames of up to 2048x2048 pixels, else 1; strips mode: 1)")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the end-to-end latency windows (a child process; profiling runs)")
    ap.add_argument("--ramp-ms", type=float, default=0.0,
                    help="opt-in: untimed frames for this long after the warm-up, so the timed region runs at "
                         "the GPU's loaded clocks (default 0: the K timed steps follow the W warm-up steps "
                         "directly); with it, the first min(K, 20) frames after the warm-up are timed before "
                         "it and reported as before_clock_ramp")
    ap.add_argument("--loaded-ms", type=float, default=100.0,
                    help="after the timed region (never inside `value`): keep the GPU loaded this long, then "
                         "time K more steps, reported beside the headline as at_loaded_clocks (0: skip)")
    ap.add_argument("--host-loop", choices=["batch", "python"], default="batch",
                    help="frames mode, one camera: 'batch' (default) enqueues a run of steps in one "
                         "xrt_render_frames_device call; 'python' calls xrt_render_rows_device once per step")
    ap.add_argument("--capi-multi", choices=["auto", "off"], default="auto",
                    help="strips mode over N > 1 ranks: after the torch path, rank 0 also times the C ABI's own "
                         "multi-GPU entry (xrt_render_rows_multi_device over devices 0..N-1 in ONE process, RCCL "
                         "gather, the split of xrt_multi_set_split) in a child process, reported as capi_multi")
    ap.add_argument("--capi-devices", default=None, metavar="LIST",
                    help="devices of the capi_multi leg, e.g. 0,0,0,0,0,0,0,0 (one GPU listed 8 times: a one-rank "
                         "RCCL rehearsal); runs the leg in any mode")
    ap.add_argument("--capi-split", choices=["balanced", "equal"], default="balanced")
    ap.add_argument("--capi-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--e2e-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--e2e-device", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--no-timing-check", action="store_true",
                    help="profiling runs of a few steps: skip the avg_kernel_ms <= ms_per_step check")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM bytes from rocprofv3 PMC runs (see DESIGN.md)")
    return ap.parse_args()


def cpu_baseline(tris, cam, W, H, budget_s, gpu_rows):
    """The CPU path timed on the box's host cores, on bounded samples of the same
    frame, each checked bit for bit against the planes the timed loop's last
    frame left on the GPU:

      kind "reference" (when oracle/_ref is built): the reference's own
        src/Ray.cxx, Triangle.cxx and TriangleMesh.cxx (compiled unmodified,
        -O2) driven by renderLoop's per-pixel loop (oracle/ref_harness.cpp),
        spans of rows on every host thread over one shared mesh -- the
        structure of main-pthreads-redo.cxx;
      kind "port": oracle/xrt_oracle.c (the C restatement of the same loop)
        threaded over 64-px blocks.

    Half of `budget_s` each; their single-thread rates beside them."""
    import numpy as np

    from oracle import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    cam = np.array(list(cam.origin) + list(cam.detector) + list(cam.up) + list(cam.right) + [cam.pixel_spacing],
                   np.float32)                         # the oracle's 13-float camera
    g_img, g_lb, g_u8 = (np.asarray(a).reshape(H, W) for a in gpu_rows)
    ref = oracle.ref_lib()
    share = budget_s / 2 if ref is not None else budget_s
    # serial rate on a span of one row (the reference main.cxx is single-threaded),
    # sized to about 1 s
    mid = H // 2
    span = int(max(8, min(W, 6.0e7 / max(len(tris), 1))))
    c0 = (W - span) // 2
    t0 = time.perf_counter()
    oracle.render_span(tris, cam, W, H, mid, c0, c0 + span, threads=1)
    serial_s = time.perf_counter() - t0
    serial_rate = span / serial_s
    # threaded sample sized to the budget
    est_rate = serial_rate * threads
    nrows = int(max(1, min(H, share * est_rate / W)))
    rows = np.unique(np.linspace(0, H - 1, nrows).astype(np.uint32))
    t0 = time.perf_counter()
    img, lb, u8, nh, odd = oracle.render_row_list(tris, cam, W, H, rows, threads=threads)
    dt = time.perf_counter() - t0
    parity = bool(np.array_equal(img.view(np.uint32), g_img[rows].ravel().view(np.uint32))
                  and np.array_equal(lb.view(np.uint32), g_lb[rows].ravel().view(np.uint32))
                  and np.array_equal(u8, g_u8[rows].ravel()))
    port = {
        "value": len(rows) * W / dt / 1e6,
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{len(rows)} rows x {W} px of the same {W}x{H} frame ({len(rows) * W} rays, "
                  f"{dt:.1f} s), oracle/xrt_oracle.c threaded over 64-px blocks",
        "serial_value": serial_rate / 1e6,
        "serial_sample": f"{span} rays of row {mid}, 1 thread ({serial_s:.2f} s)",
        "sample_bit_exact_vs_gpu": parity,
        "gpu_planes": "the timed loop's last frame (device planes copied back after timing)",
    }
    if ref is None:
        return port
    # the reference's own classes: serial on the same span, then every thread
    t0 = time.perf_counter()
    r_img, r_lb, _ = oracle.ref_render_spans(tris, cam, W, H, [mid], c0, c0 + span, threads=1)
    r_serial_s = time.perf_counter() - t0
    r_serial = span / r_serial_s
    ok = (np.array_equal(r_img.view(np.uint32), g_img[mid, c0:c0 + span].reshape(1, -1).view(np.uint32))
          and np.array_equal(r_lb.view(np.uint32), g_lb[mid, c0:c0 + span].reshape(1, -1).view(np.uint32)))
    rays = share * r_serial * threads
    if rays >= threads * W:                    # whole rows, spread over the frame
        n_r, b0, b1 = int(min(H, rays // W)), 0, W
    else:                                      # one centred span per thread
        n_r = threads
        w_s = int(max(8, min(W, rays // threads)))
        b0 = (W - w_s) // 2
        b1 = b0 + w_s
    rrows = np.unique(np.linspace(0, H - 1, n_r).astype(np.uint32))
    t0 = time.perf_counter()
    r_img, r_lb, _ = oracle.ref_render_spans(tris, cam, W, H, rrows, b0, b1, threads=threads)
    r_dt = time.perf_counter() - t0
    ok = ok and bool(np.array_equal(r_img.view(np.uint32), g_img[rrows, b0:b1].view(np.uint32))
                     and np.array_equal(r_lb.view(np.uint32), g_lb[rrows, b0:b1].view(np.uint32))
                     and np.array_equal(oracle.lut_u8_array(r_img.ravel()), g_u8[rrows, b0:b1].ravel()))
    return {
        "value": len(rrows) * (b1 - b0) / r_dt / 1e6,
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "reference",
        "sample": f"{len(rrows)} rows x columns [{b0}, {b1}) of the same {W}x{H} frame "
                  f"({len(rrows) * (b1 - b0)} rays, {r_dt:.1f} s): the reference's src/Ray.cxx, Triangle.cxx, "
                  f"TriangleMesh.cxx compiled unmodified (-O2, oracle/_ref) under renderLoop's per-pixel loop "
                  f"(oracle/ref_harness.cpp), one row per task on {threads} host threads over one shared mesh "
                  f"(main-pthreads-redo.cxx's structure)",
        "serial_value": r_serial / 1e6,
        "serial_sample": f"{span} rays of row {mid}, 1 thread ({r_serial_s:.2f} s)",
        "sample_bit_exact_vs_gpu": ok,
        "gpu_planes": port["gpu_planes"],
        "port": {k: port[k] for k in ("value", "cores", "sample", "serial_value", "serial_sample",
                                      "sample_bit_exact_vs_gpu")},
    }


def end_to_end(args, W, H, device_index, kernel):
    """The reference's only published numbers are whole-process runs
    (submit-serial.sh:18 /usr/bin/time; main.cxx:206-216 times the load): a fresh
    context's load + upload + first render (list sizing included) + D2H of the
    three planes, each part timed on the host (HIP already initialised), with
    the host-buffer call's own breakdown (xrt_debug_host_call_ms).  Then the
    same call again into the same host buffers (an Image rendered per frame)
    and into fresh ones, and the whole sequence once more in a second fresh
    context (what is a process's first-time cost, what is every context's)."""
    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.scenes import tiled_mesh

    def rounded(d):
        return {k: round(v, 3) for k, v in d.items()}

    def one_context(tris, t_load):
        t_c = time.perf_counter()
        c = xrt.Context(device_index)                 # streams, pinned D2H ring, copy threads
        r = {"context_create_ms": (time.perf_counter() - t_c) * 1e3}
        try:
            c.set_kernel(kernel)
            t2 = time.perf_counter()
            c.upload_mesh(tris)
            t3 = time.perf_counter()
            cam = xrt.camera_for_mesh(tris, W, H)
            t3c = time.perf_counter()
            planes = c.render_rows(cam)                   # host planes: render + D2H, synchronous
            t4 = time.perf_counter()
            r |= {"end_to_end_ms": (t_load + t4 - t2) * 1e3, "load_ms": t_load * 1e3,
                 "upload_ms": (t3 - t2) * 1e3, "camera_ms": (t3c - t3) * 1e3, "render_and_d2h_ms": (t4 - t3) * 1e3,
                 "render_and_d2h_breakdown_ms": rounded(c.host_call_ms())}
            t5 = time.perf_counter()
            c.render_rows(cam, out=planes[:3])
            r["again_same_buffers_ms"] = (time.perf_counter() - t5) * 1e3
            r["again_same_buffers_breakdown_ms"] = rounded(c.host_call_ms())
            t6 = time.perf_counter()
            c.render_rows(cam)
            r["again_fresh_buffers_ms"] = (time.perf_counter() - t6) * 1e3
            r["again_fresh_buffers_breakdown_ms"] = rounded(c.host_call_ms())
        finally:
            t7 = time.perf_counter()
            c.close()
            r["context_destroy_ms"] = (time.perf_counter() - t7) * 1e3
            r["context_destroy_breakdown_ms"] = rounded(xrt.Context.last_destroy_ms())
        return r

    # Python's cyclic garbage collector, not the path, can stop the harness for
    # tens of milliseconds inside a timed window (a gen-2 pass over the objects
    # torch and the timed loop left: a 30-40 ms gap outside xrt_render_rows,
    # whose own host time xrt_debug_host_call_ms shows): collected before the
    # windows and paused inside them; a C++ caller has no such pauses.
    t_gc = time.perf_counter()
    gc.collect()
    gc_collect_ms = (time.perf_counter() - t_gc) * 1e3
    gc.disable()
    try:
        t0 = time.perf_counter()
        tris = xrt.load_ply(args.mesh)
        if args.tile_mesh > 1:
            tris = tiled_mesh(tris, args.tile_mesh)
        t_load = time.perf_counter() - t0
        out = one_context(tris, t_load)
        second = one_context(tris, t_load)
    finally:
        gc.enable()
    out["second_context"] = {k: v for k, v in second.items() if k != "load_ms"}
    out["python_gc_collect_before_ms"] = gc_collect_ms   # the size of the pause kept out of the windows
    out["what"] = ("load PLY + upload + first render of a fresh context (list sizing included) + D2H of image, "
                   "L-buffer and u8 (context creation excluded); breakdown from xrt_debug_host_call_ms; then the "
                   "same call again into the same host buffers and into fresh ones; second_context: all of it "
                   "again in another fresh context of the same process")
    return out


def band_model(xrt, torch, tris, cam, W, H, device_index, band_rows=32, transit="packed"):
    """Inputs of strips.balanced_bounds from one binned render of the whole frame
    (rank 0, untimed): per band of 32 rows, its share of the render (the waves'
    in-kernel timing records, scaled to the frame's span, in us) and the bytes
    its strip sends -- packed: a 32x32 block per region the fill plan leaves;
    hits: per such region 16 tile masks (8 B each) and 4 B per hit ray."""
    import numpy as np
    dev = torch.device("cuda", device_index)
    img = torch.empty(W * H, dtype=torch.float32, device=dev)
    lb = torch.empty(W * H, dtype=torch.float32, device=dev)
    u8 = torch.empty(W * H, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    with xrt.Context(device_index) as c:
        c.set_kernel(xrt.XRT_KERNEL_BINNED)
        c.upload_mesh(tris)
        for _ in range(6):
            c.render_rows_device(cam, 0, H, img.data_ptr(), lb.data_ptr(), u8.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        t = c.wave_times().astype(np.int64)
        span_us = c.read_stats().kernel_ms * 1e3
        rmap, n_packed = c.plan_region_map(W, H)
        tile_hits = c.plan_hit_layout()[0] if transit == "hits" else None
    rx, ry = -(-W // 32), -(-H // 32)
    dur = ((t[:, 1] - t[:, 0]) % 2**32).astype(np.float64)         # ticks, per statistics record
    per_slot = dur.reshape(-1, 16).sum(axis=1)                       # 16 records per region slot
    region_cost = np.zeros(rx * ry)
    unfilled = rmap != 0xFFFFFFFF
    region_cost[unfilled] = per_slot[rmap[unfilled].astype(np.int64)]
    if (~unfilled).any():                                            # the fill plan's regions, evenly
        region_cost[~unfilled] = per_slot[n_packed:].sum() / (~unfilled).sum()
    band_wave = region_cost.reshape(ry, rx).sum(axis=1)
    band_cost = band_wave / max(band_wave.sum(), 1e-9) * span_us
    if tile_hits is not None:
        region_bytes = np.zeros(rx * ry)
        slot_bytes = 128.0 + 4.0 * tile_hits.reshape(-1, 16).sum(axis=1)
        region_bytes[unfilled] = slot_bytes[rmap[unfilled].astype(np.int64)]
        band_bytes = region_bytes.reshape(ry, rx).sum(axis=1)
    else:
        band_bytes = 4096.0 * unfilled.reshape(ry, rx).sum(axis=1)
    return band_cost, band_bytes, span_us


def measure_link(dist, torch, world, rank, dev, nccl, nbytes=4 << 20, reps=5):
    """Bytes per microsecond one sender delivers into rank 0 while every sender
    sends at once (the gather's pattern), measured with the bench's backend."""
    import time as _t
    where = dev if nccl else "cpu"
    buf = torch.ones(nbytes // 4, dtype=torch.float32, device=where)
    bufs = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None

    def once():
        if rank == 0:
            ops = [dist.P2POp(dist.irecv, bufs[g], g) for g in range(1, world)]
        else:
            ops = [dist.P2POp(dist.isend, buf, 0)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        if nccl:
            torch.cuda.synchronize(dev)
    once()
    dist.barrier()
    t0 = _t.perf_counter()
    for _ in range(reps):
        once()
    dt = (_t.perf_counter() - t0) / reps
    rate = torch.tensor([nbytes / (dt * 1e6)], dtype=torch.float64, device=where)
    dist.broadcast(rate, src=0)
    return float(rate.item())


class GcPauses:
    """Python garbage-collector pauses (count, ms) while active: a pause inside a
    timed window is the harness's, not the render path's."""

    def __init__(self):
        self.n, self.ms, self._t, self.active = 0, 0.0, None, False

    def __call__(self, phase, info):
        if not self.active:
            return
        if phase == "start":
            self._t = time.perf_counter()
        elif self._t is not None:
            self.n += 1
            self.ms += (time.perf_counter() - self._t) * 1e3
            self._t = None


GC = GcPauses()
gc.callbacks.append(GC)

DIST_TIMEOUT_S = 120            # every collective of a multi-rank run (a hung link fails the run)
EXIT_GATHER_MISMATCH = 3        # the gathered frame differs from rank 0's own render


def planes_equal(a, b) -> bool:
    """(image f32, L-buffer f32, u8) planes equal bit for bit."""
    import numpy as np
    return (np.array_equal(np.asarray(a[0]).view(np.uint32), np.asarray(b[0]).view(np.uint32))
            and np.array_equal(np.asarray(a[1]).view(np.uint32), np.asarray(b[1]).view(np.uint32))
            and np.array_equal(np.asarray(a[2]), np.asarray(b[2])))


def device_planes_equal(ctx, cam, H, planes, scratch, stream) -> bool:
    """Device planes (img, lb, u8 tensors) against a synchronous render of `cam`
    into `scratch`, compared bit for bit ON the device: no pageable device ->
    host copy in the bench process before its latency windows (live host pages
    such a copy locked stalled a fresh context's first read-back 11-40 ms:
    tools/evict_probe.py)."""
    import torch
    ctx.render_rows_device(cam, 0, H, *(t.data_ptr() for t in scratch), stream.cuda_stream)
    stream.synchronize()
    return all(torch.equal(a.view(torch.int32), b.view(torch.int32)) if a.dtype == torch.float32 else torch.equal(a, b)
               for a, b in zip(planes, scratch))


def gather_verdict(dist, torch, rank: int, ok: bool, where) -> int:
    """Every rank learns rank 0's verdict on the gathered frame (`ok` is read on
    rank 0 only) and returns its exit code: 0, or EXIT_GATHER_MISMATCH on every
    rank when the gathered frame is wrong -- a wrong frame fails the whole job,
    not just the rank that noticed."""
    flag = torch.tensor([1 if (ok or rank != 0) else 0], dtype=torch.int32, device=where)
    dist.broadcast(flag, src=0)
    if int(flag.item()) == 1:
        return 0
    print(f"bench.py rank {rank}: the gathered frame is not bit-exact against rank 0's single-device render",
          file=sys.stderr, flush=True)
    return EXIT_GATHER_MISMATCH


def make_roofline(args, kernel, workload, stats, T, rays_per_launch, avg_kernel_s, launches):
    """The dominant kernel's roofline (DESIGN.md "Measurement").

    The culled render is bound by vector-instruction issue, not by HBM: the
    top-level entry is its VALU issue rate -- SQ_INSTS_VALU per launch (rocprofv3
    PMC, profiles/traffic.json) / the live mean launch duration -- against the
    chip's issue peak (one wave64 VALU op per SIMD every 2 cycles).  Beside it
    (flat hbm_* keys) the HBM rate on the bytes the culled algorithm must move
    per launch (outputs, each candidate triangle's cull planes and record, the
    region-list entries) and the counter-measured HBM bytes.  The brute-force
    definition of SURVEY 8(d) (36 B per ray-triangle test) only gives the work
    avoided by the cull, `work_avoided_x`."""
    traffic = traffic_low = valu = None
    try:
        with open(args.traffic_json) as f:
            tr = json.load(f).get(f"{kernel}:{workload}")
        if tr:
            traffic = tr.get("hbm_bytes_per_launch")
            traffic_low = tr.get("hbm_bytes_per_launch_low")
            valu = tr.get("valu_wave_instr_per_launch")
    except (OSError, ValueError):
        pass
    tests = stats.tile_tests * 64 if kernel != "brute" else rays_per_launch * T
    if kernel == "brute":
        alg_bytes = rays_per_launch * BYTES_OUT_PER_RAY + 64 * T
    elif kernel == "binned":
        # outputs + the region lists' entries (one 64-B footprint per region
        # candidate, read once) + the record (TriRec, 64 B) of every triangle;
        # the render's other reads (each region's entries by its 16 tile waves,
        # survivors' records) are re-reads an L2 should hold
        alg_bytes = rays_per_launch * BYTES_OUT_PER_RAY + 64 * T + 64 * stats.candidates
    else:
        # outputs + cull planes (4 float4) and TriRec (64 B) of every triangle
        # + one u32 per region candidate (the LDS list built from the footprint
        # boxes, 16 B per triangle per region swept)
        alg_bytes = rays_per_launch * BYTES_OUT_PER_RAY + 128 * T + 4 * stats.candidates
    hbm_rate = alg_bytes / avg_kernel_s / 1e9 if avg_kernel_s > 0 else 0.0
    r = {
        "kernel": "k_render_" + kernel,
        "avg_kernel_ms": avg_kernel_s * 1e3,
        "launches": launches,
        "traffic": traffic,
        # FETCH_SIZE x 1 + WRITE_SIZE: the counters' lower reading (the render's
        # record gathers are counted at full size, its contiguous reads at half)
        "traffic_low": traffic_low,
        "hbm_achieved": hbm_rate,
        "hbm_peak": HBM_PEAK_GBS,
        "hbm_unit": "GB/s",
        "hbm_frac": hbm_rate / HBM_PEAK_GBS,
        "hbm_algorithmic_bytes_per_launch": alg_bytes,
        "hbm_traffic_GBs": traffic / avg_kernel_s / 1e9 if traffic and avg_kernel_s > 0 else None,
        "ray_triangle_tests_per_launch": tests,
        "brute_force_tests_per_launch": rays_per_launch * T,
        "brute_force_bytes_per_launch": rays_per_launch * (BYTES_PER_TEST * T + BYTES_OUT_PER_RAY),
        "work_avoided_x": rays_per_launch * T / max(tests, 1),
    }
    if valu and avg_kernel_s > 0:
        rate = valu / avg_kernel_s
        r.update({"bound": "valu", "achieved": rate, "peak": VALU_PEAK_WAVE_INSTR_S,
                  "unit": "wave-instr/s", "frac": rate / VALU_PEAK_WAVE_INSTR_S,
                  "valu_wave_instr_per_launch": valu})
    else:     # no PMC record for this workload: the HBM entry leads
        r.update({"bound": "hbm", "achieved": hbm_rate, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": hbm_rate / HBM_PEAK_GBS})
    if r["frac"] > 1.0 or r["hbm_frac"] > 1.0:       # a PMC record of another build (ablation runs)
        r["pmc_record_stale"] = True
    return r


def frames_in_flight(requested, strips: bool, W: int, H: int) -> int:
    """Frames in flight of a run (main(): frame k on stream k % F): the
    requested count, else 2 for frames of up to 2048^2 pixels and 1 above or in
    strips mode (DESIGN.md "Pipelining")."""
    if requested is not None:
        if requested < 1:
            raise SystemExit("--inflight must be at least 1")
        if strips and requested != 1:
            raise SystemExit("--inflight is for frames mode")
        return requested
    return 2 if not strips and W * H <= 2048 * 2048 else 1


def end_to_end_isolated(args, W, H, device_index):
    """end_to_end() in a child process of its own (bench.py --e2e-only): the
    fresh contexts it times then share the device with nothing the timed loop
    left behind (its streams, frame sets and buffers).  The child warms HIP up
    first (a throwaway context renders a 64x64 frame), as this process was."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--e2e-only", "--e2e-device", str(device_index),
           "--size", str(W), str(H), "--mesh", args.mesh, "--tile-mesh", str(args.tile_mesh),
           "--kernel", args.kernel]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, XRT_SEGV_TRACE="1"))   # a fatal signal names its library
    if r.returncode != 0:
        raise RuntimeError(f"end-to-end child failed ({r.returncode}): {r.stderr[-2000:]}")
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["process"] = "a child process of its own (HIP warmed by a 64x64 frame of a throwaway context)"
    return out


def e2e_only(args) -> int:
    import simpleraytracing_amd as xrt
    kernel = {"auto": xrt.XRT_KERNEL_AUTO, "brute": xrt.XRT_KERNEL_BRUTE, "tiled": xrt.XRT_KERNEL_TILED,
              "binned": xrt.XRT_KERNEL_BINNED}[args.kernel]
    tris = xrt.load_ply(args.mesh)
    with xrt.Context(args.e2e_device) as warm:      # HIP init, code objects, first launches
        warm.set_kernel(kernel)
        warm.upload_mesh(tris)
        warm.render_rows(xrt.camera_for_mesh(tris, 64, 64))
    W, H = args.size
    print(json.dumps(end_to_end(args, W, H, args.e2e_device, kernel)), flush=True)
    return 0


def child_exit(code: int) -> None:
    """A measurement child's exit once its JSON line is out: its contexts are
    closed, so nothing of the path is left to tear down -- os._exit skips the
    interpreter's and the shared libraries' finalizers (the HIP runtime's, a
    profiler's), whose order no caller controls."""
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)


def capi_multi_only(args) -> int:
    """bench.py --capi-only: the C ABI's multi-GPU entry timed in this process --
    one xrt_multi over --capi-devices (its own RCCL communicators from
    ncclCommInitAll, or one rank when one device is listed n times), the strips
    of xrt_multi_set_split, device-0 planes on one stream, W untimed frames (the
    first plans the split and sizes the lists), then K frames timed with the
    frames' gathers overlapping the next frames' renders; the last frame is
    compared bit for bit with one device's render of the whole frame."""
    import numpy as np
    import torch

    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.scenes import tiled_mesh
    devices = [int(d) for d in args.capi_devices.split(",")]
    kernel = {"auto": xrt.XRT_KERNEL_AUTO, "brute": xrt.XRT_KERNEL_BRUTE, "tiled": xrt.XRT_KERNEL_TILED,
              "binned": xrt.XRT_KERNEL_BINNED}[args.kernel]
    tris = xrt.load_ply(args.mesh)
    if args.tile_mesh > 1:
        tris = tiled_mesh(tris, args.tile_mesh)
    W, H = args.size
    cam = xrt.camera_for_mesh(tris, W, H)
    with xrt.Context(devices[0]) as one:
        one.set_kernel(kernel)
        one.upload_mesh(tris)
        ref = one.render_rows(cam)
    distinct = len(set(devices))
    dev = torch.device("cuda", devices[0])
    with xrt.MultiContext(devices) as m:
        m.set_kernel(kernel)
        m.upload_mesh(tris)
        if distinct == 1 and len(devices) > 1:
            m.set_gather(xrt.XRT_GATHER_RCCL)          # one-rank communicator: the RCCL calls on one GPU
        m.set_split(xrt.XRT_SPLIT_BALANCED if args.capi_split == "balanced" else xrt.XRT_SPLIT_EQUAL)
        # (--transit dense has no C-ABI counterpart: the blocks of the fill plan)
        m.set_transit(xrt.XRT_TRANSIT_HITS if args.transit == "hits" else xrt.XRT_TRANSIT_PACKED)
        img = torch.empty(W * H, dtype=torch.float32, device=dev)
        lb = torch.empty(W * H, dtype=torch.float32, device=dev)
        u8 = torch.empty(W * H, dtype=torch.uint8, device=dev)
        s = torch.cuda.Stream(dev)
        ptrs = (img.data_ptr(), lb.data_ptr(), u8.data_ptr(), s.cuda_stream)
        # the first frame splits equally and models the split from its strips'
        # records; the next frames take the balanced split planned from them
        t_w = time.perf_counter()
        for _ in range(max(args.warmup, 1)):
            m.render_device(cam, *ptrs)
        s.synchronize()
        warm_ms = (time.perf_counter() - t_w) * 1e3
        bounds, info = m.plan(cam)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            m.render_device(cam, *ptrs)
        s.synchronize()
        dt = time.perf_counter() - t0
        st = m.read_stats()
        transit = m.transit_stats()
        plan_stats = m.plan_stats()
    ok = (np.array_equal(img.cpu().numpy().view(np.uint32), ref[0].view(np.uint32))
          and np.array_equal(lb.cpu().numpy().view(np.uint32), ref[1].view(np.uint32))
          and np.array_equal(u8.cpu().numpy(), ref[2]))
    out = {"entry": "xrt_render_rows_multi_device (include/xrt.h), one process",
           "devices": devices,
           "gather": "RCCL, one communicator per device (ncclCommInitAll)" if distinct == len(devices) and distinct > 1
           else "RCCL, one rank (a device listed n times)" if distinct == 1 and len(devices) > 1 else "device copies",
           "split": args.capi_split, "strips": bounds, "strip_rows": [e - b for b, e in bounds],
           "plan": info, "plan_stats": plan_stats, "warmup_ms": warm_ms, "steps": args.steps, "warmup": max(args.warmup, 1),
           "ms_per_step": dt / args.steps * 1e3, "value": W * H * args.steps / dt / 1e6, "unit": "Mrays/s",
           "hit_rays": st.hit_rays, "transit": "hits" if args.transit == "hits" else "packed",
           "bytes_gathered_per_step": transit["last_bytes"], "transit_frames": transit,
           "bit_exact_vs_single_device_frame": bool(ok and transit["bad"] == 0)}
    print(json.dumps(out), flush=True)
    return 0


def capi_multi_isolated(args, W, H, devices, timeout_s=100):
    """capi_multi_only() in a child process (bounded by timeout_s): its RCCL
    communicators and device contexts are its own, and a failure or a hang there
    is recorded instead of ending this rank's run."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--capi-only", "--capi-devices", ",".join(map(str, devices)),
           "--size", str(W), str(H), "--mesh", args.mesh, "--tile-mesh", str(args.tile_mesh), "--kernel", args.kernel,
           "--steps", str(args.steps), "--warmup", str(args.warmup), "--capi-split", args.capi_split,
           "--transit", args.transit]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s,
                           env=dict(os.environ, XRT_SEGV_TRACE="1"))
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout_s} s", "devices": devices}
    if r.returncode != 0:
        return {"error": f"exit {r.returncode}: {r.stderr[-1500:]}", "devices": devices}
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    args = parse()
    if args.e2e_only:
        child_exit(e2e_only(args))
    if args.capi_only:
        child_exit(capi_multi_only(args))
    import numpy as np
    import torch
    import torch.distributed as dist

    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.scenes import orbit_camera, tiled_mesh
    from simpleraytracing_amd.strips import (balanced_bounds, gather_step_us, hit_descriptors, root_share,
                                             strip_bounds, unpack_descriptors, weighted_bounds)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # N > 1: BASELINE configs[3] -- one frame split into row strips, gathered to rank 0
    mode = args.mode or ("strips" if world > 1 and args.model == "attenuation" else "frames")
    if args.model == "signed" and mode == "strips":
        raise SystemExit("--model signed measures frames (the strip gather is the attenuation model's)")
    W, H = args.size or ((4096, 4096) if mode == "strips" and world > 1 else (2048, 2048))
    device_index = 0 if args.same_device else local_rank
    torch.cuda.set_device(device_index)
    dev = torch.device("cuda", device_index)
    nccl = args.dist_backend == "nccl"
    if world > 1:
        # a bounded wait on every collective: a lost rank or a stuck link ends
        # the run (non-zero exit) instead of hanging it
        timeout = datetime.timedelta(seconds=DIST_TIMEOUT_S)
        if nccl:
            dist.init_process_group("nccl", device_id=dev, timeout=timeout)
        else:
            dist.init_process_group("gloo", timeout=timeout)
        # a collective of every rank first: the point-to-point traffic below
        # (map exchange, batch_isend_irecv on rank 0 only) must not be the
        # group's first operation
        dist.barrier()
    # host-side waits (no GPU kernel spinning on the other ranks' devices while
    # rank 0's capi_multi leg uses them)
    cpu_group = (dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=DIST_TIMEOUT_S))
                 if world > 1 and nccl else None)

    tris = xrt.load_ply(args.mesh)
    if args.tile_mesh > 1:
        tris = tiled_mesh(tris, args.tile_mesh)
    T = len(tris)
    cam = xrt.camera_for_mesh(tris, W, H)
    strips = mode == "strips"
    if args.orbit and (strips or args.model != "attenuation"):
        raise SystemExit("--orbit is for frames mode, attenuation model")
    orbit_cams = None
    if args.orbit:
        lo, hi = xrt.mesh_bbox(tris)
        orbit_cams = [orbit_camera(cam, 0.5 * (np.asarray(lo, np.float64) + np.asarray(hi, np.float64)),
                                   k * args.orbit) for k in range(max(args.warmup, 1) + args.steps)]
    gathering = strips and world > 1
    # Row strips.  The root's own rows need no transfer: by default it renders a
    # larger first strip (strips.root_share), the others split the rest.
    split_info = None
    balanced = (strips and world > 1 and args.root_share == "balanced" and args.kernel in ("auto", "binned")
                and -(-H // 32) >= world)
    if args.root_share == "equal" or not strips:
        share0 = None
        bounds = [strip_bounds(H, world, g) for g in range(world)]
    elif balanced:
        # the frame's per-band cost and bytes (rank 0) and the link rate (every
        # rank): strips that balance the root's render against the senders'
        # renders and transfers (strips.balanced_bounds), sent to every rank
        share0 = None
        link = measure_link(dist, torch, world, rank, dev, nccl)
        flat = torch.zeros(2 * world, dtype=torch.int64, device=dev if nccl else "cpu")
        if rank == 0:
            band_cost, band_bytes, span_us = band_model(xrt, torch, tris, cam, W, H, device_index,
                                                        transit=args.transit)
            b = balanced_bounds(band_cost, band_bytes, world, link, H, unpack_us=5.0)
            flat.copy_(torch.tensor([v for be in b for v in be], dtype=torch.int64))
            split_info = {"link_bytes_per_us": link, "frame_span_us": span_us,
                          "predicted_step_us": gather_step_us(b, band_cost, band_bytes, link),
                          "band_rows": 32}
        dist.broadcast(flat, src=0)
        v = flat.cpu().tolist()
        bounds = [(int(v[2 * g]), int(v[2 * g + 1])) for g in range(world)]
    else:
        share0 = root_share(world) if args.root_share == "auto" else float(args.root_share)
        bounds = [weighted_bounds(H, world, g, share0) for g in range(world)]
    r0, r1 = bounds[rank] if strips else (0, H)

    ctx = xrt.Context(device_index)
    ctx.set_kernel({"auto": xrt.XRT_KERNEL_AUTO, "brute": xrt.XRT_KERNEL_BRUTE,
                    "tiled": xrt.XRT_KERNEL_TILED, "binned": xrt.XRT_KERNEL_BINNED}[args.kernel])
    ctx.upload_mesh(tris)
    signed = args.model == "signed"
    if signed:
        ctx.set_model(xrt.XRT_MODEL_SIGNED, 0.1037)   # main-pthreads-lbuffer.cxx:800
    stream = torch.cuda.current_stream(dev)

    # Rank 0 (and every rank in frames mode) holds a whole frame's planes.  In
    # strips mode the other ranks render L-buffer strips with misses coded
    # XRT_MISS_TRANSIT (4 B per pixel: image and u8 are functions of L) into
    # two alternating buffers and send them to rank 0, which receives them into
    # its frame's L plane and expands the image and u8 planes from them
    # (xrt_expand_rows_device) -- frame k's gather overlaps frame k+1's render.
    root = rank == 0 or not strips
    hits = gathering and args.transit == "hits"
    packed = gathering and args.transit in ("packed", "hits")     # the hit layout travels by the fill plan too
    # Frames in flight (frames mode): frame k renders on stream k % F into its
    # own planes, so consecutive renders are not serialised by one stream -- a
    # frame's first waves start while the previous frame's last ones run.  The
    # context keeps each frame's lists, records and statistics in its own
    # frame set (include/xrt.h).  It pays where a frame's ramp and tail are a
    # large part of its span (up to 2048^2: a few rounds of the GPU's wave
    # slots); two larger frames overlapping all along only share the L2s
    # (4096^2 step 105 -> 113 us, 1.12 M triangles 1,032 -> 1,057 us: DESIGN.md
    # "Frames in flight"), so they keep one stream.  Strips mode keeps one
    # stream (the gather already overlaps the next frame's render).
    inflight = frames_in_flight(args.inflight, strips, W, H)
    planes_of = []
    if root:
        for f in range(inflight):
            planes_of.append((torch.zeros(W * H, dtype=torch.float32, device=dev),
                              torch.zeros(W * H, dtype=torch.float32, device=dev),
                              torch.zeros(W * H, dtype=torch.uint8, device=dev),
                              stream if f == 0 else torch.cuda.Stream(dev)))
        img, lb, u8, _ = planes_of[0]
    else:
        ctx.set_miss_code(xrt.XRT_MISS_TRANSIT)
        tbufs = [torch.zeros((r1 - r0) * W, dtype=torch.float32, device=dev) for _ in range(2)]
        pending = [None, None]
    rest = W * H - (r1 - r0) * W if strips else 0     # pixels of the other ranks' strips
    frame_no = [0]

    # Packed transit: a sender's strip travels as the 32x32 blocks of the regions
    # its fill plan did not fill (those hold only misses).  The map of each
    # strip is a function of its geometry: one untimed frame sizes it, and the
    # senders send their maps to rank 0 once.
    # Hit transit (--transit hits): per tile of the fill plan a 64-bit hit mask,
    # then the hit rays' L values; the hit counts are a function of the
    # geometry too (xrt_plan_hit_layout), so the senders send them once with
    # their maps and rank 0 builds one set of unpack descriptors.
    if packed:
        if not root:
            ctx.render_rows_device(cam, r0, r1, 0, tbufs[0].data_ptr(), 0, stream.cuda_stream)
            rmap, n_packed = ctx.plan_region_map(W, r1 - r0)
            expect_fill = len(rmap) - n_packed
            d_map = torch.from_numpy(rmap.view(np.int32)).to(dev)
            words = 0
            if hits:
                tile_hits, words = ctx.plan_hit_layout()
                # the message, and room for one tile's hits past it (xrt.h)
                hbufs = [torch.zeros(max(words, 4) + 64, dtype=torch.float32, device=dev) for _ in range(2)]
                pbufs = [hb[:max(words, 4)] for hb in hbufs]
                ctx.set_transit_hits(hbufs[0].numel())
            else:
                pbufs = [torch.zeros(max(n_packed, 1) * 1024, dtype=torch.float32, device=dev) for _ in range(2)]
                # later frames render their L-buffer straight into the packed layout
                if expect_fill:
                    ctx.set_transit_layout(pbufs[0].numel())
            meta = torch.tensor([n_packed, words], dtype=torch.int64)
            dist.send(meta.to(dev) if nccl else meta, dst=0)
            dist.send(d_map if nccl else d_map.cpu(), dst=0)
            if hits:
                th = torch.from_numpy(tile_hits.view(np.int32))
                if th.numel():
                    dist.send(th.to(dev) if nccl else th, dst=0)
        else:
            # every sender's blocks back to back in one buffer, one unpack launch
            maps, counts, plans = [], [], []
            for g, (b, e) in enumerate(bounds):
                if not g:
                    continue
                meta = torch.zeros(2, dtype=torch.int64, device=dev if nccl else "cpu")
                dist.recv(meta, src=g)
                n_regions = -(-W // 32) * -(-(e - b) // 32)
                m = torch.zeros(n_regions, dtype=torch.int32, device=dev if nccl else "cpu")
                dist.recv(m, src=g)
                maps.append(m.cpu().numpy().view(np.uint32))
                counts.append(int(meta[0].item()))
                if hits:
                    th = torch.zeros(16 * counts[-1], dtype=torch.int32, device=dev if nccl else "cpu")
                    if th.numel():
                        dist.recv(th, src=g)
                    plans.append(th.cpu().numpy().view(np.uint32))
            if hits:
                desc, tdesc, bases, msg_words, total = hit_descriptors(W, bounds[1:], maps, plans)
                d_tdesc = torch.from_numpy(tdesc.reshape(-1).view(np.int32)).to(dev)
                d_bad = torch.zeros(1, dtype=torch.int32, device=dev)
                rbuf = torch.zeros(max(total, 4), dtype=torch.float32, device=dev)
                segs = {g + 1: rbuf[bases[g]:bases[g] + msg_words[g]] for g in range(world - 1)}
            else:
                desc, bases, total = unpack_descriptors(W, bounds[1:], maps)
                rbuf = torch.zeros(max(total, 1) * 1024, dtype=torch.float32, device=dev)
                segs = {g + 1: rbuf[bases[g] * 1024:(bases[g] + max(counts[g], 1)) * 1024]
                        for g in range(world - 1)}
            d_desc = torch.from_numpy(desc.reshape(-1).view(np.int32)).to(dev)
            n_desc = len(desc)

    def send_strip(t):
        if nccl:
            return dist.isend(t, dst=0)
        dist.send(t.cpu(), dst=0)             # gloo rehearsal: staged through the host
        return None

    recv_ops = []
    if gathering and root and nccl:           # the same receives every frame: built once
        bufs = segs if packed else {g: lb[b * W:e * W] for g, (b, e) in enumerate(bounds) if g}
        recv_ops = [dist.P2POp(dist.irecv, t, g) for g, t in bufs.items()]

    def post_recvs():
        """RCCL: the frame's receives, posted before the root renders its own strip."""
        return dist.batch_isend_irecv(recv_ops) if recv_ops else None

    def finish_recvs(works):
        if nccl:
            for w in works:
                w.wait()                      # the current stream waits for the receives
        else:                                 # gloo rehearsal: staged through the host
            bufs = segs if packed else {g: lb[b * W:e * W] for g, (b, e) in enumerate(bounds) if g}
            for g, t in bufs.items():
                host = torch.empty(t.numel(), dtype=torch.float32)
                dist.recv(host, src=g)
                t.copy_(host, non_blocking=False)
        if hits:
            ctx.unpack_hits_device(W, n_desc, d_desc.data_ptr(), d_tdesc.data_ptr(), rbuf.data_ptr(), lb.data_ptr(),
                                   img.data_ptr(), u8.data_ptr(), d_bad.data_ptr(), stream.cuda_stream)
        elif packed:
            ctx.unpack_blocks_device(W, n_desc, d_desc.data_ptr(), rbuf.data_ptr(), lb.data_ptr(), img.data_ptr(),
                                     u8.data_ptr(), stream.cuda_stream)
        else:                                 # the received rows, above and below the root's strip
            for b0, e0 in ((0, bounds[0][0]), (bounds[0][1], H)):
                if e0 > b0:
                    ctx.expand_rows_device((e0 - b0) * W, lb.data_ptr() + 4 * b0 * W, img.data_ptr() + 4 * b0 * W,
                                           u8.data_ptr() + b0 * W, stream.cuda_stream)

    # each buffer set's device pointers (the root's rows) and stream handle,
    # looked up once: the harness's own per-step host time stays small next to
    # a 20-40 us frame
    o_root = r0 * W
    ptrs_of = [(img_f.data_ptr(), lb_f.data_ptr(), u8_f.data_ptr(), s_f.cuda_stream)
               for img_f, lb_f, u8_f, s_f in planes_of]

    def step():
        k = frame_no[0]
        frame_no[0] += 1
        if root:
            img_k, lb_k, u8_k, s_k = ptrs_of[k % inflight]
        if signed:                            # the fork: signed L-buffer, then the hole fill
            ctx.render_rows_device(cam, 0, H, 0, lb_k, 0, s_k)
            ctx.hole_fill_device(W, H, lb_k, img_k, u8_k, s_k)
        elif root:
            works = post_recvs() if gathering else None
            ctx.render_rows_device(orbit_cams[k % len(orbit_cams)] if orbit_cams else cam, r0, r1,
                                   img_k + 4 * o_root, lb_k + 4 * o_root, u8_k + o_root, s_k)
            if gathering:
                finish_recvs(works)
        else:
            b = k % 2
            if pending[b] is not None:
                pending[b].wait()             # the send of frame k-2 has read this buffer
            if hits or (packed and expect_fill):   # the render writes the message itself
                ctx.render_rows_device(cam, r0, r1, 0, pbufs[b].data_ptr(), 0, stream.cuda_stream)
                if ctx.fill_regions() != expect_fill:   # the map assumes this frame filled them
                    raise RuntimeError(f"rank {rank}: the strip's fill plan did not hold for frame {k}")
                pending[b] = send_strip(pbufs[b])
            elif packed:                      # no plan (every region travels): pack the row-major strip
                ctx.render_rows_device(cam, r0, r1, 0, tbufs[b].data_ptr(), 0, stream.cuda_stream)
                ctx.pack_regions_device(W, r1 - r0, d_map.data_ptr(), tbufs[b].data_ptr(), pbufs[b].data_ptr(),
                                        stream.cuda_stream)
                pending[b] = send_strip(pbufs[b])
            else:
                ctx.render_rows_device(cam, r0, r1, 0, tbufs[b].data_ptr(), 0, stream.cuda_stream)
                pending[b] = send_strip(tbufs[b])

    # Frames mode with one camera: n steps in ONE call (xrt_render_frames_device,
    # frame k into plane set k % F on stream k % F -- every frame prepared and
    # rendered in full, the host side of all n in one pass instead of a Python
    # loop around one call per frame); otherwise one step() per frame.
    batch = (args.host_loop == "batch" and root and not strips and not signed and not orbit_cams)

    def run_steps(n):
        if n <= 0:
            return
        if batch:
            k0 = frame_no[0]
            ctx.render_frames_device(cam, 0, H, n, [ptrs_of[(k0 + j) % inflight] for j in range(inflight)])
            frame_no[0] += n
        else:
            for _ in range(n):
                step()

    # the first frame of this context (list sizing included), then the warm-up
    torch.cuda.synchronize(dev)
    t_first = time.perf_counter()
    step()
    torch.cuda.synchronize(dev)
    first_frame_ms = (time.perf_counter() - t_first) * 1e3
    run_steps(max(args.warmup - 1, 0))
    torch.cuda.synchronize(dev)
    # Clock ramp (DESIGN.md "Measurement"): an idle GPU runs at low clocks and
    # needs ~30 ms of sustained load to reach its steady rate (2048^2: ~38 us per
    # frame at first, 29.5 us after ~1,000 frames; an idle gap of 20 ms drops it
    # back).  By default the K timed steps follow the W warm-up steps directly
    # (`value` is that rate) and the loaded-clock rate is measured after them
    # (--loaded-ms, `at_loaded_clocks`).  Opt-in (--ramp-ms): the first min(K,
    # 20) frames after the warm-up are timed as they are (`before_clock_ramp`),
    # then untimed frames keep the GPU loaded for --ramp-ms before the timed
    # region.  Frame counts are agreed over ranks (a strips run exchanges data
    # every frame).
    cold = None
    ramp_frames = 0
    if args.ramp_ms > 0 and args.steps > 0:
        n_cold = min(args.steps, 20)
        t_c = time.perf_counter()
        run_steps(n_cold)
        torch.cuda.synchronize(dev)
        per_step = (time.perf_counter() - t_c) / n_cold
        cold = {"steps": n_cold, "ms_per_step": per_step * 1e3}
        if world > 1:
            t_ps = torch.tensor([per_step], dtype=torch.float64, device=dev if nccl else "cpu")
            dist.all_reduce(t_ps, op=dist.ReduceOp.MAX)
            per_step = float(t_ps.item())
        ramp_frames = int(min(20000, max(0.0, args.ramp_ms / 1e3 / max(per_step, 1e-7))))
        t_r = time.perf_counter()
        run_steps(ramp_frames)
        torch.cuda.synchronize(dev)
        cold["ramp_frames"] = ramp_frames
        cold["ramp_ms"] = (time.perf_counter() - t_r) * 1e3
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    tp_before = ctx.tile_plan_counters()["frames"]
    ctx.timing_begin()
    GC.active = True
    t0 = time.perf_counter()
    run_steps(args.steps)
    if not root:
        for p_ in pending:
            if p_ is not None:
                p_.wait()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    GC.active = False
    gc_in_timed = {"collections": GC.n, "ms": round(GC.ms, 3)}
    kernel_ms, launches = ctx.timing_end()
    event_ms, event_launches = ctx.timing_events()
    stats = ctx.read_stats()
    # Every timed frame culls from its own preparation: none may take the
    # (opt-in) tile plan, which skips tiles an earlier identical frame found dead.
    tile_plan_timed = ctx.tile_plan_counters()["frames"] - tp_before
    if tile_plan_timed:
        raise SystemExit(f"bench.py: {tile_plan_timed} timed frames used the tile plan")

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if nccl else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max = float(t.item())
    untimed_before = max(args.warmup, 1) + (cold["steps"] if cold else 0) + ramp_frames

    # After the timed region, never inside `value`: --loaded-ms of untimed
    # steps, then K more timed steps -- the rate once the GPU's clocks have
    # ramped under sustained load (DESIGN.md "Measurement").  The frame count
    # comes from the region's max-over-ranks step, so every rank agrees.
    loaded = None
    if args.loaded_ms > 0 and args.steps > 0:
        n_load = int(min(20000, max(0.0, args.loaded_ms / 1e3 / max(elapsed_max / args.steps, 1e-7))))
        t_r = time.perf_counter()
        run_steps(n_load)
        torch.cuda.synchronize(dev)
        load_ms = (time.perf_counter() - t_r) * 1e3
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t_l = time.perf_counter()
        run_steps(args.steps)
        if not root:
            for p_ in pending:
                if p_ is not None:
                    p_.wait()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t_lt = torch.tensor([time.perf_counter() - t_l], dtype=torch.float64, device=dev if nccl else "cpu")
        if world > 1:
            dist.all_reduce(t_lt, op=dist.ReduceOp.MAX)
        el = float(t_lt.item())
        loaded = {"value": W * H * args.steps * (1 if strips else world) / el / 1e6,
                  "ms_per_step": el / args.steps * 1e3, "steps": args.steps,
                  "untimed_frames_before": n_load, "untimed_ms_before": load_ms,
                  "what": "after the timed region: --loaded-ms of untimed steps keep the GPU loaded (its clocks "
                          "ramp), then K steps timed as the region is; not the headline value"}

    # Opt-in tile plan, never `value`: the same loop with it on (its frames skip
    # the cull of tiles an earlier frame of the same camera found dead).
    with_tile_plan = None
    if root and not strips and not signed and not orbit_cams and world == 1 and args.steps > 0 and \
            args.kernel in ("auto", "binned") and not args.no_tile_plan_leg:
        ctx.set_tile_plan(True)
        run_steps(max(args.warmup, 4))
        torch.cuda.synchronize(dev)
        tp0 = ctx.tile_plan_counters()["frames"]
        t_p = time.perf_counter()
        run_steps(args.steps)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t_p
        tp_frames = ctx.tile_plan_counters()["frames"] - tp0
        ctx.set_tile_plan(False)
        with_tile_plan = {"value": W * H * args.steps / el / 1e6, "ms_per_step": el / args.steps * 1e3,
                          "steps": args.steps, "tile_plan_frames": tp_frames,
                          "what": "after at_loaded_clocks, the same loop with the opt-in tile plan "
                                  "(xrt_debug_set_tile_plan): a tile without a survivor in an earlier frame of the "
                                  "same camera skips its cull -- memoisation of an identical-frame loop, not `value`"}

    # Moving camera (a projection sweep, the X-ray renderer's repeated
    # workload): a fresh context per leg, the camera turning deg degrees per
    # frame about the mesh centre, one xrt_render_rows_device call per frame
    # (frames in flight as in the main loop), every frame prepared for its
    # own camera.  The last frames are checked bit for bit afterwards.
    orbit = None
    if root and not strips and not signed and not orbit_cams and world == 1 and args.steps > 0 and \
            args.orbit_legs:
        orbit = {"fixed_camera_ms_per_step": elapsed_max / args.steps * 1e3}
        lo_, hi_ = xrt.mesh_bbox(tris)
        centre = 0.5 * (np.asarray(lo_, np.float64) + np.asarray(hi_, np.float64))
        n_timed = args.orbit_frames            # the same sweep whatever K (a 1-degree leg turns 60 degrees)
        n_warm = 4
        # planes of their own (the main loop's last frames are checked below)
        oplanes = [(torch.zeros(W * H, dtype=torch.float32, device=dev), torch.zeros(W * H, dtype=torch.float32, device=dev),
                    torch.zeros(W * H, dtype=torch.uint8, device=dev), s_f) for _, _, _, s_f in planes_of]
        optrs = [(a.data_ptr(), b.data_ptr(), c.data_ptr(), s_f.cuda_stream) for a, b, c, s_f in oplanes]
        fplanes = [(torch.empty(W * H, dtype=torch.float32, device=dev), torch.empty(W * H, dtype=torch.float32, device=dev),
                    torch.empty(W * H, dtype=torch.uint8, device=dev), s_f) for _, _, _, s_f in planes_of]
        fptrs = [(a.data_ptr(), b.data_ptr(), c.data_ptr(), s_f.cuda_stream) for a, b, c, s_f in fplanes]
        for deg in args.orbit_legs:
            # untimed: the sweep's frames before angle n_warm * deg, as many as
            # --orbit-ramp-ms of sustained load takes at twice the main loop's step
            # (the clock ramp, DESIGN.md "Clock ramp"); timed: the n_timed frames
            # from angle n_warm * deg on (the angles of the round-6 legs)
            n_ramp = max(int(args.orbit_ramp_ms / (2.0 * orbit["fixed_camera_ms_per_step"])), 0)
            k0 = n_warm + n_ramp
            cams_o = [orbit_camera(cam, centre, (k - n_ramp) * deg) for k in range(k0 + n_timed)]
            # a fresh context beside the bench's: it shares the device's prep and
            # host streams (libxrt's acquire_streams), so it adds no hardware
            # queue (DESIGN.md "Moving camera")
            with xrt.Context(device_index) as oc:
                oc.set_kernel({"auto": xrt.XRT_KERNEL_AUTO, "brute": xrt.XRT_KERNEL_BRUTE,
                               "tiled": xrt.XRT_KERNEL_TILED, "binned": xrt.XRT_KERNEL_BINNED}[args.kernel])
                oc.upload_mesh(tris)
                for k in range(k0):
                    img_k, lb_k, u8_k, s_k = optrs[k % inflight]
                    oc.render_rows_device(cams_o[k], 0, H, img_k, lb_k, u8_k, s_k)
                g0, q0 = oc.geometry_counters(), oc.pipeline_counters()
                t_o = time.perf_counter()
                for k in range(k0, k0 + n_timed):
                    img_k, lb_k, u8_k, s_k = optrs[k % inflight]
                    oc.render_rows_device(cams_o[k], 0, H, img_k, lb_k, u8_k, s_k)
                enq = time.perf_counter() - t_o
                torch.cuda.synchronize(dev)
                el = time.perf_counter() - t_o
                g1, q1 = oc.geometry_counters(), oc.pipeline_counters()
                # the same context at the same clocks, the camera held still: a few
                # untimed frames (the still camera's list sizing, frames prepared
                # ahead), then n_timed timed ones -- the moving camera's cost per se
                cam_f = cams_o[-1]
                for j in range(8):
                    img_k, lb_k, u8_k, s_k = fptrs[j % inflight]
                    oc.render_rows_device(cam_f, 0, H, img_k, lb_k, u8_k, s_k)
                torch.cuda.synchronize(dev)
                gf0, qf0 = oc.geometry_counters(), oc.pipeline_counters()
                t_f = time.perf_counter()
                for j in range(n_timed):
                    img_k, lb_k, u8_k, s_k = fptrs[j % inflight]
                    oc.render_rows_device(cam_f, 0, H, img_k, lb_k, u8_k, s_k)
                torch.cuda.synchronize(dev)
                el_f = time.perf_counter() - t_f
                gf1, qf1 = oc.geometry_counters(), oc.pipeline_counters()
                fixed_paths = {k_: v_ - gf0[k_] for k_, v_ in gf1.items() if v_ != gf0[k_]}
                fixed_paths.update({k_: v_ - qf0[k_] for k_, v_ in qf1.items() if v_ != qf0[k_]})
                exact = True
                scratch = (torch.empty(W * H, dtype=torch.float32, device=dev),
                           torch.empty(W * H, dtype=torch.float32, device=dev),
                           torch.empty(W * H, dtype=torch.uint8, device=dev))
                for j in range(inflight):
                    k = k0 + n_timed - 1 - j
                    with xrt.Context(device_index) as ref_ctx:       # a fresh context's synchronous render
                        ref_ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
                        ref_ctx.upload_mesh(tris)
                        exact &= device_planes_equal(ref_ctx, cams_o[k], H, oplanes[k % inflight][:3], scratch,
                                                     planes_of[0][3])
                del scratch
            if not exact:
                raise SystemExit(f"bench.py: an orbit frame ({deg:g} deg per frame) differs from its synchronous render")
            ms = el / n_timed * 1e3
            ms_f = el_f / n_timed * 1e3
            orbit[f"deg_{deg:g}"] = {
                "ms_per_step": ms, "value": W * H * n_timed / el / 1e6, "frames": n_timed, "warmup": n_warm,
                "ramp_frames": n_ramp, "fixed_camera_same_context_ms_per_step": ms_f,
                "fixed_camera_same_context_paths": fixed_paths,
                "vs_fixed_camera": ms / ms_f,
                "vs_main_loop_step": ms / orbit["fixed_camera_ms_per_step"],
                "sizings": g1["sizings"] - g0["sizings"], "reused_lists": g1["reused"] - g0["reused"],
                "plan_misses": g1["plan_misses"] - g0["plan_misses"], "overflows": g1["overflows"] - g0["overflows"],
                "host_waits": q1["host_waits"] - q0["host_waits"], "last_frames_bit_exact": bool(exact),
                "host_enqueue_ms_per_step": enq / n_timed * 1e3}
        del oplanes, fplanes
        orbit["what"] = ("a fresh context per leg (beside the bench's, on the device's shared streams); the camera "
                         "turns deg degrees per frame about the mesh centre "
                         "(scenes.orbit_camera); one xrt_render_rows_device call per frame, frames in flight as in "
                         "the main loop; each frame's k_prep bins its own camera; untimed frames of the sweep until "
                         "--orbit-ramp-ms of load (clock ramp), then `frames` timed ones; then, in the same context, "
                         "the last camera held still for 8 untimed and `frames` timed frames "
                         "(fixed_camera_same_context_ms_per_step): vs_fixed_camera = the moving step / that step; "
                         "vs_main_loop_step = the moving step / the main loop's; counters over the timed moving frames")

    # untimed: the gathered frame against rank 0's own render of the whole frame
    gather = None
    if gathering and rank == 0:
        full = ctx.render_rows(cam)
        ok = planes_equal((img.cpu().numpy(), lb.cpu().numpy(), u8.cpu().numpy()), full)
        if hits and int(d_bad.item()) != 0:   # a mask disagreed with its sender's plan
            ok = False
        if os.environ.get("XRT_BENCH_CORRUPT_GATHER") == "1":    # test hook: a wrong strip must fail the job
            ok = False
        moved = (4 * sum(msg_words) if hits else 4096 * sum(max(c, 1) for c in counts)) if packed else 4 * rest
        gather = {"bit_exact_vs_single_device_frame": bool(ok),
                  "bytes_gathered_per_step": moved, "dense_bytes_per_step": 4 * rest,
                  "transit": ("per tile of each strip's fill plan a 64-bit hit mask, then the hit rays' L values "
                              "(xrt_set_transit_hits)") if hits
                  else ("L-buffer strips, misses as XRT_MISS_TRANSIT, packed by region (the regions "
                        "each strip's fill plan filled stay behind)") if packed
                  else "L-buffer strips, misses as XRT_MISS_TRANSIT",
                  "strip_rows": [e - b for b, e in bounds], "strips": bounds, "root_share": share0,
                  "split": split_info or ("balanced" if balanced else args.root_share)}

    result = None
    if rank == 0:
        rays_total = W * H * args.steps * (1 if strips else world)
        value = rays_total / elapsed_max / 1e6
        rays_per_launch = (r1 - r0) * W
        avg_kernel_s = kernel_ms / max(launches, 1) / 1e3
        result_kernel = {1: "brute", 2: "tiled", 3: "binned"}[stats.kernel]
        workload = f"{os.path.basename(args.mesh)}" + (f" tiled {args.tile_mesh}x{args.tile_mesh}"
                                                         if args.tile_mesh > 1 else "") + f" {W}x{H}" + \
            (" signed L-buffer + hole fill" if signed else "") + \
            (f", orbit {args.orbit:g} deg per frame" if args.orbit else "")
        roofline = make_roofline(args, result_kernel, workload, stats, T, rays_per_launch, avg_kernel_s,
                                 launches)
        roofline["kernel_timing"] = ("in-kernel span of every timed render: its waves' s_memrealtime "
                                     "(100 MHz) start/end records, first start to last end; "
                                     "avg_kernel_ms_hip_events: HIP start/stop events on every 16th dispatch")
        roofline["avg_kernel_ms_hip_events"] = event_ms / event_launches if event_launches else None
        roofline["hip_event_launches"] = event_launches
        ms_per_step = elapsed_max / args.steps * 1e3
        # (frames past the record space are not sampled: a mean over the first
        # frames may sit a little above the whole region's step)
        slack = 1.0 if launches >= args.steps else 1.03
        if not strips and not args.no_timing_check and roofline["avg_kernel_ms"] > slack * inflight * ms_per_step:
            # at most `inflight` renders overlap: their mean duration cannot
            # exceed that many steps -- an event sample that says so is not
            # the kernel's duration
            raise SystemExit(f"bench.py: avg_kernel_ms {roofline['avg_kernel_ms']:.4f} > {inflight} x ms_per_step "
                             f"{ms_per_step:.4f} ({launches} sampled launches): inconsistent timing")
        roofline["frames_in_flight"] = inflight
        if roofline.get("bound") == "valu":
            # the chip's issue rate over the timed region: one render per step
            chip = roofline["valu_wave_instr_per_launch"] / (ms_per_step / 1e3)
            roofline["chip_achieved"] = chip
            roofline["chip_frac"] = chip / VALU_PEAK_WAVE_INSTR_S
            if inflight > 1:
                # Renders overlap in pairs, so a launch's span (avg_kernel_ms) is
                # shared with its neighbours and work / span undercounts the
                # issue rate the chip sustains: `achieved` is the chip's rate over
                # the timed region (the launch's work / the step; the span-based
                # figures stay beside it as span_*).
                roofline["span_achieved"] = roofline["achieved"]
                roofline["span_frac"] = roofline["frac"]
                roofline["achieved"] = chip
                roofline["frac"] = roofline["chip_frac"]
                roofline["achieved_is"] = "valu_wave_instr_per_launch / ms_per_step (launches overlap in pairs)"
        result = {
            "metric": "Mrays/s (dragon.ply render, whole job)",
            "value": value,
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if strips else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "dragon.ply from the reference repo (deterministic mesh; no synthetic noise)"
                    if args.tile_mesh == 1 else "tiled copies of dragon.ply (scenes.tiled_mesh)",
            "config": {
                "workload": workload,
                "kernel": {0: "auto", 1: "brute", 2: "tiled", 3: "binned"}[stats.kernel],
                "mode": mode,
                "triangles": T,
                "image": [W, H],
                "rays_per_step": W * H * (1 if strips else world),
                "parallelism": (f"row strips x{world}, L-buffer strips gathered to rank 0 over "
                                f"{'RCCL (xGMI)' if nccl else 'gloo (host-staged rehearsal)'}, overlapped with "
                                f"the next frame's render" if gathering
                                else f"one frame per rank x{world} (weak)" if world > 1 else "one GPU"),
                "frames_in_flight": inflight,
                "host_loop": ("xrt_render_frames_device: the timed steps in one call" if batch
                              else "one xrt_render_rows_device call per step"),
            },
            "frames_in_flight_exact": None,
            "roofline": roofline,
            "render_stats": {
                "hit_rays": stats.hit_rays, "odd_rays": stats.odd_rays, "max_hits": stats.max_hits,
                "overflow_rays": stats.overflow_rays,
                "region_candidates": stats.candidates, "global_triangles": stats.global_triangles,
                "wave_tile_tests": stats.tile_tests,
                "ray_triangle_tests_per_ray": stats.tile_tests * 64 / max(stats.rays, 1),
            },
            "python_gc_in_timed_region": gc_in_timed,
            # every frame rendered before the timed region: the first frame +
            # the warm-up steps (+ the opt-in --ramp-ms frames and their cold sample)
            "untimed_frames_before_timed_region": untimed_before,
            "before_clock_ramp": cold,
            "at_loaded_clocks": loaded,
            "tile_plan_frames_in_timed_region": tile_plan_timed,
            "with_tile_plan": with_tile_plan,
            "orbit": orbit,
            "latency": {"first_frame_ms": first_frame_ms,
                        "first_frame": "this context's first frame: k_prep, the synchronous list sizing, "
                                       "k_prep again and the render (device planes, synchronised)"},
            "cpu_baseline": None,
            "gather_check": gather,
            "dist_backend": args.dist_backend if world > 1 else None,
        }

    if rank == 0 and world == 1 and not signed:
        # the timed loop's own planes (its last frame), checked against the oracle's rows
        last_cam = orbit_cams[(frame_no[0] - 1) % len(orbit_cams)] if orbit_cams else cam
        img_l, lb_l, u8_l, _ = planes_of[(frame_no[0] - 1) % inflight]
        # (its host copy is taken after the latency windows: host pages that a
        # pageable device -> host copy locked, alive while a fresh context makes
        # its first synchronous read-back, stalled that read-back 23-40 ms --
        # tools/evict_probe.py, DESIGN.md "Measurement")
        if not args.no_latency:
            # in this process, right after the timed loop's streams and frame
            # sets (what a drop-in caller that renders an Image after streaming
            # device frames sees), and beside it in a child process of its own
            kernel_id = {"auto": xrt.XRT_KERNEL_AUTO, "brute": xrt.XRT_KERNEL_BRUTE, "tiled": xrt.XRT_KERNEL_TILED,
                         "binned": xrt.XRT_KERNEL_BINNED}[args.kernel]
            result["latency"].update(end_to_end(args, W, H, device_index, kernel_id))
            result["latency"]["process"] = "the bench process, after the timed loop (its contexts still open)"
            result["latency"]["child_process"] = end_to_end_isolated(args, W, H, device_index)
        if not args.no_cpu_baseline:
            planes = (img_l.cpu().numpy(), lb_l.cpu().numpy(), u8_l.cpu().numpy())
            result["cpu_baseline"] = cpu_baseline(tris, last_cam, W, H, args.cpu_seconds, planes)

    if root and not strips and not signed and inflight > 1:
        # untimed: each in-flight buffer set's last frame against a synchronous
        # render of its camera (frames that overlapped must not change a bit)
        ok = True
        for j in range(inflight):
            k = frame_no[0] - 1 - j
            img_k, lb_k, u8_k, _ = planes_of[k % inflight]
            ok &= planes_equal((img_k.cpu().numpy(), lb_k.cpu().numpy(), u8_k.cpu().numpy()),
                               ctx.render_rows(orbit_cams[k % len(orbit_cams)] if orbit_cams else cam))
        if not ok:
            raise SystemExit("bench.py: a frame rendered in flight differs from its synchronous render")
        if result is not None:
            result["frames_in_flight_exact"] = True

    code = 0
    if gathering:
        code = gather_verdict(dist, torch, rank, bool(gather and gather["bit_exact_vs_single_device_frame"]),
                              dev if nccl else "cpu")
    # The C ABI's own multi-GPU entry (the drop-in's renderLoopMultiGPU / xrt_main
    # -g N path) beside the torch path: rank 0 times it in a child process over
    # every rank's device while the other ranks wait on the host.
    capi_devices = ([int(d) for d in args.capi_devices.split(",")] if args.capi_devices
                    else ([device_index] * world if args.same_device else list(range(world)))
                    if gathering and args.capi_multi == "auto" else None)
    if capi_devices:
        torch.cuda.synchronize(dev)
        if rank == 0:
            result["capi_multi"] = capi_multi_isolated(args, W, H, capi_devices)
        if world > 1:
            dist.barrier(group=cpu_group)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    return code


def run() -> int:
    """main() with a failing rank's exit made prompt and non-zero: an exception
    prints its traceback and leaves through os._exit, so no collective or RCCL
    teardown of this rank can hang, and torch.distributed.run then ends the
    other ranks (a multi-rank run fails as a whole)."""
    try:
        return main()
    except SystemExit:
        raise
    except BaseException:
        rank = os.environ.get("RANK", "0")
        print(f"bench.py rank {rank} failed:", file=sys.stderr, flush=True)
        traceback.print_exc()
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(1)


if __name__ == "__main__":
    sys.exit(run())
