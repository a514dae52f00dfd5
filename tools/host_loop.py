#!/usr/bin/env python3
"""Host cost of the enqueue path: per-call host time of render_rows_device
(no sync between calls) and the wall time per frame over a long run."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import simpleraytracing_amd as xrt
from simpleraytracing_amd.strips import views

W = H = int(os.environ.get("SIZE", "2048"))
N = int(os.environ.get("FRAMES", "400"))
tris = xrt.load_ply(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "dragon.ply"))
cam = xrt.camera_for_mesh(tris, W, H)
dev = torch.device("cuda", 0)
ctx = xrt.Context(0)
ctx.set_kernel(xrt.XRT_KERNEL_BINNED)
ctx.upload_mesh(tris)
buf = torch.zeros(9 * W * H, dtype=torch.uint8, device=dev)
img, lb, u8 = views(buf, W * H)
s = torch.cuda.current_stream(dev).cuda_stream
for _ in range(5):
    ctx.render_rows_device(cam, 0, H, img.data_ptr(), lb.data_ptr(), u8.data_ptr(), s)
torch.cuda.synchronize()
for label in ("plain", "timed"):
    if label == "timed":
        ctx.timing_begin()
    per = np.zeros(N)
    t0 = time.perf_counter()
    for i in range(N):
        a = time.perf_counter()
        ctx.render_rows_device(cam, 0, H, img.data_ptr(), lb.data_ptr(), u8.data_ptr(), s)
        per[i] = time.perf_counter() - a
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    extra = ""
    if label == "timed":
        ms, n = ctx.timing_end()
        extra = f" kernel {ms / max(n, 1) * 1e3:.1f} us over {n}"
    print(f"{label}: wall/frame {wall / N * 1e6:.1f} us  enqueue/frame {t_enq / N * 1e6:.1f} us  "
          f"call p50 {np.percentile(per, 50) * 1e6:.1f} p90 {np.percentile(per, 90) * 1e6:.1f} "
          f"max {per.max() * 1e6:.1f} us{extra}", flush=True)
