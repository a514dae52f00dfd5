#!/usr/bin/env python3
"""Debug: is the first render of a context written when timing is on?"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
import simpleraytracing_amd as xrt
W = H = 512
tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
cam = xrt.camera_for_mesh(tris, W, H)
dev = torch.device("cuda", 0)
for timing in (True, False):
    for kernel in (2, 1):
        ctx = xrt.Context(0)
        ctx.upload_mesh(tris)
        ctx.set_kernel(kernel)
        img = torch.full((W * H,), -1.0, dtype=torch.float32, device=dev)
        s = torch.cuda.current_stream(dev)
        if timing:
            ctx.timing_begin()
        for k in range(3):
            ctx.render_rows_device(cam, 0, H, img.data_ptr(), 0, 0, s.cuda_stream)
            if k == 0:
                torch.cuda.synchronize(dev)
                a = img.cpu().numpy()
                print("timing", timing, "kernel", kernel, "after 1st render: unwritten", int((a == -1.0).sum()), "min", a.min(), flush=True)
        if timing:
            print("timing_end", ctx.timing_end())
        torch.cuda.synchronize(dev)
        a = img.cpu().numpy()
        print("   after 3 renders: unwritten", int((a == -1.0).sum()), flush=True)
        ctx.close()
