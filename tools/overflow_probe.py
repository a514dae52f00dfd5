import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
import simpleraytracing_amd as xrt
tris = xrt.load_ply("data/dragon.ply")
for W in (512, 1024, 2048):
    cam = xrt.camera_for_mesh(tris, W, W)
    ctx = xrt.Context(0); ctx.set_kernel(xrt.XRT_KERNEL_BINNED); ctx.upload_mesh(tris)
    for _ in range(3):
        img, lb, u8, st = ctx.render_rows(cam)
    print(W, "overflow_rays", st.overflow_rays, "max_hits", st.max_hits, "kernel_ms", round(st.kernel_ms, 4), "tile_tests", st.tile_tests, flush=True)
    ctx.close()
