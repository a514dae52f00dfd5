#!/usr/bin/env python3
"""Render statistics (tile tests, candidates, hits) of one library build."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import simpleraytracing_amd as xrt
tris = xrt.load_ply(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "dragon.ply"))
W = int(os.environ.get("SIZE", "2048"))
cam = xrt.camera_for_mesh(tris, W, W)
ctx = xrt.Context(0); ctx.set_kernel(xrt.XRT_KERNEL_BINNED); ctx.upload_mesh(tris)
img, lb, u8, st = ctx.render_rows(cam)
print(f"tile_tests {st.tile_tests} per-ray {st.tile_tests * 64 / st.rays:.3f} hits {st.hits} hit_rays {st.hit_rays} candidates {st.candidates}")
