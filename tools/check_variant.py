#!/usr/bin/env python3
"""Checks libxrt.so variants against the oracle on sampled rows of a frame
rendered into device buffers (the bench/ab path).  Test tooling."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import simpleraytracing_amd as xrt
from simpleraytracing_amd import _abi
from oracle import oracle

W = H = int(os.environ.get("SIZE", "2048"))
kid = int(os.environ.get("KERNEL", "2"))
tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
cam = xrt.camera_for_mesh(tris, W, H)
rows = [0, H // 3, H // 2, H - 1]
ref = oracle.render_row_list(tris, oracle.camera_for_mesh(tris, W, H), W, H, rows)
dev = torch.device("cuda", 0)
for spec in sys.argv[1:]:
    name, path = spec.split("=", 1)
    need = ["xrt_create", "xrt_last_error", "xrt_upload_mesh", "xrt_set_kernel", "xrt_render_rows_device"]
    L = _abi._bind(ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL), {k: _abi.XRT_SYMBOLS[k] for k in need})
    ctx = _abi._CtxP()
    assert L.xrt_create(0, ctypes.byref(ctx)) == 0
    t = np.ascontiguousarray(tris)
    L.xrt_upload_mesh(ctx, t.ctypes.data_as(_abi._fp), len(t))
    L.xrt_set_kernel(ctx, kid)
    img = torch.full((W * H,), -1.0, dtype=torch.float32, device=dev)
    lb = torch.full((W * H,), -1.0, dtype=torch.float32, device=dev)
    u8 = torch.zeros(W * H, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    rc = L.xrt_render_rows_device(ctx, ctypes.byref(cam), 0, H, img.data_ptr(), lb.data_ptr(), u8.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize(dev)
    g = img.cpu().numpy().reshape(H, W)[rows].ravel()
    ok = np.array_equal(g.view(np.uint32), ref[0].view(np.uint32))
    bad = np.nonzero(g.view(np.uint32) != ref[0].view(np.uint32))[0]
    print(name, "rc", rc, "image rows match oracle:", ok, "mismatches", len(bad), bad[:5], g[bad[:3]], ref[0][bad[:3]])

# full-frame comparison between variants, repeated renders
frames = {}
for spec in sys.argv[1:]:
    name, path = spec.split("=", 1)
    need = ["xrt_create", "xrt_last_error", "xrt_upload_mesh", "xrt_set_kernel", "xrt_render_rows_device"]
    L = _abi._bind(ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL), {k: _abi.XRT_SYMBOLS[k] for k in need})
    ctx = _abi._CtxP()
    assert L.xrt_create(0, ctypes.byref(ctx)) == 0
    t = np.ascontiguousarray(tris)
    L.xrt_upload_mesh(ctx, t.ctypes.data_as(_abi._fp), len(t))
    L.xrt_set_kernel(ctx, kid)
    outs = []
    for rep in range(3):
        img = torch.full((W * H,), -1.0, dtype=torch.float32, device=dev)
        s = torch.cuda.current_stream(dev)
        L.xrt_render_rows_device(ctx, ctypes.byref(cam), 0, H, img.data_ptr(), None, None, s.cuda_stream)
        torch.cuda.synchronize(dev)
        outs.append(img.cpu().numpy().view(np.uint32).copy())
    print(name, "repeat-stable:", all(np.array_equal(outs[0], o) for o in outs[1:]),
          "unwritten:", int(np.count_nonzero(outs[0] == np.float32(-1.0).view(np.uint32))))
    frames[name] = outs[0]
names = list(frames)
for n in names[1:]:
    d = np.nonzero(frames[n] != frames[names[0]])[0]
    print(names[0], "vs", n, "differ at", len(d), d[:10])
