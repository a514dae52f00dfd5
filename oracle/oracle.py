"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the CPU oracle.

``liboracle.so`` is the plain-C restatement of the reference's render path
(oracle/xrt_oracle.c); ``_ref/libxrt_ref.so`` is the reference's own
src/Ray.cxx, src/Triangle.cxx and src/TriangleMesh.cxx compiled unmodified with
a harness (oracle/ref_harness.cpp).  Both are built by oracle/Makefile.  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use them.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_F = ctypes.POINTER(ctypes.c_float)
_U8 = ctypes.POINTER(ctypes.c_uint8)
_I32 = ctypes.POINTER(ctypes.c_int32)
_U32 = ctypes.POINTER(ctypes.c_uint32)
_U64 = ctypes.POINTER(ctypes.c_uint64)
_D = ctypes.POINTER(ctypes.c_double)

_orc = None
_ref = None


def _fp(a):
    return None if a is None else a.ctypes.data_as(_F)


def lib():
    global _orc
    if _orc is None:
        # XRT_ORACLE_LIB: a sanitizer build (make -C oracle SAN=1, tools/san_check.sh)
        path = os.environ.get("XRT_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        L.orc_load_ply.argtypes = [ctypes.c_char_p, ctypes.POINTER(_F), ctypes.POINTER(ctypes.c_uint64)]
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_bbox.argtypes = [_F, ctypes.c_uint64, _F, _F]
        L.orc_camera.argtypes = [_F, _F, ctypes.c_uint32, ctypes.c_uint32, _F]
        L.orc_render_rows.restype = ctypes.c_int64
        L.orc_render_rows.argtypes = [_F, ctypes.c_uint64, _F, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, _F, _F, _U8, _I32, ctypes.c_int]
        L.orc_render_row_list.restype = ctypes.c_int64
        L.orc_render_row_list.argtypes = [_F, ctypes.c_uint64, _F, ctypes.c_uint32, ctypes.c_uint32,
                                          _U32, ctypes.c_uint32, _F, _F, _U8, _I32, ctypes.c_int]
        L.orc_render_span.restype = ctypes.c_int64
        L.orc_render_span.argtypes = [_F, ctypes.c_uint64, _F, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _F, _F, _U8,
                                      _I32, ctypes.c_int]
        L.orc_render_row_list_span.restype = ctypes.c_int64
        L.orc_render_row_list_span.argtypes = [_F, ctypes.c_uint64, _F, ctypes.c_uint32, ctypes.c_uint32,
                                               _U32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                               _F, _F, _U8, _I32, ctypes.c_int]
        L.orc_hit_pairs.restype = ctypes.c_int64
        L.orc_hit_pairs.argtypes = [_F, ctypes.c_uint64, _F, ctypes.c_uint32, ctypes.c_uint32, _U32,
                                    ctypes.c_uint32, _U32, _U32, ctypes.c_uint64, ctypes.c_int]
        L.orc_intersect_batch.argtypes = [_F, _F, ctypes.c_uint64, _U8, _F]
        L.orc_save_text.argtypes = [_F, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p]
        L.orc_expf_batch.argtypes = [_F, _F, ctypes.c_uint64]
        L.orc_render_scene_rows.restype = ctypes.c_int64
        L.orc_render_scene_rows.argtypes = [_F, _U64, ctypes.c_uint32, _F, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, _F, _F, _U8, _I32, ctypes.c_int]
        L.orc_render_signed_rows.restype = ctypes.c_int64
        L.orc_render_signed_rows.argtypes = [_F, _U64, ctypes.c_uint32, _F, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_uint32, _F, _I32, ctypes.c_int]
        L.orc_hole_fill.argtypes = [_F, ctypes.c_uint32, ctypes.c_uint32, _F]
        L.orc_scene_bbox.argtypes = [_F, _U64, ctypes.c_uint32, _F, _F]
        L.orc_exp_batch.argtypes = [_D, _D, ctypes.c_uint64]
        L.orc_triangle_normals.argtypes = [_F, ctypes.c_uint64, _F]
        L.orc_lut_u8.restype = ctypes.c_uint8
        L.orc_lut_u8.argtypes = [ctypes.c_float]
        _orc = L
    return _orc


def ref_lib():
    """The reference's own classes (oracle/_ref); None when not built."""
    global _ref
    if _ref is None:
        path = os.path.join(HERE, "_ref", "libxrt_ref.so")
        # sanitizer runs (tools/san_check.sh): RTLD_DEEPBIND is incompatible with
        # the sanitizer runtimes, and the reference's classes are not this repo's code
        if not os.path.exists(path) or os.environ.get("XRT_ORACLE_NO_REF"):
            return None
        # RTLD_DEEPBIND: the reference's classes (TriangleMesh, Vec3, ...) bind
        # to their own definitions, not to the same-named drop-in classes of
        # libxrt_host.so when that is already loaded RTLD_GLOBAL.
        R = ctypes.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_DEEPBIND)
        R.ref_intersect_batch.argtypes = [_F, _F, ctypes.c_uint64, _U8, _F]
        R.ref_mesh_bbox.argtypes = [_F, ctypes.c_uint64, _F, _F]
        R.ref_camera.argtypes = [_F, _F, ctypes.c_uint32, ctypes.c_uint32, _F]
        R.ref_triangle_normals.argtypes = [_F, ctypes.c_uint64, _F]
        R.ref_render_signed_rows.restype = ctypes.c_int64
        R.ref_render_signed_rows.argtypes = [_F, _U64, ctypes.c_uint32, _F, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_uint32, _F]
        R.ref_render_rows.restype = ctypes.c_int64
        R.ref_render_rows.argtypes = [_F, ctypes.c_uint64, _F, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, _F, _F]
        R.ref_mesh_create.restype = ctypes.c_void_p
        R.ref_mesh_create.argtypes = [_F, ctypes.c_uint64]
        R.ref_mesh_destroy.restype = None
        R.ref_mesh_destroy.argtypes = [ctypes.c_void_p]
        R.ref_render_span.restype = ctypes.c_int64
        R.ref_render_span.argtypes = [ctypes.c_void_p, _F, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, _F, _F]
        _ref = R
    return _ref


def load_ply(path):
    L = lib()
    p = _F()
    n = ctypes.c_uint64()
    rc = L.orc_load_ply(str(path).encode(), ctypes.byref(p), ctypes.byref(n))
    if rc != 0:
        raise RuntimeError(f"oracle: cannot load {path} ({rc})")
    T = n.value
    out = np.ctypeslib.as_array(p, shape=(max(T, 1) * 9,))[: T * 9].copy()
    L.orc_free(ctypes.cast(p, ctypes.c_void_p))
    return out.reshape(T, 9)


def bbox(tris):
    tris = np.ascontiguousarray(tris, np.float32)
    lo = np.zeros(3, np.float32)
    hi = np.zeros(3, np.float32)
    lib().orc_bbox(_fp(tris), len(tris), _fp(lo), _fp(hi))
    return lo, hi


def camera(lower, upper, width, height):
    """13 floats: origin, detector, up, right, pixel spacing."""
    lo = np.ascontiguousarray(lower, np.float32)
    hi = np.ascontiguousarray(upper, np.float32)
    cam = np.zeros(13, np.float32)
    lib().orc_camera(_fp(lo), _fp(hi), width, height, _fp(cam))
    return cam


def camera_for_mesh(tris, width, height):
    lo, hi = bbox(tris)
    return camera(lo, hi, width, height)


def render_rows(tris, cam13, width, height, row_begin=0, row_end=None, threads=None):
    """(image f32, lbuffer f32, u8, nhits i32, odd) for rows [row_begin, row_end)."""
    if row_end is None:
        row_end = height
    tris = np.ascontiguousarray(tris, np.float32)
    cam13 = np.ascontiguousarray(cam13, np.float32)
    n = (row_end - row_begin) * width
    img = np.empty(n, np.float32)
    lb = np.empty(n, np.float32)
    u8 = np.empty(n, np.uint8)
    nh = np.empty(n, np.int32)
    threads = threads or os.cpu_count() or 1
    odd = lib().orc_render_rows(_fp(tris), len(tris), _fp(cam13), width, height, row_begin, row_end,
                                _fp(img), _fp(lb), u8.ctypes.data_as(_U8), nh.ctypes.data_as(_I32),
                                threads)
    if odd < 0:
        raise ValueError("bad row range")
    return img, lb, u8, nh, odd


def render_row_list(tris, cam13, width, height, rows, threads=None):
    rows = np.ascontiguousarray(rows, np.uint32)
    tris = np.ascontiguousarray(tris, np.float32)
    cam13 = np.ascontiguousarray(cam13, np.float32)
    n = len(rows) * width
    img = np.empty(n, np.float32)
    lb = np.empty(n, np.float32)
    u8 = np.empty(n, np.uint8)
    nh = np.empty(n, np.int32)
    threads = threads or os.cpu_count() or 1
    odd = lib().orc_render_row_list(_fp(tris), len(tris), _fp(cam13), width, height,
                                    rows.ctypes.data_as(_U32), len(rows), _fp(img), _fp(lb),
                                    u8.ctypes.data_as(_U8), nh.ctypes.data_as(_I32), threads)
    return img, lb, u8, nh, odd


def render_row_list_span(tris, cam13, width, height, rows, col_begin, col_end, threads=None):
    """Columns [col_begin, col_end) of each row in `rows`: (image, lbuffer, u8, nhits, odd),
    row-major (len(rows), col_end - col_begin)."""
    rows = np.ascontiguousarray(rows, np.uint32)
    tris = np.ascontiguousarray(tris, np.float32)
    cam13 = np.ascontiguousarray(cam13, np.float32)
    n = len(rows) * (col_end - col_begin)
    img = np.empty(n, np.float32)
    lb = np.empty(n, np.float32)
    u8 = np.empty(n, np.uint8)
    nh = np.empty(n, np.int32)
    odd = lib().orc_render_row_list_span(_fp(tris), len(tris), _fp(cam13), width, height,
                                         rows.ctypes.data_as(_U32), len(rows), col_begin, col_end,
                                         _fp(img), _fp(lb), u8.ctypes.data_as(_U8),
                                         nh.ctypes.data_as(_I32), threads or os.cpu_count() or 1)
    if odd < 0:
        raise ValueError("bad rows or span")
    return img, lb, u8, nh, odd


def render_span(tris, cam13, width, height, row, col_begin, col_end, threads=1):
    tris = np.ascontiguousarray(tris, np.float32)
    cam13 = np.ascontiguousarray(cam13, np.float32)
    n = col_end - col_begin
    img = np.empty(n, np.float32)
    lb = np.empty(n, np.float32)
    u8 = np.empty(n, np.uint8)
    nh = np.empty(n, np.int32)
    odd = lib().orc_render_span(_fp(tris), len(tris), _fp(cam13), width, height, row, col_begin,
                                col_end, _fp(img), _fp(lb), u8.ctypes.data_as(_U8),
                                nh.ctypes.data_as(_I32), threads)
    if odd < 0:
        raise ValueError("bad span")
    return img, lb, u8, nh, odd


def hit_pairs(tris, cam13, width, height, rows, cap=1 << 24, threads=None):
    """(pixel index within the row list, triangle index) of every hit with t > 1e-7."""
    rows = np.ascontiguousarray(rows, np.uint32)
    tris = np.ascontiguousarray(tris, np.float32)
    cam13 = np.ascontiguousarray(cam13, np.float32)
    px = np.zeros(cap, np.uint32)
    tr = np.zeros(cap, np.uint32)
    n = lib().orc_hit_pairs(_fp(tris), len(tris), _fp(cam13), width, height, rows.ctypes.data_as(_U32),
                            len(rows), px.ctypes.data_as(_U32), tr.ctypes.data_as(_U32), cap,
                            threads or os.cpu_count() or 1)
    if n > cap:
        raise ValueError("capacity exceeded")
    return px[:n], tr[:n]


def intersect_batch(rays, tris):
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    hit = np.zeros(len(rays), np.uint8)
    t = np.zeros(len(rays), np.float32)
    lib().orc_intersect_batch(_fp(rays), _fp(tris), len(rays), hit.ctypes.data_as(_U8), _fp(t))
    return hit, t


def ref_intersect_batch(rays, tris):
    R = ref_lib()
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    hit = np.zeros(len(rays), np.uint8)
    t = np.zeros(len(rays), np.float32)
    R.ref_intersect_batch(_fp(rays), _fp(tris), len(rays), hit.ctypes.data_as(_U8), _fp(t))
    return hit, t


def ref_render_spans(tris, cam13, width, height, rows, col_begin=0, col_end=None, threads=1):
    """Pixels [col_begin, col_end) of each of `rows` through the reference's own
    compiled classes (oracle/_ref), one row per task on `threads` host threads
    over one shared TriangleMesh (main-pthreads-redo.cxx's threads share theirs):
    (image, lbuffer) as (len(rows), span) float32 arrays, and the odd-ray count.
    ctypes releases the GIL for every call."""
    from concurrent.futures import ThreadPoolExecutor
    R = ref_lib()
    if R is None:
        raise RuntimeError("oracle/_ref is not built")
    if col_end is None:
        col_end = width
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    cam = np.ascontiguousarray(cam13, np.float32)
    rows = [int(r) for r in rows]
    span = col_end - col_begin
    img = np.empty((len(rows), span), np.float32)
    lb = np.empty((len(rows), span), np.float32)
    mesh = R.ref_mesh_create(_fp(tris), len(tris))
    try:
        def one(i):
            return R.ref_render_span(mesh, _fp(cam), width, height, rows[i], col_begin, col_end,
                                     _fp(img[i]), _fp(lb[i]))
        with ThreadPoolExecutor(max(1, int(threads))) as ex:
            odd = sum(ex.map(one, range(len(rows))))
    finally:
        R.ref_mesh_destroy(mesh)
    return img, lb, odd


def expf(x):
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    lib().orc_expf_batch(_fp(x), _fp(out), x.size)
    return out


def save_text(img, width, height, path):
    img = np.ascontiguousarray(img, np.float32)
    return lib().orc_save_text(_fp(img), width, height, str(path).encode())


def text_bytes(img, width, height):
    """Image::saveTextFile's bytes for a float image (via a temp file)."""
    import tempfile
    with tempfile.NamedTemporaryFile(suffix=".txt", delete=False) as f:
        path = f.name
    try:
        save_text(img, width, height, path)
        with open(path, "rb") as f:
            return f.read()
    finally:
        os.unlink(path)


def lut_u8(v):
    return lib().orc_lut_u8(float(v))


def lut_u8_array(v):
    """lut_u8 over an array: Image::applyLUT's per-pixel formula (include/Image.inl:195-211)
    with vmin 0, vmax 80 -- round(255 * (v - 0) / 80) in f64, half away from zero, clamped
    to [0, 255], NaN -> 0.  255 * v is exact in f64 and the quotient is rounded once, as in
    the reference; for v >= 0 the half-away rounding is floor(x + 0.5)."""
    x = 255.0 * (np.asarray(v, np.float32) - np.float32(0.0)).astype(np.float64) / 80.0
    out = np.where(x >= 0, np.floor(x + 0.5), -np.floor(-x + 0.5))
    out = np.where(np.isnan(x), 0.0, np.clip(out, 0.0, 255.0))
    return out.astype(np.uint8)


# --- scenes of several meshes, the signed L-buffer fork -----------------------

def scene_arrays(meshes):
    """(concatenated soup f32 (T, 9), triangles per mesh u64) of a list of soups."""
    meshes = [np.ascontiguousarray(m, np.float32).reshape(-1, 9) for m in meshes]
    counts = np.array([len(m) for m in meshes], np.uint64)
    tris = np.concatenate(meshes) if meshes else np.zeros((0, 9), np.float32)
    return np.ascontiguousarray(tris, np.float32), counts


def scene_bbox(meshes):
    tris, counts = scene_arrays(meshes)
    lo = np.zeros(3, np.float32)
    hi = np.zeros(3, np.float32)
    lib().orc_scene_bbox(_fp(tris), counts.ctypes.data_as(_U64), len(counts), _fp(lo), _fp(hi))
    return lo, hi


def camera_for_scene(meshes, width, height):
    lo, hi = scene_bbox(meshes)
    return camera(lo, hi, width, height)


def render_scene_rows(meshes, cam13, width, height, row_begin=0, row_end=None, threads=None):
    """renderLoop over a scene (hits on mesh 0 only): (image, lbuffer, u8, nhits, odd)."""
    if row_end is None:
        row_end = height
    tris, counts = scene_arrays(meshes)
    cam13 = np.ascontiguousarray(cam13, np.float32)
    n = (row_end - row_begin) * width
    img = np.empty(n, np.float32)
    lb = np.empty(n, np.float32)
    u8 = np.empty(n, np.uint8)
    nh = np.empty(n, np.int32)
    odd = lib().orc_render_scene_rows(_fp(tris), counts.ctypes.data_as(_U64), len(counts), _fp(cam13), width,
                                      height, row_begin, row_end, _fp(img), _fp(lb), u8.ctypes.data_as(_U8),
                                      nh.ctypes.data_as(_I32), threads or os.cpu_count() or 1)
    if odd < 0:
        raise ValueError("bad row range")
    return img, lb, u8, nh, odd


def render_signed_rows(meshes, cam13, width, height, row_begin=0, row_end=None, threads=None):
    """The L-buffer fork's signed L-buffer: (lbuffer f32 with -1 flags, nhits i32, flagged)."""
    if row_end is None:
        row_end = height
    tris, counts = scene_arrays(meshes)
    cam13 = np.ascontiguousarray(cam13, np.float32)
    n = (row_end - row_begin) * width
    lb = np.empty(n, np.float32)
    nh = np.empty(n, np.int32)
    flagged = lib().orc_render_signed_rows(_fp(tris), counts.ctypes.data_as(_U64), len(counts), _fp(cam13),
                                           width, height, row_begin, row_end, _fp(lb),
                                           nh.ctypes.data_as(_I32), threads or os.cpu_count() or 1)
    if flagged < 0:
        raise ValueError("bad row range")
    return lb, nh, flagged


def hole_fill(lbuffer, width, height):
    """The fork's -1 hole fill: the final image (f32) from a full-frame L-buffer."""
    lb = np.ascontiguousarray(lbuffer, np.float32).reshape(-1)
    assert lb.size == width * height
    out = np.empty_like(lb)
    lib().orc_hole_fill(_fp(lb), width, height, _fp(out))
    return out


def exp(x):
    """glibc exp (double)."""
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty_like(x)
    lib().orc_exp_batch(x.ctypes.data_as(_D), out.ctypes.data_as(_D), x.size)
    return out


def triangle_normals(tris):
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    out = np.empty((len(tris), 3), np.float32)
    lib().orc_triangle_normals(_fp(tris), len(tris), _fp(out))
    return out


def ref_triangle_normals(tris):
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    out = np.empty((len(tris), 3), np.float32)
    ref_lib().ref_triangle_normals(_fp(tris), len(tris), _fp(out))
    return out


def ref_render_signed_rows(meshes, cam13, width, height, row_begin=0, row_end=None):
    if row_end is None:
        row_end = height
    tris, counts = scene_arrays(meshes)
    cam13 = np.ascontiguousarray(cam13, np.float32)
    lb = np.empty((row_end - row_begin) * width, np.float32)
    flagged = ref_lib().ref_render_signed_rows(_fp(tris), counts.ctypes.data_as(_U64), len(counts), _fp(cam13),
                                               width, height, row_begin, row_end, _fp(lb))
    return lb, flagged
