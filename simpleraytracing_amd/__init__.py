"""simpleraytracing_amd -- MI355X-native X-ray attenuation render path.

A drop-in for the reference's per-pixel ``renderLoop`` (Brandagot/
SimpleRayTracing, src/main.cxx:626-743): ray generation -> brute-force
Moller-Trumbore over the whole mesh -> L-buffer path length -> Beer-Lambert
shade -> image store, bit-identical to the serial CPU program.

The product is native: HIP kernels for gfx950 behind the C ABI of
``include/xrt.h`` (``lib/libxrt.so``) and the C++ host API of
``csrc/host`` (``lib/libxrt_host.so``, ``lib/xrt_main``).  This Python module is
thin plumbing over that ABI for tests, ``bench.py`` and scripting; it never
computes pixels itself.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _abi
from ._abi import (Camera, Stats, XRT_KERNEL_AUTO, XRT_KERNEL_BINNED,  # noqa: F401
                   XRT_KERNEL_BRUTE, XRT_KERNEL_TILED, XRT_MISS_TRANSIT, XRT_MODEL_ATTENUATION,
                   XRT_MODEL_SIGNED, XRT_GATHER_AUTO, XRT_GATHER_COPY, XRT_GATHER_RCCL, XRT_SPLIT_EQUAL,
                   XRT_SPLIT_BALANCED, XRT_TRANSIT_HITS, XRT_TRANSIT_PACKED)

__all__ = [
    "Camera", "Stats", "Context", "MultiContext", "XrtError", "load_ply", "mesh_bbox", "camera_from_bbox",
    "camera_for_mesh", "device_count", "XRT_KERNEL_AUTO", "XRT_KERNEL_BRUTE", "XRT_KERNEL_TILED",
    "XRT_KERNEL_BINNED", "XRT_MISS_TRANSIT", "load_meshes", "scene_bbox", "camera_for_scene",
    "XRT_MODEL_ATTENUATION", "XRT_MODEL_SIGNED", "XRT_GATHER_AUTO", "XRT_GATHER_COPY", "XRT_GATHER_RCCL",
    "XRT_SPLIT_EQUAL", "XRT_SPLIT_BALANCED", "XRT_TRANSIT_HITS", "XRT_TRANSIT_PACKED",
]


class XrtError(RuntimeError):
    def __init__(self, code, message):
        super().__init__(f"xrt error {code}: {message}")
        self.code = code


def _fptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _u8ptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def device_count() -> int:
    return _abi.load().xrt_device_count()


def load_ply(path: str) -> np.ndarray:
    """Mesh 0 of a PLY file as a (T, 9) float32 triangle soup (p1, p2, p3)."""
    host = _abi.load_host()
    p = ctypes.POINTER(ctypes.c_float)()
    n = ctypes.c_uint64()
    rc = host.xrt_host_load_ply(str(path).encode(), ctypes.byref(p), ctypes.byref(n))
    if rc != _abi.XRT_OK:
        raise XrtError(rc, f"cannot load {path}")
    try:
        count = n.value
        out = np.ctypeslib.as_array(p, shape=(max(count, 1) * 9,))[: count * 9].copy()
    finally:
        host.xrt_host_free(ctypes.cast(p, ctypes.c_void_p))
    return out.reshape(count, 9)


def load_meshes(path: str) -> list:
    """Every mesh of a PLY (one) or OBJ (one per object) file, as (T, 9) float32 soups."""
    host = _abi.load_host()
    p = ctypes.POINTER(ctypes.c_float)()
    c = ctypes.POINTER(ctypes.c_uint64)()
    m = ctypes.c_uint32()
    rc = host.xrt_host_load_meshes(str(path).encode(), ctypes.byref(p), ctypes.byref(c), ctypes.byref(m))
    if rc != _abi.XRT_OK:
        raise XrtError(rc, f"cannot load {path}")
    try:
        counts = [int(c[i]) for i in range(m.value)]
        total = sum(counts)
        flat = np.ctypeslib.as_array(p, shape=(max(total, 1) * 9,))[: total * 9].copy().reshape(total, 9)
    finally:
        host.xrt_host_free(ctypes.cast(p, ctypes.c_void_p))
        host.xrt_host_free(ctypes.cast(c, ctypes.c_void_p))
    out, first = [], 0
    for n in counts:
        out.append(flat[first:first + n])
        first += n
    return out


def scene_bbox(meshes):
    """getBBox over several meshes (src/main.cxx:538-563)."""
    meshes = [np.ascontiguousarray(m, dtype=np.float32).reshape(-1, 9) for m in meshes]
    counts = np.array([len(m) for m in meshes], np.uint64)
    tris = np.ascontiguousarray(np.concatenate(meshes) if meshes else np.zeros((0, 9), np.float32))
    lo = np.zeros(3, np.float32)
    hi = np.zeros(3, np.float32)
    rc = _abi.load().xrt_scene_bbox(_fptr(tris), counts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                    len(counts), _fptr(lo), _fptr(hi))
    if rc != _abi.XRT_OK:
        raise XrtError(rc, "xrt_scene_bbox")
    return lo, hi


def camera_for_scene(meshes, width: int, height: int) -> Camera:
    """The camera of a scene: from the box of every mesh (main.cxx:634)."""
    lo, hi = scene_bbox(meshes)
    return camera_from_bbox(lo, hi, width, height)


def mesh_bbox(tris: np.ndarray):
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    lo = np.zeros(3, np.float32)
    hi = np.zeros(3, np.float32)
    rc = _abi.load().xrt_mesh_bbox(_fptr(tris), len(tris), _fptr(lo), _fptr(hi))
    if rc != _abi.XRT_OK:
        raise XrtError(rc, "xrt_mesh_bbox")
    return lo, hi


def camera_from_bbox(lower, upper, width: int, height: int) -> Camera:
    lo = np.ascontiguousarray(lower, dtype=np.float32)
    hi = np.ascontiguousarray(upper, dtype=np.float32)
    cam = Camera()
    rc = _abi.load().xrt_camera_from_bbox(_fptr(lo), _fptr(hi), width, height, ctypes.byref(cam))
    if rc != _abi.XRT_OK:
        raise XrtError(rc, "xrt_camera_from_bbox")
    return cam


def camera_for_mesh(tris: np.ndarray, width: int, height: int) -> Camera:
    lo, hi = mesh_bbox(tris)
    return camera_from_bbox(lo, hi, width, height)


class Context:
    """One xrt_context (one device).  Not thread-safe."""

    def __init__(self, device: int = 0):
        self._lib = _abi.load()
        self._ctx = _abi._CtxP()
        rc = self._lib.xrt_create(device, ctypes.byref(self._ctx))
        if rc != _abi.XRT_OK:
            raise XrtError(rc, self._lib.xrt_last_error(None).decode())
        self.device = device

    def close(self):
        if self._ctx:
            self._lib.xrt_destroy(self._ctx)
            self._ctx = _abi._CtxP()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != _abi.XRT_OK:
            raise XrtError(rc, f"{what}: {self._lib.xrt_last_error(self._ctx).decode()}")

    def upload_mesh(self, tris: np.ndarray):
        tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
        self._check(self._lib.xrt_upload_mesh(self._ctx, _fptr(tris), len(tris)), "xrt_upload_mesh")

    def set_kernel(self, kernel: int):
        self._check(self._lib.xrt_set_kernel(self._ctx, int(kernel)), "xrt_set_kernel")

    def set_model(self, model: int, mu: float = 0.1037):
        """XRT_MODEL_ATTENUATION (main.cxx) or XRT_MODEL_SIGNED (the L-buffer fork, mesh-0 mu)."""
        self._check(self._lib.xrt_set_model(self._ctx, int(model), float(np.float32(mu))), "xrt_set_model")

    def render_signed(self, cam: Camera):
        """The L-buffer fork end to end: (image f32, lbuffer f32 with -1 flags, u8, Stats)."""
        n = cam.width * cam.height
        img = np.empty(n, np.float32)
        lb = np.empty(n, np.float32)
        u8 = np.empty(n, np.uint8)
        st = Stats()
        self._check(self._lib.xrt_render_signed(self._ctx, ctypes.byref(cam), _fptr(img), _fptr(lb), _u8ptr(u8),
                                                ctypes.byref(st)), "xrt_render_signed")
        return img, lb, u8, st

    def hole_fill(self, lbuffer: np.ndarray, width: int, height: int):
        """The fork's hole fill of a whole-frame L-buffer: (image f32, u8)."""
        lb = np.ascontiguousarray(lbuffer, dtype=np.float32).reshape(-1)
        if lb.size != width * height:
            raise ValueError("L-buffer size does not match width x height")
        img = np.empty_like(lb)
        u8 = np.empty(lb.size, np.uint8)
        self._check(self._lib.xrt_hole_fill(self._ctx, width, height, _fptr(lb), _fptr(img), _u8ptr(u8)),
                    "xrt_hole_fill")
        return img, u8

    def hole_fill_device(self, width: int, height: int, d_lbuffer: int, d_image: int, d_u8: int, stream: int = 0):
        self._check(self._lib.xrt_hole_fill_device(self._ctx, width, height, d_lbuffer, d_image, d_u8, stream),
                    "xrt_hole_fill_device")

    def set_hit_capacity(self, capacity: int):
        self._check(self._lib.xrt_set_hit_capacity(self._ctx, int(capacity)), "xrt_set_hit_capacity")

    def set_bin_capacity(self, entries: int):
        self._check(self._lib.xrt_set_bin_capacity(self._ctx, int(entries)), "xrt_set_bin_capacity")

    def set_fill_plan(self, mode: int):
        """BINNED fill plan: 1 on (default), 0 off, 2 every region planned empty (test hook)."""
        self._check(self._lib.xrt_set_fill_plan(self._ctx, int(mode)), "xrt_set_fill_plan")

    def fill_regions(self) -> int:
        """Regions the last enqueued BINNED frame rendered through the fill plan."""
        n = ctypes.c_uint32()
        self._check(self._lib.xrt_debug_fill_regions(self._ctx, ctypes.byref(n)), "xrt_debug_fill_regions")
        return n.value

    def geometry_counters(self) -> dict:
        """BINNED frames by geometry path: sized, reused (moving camera), plan misses, list overflows."""
        c = (ctypes.c_uint64 * 4)()
        self._check(self._lib.xrt_debug_geometry_counters(self._ctx, c), "xrt_debug_geometry_counters")
        return dict(zip(("sizings", "reused", "plan_misses", "overflows"), (int(v) for v in c)))

    def first_frames(self) -> dict:
        """Frames of a new geometry sized on the device, and those whose pool was regrown (xrt_debug_first_frames)."""
        c = (ctypes.c_uint64 * 4)()
        self._check(self._lib.xrt_debug_first_frames(self._ctx, c), "xrt_debug_first_frames")
        return {"device_sized": int(c[0]), "recounted": int(c[1]), "last_pairs": int(c[2]), "last_pool": int(c[3])}

    def wave_times(self, frames_back: int = 0) -> np.ndarray:
        """Timing records of the render frames_back frames before the last (xrt_debug_wave_times):
        (n, 2) u32 s_memrealtime start / end (100 MHz, low 32 bits), one per statistics record."""
        n = ctypes.c_uint64()
        self._check(self._lib.xrt_debug_wave_times(self._ctx, frames_back, None, 0, ctypes.byref(n)),
                    "xrt_debug_wave_times")
        out = np.zeros((n.value, 2), np.uint32)
        self._check(self._lib.xrt_debug_wave_times(self._ctx, frames_back,
                                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                                   n.value, ctypes.byref(n)), "xrt_debug_wave_times")
        return out

    def block_records(self) -> np.ndarray:
        """The last render's statistics records (xrt_debug_block_records): (n, 8) u32 -- rays,
        hit rays, odd rays, overflow rays, hits, tile tests, candidates, max hits."""
        n = ctypes.c_uint64()
        self._check(self._lib.xrt_debug_block_records(self._ctx, None, 0, ctypes.byref(n)),
                    "xrt_debug_block_records")
        out = np.zeros((n.value, 8), np.uint32)
        self._check(self._lib.xrt_debug_block_records(self._ctx, out.ctypes.data, out.nbytes, ctypes.byref(n)),
                    "xrt_debug_block_records")
        return out

    def tile_plan_counters(self) -> dict:
        """Binned frames rendered with a tile plan, tile plans taken (xrt_debug_tile_plan)."""
        c = (ctypes.c_uint64 * 2)()
        self._check(self._lib.xrt_debug_tile_plan(self._ctx, c), "xrt_debug_tile_plan")
        return {"frames": int(c[0]), "plans": int(c[1])}

    def prep_times(self, enable=None) -> np.ndarray:
        """k_prep's per-wave timestamps of the last recorded launch (xrt_debug_prep_times):
        (n, 8) u32 stamps (xrt_debug.h); enable turns recording on / off."""
        n = ctypes.c_uint64()
        en = -1 if enable is None else int(bool(enable))
        self._check(self._lib.xrt_debug_prep_times(self._ctx, en, None, 0, ctypes.byref(n)), "xrt_debug_prep_times")
        out = np.zeros((n.value, 8), np.uint32)
        if n.value and enable is None:
            self._check(self._lib.xrt_debug_prep_times(self._ctx, -1, out.ctypes.data, n.value, ctypes.byref(n)),
                        "xrt_debug_prep_times")
        return out

    def set_tile_plan(self, on: bool):
        """The tile plan on / off for later frames (off by default: xrt_debug_set_tile_plan)."""
        self._check(self._lib.xrt_debug_set_tile_plan(self._ctx, 1 if on else 0), "xrt_debug_set_tile_plan")

    def pipeline_counters(self) -> dict:
        """Frames rendered from a preparation made ahead, preparations dropped, renders
        launched with no wait, renders launched after a host wait (xrt_debug_pipeline_counters)."""
        c = (ctypes.c_uint64 * 4)()
        self._check(self._lib.xrt_debug_pipeline_counters(self._ctx, c), "xrt_debug_pipeline_counters")
        return dict(zip(("ahead_used", "ahead_dropped", "no_wait", "host_waits"), (int(v) for v in c)))

    def host_call_ms(self) -> dict:
        """Host time of the last render_rows call, ms (xrt_debug_host_call_ms)."""
        ms = (ctypes.c_double * 16)()
        self._check(self._lib.xrt_debug_host_call_ms(self._ctx, ms), "xrt_debug_host_call_ms")
        keys = ("device_planes", "enqueue", "render_wait", "d2h", "d2h_copy_threads", "d2h_mb", "stats", "total",
                "of_which_hipmalloc", "of_which_list_sizing", "of_which_device_sync", "of_which_prep_wait",
                "of_which_launches", "device_sync_prep_stream", "device_sync_set_events",
                "device_sync_last_stream")
        return dict(zip(keys, (float(v) for v in ms)))

    @staticmethod
    def last_destroy_ms() -> dict:
        """Phases of the last xrt_destroy in this process, ms (xrt_debug_destroy_ms)."""
        ms = (ctypes.c_double * 4)()
        _abi.load().xrt_debug_destroy_ms(ms)
        return dict(zip(("wait_for_work", "device_frees", "pinned_host_frees", "streams_events"),
                        (float(v) for v in ms)))

    def render_rows(self, cam: Camera, row_begin: int = 0, row_end: int | None = None,
                    image=True, lbuffer=True, u8=True, out=None):
        """Host-buffer render of rows [row_begin, row_end); returns (image, lbuffer, u8, stats).
        `out`: (image, lbuffer, u8) arrays to render into instead of new ones."""
        if row_end is None:
            row_end = cam.height
        n = max(row_end - row_begin, 0) * cam.width
        if out is not None:
            img, lb, u = out
            for a, dt in ((img, np.float32), (lb, np.float32), (u, np.uint8)):
                if a is not None and (a.dtype != dt or a.size != n or not a.flags.c_contiguous):
                    raise ValueError("out arrays must be contiguous, of the strip's size and dtype")
        else:
            img = np.empty(n, np.float32) if image else None
            lb = np.empty(n, np.float32) if lbuffer else None
            u = np.empty(n, np.uint8) if u8 else None
        st = Stats()
        rc = self._lib.xrt_render_rows(
            self._ctx, ctypes.byref(cam), row_begin, row_end,
            _fptr(img) if img is not None else None,
            _fptr(lb) if lb is not None else None,
            _u8ptr(u) if u is not None else None, ctypes.byref(st))
        self._check(rc, "xrt_render_rows")
        return img, lb, u, st

    def render_rows_device(self, cam: Camera, row_begin: int, row_end: int, d_image: int,
                           d_lbuffer: int, d_u8: int, stream: int = 0):
        """Device-buffer render (raw device pointers, hipStream_t as int); asynchronous."""
        rc = self._lib.xrt_render_rows_device(self._ctx, ctypes.byref(cam), row_begin, row_end,
                                              d_image or None, d_lbuffer or None, d_u8 or None,
                                              stream or None)
        self._check(rc, "xrt_render_rows_device")

    def read_stats(self) -> Stats:
        st = Stats()
        self._check(self._lib.xrt_read_stats(self._ctx, ctypes.byref(st)), "xrt_read_stats")
        return st

    def render_frames_device(self, cam: Camera, row_begin: int, row_end: int, n_frames: int, sets):
        """n_frames frames of one geometry in one call (xrt_render_frames_device); frame k into
        sets[k % len(sets)] = (d_image, d_lbuffer, d_u8, stream) raw pointers (0 = none / default)."""
        ns = len(sets)
        arrs = [(ctypes.c_void_p * ns)(*[(s[i] or None) for s in sets]) for i in range(4)]
        rc = self._lib.xrt_render_frames_device(self._ctx, ctypes.byref(cam), row_begin, row_end, int(n_frames), ns,
                                                *arrs)
        self._check(rc, "xrt_render_frames_device")

    def render_frames(self, cam: Camera, n_frames: int, row_begin: int = 0, row_end: int | None = None):
        """n_frames frames back to back, the last one's host planes: (image, lbuffer, u8, stats, ms_per_frame)."""
        if row_end is None:
            row_end = cam.height
        n = max(row_end - row_begin, 0) * cam.width
        img, lb, u = np.empty(n, np.float32), np.empty(n, np.float32), np.empty(n, np.uint8)
        st = Stats()
        ms = ctypes.c_double()
        self._check(self._lib.xrt_render_frames(self._ctx, ctypes.byref(cam), row_begin, row_end, int(n_frames),
                                                _fptr(img), _fptr(lb), _u8ptr(u), ctypes.byref(st), ctypes.byref(ms)),
                    "xrt_render_frames")
        return img, lb, u, st, ms.value

    def set_miss_code(self, bits: int):
        """L-buffer bits of a miss in later renders: 0 (+inf) or XRT_MISS_TRANSIT."""
        self._check(self._lib.xrt_set_miss_code(self._ctx, int(bits)), "xrt_set_miss_code")

    def expand_rows_device(self, num_pixels: int, d_lbuffer: int, d_image: int, d_u8: int, stream: int = 0):
        """A received transit L-buffer into image / u8 planes, in place (device pointers)."""
        rc = self._lib.xrt_expand_rows_device(self._ctx, int(num_pixels), d_lbuffer or None, d_image or None,
                                              d_u8 or None, stream or None)
        self._check(rc, "xrt_expand_rows_device")

    def plan_region_map(self, width: int, rows: int):
        """(map, n_packed) of the last frame's strip: map[r] = packed index of region r
        (row-major 32x32 regions), 0xFFFFFFFF for a region its fill plan filled."""
        n = -(-width // 32) * -(-rows // 32)
        m = np.zeros(n, np.uint32)
        k = ctypes.c_uint32()
        self._check(self._lib.xrt_plan_region_map(self._ctx, width, rows,
                                                  m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n,
                                                  ctypes.byref(k)), "xrt_plan_region_map")
        return m, k.value

    def pack_regions_device(self, width: int, rows: int, d_map: int, d_lbuffer: int, d_packed: int, stream: int = 0):
        """A transit L-buffer strip into its packed regions (device pointers)."""
        self._check(self._lib.xrt_pack_regions_device(self._ctx, width, rows, d_map, d_lbuffer, d_packed,
                                                      stream or None), "xrt_pack_regions_device")

    def unpack_regions_device(self, width: int, rows: int, d_map: int, d_packed: int, d_lbuffer: int, d_image: int,
                              d_u8: int, stream: int = 0):
        """Packed regions into a strip's L / image / u8 planes (device pointers; 0 skips a plane)."""
        self._check(self._lib.xrt_unpack_regions_device(self._ctx, width, rows, d_map, d_packed, d_lbuffer or None,
                                                        d_image or None, d_u8 or None, stream or None),
                    "xrt_unpack_regions_device")

    def set_transit_layout(self, packed_floats: int):
        """Render L-buffers in the packed layout (capacity in floats; 0: row-major)."""
        self._check(self._lib.xrt_set_transit_layout(self._ctx, int(packed_floats)), "xrt_set_transit_layout")

    def unpack_blocks_device(self, width: int, n_blocks: int, d_desc: int, d_packed: int, d_lbuffer: int,
                             d_image: int, d_u8: int, stream: int = 0):
        """Many strips' packed regions into whole-frame planes in one launch (see xrt.h)."""
        self._check(self._lib.xrt_unpack_blocks_device(self._ctx, width, n_blocks, d_desc, d_packed,
                                                       d_lbuffer or None, d_image or None, d_u8 or None,
                                                       stream or None), "xrt_unpack_blocks_device")

    def plan_hit_layout(self):
        """(tile_hits, words) of the last frame's geometry (xrt_plan_hit_layout): the
        hit count of each tile of its fill plan (16 per tile slot) and the words of
        its hit-layout message."""
        n, w = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self._lib.xrt_plan_hit_layout(self._ctx, None, 0, ctypes.byref(n), ctypes.byref(w)),
                    "xrt_plan_hit_layout")
        hits = np.zeros(n.value, np.uint32)
        self._check(self._lib.xrt_plan_hit_layout(self._ctx, hits.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                                  n.value, ctypes.byref(n), ctypes.byref(w)), "xrt_plan_hit_layout")
        return hits, w.value

    def set_transit_hits(self, capacity_words: int):
        """Render L-buffers in the hit layout (message capacity in 32-bit words; 0: off)."""
        self._check(self._lib.xrt_set_transit_hits(self._ctx, int(capacity_words)), "xrt_set_transit_hits")

    def unpack_hits_device(self, width: int, n_blocks: int, d_desc: int, d_tdesc: int, d_msg: int, d_lbuffer: int,
                           d_image: int, d_u8: int, d_bad: int = 0, stream: int = 0):
        """Many strips' hit-layout messages into whole-frame planes in one launch (see xrt.h)."""
        self._check(self._lib.xrt_unpack_hits_device(self._ctx, width, n_blocks, d_desc, d_tdesc, d_msg,
                                                     d_lbuffer or None, d_image or None, d_u8 or None,
                                                     d_bad or None, stream or None), "xrt_unpack_hits_device")

    def timing_begin(self):
        self._check(self._lib.xrt_timing_begin(self._ctx), "xrt_timing_begin")

    def timing_end(self):
        """(summed kernel spans in ms, sampled launches) of the render kernel since
        timing_begin: every render's in-kernel span (its waves' s_memrealtime
        records, first start to last end)."""
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        self._check(self._lib.xrt_timing_end(self._ctx, ctypes.byref(ms), ctypes.byref(n)),
                    "xrt_timing_end")
        return ms.value, n.value

    def timing_events(self):
        """(summed ms, launches) of the HIP start/stop event pairs on every 16th render
        dispatch of the last timed region (a cross-check of timing_end)."""
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        self._check(self._lib.xrt_timing_events(self._ctx, ctypes.byref(ms), ctypes.byref(n)),
                    "xrt_timing_events")
        return ms.value, n.value

    def probe_intersect(self, rays: np.ndarray, tris: np.ndarray):
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
        n = len(rays)
        hit = np.zeros(n, np.uint8)
        t = np.zeros(n, np.float32)
        self._check(self._lib.xrt_probe_intersect(self._ctx, _fptr(rays), _fptr(tris), n,
                                                  _u8ptr(hit), _fptr(t)), "xrt_probe_intersect")
        return hit, t

    def probe_prep(self, cam: Camera, n: int):
        """(records (n,16), footprint (n,16)) of the uploaded mesh (n triangles) for `cam`."""
        rec = np.zeros((n, 16), np.float32)
        fp = np.zeros((n, 16), np.float32)
        self._check(self._lib.xrt_probe_prep(self._ctx, ctypes.byref(cam), _fptr(rec), _fptr(fp)),
                    "xrt_probe_prep")
        return rec, fp

    def probe_math(self, op: int, x: np.ndarray):
        x = np.ascontiguousarray(x, dtype=np.float32)
        out = np.empty_like(x)
        self._check(self._lib.xrt_probe_math(self._ctx, int(op), _fptr(x), _fptr(out), x.size),
                    "xrt_probe_math")
        return out


class MultiContext:
    """xrt_multi: row strips over several devices, gathered into device 0's
    frame with RCCL (include/xrt.h, "multi-GPU").  A device listed twice
    rehearses the strip logic on one GPU (device-copy gather)."""

    def __init__(self, devices):
        self._lib = _abi.load()
        self._m = _abi._MultiP()
        arr = (ctypes.c_int * len(devices))(*devices)
        rc = self._lib.xrt_multi_create(arr, len(devices), ctypes.byref(self._m))
        if rc != _abi.XRT_OK:
            raise XrtError(rc, self._lib.xrt_multi_last_error(None).decode())
        self.devices = list(devices)

    def close(self):
        if self._m:
            self._lib.xrt_multi_destroy(self._m)
            self._m = _abi._MultiP()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != _abi.XRT_OK:
            raise XrtError(rc, f"{what}: {self._lib.xrt_multi_last_error(self._m).decode()}")

    def upload_mesh(self, tris: np.ndarray):
        tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
        self._check(self._lib.xrt_multi_upload_mesh(self._m, _fptr(tris), len(tris)), "xrt_multi_upload_mesh")

    def set_kernel(self, kernel: int):
        self._check(self._lib.xrt_multi_set_kernel(self._m, int(kernel)), "xrt_multi_set_kernel")

    def set_gather(self, mode: int):
        """XRT_GATHER_AUTO / _COPY / _RCCL (a one-rank RCCL communicator when one
        device is listed n times)."""
        self._check(self._lib.xrt_multi_set_gather(self._m, int(mode)), "xrt_multi_set_gather")

    def set_model(self, model: int, mu: float = 0.1037):
        self._check(self._lib.xrt_multi_set_model(self._m, int(model), float(np.float32(mu))), "xrt_multi_set_model")

    def set_split(self, mode: int, link_bytes_per_us: float = 0.0):
        """XRT_SPLIT_EQUAL (the reference's H/N rows) or XRT_SPLIT_BALANCED (the default;
        link rate in bytes/us, 0 = measured once)."""
        self._check(self._lib.xrt_multi_set_split(self._m, int(mode), float(link_bytes_per_us)), "xrt_multi_set_split")

    def set_transit(self, mode: int):
        """XRT_TRANSIT_HITS (the default: hit masks and hit values once a strip geometry
        repeats) or XRT_TRANSIT_PACKED (the fill plan's 32x32 blocks)."""
        self._check(self._lib.xrt_multi_set_transit(self._m, int(mode)), "xrt_multi_set_transit")

    def transit_stats(self):
        """{frames_hits, frames_packed, last_bytes, bad} (xrt_multi_transit_stats)."""
        out = (ctypes.c_uint64 * 4)()
        self._check(self._lib.xrt_multi_transit_stats(self._m, out), "xrt_multi_transit_stats")
        return {"frames_hits": int(out[0]), "frames_packed": int(out[1]), "last_bytes": int(out[2]),
                "bad": int(out[3])}

    def plan_stats(self):
        """{plans, equal_no_model, link_probes, models} (xrt_multi_plan_stats)."""
        out = (ctypes.c_uint64 * 4)()
        self._check(self._lib.xrt_multi_plan_stats(self._m, out), "xrt_multi_plan_stats")
        return dict(zip(("plans", "equal_no_model", "link_probes", "models"), (int(v) for v in out)))

    def corrupt_hit_plan(self):
        """Test hook: the next hit frame's receive disagrees with its plan (xrt_multi_debug_corrupt_hit_plan)."""
        self._check(self._lib.xrt_multi_debug_corrupt_hit_plan(self._m), "xrt_multi_debug_corrupt_hit_plan")

    def plan(self, cam: Camera):
        """The strips of cam's frame: ([(begin, end) per device], {link, span_us, step_us})."""
        n = len(self.devices)
        b = (ctypes.c_uint32 * (2 * n))()
        info = (ctypes.c_double * 3)()
        self._check(self._lib.xrt_multi_plan(self._m, ctypes.byref(cam), b, info), "xrt_multi_plan")
        return ([(int(b[2 * g]), int(b[2 * g + 1])) for g in range(n)],
                {"link_bytes_per_us": info[0], "frame_span_us": info[1], "predicted_step_us": info[2]})

    def render(self, cam: Camera, image=True, lbuffer=True, u8=True):
        """The whole frame, gathered to the host: (image, lbuffer, u8, stats)."""
        n = cam.width * cam.height
        img = np.empty(n, np.float32) if image else None
        lb = np.empty(n, np.float32) if lbuffer else None
        u = np.empty(n, np.uint8) if u8 else None
        st = Stats()
        rc = self._lib.xrt_render_rows_multi(self._m, ctypes.byref(cam),
                                             _fptr(img) if img is not None else None,
                                             _fptr(lb) if lb is not None else None,
                                             _u8ptr(u) if u is not None else None, ctypes.byref(st))
        self._check(rc, "xrt_render_rows_multi")
        return img, lb, u, st

    def render_device(self, cam: Camera, d_image: int, d_lbuffer: int, d_u8: int, stream: int = 0):
        """Into device-0 planes (raw pointers), ordered on device 0's stream; asynchronous."""
        rc = self._lib.xrt_render_rows_multi_device(self._m, ctypes.byref(cam), d_image or None,
                                                    d_lbuffer or None, d_u8 or None, stream or None)
        self._check(rc, "xrt_render_rows_multi_device")

    def read_stats(self) -> Stats:
        st = Stats()
        self._check(self._lib.xrt_multi_read_stats(self._m, ctypes.byref(st)), "xrt_multi_read_stats")
        return st
