"""ctypes bindings of the C ABI (include/xrt.h, include/xrt_host.h).

The shared libraries are built in-tree by ``simpleraytracing_amd/csrc/Makefile``
into ``simpleraytracing_amd/lib/``.  Loading fails loudly when they are
missing: there is no Python or CPU fallback for the render path.
"""
from __future__ import annotations

import ctypes
import os

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")

XRT_OK = 0
XRT_ERR_ARGUMENT = 1
XRT_ERR_DEVICE = 2
XRT_ERR_NO_MESH = 3
XRT_ERR_OVERFLOW = 4
XRT_ERR_IO = 5
XRT_ERR_FORMAT = 6

XRT_KERNEL_AUTO = 0
XRT_KERNEL_BRUTE = 1
XRT_KERNEL_TILED = 2
XRT_KERNEL_BINNED = 3

XRT_MISS_TRANSIT = 0x7F800001

XRT_PROBE_EXPF = 0
XRT_PROBE_SQRTF = 1
XRT_PROBE_RCP = 2
XRT_PROBE_LUT_U8 = 3
XRT_PROBE_RCP_FAST = 4
XRT_PROBE_SIGNED_L = 5

XRT_MODEL_ATTENUATION = 0
XRT_MODEL_SIGNED = 1

XRT_GATHER_AUTO = 0
XRT_GATHER_COPY = 1
XRT_GATHER_RCCL = 2

XRT_SPLIT_EQUAL = 0
XRT_SPLIT_BALANCED = 1

XRT_TRANSIT_PACKED = 0
XRT_TRANSIT_HITS = 1

XRT_IMAGE_TEXT = 0
XRT_IMAGE_TGA = 1
XRT_IMAGE_PGM = 2
XRT_IMAGE_JPEG = 3

_f = ctypes.c_float
_fp = ctypes.POINTER(ctypes.c_float)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_vp = ctypes.c_void_p
_dp = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


class Camera(ctypes.Structure):
    """xrt_camera: RayTracerInfo (src/main.cxx:111-121) + pixel spacing + size."""

    _fields_ = [
        ("origin", _f * 3),
        ("detector", _f * 3),
        ("up", _f * 3),
        ("right", _f * 3),
        ("pixel_spacing", _f),
        ("width", _u32),
        ("height", _u32),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("rays", _u64),
        ("hit_rays", _u64),
        ("odd_rays", _u64),
        ("overflow_rays", _u64),
        ("hits", _u64),
        ("max_hits", _u32),
        ("kernel", _u32),
        ("kernel_ms", ctypes.c_double),
        ("candidates", _u64),
        ("tile_tests", _u64),
        ("global_triangles", _u64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class _Context(ctypes.Structure):
    pass


class _Multi(ctypes.Structure):
    pass


_CtxP = ctypes.POINTER(_Context)
_MultiP = ctypes.POINTER(_Multi)

# name -> (restype, argtypes); every symbol declared in include/xrt.h
XRT_SYMBOLS = {
    "xrt_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_CtxP)]),
    "xrt_destroy": (None, [_CtxP]),
    "xrt_last_error": (ctypes.c_char_p, [_CtxP]),
    "xrt_abi_version": (ctypes.c_int, []),
    "xrt_device_count": (ctypes.c_int, []),
    "xrt_upload_mesh": (ctypes.c_int, [_CtxP, _fp, _u64]),
    "xrt_mesh_bbox": (ctypes.c_int, [_fp, _u64, _fp, _fp]),
    "xrt_scene_bbox": (ctypes.c_int, [_fp, _u64p, _u32, _fp, _fp]),
    "xrt_camera_from_bbox": (ctypes.c_int, [_fp, _fp, _u32, _u32, ctypes.POINTER(Camera)]),
    "xrt_set_kernel": (ctypes.c_int, [_CtxP, ctypes.c_int]),
    "xrt_render_rows": (ctypes.c_int, [_CtxP, ctypes.POINTER(Camera), _u32, _u32, _fp, _fp, _u8p,
                                       ctypes.POINTER(Stats)]),
    "xrt_render_rows_device": (ctypes.c_int, [_CtxP, ctypes.POINTER(Camera), _u32, _u32, _vp, _vp,
                                              _vp, _vp]),
    "xrt_read_stats": (ctypes.c_int, [_CtxP, ctypes.POINTER(Stats)]),
    "xrt_render_frames_device": (ctypes.c_int, [_CtxP, ctypes.POINTER(Camera), _u32, _u32, _u32, _u32,
                                                ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                                ctypes.POINTER(_vp)]),
    "xrt_render_frames": (ctypes.c_int, [_CtxP, ctypes.POINTER(Camera), _u32, _u32, _u32, _fp, _fp, _u8p,
                                         ctypes.POINTER(Stats), _dp]),
    "xrt_timing_begin": (ctypes.c_int, [_CtxP]),
    "xrt_timing_end": (ctypes.c_int, [_CtxP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_u64)]),
    "xrt_timing_events": (ctypes.c_int, [_CtxP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_u64)]),
    "xrt_probe_intersect": (ctypes.c_int, [_CtxP, _fp, _fp, _u64, _u8p, _fp]),
    "xrt_probe_math": (ctypes.c_int, [_CtxP, ctypes.c_int, _fp, _fp, _u64]),
    "xrt_probe_prep": (ctypes.c_int, [_CtxP, ctypes.POINTER(Camera), _fp, _fp]),
    "xrt_host_expf_batch": (None, [_fp, _fp, _u64]),
    "xrt_host_exp_batch": (None, [_dp, _dp, _u64]),
    "xrt_host_signed_lbuffer_batch": (None, [_fp, _i32p, _f, _fp, _u64]),
    "xrt_set_model": (ctypes.c_int, [_CtxP, ctypes.c_int, _f]),
    "xrt_hole_fill": (ctypes.c_int, [_CtxP, _u32, _u32, _fp, _fp, _u8p]),
    "xrt_hole_fill_device": (ctypes.c_int, [_CtxP, _u32, _u32, _vp, _vp, _vp, _vp]),
    "xrt_render_signed": (ctypes.c_int, [_CtxP, ctypes.POINTER(Camera), _fp, _fp, _u8p, ctypes.POINTER(Stats)]),
    "xrt_host_mt_check": (None, [_fp, _fp, _fp, _fp, _u64, ctypes.POINTER(ctypes.c_uint8),
                                 ctypes.POINTER(ctypes.c_uint8), _fp]),
    "xrt_set_hit_capacity": (ctypes.c_int, [_CtxP, _u32]),
    "xrt_set_bin_capacity": (ctypes.c_int, [_CtxP, _u64]),
    "xrt_set_fill_plan": (ctypes.c_int, [_CtxP, ctypes.c_int]),
    "xrt_debug_fill_regions": (ctypes.c_int, [_CtxP, ctypes.POINTER(ctypes.c_uint32)]),
    "xrt_debug_geometry_counters": (ctypes.c_int, [_CtxP, ctypes.POINTER(ctypes.c_uint64)]),
    "xrt_debug_first_frames": (ctypes.c_int, [_CtxP, ctypes.POINTER(ctypes.c_uint64)]),
    "xrt_debug_pipeline_counters": (ctypes.c_int, [_CtxP, ctypes.POINTER(ctypes.c_uint64)]),
    "xrt_debug_host_call_ms": (ctypes.c_int, [_CtxP, _dp]),
    "xrt_debug_destroy_ms": (ctypes.c_int, [_dp]),
    "xrt_debug_tile_plan": (ctypes.c_int, [_CtxP, ctypes.POINTER(ctypes.c_uint64)]),
    "xrt_debug_set_tile_plan": (ctypes.c_int, [_CtxP, ctypes.c_int]),
    "xrt_debug_direction_grid": (ctypes.c_int, [ctypes.POINTER(Camera), ctypes.POINTER(ctypes.c_int)]),
    "xrt_debug_prep_times": (ctypes.c_int, [_CtxP, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.POINTER(ctypes.c_uint64)]),
    "xrt_debug_block_records": (ctypes.c_int, [_CtxP, _vp, _u64, ctypes.POINTER(_u64)]),
    "xrt_debug_wave_times": (ctypes.c_int, [_CtxP, _u32, ctypes.POINTER(_u32), _u64, ctypes.POINTER(_u64)]),
    "xrt_set_miss_code": (ctypes.c_int, [_CtxP, _u32]),
    "xrt_expand_rows_device": (ctypes.c_int, [_CtxP, _u64, _vp, _vp, _vp, _vp]),
    "xrt_plan_region_map": (ctypes.c_int, [_CtxP, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.POINTER(ctypes.c_uint32), _u64, ctypes.POINTER(ctypes.c_uint32)]),
    "xrt_pack_regions_device": (ctypes.c_int, [_CtxP, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp, _vp]),
    "xrt_unpack_regions_device": (ctypes.c_int, [_CtxP, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp,
                                                 _vp]),
    "xrt_set_transit_layout": (ctypes.c_int, [_CtxP, _u64]),
    "xrt_unpack_blocks_device": (ctypes.c_int, [_CtxP, ctypes.c_uint32, _u64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "xrt_plan_hit_layout": (ctypes.c_int, [_CtxP, ctypes.POINTER(_u32), _u64, ctypes.POINTER(_u64),
                                           ctypes.POINTER(_u64)]),
    "xrt_set_transit_hits": (ctypes.c_int, [_CtxP, _u64]),
    "xrt_unpack_hits_device": (ctypes.c_int, [_CtxP, ctypes.c_uint32, _u64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                              _vp]),
    "xrt_multi_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(_MultiP)]),
    "xrt_multi_destroy": (None, [_MultiP]),
    "xrt_multi_last_error": (ctypes.c_char_p, [_MultiP]),
    "xrt_multi_num_devices": (ctypes.c_int, [_MultiP]),
    "xrt_multi_upload_mesh": (ctypes.c_int, [_MultiP, _fp, _u64]),
    "xrt_multi_set_kernel": (ctypes.c_int, [_MultiP, ctypes.c_int]),
    "xrt_multi_set_model": (ctypes.c_int, [_MultiP, ctypes.c_int, _f]),
    "xrt_render_rows_multi": (ctypes.c_int, [_MultiP, ctypes.POINTER(Camera), _fp, _fp, _u8p,
                                             ctypes.POINTER(Stats)]),
    "xrt_render_rows_multi_device": (ctypes.c_int, [_MultiP, ctypes.POINTER(Camera), _vp, _vp, _vp, _vp]),
    "xrt_multi_read_stats": (ctypes.c_int, [_MultiP, ctypes.POINTER(Stats)]),
    "xrt_multi_set_gather": (ctypes.c_int, [_MultiP, ctypes.c_int]),
    "xrt_multi_set_split": (ctypes.c_int, [_MultiP, ctypes.c_int, ctypes.c_double]),
    "xrt_multi_set_transit": (ctypes.c_int, [_MultiP, ctypes.c_int]),
    "xrt_multi_transit_stats": (ctypes.c_int, [_MultiP, ctypes.POINTER(_u64)]),
    "xrt_multi_plan_stats": (ctypes.c_int, [_MultiP, ctypes.POINTER(_u64)]),
    "xrt_multi_debug_corrupt_hit_plan": (ctypes.c_int, [_MultiP]),
    "xrt_multi_plan": (ctypes.c_int, [_MultiP, ctypes.POINTER(Camera), ctypes.POINTER(_u32), _dp]),
    "xrt_balanced_bounds": (ctypes.c_int, [_dp, _dp, _u32, _u32, ctypes.c_double, _u32, _u32, ctypes.c_double,
                                           ctypes.POINTER(_u32), _dp]),
}

# every C symbol declared in include/xrt_host.h
XRT_HOST_SYMBOLS = {
    "xrt_host_load_ply": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_fp), ctypes.POINTER(_u64)]),
    "xrt_host_load_meshes": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_fp), ctypes.POINTER(_u64p),
                                            ctypes.POINTER(_u32)]),
    "xrt_host_free": (None, [_vp]),
    "xrt_host_intersect_batch": (None, [_fp, _fp, _u64, _u8p, _fp]),
    "xrt_host_save_image": (ctypes.c_int, [_fp, _u32, _u32, ctypes.c_char_p, ctypes.c_int, _f, _f]),
}

_lib = None
_host = None


def _bind(lib, table):
    variant = bool(os.environ.get("XRT_LIB"))
    for name, (res, args) in table.items():
        if variant and not hasattr(lib, name):     # an A/B build of an older ABI: its entry points only
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def lib_path(name="libxrt.so"):
    return os.path.join(LIB_DIR, name)


def load():
    """Returns the bound libxrt.so; raises if it has not been built."""
    global _lib
    if _lib is None:
        # XRT_LIB: a variant build (tools/build_variants.sh) for A/B timing only
        path = os.environ.get("XRT_LIB") or lib_path("libxrt.so")
        if not os.path.exists(path):
            raise RuntimeError(
                f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C simpleraytracing_amd/csrc` (there is no CPU fallback)")
        # torch's ROCm libraries first: they are NEEDED by unversioned names
        # (libamdhip64.so, librccl.so), so a torch imported after libxrt.so
        # (which needs libamdhip64.so.7, librccl.so.1) would load a second HIP
        # and HSA runtime into the process -- two runtimes that corrupt the heap
        # at exit.  Imported first, torch's copies carry the versioned sonames
        # and libxrt.so binds to them.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _lib = _bind(ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL), XRT_SYMBOLS)
    return _lib


def load_host():
    """Returns the bound libxrt_host.so (C++ host API's C entry points)."""
    global _host
    if _host is None:
        load()
        # XRT_HOST_LIB: a sanitizer build (make -C simpleraytracing_amd/csrc SAN=1, tools/san_check.sh)
        path = os.environ.get("XRT_HOST_LIB") or lib_path("libxrt_host.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: build simpleraytracing_amd/csrc first")
        _host = _bind(ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL), XRT_HOST_SYMBOLS)
    return _host
