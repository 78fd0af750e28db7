"""ctypes binding of libvr.so (include/vr.h).

The library is built in-tree by ``csrc/Makefile`` (``__graft_entry__.build()``).
There is no fallback: if the HIP library is missing or fails to load, every
entry point raises, so nothing can silently run on the CPU.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# VRDD_LIB overrides the library path (tools/bench_variants.py loads tuning builds)
LIB_PATH = os.environ.get("VRDD_LIB") or os.path.join(_HERE, "csrc", "build", "libvr.so")

VR_OK = 0
VR_ERR_ARG = -1
VR_ERR_STATE = -2
VR_ERR_HIP = -3
VR_ERR_UNSUPPORTED = -4


class VRError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"libvr status {status}: {message}")
        self.status = status


class Dim3(ctypes.Structure):
    """Layout of dim3 (3 x uint32)."""
    _fields_ = [("x", ctypes.c_uint32), ("y", ctypes.c_uint32), ("z", ctypes.c_uint32)]


class Extent(ctypes.Structure):
    """Layout of cudaExtent / hipExtent (3 x size_t)."""
    _fields_ = [("width", ctypes.c_size_t), ("height", ctypes.c_size_t),
                ("depth", ctypes.c_size_t)]


class RenderDesc(ctypes.Structure):
    """vr_render_desc of include/vr.h."""
    _fields_ = [
        ("d_output", ctypes.c_void_p),
        ("d_output_f", ctypes.c_void_p),
        ("d_steps", ctypes.c_void_p),
        ("width", ctypes.c_uint32),
        ("height", ctypes.c_uint32),
        ("inv_view", ctypes.c_float * 12),
        ("density", ctypes.c_float),
        ("brightness", ctypes.c_float),
        ("transfer_offset", ctypes.c_float),
        ("transfer_scale", ctypes.c_float),
        ("query_method", ctypes.c_int),
        ("volume_size", Extent),
        ("d_tile_list", ctypes.c_void_p),
        ("n_tiles", ctypes.c_uint32),
    ]


class GmmSlab(ctypes.Structure):
    """vr_gmm_slab (include/vr.h): one slab of a slab-chained GMM render"""
    _fields_ = [
        ("z_lo", ctypes.c_int),
        ("z_hi", ctypes.c_int),
        ("d_rays_in", ctypes.c_void_p),
        ("n_rays_in", ctypes.c_uint32),
        ("d_rays_out", ctypes.c_void_p),
        ("d_n_rays_out", ctypes.c_void_p),
    ]


GMM_RAY_BYTES = 36  # alive-list entry: float sum[4], t, pos[3]; uint32 pixel | samples << 23


class FlexTables(ctypes.Structure):
    """vr_flex_tables (include/vr.h)"""
    _fields_ = [
        ("dim", ctypes.c_int), ("nbins", ctypes.c_int),
        ("n_fractal", ctypes.c_int),
        ("fractal_low", ctypes.c_void_p), ("fractal_high", ctypes.c_void_p),
        ("fractal_code", ctypes.c_void_p), ("fractal_errors", ctypes.c_void_p),
        ("n_simple", ctypes.c_int),
        ("simple_low", ctypes.c_void_p), ("simple_high", ctypes.c_void_p),
        ("simple_count", ctypes.c_void_p), ("simple_hist", ctypes.c_void_p),
        ("templates", ctypes.c_void_p), ("ntemplates", ctypes.c_int),
    ]


# every symbol include/vr.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "render_kernel", "copyInvViewMatrix", "initCuda", "freeCudaBuffers",
    "setTextureFilterMode", "basicDataProcessing", "dataProcessing",
    "vr_last_error", "vr_last_status", "vr_clear_error", "vr_init_distribution", "vr_init_codec", "vr_synthesize_codec", "vr_codec_info",
    "vr_synthesize", "vr_volume_info", "vr_footprint_bytes", "vr_volume_layout", "vr_set_stream", "vr_render", "vr_count_footprint",
    "vr_unscatter_tiles", "vr_tiles_x", "vr_tiles_y", "vr_version", "vr_last_kernel", "vr_selftest_logf", "vr_parse_codebook", "vr_parse_templates",
    "vr_load_reference_files", "vr_init_flex", "vr_flex_process", "vr_flex_info",
    "vr_parse_span_list", "vr_parse_fractal_histogram", "vr_parse_simple_histogram",
    "vr_load_flex_files", "vr_debug_wave_clock", "vr_debug_box_check",
    "vr_init_gmm", "vr_synthesize_gmm", "vr_gmm_info", "vr_free_gmm", "vr_gmm_select", "vr_render_gmm",
    "vr_gmm_count_footprint", "vr_gmm_count_footprint_slab", "vr_bake_stats", "vr_release_stats", "vr_stats_info",
    "vr_set_tuning", "vr_clear_tuning", "vr_stream_read", "vr_set_layout_budget",
    "vr_layout_info",
]

_lib = None


def load() -> ctypes.CDLL:
    """Load libvr.so (raises OSError / FileNotFoundError when absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(
            f"{LIB_PATH} is missing: build the HIP library first (__graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, f32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_float, ctypes.c_int
    L.render_kernel.argtypes = [Dim3, Dim3, vp, u32, u32, f32, f32, f32, f32, i32, Extent]
    L.render_kernel.restype = None
    L.copyInvViewMatrix.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_size_t]
    L.copyInvViewMatrix.restype = None
    L.initCuda.argtypes = [vp, Extent, Extent, vp, Extent, vp, Extent, vp, Extent,
                           vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.initCuda.restype = None
    L.freeCudaBuffers.argtypes = []
    L.freeCudaBuffers.restype = None
    L.setTextureFilterMode.argtypes = [ctypes.c_bool]
    L.setTextureFilterMode.restype = None
    L.basicDataProcessing.argtypes = []
    L.basicDataProcessing.restype = None
    L.dataProcessing.argtypes = []
    L.dataProcessing.restype = None
    L.vr_last_error.argtypes = []
    L.vr_last_error.restype = ctypes.c_char_p
    L.vr_last_status.argtypes = []
    L.vr_last_status.restype = i32
    L.vr_clear_error.argtypes = []
    L.vr_clear_error.restype = None
    L.vr_init_distribution.argtypes = [vp, Extent, i32, i32]
    L.vr_init_distribution.restype = i32
    L.vr_synthesize.argtypes = [Extent, i32, ctypes.c_uint64]
    L.vr_synthesize.restype = i32
    L.vr_volume_info.argtypes = [ctypes.POINTER(Extent), ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(ctypes.c_void_p)]
    L.vr_volume_info.restype = i32
    L.vr_volume_layout.argtypes = [ctypes.POINTER(ctypes.c_size_t),
                                   ctypes.POINTER(ctypes.c_size_t)]
    L.vr_volume_layout.restype = i32
    L.vr_set_stream.argtypes = [vp]
    L.vr_set_stream.restype = i32
    L.vr_render.argtypes = [ctypes.POINTER(RenderDesc)]
    L.vr_render.restype = i32
    L.vr_count_footprint.argtypes = [ctypes.POINTER(RenderDesc)]
    L.vr_count_footprint.restype = ctypes.c_int64
    L.vr_unscatter_tiles.argtypes = [vp, vp, u32, u32, vp, u32, u32]
    L.vr_unscatter_tiles.restype = i32
    L.vr_tiles_x.argtypes = [u32]
    L.vr_tiles_x.restype = u32
    L.vr_tiles_y.argtypes = [u32]
    L.vr_tiles_y.restype = u32
    L.vr_version.argtypes = []
    L.vr_version.restype = ctypes.c_char_p
    L.vr_parse_codebook.argtypes = [ctypes.c_char_p, i32, ctypes.c_longlong, vp, vp]
    L.vr_parse_codebook.restype = ctypes.c_longlong
    L.vr_parse_templates.argtypes = [ctypes.c_char_p, i32, ctypes.c_longlong, vp]
    L.vr_parse_templates.restype = ctypes.c_longlong
    L.vr_load_reference_files.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                          Extent, i32]
    L.vr_load_reference_files.restype = i32
    L.vr_stream_read.argtypes = [i32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint64)]
    L.vr_stream_read.restype = i32
    L.vr_selftest_logf.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    L.vr_selftest_logf.restype = ctypes.c_int
    L.vr_init_codec.argtypes = [vp, Extent, vp, i32, vp, i32, i32, i32]
    L.vr_init_codec.restype = i32
    L.vr_synthesize_codec.argtypes = [Extent, i32, i32, i32, ctypes.c_uint64]
    L.vr_synthesize_codec.restype = i32
    L.vr_codec_info.argtypes = [vp] * 7
    L.vr_codec_info.restype = i32
    L.vr_footprint_bytes.argtypes = [ctypes.POINTER(RenderDesc)]
    L.vr_footprint_bytes.restype = ctypes.c_int64
    L.vr_init_flex.argtypes = [ctypes.POINTER(FlexTables)]
    L.vr_init_flex.restype = i32
    L.vr_flex_process.argtypes = [i32]
    L.vr_flex_process.restype = i32
    L.vr_flex_info.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), vp]
    L.vr_flex_info.restype = i32
    ll = ctypes.c_longlong
    L.vr_parse_span_list.argtypes = [ctypes.c_char_p, ll, vp, vp]
    L.vr_parse_span_list.restype = ll
    L.vr_parse_fractal_histogram.argtypes = [ctypes.c_char_p, vp, vp, ll, i32, ll, vp, vp, vp, vp]
    L.vr_parse_fractal_histogram.restype = ll
    L.vr_parse_simple_histogram.argtypes = [ctypes.c_char_p] * 3 + [i32, ll, vp, vp, vp, vp]
    L.vr_parse_simple_histogram.restype = ll
    L.vr_load_flex_files.argtypes = [ctypes.c_char_p] * 6 + [i32, i32]
    L.vr_load_flex_files.restype = i32
    L.vr_debug_wave_clock.argtypes = [ctypes.c_void_p]
    L.vr_debug_wave_clock.restype = ctypes.c_int
    L.vr_debug_box_check.argtypes = [ctypes.c_void_p]
    L.vr_debug_box_check.restype = ctypes.c_int
    L.vr_last_kernel.argtypes = []
    L.vr_last_kernel.restype = ctypes.c_char_p
    L.vr_init_gmm.argtypes = [vp, vp, Extent, i32, i32, i32, i32]
    L.vr_init_gmm.restype = i32
    L.vr_synthesize_gmm.argtypes = [Extent, i32, ctypes.c_uint64, i32, i32]
    L.vr_synthesize_gmm.restype = i32
    L.vr_gmm_info.argtypes = [vp] * 6
    L.vr_gmm_info.restype = i32
    L.vr_free_gmm.argtypes = []
    L.vr_free_gmm.restype = i32
    L.vr_render_gmm.argtypes = [ctypes.POINTER(RenderDesc), ctypes.POINTER(GmmSlab)]
    L.vr_render_gmm.restype = i32
    L.vr_gmm_count_footprint.argtypes = [ctypes.POINTER(RenderDesc)]
    L.vr_gmm_count_footprint.restype = ctypes.c_int64
    L.vr_gmm_select.argtypes = [ctypes.c_int]
    L.vr_gmm_select.restype = ctypes.c_int
    L.vr_gmm_count_footprint_slab.argtypes = [ctypes.POINTER(RenderDesc), ctypes.POINTER(GmmSlab)]
    L.vr_gmm_count_footprint_slab.restype = ctypes.c_int64
    L.vr_bake_stats.argtypes = []
    L.vr_bake_stats.restype = i32
    L.vr_release_stats.argtypes = []
    L.vr_release_stats.restype = i32
    L.vr_stats_info.argtypes = [vp] * 4
    L.vr_stats_info.restype = i32
    L.vr_set_layout_budget.argtypes = [ctypes.c_uint64]
    L.vr_set_layout_budget.restype = i32
    L.vr_layout_info.argtypes = [vp] * 4
    L.vr_layout_info.restype = i32
    L.vr_set_tuning.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    L.vr_set_tuning.restype = i32
    L.vr_clear_tuning.argtypes = []
    L.vr_clear_tuning.restype = None
    _lib = L
    return L


def last_error() -> str:
    return load().vr_last_error().decode()


def check(status: int) -> int:
    """Raise VRError for a negative status (message from vr_last_error)."""
    if status < 0:
        msg = last_error()
        load().vr_clear_error()
        raise VRError(int(status), msg)
    return status


def check_last() -> None:
    """Raise if a void reference entry point recorded an error."""
    L = load()
    st = L.vr_last_status()
    if st != VR_OK:
        msg = last_error()
        L.vr_clear_error()
        raise VRError(st, msg)
