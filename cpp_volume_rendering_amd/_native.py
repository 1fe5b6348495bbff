"""ctypes binding of the C-ABI in include/cvr.h (libcvr.so, built in-tree).

The shared library is the product: HIP kernels for gfx950 plus the C-ABI.
There is no fallback — if libcvr.so is missing or cannot be loaded the import
fails loudly (run ``python -c "import __graft_entry__ as g; g.build()"``).

torch is imported before the library is loaded so that libcvr.so binds to the
HIP runtime torch already carries (both have SONAME libamdhip64.so.7); device
pointers and streams can then be shared with torch tensors.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen below, see module docstring)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libcvr.so")
# tools/ab_builds.sh: A/B timing of two builds of the library in one GPU session
LIB_PATH = os.environ.get("CVR_LIB_OVERRIDE", LIB_PATH)

# include/cvr.h CVR_ABI_VERSION: the struct layouts declared below
ABI_VERSION = 2

CVR_OK, CVR_ERR_ARG, CVR_ERR_HIP, CVR_ERR_OOM, CVR_ERR_STATE, CVR_ERR_IO = range(6)
GRADIENT_NONE, GRADIENT_FINITE_DIFFERENCES, GRADIENT_SOBEL_FELDMAN = 0, 1, 2

# Every symbol include/cvr.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "cvr_abi_version", "cvr_status_string", "cvr_create", "cvr_destroy", "cvr_last_error",
    "cvr_set_stream", "cvr_set_option", "cvr_get_option", "cvr_synchronize", "cvr_set_volume", "cvr_set_volume_device",
    "cvr_set_transfer_function", "cvr_set_gradient", "cvr_device_bytes", "cvr_copy_cells", "cvr_tiles_for_rank",
    "cvr_render_rc1pass", "cvr_render_rc1pass_frames", "cvr_unpack_tiles_device", "cvr_copy_tile_stats", "cvr_read_kernel_times", "cvr_read_shade_counters", "cvr_selftest_arith", "cvr_camera_lookat", "cvr_default_step",
    "cvr_tf1d_build_rgbt", "cvr_read_tf1d", "cvr_read_raw", "cvr_read_syn", "cvr_read_pvm",
    "cvr_read_camera_state", "cvr_read_light_position", "cvr_read_light", "cvr_build_cone_tables",
    "cvr_set_extinction_volume", "cvr_copy_extinction_level", "cvr_render_dosct",
    "cvr_tf1d_ext_lut", "cvr_set_extinction_sat", "cvr_copy_extinction_sat", "cvr_sat_layout_check", "cvr_render_extbsd",
    "cvr_comm_unique_id", "cvr_comm_init", "cvr_comm_destroy", "cvr_gather_tiles",
    "cvr_gather_tiles_n", "cvr_unpack_tiles_device_n", "cvr_tile_code_bound", "cvr_encode_tiles",
    "cvr_decode_tiles", "cvr_comm_init_local", "cvr_create_group", "cvr_group_size",
    "cvr_group_member",
    "cvr_gather_sync", "cvr_multiscale_resolution", "cvr_multiscale_filter",
    "cvr_screenshot_rgb8", "cvr_iso_params_default", "cvr_render_iso", "cvr_iso_block_ranges",
)
SINGLE_RAY_PER_PIXEL, MULTIPLE_RAYS_PER_PIXEL, DOWN_SCALING_RENDER, UP_SCALING_RENDER = range(4)
(FILTER_BOX, FILTER_HAT, FILTER_CATMULL_ROM, FILTER_MITCHELL_NETRAVALI, FILTER_CARDINAL_BSPLINE_3,
 FILTER_CARDINAL_OMOMS3) = range(6)
COMM_ID_BYTES = 128
MAX_GATHER_SETS = 64   # cvr.h CVR_MAX_GATHER_SETS


class CvrError(RuntimeError):
    def __init__(self, status: int, where: str, detail: str = ""):
        self.status = status
        super().__init__(f"{where}: {_status_name(status)}" + (f" — {detail}" if detail else ""))


class Camera(ctypes.Structure):
    _fields_ = [("eye", ctypes.c_float * 3), ("center", ctypes.c_float * 3),
                ("up", ctypes.c_float * 3), ("fovy_deg", ctypes.c_float),
                ("aspect", ctypes.c_float)]


class Frame(ctypes.Structure):
    _fields_ = [("camera", Camera), ("width", ctypes.c_int), ("height", ctypes.c_int),
                ("tile_size", ctypes.c_int), ("rank", ctypes.c_int), ("nranks", ctypes.c_int),
                ("use_view", ctypes.c_int), ("view", ctypes.c_float * 16)]


FORMAT_RGBA32F = 0
FORMAT_RGBA16F = 1   # the reference's RGBA16F frame (imageStore rounding: nearest even)


class Output(ctypes.Structure):
    _fields_ = [("rgba", ctypes.c_void_p), ("samples", ctypes.c_void_p),
                ("total", ctypes.c_void_p), ("on_device", ctypes.c_int),
                ("format", ctypes.c_int)]


class Rc1passParams(ctypes.Structure):
    _fields_ = [("step", ctypes.c_float), ("apply_gradient_shading", ctypes.c_int),
                ("ka", ctypes.c_float), ("kd", ctypes.c_float), ("ks", ctypes.c_float),
                ("shininess", ctypes.c_float), ("ispecular", ctypes.c_float * 3),
                ("light_pos", ctypes.c_float * 3)]


MAX_CONE_SECTIONS = 1024


class ConeParams(ctypes.Structure):
    _fields_ = [("half_angle_deg", ctypes.c_float), ("max_packing", ctypes.c_int),
                ("covered_distance", ctypes.c_float), ("ui_weight", ctypes.c_float),
                ("initial_step", ctypes.c_float)]


class ConeTables(ctypes.Structure):
    _fields_ = [("n_sections", ctypes.c_int), ("counts", ctypes.c_int * 3),
                ("initial_step", ctypes.c_float), ("ray7_adj_weight", ctypes.c_float),
                ("ui_weight", ctypes.c_float), ("axes", (ctypes.c_float * 3) * 10),
                ("sections", (ctypes.c_float * 4) * MAX_CONE_SECTIONS)]


class Light(ctypes.Structure):
    _fields_ = [("position", ctypes.c_float * 3), ("forward", ctypes.c_float * 3),
                ("up", ctypes.c_float * 3), ("right", ctypes.c_float * 3),
                ("spot_angle_deg", ctypes.c_float)]


class DosParams(ctypes.Structure):
    _fields_ = [("step", ctypes.c_float), ("apply_gradient_shading", ctypes.c_int),
                ("ka", ctypes.c_float), ("kd", ctypes.c_float), ("ks", ctypes.c_float),
                ("shininess", ctypes.c_float), ("ispecular", ctypes.c_float * 3),
                ("light", Light), ("apply_occlusion", ctypes.c_int),
                ("apply_shadow", ctypes.c_int), ("shadow_type", ctypes.c_int),
                ("occlusion", ConeParams), ("shadow", ConeParams)]


class EbsParams(ctypes.Structure):
    _fields_ = [("step", ctypes.c_float), ("apply_gradient_shading", ctypes.c_int),
                ("ka", ctypes.c_float), ("kd", ctypes.c_float), ("ks", ctypes.c_float),
                ("shininess", ctypes.c_float), ("ispecular", ctypes.c_float * 3),
                ("light_pos", ctypes.c_float * 3), ("light_forward", ctypes.c_float * 3),
                ("apply_occlusion", ctypes.c_int), ("occlusion_shells", ctypes.c_int),
                ("occlusion_radius", ctypes.c_float), ("apply_shadow", ctypes.c_int),
                ("shadow_type", ctypes.c_int), ("shadow_cone_angle_deg", ctypes.c_float),
                ("shadow_sample_interval", ctypes.c_float), ("shadow_initial_step", ctypes.c_float),
                ("shadow_ui_weight", ctypes.c_float), ("shadow_max_distance", ctypes.c_float)]


class IsoParams(ctypes.Structure):
    _fields_ = [("variant", ctypes.c_int), ("num_blocks", ctypes.c_int * 3),
                ("isovalue", ctypes.c_float), ("step_small", ctypes.c_float),
                ("step_large", ctypes.c_float), ("step_range", ctypes.c_float),
                ("color", ctypes.c_float * 4), ("apply_gradient_shading", ctypes.c_int),
                ("ka", ctypes.c_float), ("kd", ctypes.c_float), ("ks", ctypes.c_float),
                ("shininess", ctypes.c_float), ("ispecular", ctypes.c_float * 3),
                ("light_pos", ctypes.c_float * 3)]


_lib = None


def _status_name(st: int) -> str:
    names = {0: "CVR_OK", 1: "CVR_ERR_ARG", 2: "CVR_ERR_HIP", 3: "CVR_ERR_OOM",
             4: "CVR_ERR_STATE", 5: "CVR_ERR_IO"}
    return names.get(st, f"status {st}")


def lib() -> ctypes.CDLL:
    """Load libcvr.so (once) and declare the C signatures."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libcvr.so not built: {LIB_PATH} is missing "
                          "(build with __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P, I, F, V = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, None
    FP = ctypes.POINTER(ctypes.c_float)
    DP = ctypes.POINTER(ctypes.c_double)
    IP = ctypes.POINTER(ctypes.c_int)
    sig = {
        "cvr_abi_version": ([], I),
        "cvr_status_string": ([I], ctypes.c_char_p),
        "cvr_create": ([I, ctypes.POINTER(P)], I),
        "cvr_destroy": ([P], V),
        "cvr_last_error": ([P], ctypes.c_char_p),
        "cvr_set_stream": ([P, P], I),
        "cvr_synchronize": ([P], I),
        "cvr_set_option": ([P, ctypes.c_char_p, I], I),
        "cvr_get_option": ([P, ctypes.c_char_p], I),
        "cvr_set_volume": ([P, P, I, I, I, I, FP], I),
        "cvr_set_volume_device": ([P, P, I, I, I, I, FP], I),
        "cvr_set_transfer_function": ([P, FP, I], I),
        "cvr_set_gradient": ([P, I], I),
        "cvr_device_bytes": ([P], ctypes.c_size_t),
        "cvr_copy_cells": ([P, P, ctypes.c_size_t], I),
        "cvr_tiles_for_rank": ([ctypes.POINTER(Frame), I], I),
        "cvr_render_rc1pass": ([P, ctypes.POINTER(Frame), ctypes.POINTER(Rc1passParams),
                                ctypes.POINTER(Output)], I),
        "cvr_render_rc1pass_frames": ([P, ctypes.POINTER(Frame), I, ctypes.POINTER(Rc1passParams),
                                       ctypes.POINTER(Output)], I),
        "cvr_unpack_tiles_device": ([P, ctypes.POINTER(Frame), P, I, I, P], I),
        "cvr_comm_unique_id": ([ctypes.c_char_p], I),
        "cvr_comm_init": ([P, I, I, ctypes.c_char_p], I),
        "cvr_comm_destroy": ([P], I),
        "cvr_comm_init_local": ([ctypes.POINTER(P), I], I),
        "cvr_create_group": ([IP, I, ctypes.POINTER(P)], I),
        "cvr_group_size": ([P], I),
        "cvr_group_member": ([P, I], P),
        "cvr_gather_tiles": ([P, ctypes.POINTER(Frame), P, I, I, P, P], I),
        "cvr_gather_sync": ([P], I),
        "cvr_unpack_tiles_device_n": ([P, ctypes.POINTER(Frame), P, I, I, I, I, P], I),
        "cvr_tile_code_bound": ([I, I], ctypes.c_size_t),
        "cvr_encode_tiles": ([P, P, I, I, P, P], I),
        "cvr_decode_tiles": ([P, P, I, I, P], I),
        "cvr_gather_tiles_n": ([P, ctypes.POINTER(Frame), I, P, I, I, P,
                                ctypes.POINTER(ctypes.c_void_p)], I),
        "cvr_multiscale_resolution": ([I, I, I, IP, IP], I),
        "cvr_multiscale_filter": ([P, I, I, P, I, I, P, I, I], I),
        "cvr_screenshot_rgb8": ([P, P, I, I, I, P], I),
        "cvr_copy_tile_stats": ([P, P, I, IP], I),
        "cvr_read_kernel_times": ([P, FP, I, IP], I),
        "cvr_read_shade_counters": ([P, ctypes.POINTER(ctypes.c_uint64)], I),
        "cvr_selftest_arith": ([P, ctypes.POINTER(ctypes.c_uint64)], I),
        "cvr_camera_lookat": ([ctypes.POINTER(Camera), FP, FP], I),
        "cvr_default_step": ([FP], F),
        "cvr_tf1d_build_rgbt": ([DP, I, DP, I, I, I, FP], I),
        "cvr_read_tf1d": ([ctypes.c_char_p, FP, IP], I),
        "cvr_read_raw": ([ctypes.c_char_p, P, ctypes.c_size_t, IP, IP, IP, IP], I),
        "cvr_read_syn": ([ctypes.c_char_p, P, ctypes.c_size_t, IP, IP, IP], I),
        "cvr_read_pvm": ([ctypes.c_char_p, P, ctypes.c_size_t, IP, IP, IP, IP, FP], I),
        "cvr_read_camera_state": ([ctypes.c_char_p, I, ctypes.POINTER(Camera), ctypes.c_char_p,
                                   I, IP], I),
        "cvr_read_light_position": ([ctypes.c_char_p, I, I, FP, IP], I),
        "cvr_read_light": ([ctypes.c_char_p, I, I, ctypes.POINTER(Light), IP], I),
        "cvr_build_cone_tables": ([ctypes.POINTER(ConeParams), F, ctypes.POINTER(ConeTables)], I),
        "cvr_set_extinction_volume": ([P, FP, I, IP, F], I),
        "cvr_copy_extinction_level": ([P, I, FP, IP, IP], I),
        "cvr_render_dosct": ([P, ctypes.POINTER(Frame), ctypes.POINTER(DosParams),
                              ctypes.POINTER(Output)], I),
        "cvr_tf1d_ext_lut": ([DP, I, DP, I, I, I, I, FP], I),
        "cvr_set_extinction_sat": ([P, FP, I], I),
        "cvr_copy_extinction_sat": ([P, FP, ctypes.c_size_t, IP], I),
        "cvr_sat_layout_check": ([IP, I, I, ctypes.POINTER(ctypes.c_ulonglong)], I),
        "cvr_render_extbsd": ([P, ctypes.POINTER(Frame), ctypes.POINTER(EbsParams),
                               ctypes.POINTER(Output)], I),
        "cvr_iso_params_default": ([I, ctypes.POINTER(IsoParams)], None),
        "cvr_render_iso": ([P, ctypes.POINTER(Frame), ctypes.POINTER(IsoParams),
                            ctypes.POINTER(Output)], I),
        "cvr_iso_block_ranges": ([P, IP, FP, FP], I),
    }
    for name, (args, res) in sig.items():
        if "CVR_LIB_OVERRIDE" in os.environ and not hasattr(L, name):
            continue   # A/B timing against an older build that predates this entry point
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    got = L.cvr_abi_version()
    if got != ABI_VERSION:
        raise ImportError(f"{LIB_PATH}: ABI version {got}, this binding declares {ABI_VERSION} "
                          "(struct layouts differ; rebuild the library)")
    _lib = L
    return L


def check(status: int, where: str, ctx=None) -> None:
    if status != CVR_OK:
        detail = ""
        if ctx:
            msg = lib().cvr_last_error(ctx)
            detail = msg.decode(errors="replace") if msg else ""
        raise CvrError(status, where, detail)


def fptr(arr):
    """ctypes float* of a C-contiguous float32 numpy array."""
    return arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def dptr(arr):
    return arr.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
