"""Loader for libgs_raster.so, the gfx950 kernels behind include/gs_raster.h.

There is deliberately NO fallback: if the shared library is missing or no
ROCm GPU is visible, every entry point raises.  (The CPU restatement under
``oracle/`` is test infrastructure and is never imported from here.)
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# DGE_AMD_LIB: an alternative in-tree build of the same ABI (A/B kernel experiments)
LIB_PATH = os.environ.get("DGE_AMD_LIB") or os.path.join(_HERE, "lib", "libgs_raster.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "gs_raster.h")

ABI_VERSION = 21  # GS_RASTER_ABI_VERSION of include/gs_raster.h this binding is written against


def source_stamp() -> str:
    """A stamp of the kernel sources the library is built from (sha1 of dge_amd/csrc/*.hip and *.h, by name):
    profiles/pmc_traffic.json records the stamp of the build it measured, and bench.py reports whether the
    running build still has it."""
    import glob
    import hashlib

    h = hashlib.sha1()
    csrc = os.path.join(_HERE, "csrc")
    for f in sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]

GS_OK = 0
GS_ERR_INVALID_ARG = 1
GS_ERR_HIP = 2
GS_ERR_ALLOC = 3
GS_ERR_PREFILTERED = 4
GS_ERR_UNSUPPORTED = 5
GS_ERR_RETRY = 6

MAX_VIEWS = 8  # GS_MAX_VIEWS
VIEWS_EXACT, VIEWS_SPECULATE = 0, 1

_fp = ctypes.c_void_p  # device pointers travel as opaque addresses


class GsSettings(ctypes.Structure):
    """struct gs_settings (include/gs_raster.h)."""

    _fields_ = [
        ("image_height", ctypes.c_int),
        ("image_width", ctypes.c_int),
        ("tanfovx", ctypes.c_float),
        ("tanfovy", ctypes.c_float),
        ("bg", _fp),
        ("scale_modifier", ctypes.c_float),
        ("viewmatrix", _fp),
        ("projmatrix", _fp),
        ("sh_degree", ctypes.c_int),
        ("campos", _fp),
        ("prefiltered", ctypes.c_int),
        ("debug", ctypes.c_int),
    ]


class GsParams(ctypes.Structure):
    """struct gs_params (include/gs_raster.h)."""

    _fields_ = [
        ("P", ctypes.c_int),
        ("M", ctypes.c_int),
        ("means3D", _fp),
        ("sh_dc", _fp),
        ("sh_rest", _fp),
        ("sh_dc_stride", ctypes.c_int),
        ("sh_rest_stride", ctypes.c_int),
        ("colors_precomp", _fp),
        ("opacities", _fp),
        ("scales", _fp),
        ("rotations", _fp),
        ("cov3D_precomp", _fp),
        ("activation", ctypes.c_int),
        ("sh_half", ctypes.c_int),
        ("index", ctypes.c_void_p),
        ("visible_out", ctypes.c_void_p),
        ("forward_only", ctypes.c_int),
        ("aux_mask", ctypes.c_void_p),
    ]


# gs_grads.accumulate bits (include/gs_raster.h)
ACC_MEANS2D, ACC_COLORS, ACC_OPACITY, ACC_MEANS3D, ACC_COV3D, ACC_SH = 1, 2, 4, 8, 16, 32
ACC_SCALES, ACC_ROTATIONS = 128, 256


class GsGrads(ctypes.Structure):
    """struct gs_grads (include/gs_raster.h)."""

    _fields_ = [
        ("dL_dmeans2D", _fp),
        ("dL_dcolors", _fp),
        ("dL_dopacity", _fp),
        ("dL_dmeans3D", _fp),
        ("dL_dcov3D", _fp),
        ("dL_dsh_dc", _fp),
        ("dL_dsh_rest", _fp),
        ("dsh_dc_stride", ctypes.c_int),
        ("dsh_rest_stride", ctypes.c_int),
        ("dL_dscales", _fp),
        ("dL_drotations", _fp),
        ("accumulate", ctypes.c_uint),
        ("grad_mask", ctypes.c_void_p),
        ("mask_bits", ctypes.c_uint),
        ("dL_dconic", _fp),
        ("writes_after", ctypes.c_void_p),
        ("zeroed", ctypes.c_uint),
        ("pitch_means3D", ctypes.c_int),
        ("pitch_opacity", ctypes.c_int),
        ("pitch_scales", ctypes.c_int),
        ("pitch_rotations", ctypes.c_int),
        ("dirty_rows", ctypes.c_void_p),
    ]


class AdamSegment(ctypes.Structure):
    """struct gs_adam_segment (include/gs_raster.h)."""

    _fields_ = [
        ("param", ctypes.c_void_p),
        ("grad", ctypes.c_void_p),
        ("exp_avg", ctypes.c_void_p),
        ("exp_avg_sq", ctypes.c_void_p),
        ("n", ctypes.c_longlong),
        ("step_size", ctypes.c_float),
        ("bias_correction2_sqrt", ctypes.c_float),
        ("grad_width", ctypes.c_int),
        ("grad_pitch", ctypes.c_int),
    ]


class RowsRegion(ctypes.Structure):
    """struct gs_rows_region (include/gs_raster.h)."""

    _fields_ = [("base", ctypes.c_void_p), ("width", ctypes.c_int), ("pitch", ctypes.c_int)]


ROWS_MAX_REGIONS = 8

ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t)

# Every symbol include/gs_raster.h declares, with its ctypes signature.
SIGNATURES = {
    "gs_rasterize_forward": (ctypes.c_int, [ctypes.POINTER(GsSettings), ctypes.c_int, ctypes.c_int] + [_fp] * 10
                             + [ALLOC_FN, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "gs_rasterize_backward": (ctypes.c_int, [ctypes.POINTER(GsSettings), ctypes.c_int, ctypes.c_int, ctypes.c_int]
                              + [_fp] * 19 + [ctypes.c_void_p]),
    "gs_rasterize_forward_ex": (ctypes.c_int, [ctypes.POINTER(GsSettings), ctypes.POINTER(GsParams), _fp, _fp, _fp,
                                                ALLOC_FN, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.POINTER(ctypes.c_int)]),
    "gs_rasterize_forward_begin": (ctypes.c_int, [ctypes.POINTER(GsSettings), ctypes.POINTER(GsParams), _fp, ALLOC_FN,
                                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "gs_rasterize_forward_end": (ctypes.c_int, [ctypes.c_void_p, _fp, _fp, ALLOC_FN, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.POINTER(ctypes.c_int)]),
    "gs_rasterize_forward_release": (None, [ctypes.c_void_p]),
    "gs_rasterize_backward_ex": (ctypes.c_int, [ctypes.POINTER(GsSettings), ctypes.POINTER(GsParams), ctypes.c_int,
                                                 _fp, _fp, _fp, _fp, _fp, ctypes.POINTER(GsGrads), ctypes.c_void_p]),
    "gs_rasterize_backward_replay": (ctypes.c_int, [ctypes.POINTER(GsSettings), ctypes.POINTER(GsParams), ctypes.c_int,
                                                     _fp, _fp, _fp, _fp, _fp, ctypes.POINTER(GsGrads), ctypes.c_void_p]),
    "gs_rasterize_backward_passes": (ctypes.c_int, [ctypes.c_int] + [ctypes.c_void_p] * 8),
    "gs_views_forward": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ALLOC_FN, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "gs_views_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "gs_views_backward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "gs_views_overflow": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gs_views_buffer": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "gs_views_layout": (ctypes.c_longlong, [ctypes.c_void_p, ctypes.c_int]),
    "gs_views_release": (None, [ctypes.c_void_p]),
    "gs_mark_visible": (ctypes.c_int, [ctypes.c_int, _fp, _fp, _fp, _fp, ctypes.c_void_p]),
    "gs_apply_weights": (ctypes.c_int, [ctypes.POINTER(GsSettings), ctypes.c_int, ctypes.c_int, _fp, _fp, ctypes.c_int]
                         + [_fp] * 7 + [ALLOC_FN, ctypes.c_void_p, ctypes.c_void_p]),
    "gs_geometry_buffer_size": (ctypes.c_size_t, [ctypes.c_int]),
    "gs_image_buffer_size": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]),
    "gs_binning_buffer_size": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]),
    "gs_buffer_offset": (ctypes.c_longlong, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int]),
    "gs_profile_enable": (ctypes.c_int, [ctypes.c_int]),
    "gs_profile_set_stages": (ctypes.c_int, [ctypes.c_uint]),
    "gs_profile_num_stages": (ctypes.c_int, []),
    "gs_profile_stage_name": (ctypes.c_char_p, [ctypes.c_int]),
    "gs_profile_collect": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "gs_host_wait_ns": (ctypes.c_longlong, []),
    "gs_profile_diag_enable": (ctypes.c_int, [ctypes.c_int]),
    "gs_profile_diag_read": (ctypes.c_longlong, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_longlong]),
    "gs_timer_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p)]),
    "gs_timer_record": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "gs_timer_elapsed_ms": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]),
    "gs_timer_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "gs_adam_step": (ctypes.c_int, [ctypes.POINTER(AdamSegment), ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_float, ctypes.c_void_p]),
    "gs_rows_live": (ctypes.c_int, [ctypes.POINTER(RowsRegion), ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p,
                                    ctypes.c_void_p]),
    "gs_rows_gather": (ctypes.c_int, [ctypes.POINTER(RowsRegion), ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    "gs_rows_scatter": (ctypes.c_int, [ctypes.POINTER(RowsRegion), ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    "gs_rows_zero_dirty": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_longlong, ctypes.c_void_p]),
    "gs_rows_mark_dirty": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    "gs_rows_compact": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p]),
    "gs_rows_gather_dev": (ctypes.c_int, [ctypes.POINTER(RowsRegion), ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gs_rows_scatter_dev": (ctypes.c_int, [ctypes.POINTER(RowsRegion), ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gs_blend_exp": (ctypes.c_int, [ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gs_activate_params": (ctypes.c_int, [ctypes.c_int] + [ctypes.c_void_p] * 7),
    "gs_render_recolor": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 9),
    "gs_last_error": (ctypes.c_char_p, []),
    "gs_abi_version": (ctypes.c_int, []),
}

_lib = None
_lock = threading.Lock()


class NativeError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH):
    """dlopen libgs_raster.so and bind every exported symbol (no GPU needed)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise ImportError(
                f"dge_amd: {path} is missing. Build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()' or make -C dge_amd/csrc). "
                "There is no CPU fallback.")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def lib():
    return _lib if _lib is not None else load_library()


def last_error() -> str:
    msg = lib().gs_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> None:
    if rc != GS_OK:
        raise NativeError(f"{what} failed (code {rc}): {last_error()}")


_gpu_ok = False


def require_gpu(t) -> None:
    """The product path runs only on a ROCm GPU; fail loudly otherwise."""
    global _gpu_ok
    if not _gpu_ok:
        import torch

        if not torch.cuda.is_available():
            raise NativeError("dge_amd requires a ROCm GPU (torch.cuda.is_available() is False); "
                              "no CPU fallback exists")
        _gpu_ok = True
    if not getattr(t, "is_cuda", False):
        raise NativeError("dge_amd: tensors must live on the GPU")


class StepTimer:
    """A timing event without the system-scope fence (gs_timer_*): record(stream), elapsed_ms(end)."""

    def __init__(self):
        h = ctypes.c_void_p(None)
        check(lib().gs_timer_create(ctypes.byref(h)), "gs_timer_create")
        self.h = h.value

    def record(self, stream) -> None:
        check(lib().gs_timer_record(self.h, stream.cuda_stream), "gs_timer_record")

    def elapsed_ms(self, end: "StepTimer") -> float:
        ms = ctypes.c_float()
        check(lib().gs_timer_elapsed_ms(self.h, end.h, ctypes.byref(ms)), "gs_timer_elapsed_ms")
        return float(ms.value)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.gs_timer_destroy(self.h)


def profile_enable(on: bool = True) -> None:
    lib().gs_profile_enable(int(on))


def profile_stages(names=None) -> None:
    """Profile only the named stages (None: all)."""
    L = lib()
    if names is None:
        L.gs_profile_set_stages(0xFFFFFFFF)
        return
    all_names = [L.gs_profile_stage_name(i).decode() for i in range(L.gs_profile_num_stages())]
    L.gs_profile_set_stages(sum(1 << all_names.index(n) for n in names))


def profile_collect() -> dict:
    """{stage: (total_ms, launches)} since the last collect (see gs_profile_collect)."""
    L = lib()
    n = L.gs_profile_num_stages()
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int * n)()
    check(L.gs_profile_collect(ms, cnt, n), "gs_profile_collect")
    return {L.gs_profile_stage_name(i).decode(): (ms[i], cnt[i]) for i in range(n)}


def diag_enable(on: bool = True) -> None:
    lib().gs_profile_diag_enable(int(on))


def diag_read(which: int, max_u64: int = 1 << 20):
    """Per-wave diagnostics of the last forward (which=0) / backward (which=1) blend launch
    (which=2: k_gauss_bwd_live phase stamps, see gs_backward.hip):
    numpy [n, 8] of (start, end) in 10 ns ticks, kept entries, rounds, loop cycles, total cycles, 0, 0."""
    import numpy as np

    buf = (ctypes.c_uint64 * max_u64)()
    n = lib().gs_profile_diag_read(int(which), buf, max_u64)
    return np.frombuffer(buf, dtype=np.uint64, count=n).reshape(-1, 8).copy()
