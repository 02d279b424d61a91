"""ctypes binding of the C ABI declared in include/sks_homography.h.

The product path is the HIP library only: if lib/libsks_homography_amd.so is
missing or fails to load, every entry point raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libsks_homography_amd.so")
TORCH_LIB_PATH = os.path.join(HERE, "lib", "libsks_homography_torch.so")
TUNE_LIB_PATH = os.path.join(HERE, "lib", "libsks_homography_tune.so")
MULTI_LIB_PATH = os.path.join(HERE, "lib", "libsks_homography_multi.so")

HG_LAYOUT_AOS = 0
HG_LAYOUT_SOA = 1
HG_FLAG_NORMALIZE = 1
HG_FLAG_HOST_REGISTER = 2  # hg_solve_host_* only: register pageable pages instead of staging

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int

# name -> (argtypes, restype); mirrors include/sks_homography.h one for one.
SIGNATURES = {
    "hg_aca_f32": ([_vp, _vp, _vp, _i64, _int, _int, _vp], _int),
    "hg_aca_f64": ([_vp, _vp, _vp, _i64, _int, _int, _vp], _int),
    "hg_sks_f32": ([_vp, _vp, _vp, _i64, _int, _int, _vp], _int),
    "hg_sks_f64": ([_vp, _vp, _vp, _i64, _int, _int, _vp], _int),
    "hg_ge_f32": ([_vp, _vp, _vp, _i64, _int, _int, _vp], _int),
    "hg_ge_f64": ([_vp, _vp, _vp, _i64, _int, _int, _vp], _int),
    "hg_gpt_f64": ([_vp, _vp, _vp, _i64, _int, _int, _vp], _int),
    "hg_tensor_aca_rect_f32": ([_vp, _vp, _vp, _i64, _vp, _vp, _vp], _int),
    "hg_tensor_aca_rect_f32_hostscalar": ([_vp, _vp, _vp, _i64, ctypes.c_float, ctypes.c_float,
                                           _vp], _int),
    "hg_tensor_aca_rect_backward_f32": ([_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp], _int),
    "hg_tensor_aca_rect_backward_terms_f32": ([_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp], _int),
    "hg_tensor_aca_rect_backward_sum_f32": ([_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _int, _int, _vp, _vp], _int),
    "hg_tensor_aca_rect_bcast_f32": ([_vp, _vp, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp],
                                     _int),
    "hg_tensor_aca_rect_bcast_backward_f32": ([_vp, _vp, _vp, _i64, _vp, _i64, _i64, _vp, _i64,
                                               _i64, _vp, _vp, _vp, _int, _vp, _int, _vp], _int),
    "hg_tensor_aca_rect_order_f32": ([_vp, _vp, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _int,
                                      _vp], _int),
    "hg_tensor_aca_rect_backward_order_f32": ([_vp, _vp, _vp, _i64, _vp, _i64, _i64, _vp, _i64,
                                               _i64, _vp, _vp, _vp, _int, _vp, _int, _int, _vp],
                                              _int),
    "hg_sum_rocm_f32": ([_vp, _i64, _int, _vp, _vp, _vp], _int),
    "hg_sum_rocm_plan": ([_i64, _int, _int, _int, _vp], _int),
    "hg_tensor_aca_offsets_f32": ([_vp, _vp, _vp, _i64, ctypes.c_float, ctypes.c_float, _vp],
                                  _int),
    "hg_tensor_aca_offsets_backward_f32": ([_vp, _vp, _vp, _i64, ctypes.c_float, ctypes.c_float,
                                           _vp, _vp, _vp], _int),
    "hg_aca_backward_f32": ([_vp, _vp, _vp, _i64, _vp, _vp, _vp], _int),
    "hg_aca_backward_f64": ([_vp, _vp, _vp, _i64, _vp, _vp, _vp], _int),
    "hg_fill_uniform_f32": ([_vp, _i64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_float,
                             ctypes.c_float, _vp], _int),
    "hg_fill_bits_u32": ([_vp, _i64, ctypes.c_uint64, ctypes.c_uint64, _vp], _int),
    "hg_sample_solve_f32": ([_vp, _vp, ctypes.c_uint32, _vp, _vp, _i64, _int, _int, _vp], _int),
    "hg_sample_solve_seeded_f32": ([_vp, _vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                    _vp, _i64, _int, _int, _vp], _int),
    "hg_ransac_score_f32": ([_vp, _i64, _vp, _vp, ctypes.c_uint32, ctypes.c_float, _vp, _vp],
                            _int),
    "hg_rand_mrg32k3a_u32": ([_vp, _i64, ctypes.c_uint64, _vp], _int),
    "hg_mrg32k3a_state": ([ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _vp], _int),
    "hg_rand_gather_solve_f64": ([_int, _vp, _vp, ctypes.c_uint32, ctypes.c_uint64, _vp, _i64, _int,
                                  _vp], _int),
    "hg_get_rand_list_f64": ([_vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _i64, _vp], _int),
    "hg_gather_solve_f64": ([_int, _vp, _vp, ctypes.c_uint32, _vp, _vp, _i64, _int, _vp], _int),
    "hg_solve_one_f32": ([_int, _vp, _vp, _vp, _int, _vp], _int),
    "hg_solve_one_f64": ([_int, _vp, _vp, _vp, _int, _vp], _int),
    "hg_solve_host_f32": ([_int, _vp, _vp, _vp, _i64, _int, _int, _vp], _int),
    "hg_solve_host_f64": ([_int, _vp, _vp, _vp, _i64, _int, _int, _vp], _int),
    "hg_solve_grouped_f32": ([_int, _vp, _vp, _vp, _vp, _int, _int, _int, _vp], _int),
    "hg_solve_grouped_f64": ([_int, _vp, _vp, _vp, _vp, _int, _int, _int, _vp], _int),
    "hg_sum_rows_f32": ([_vp, _i64, _i64, _vp, _vp], _int),
    "hg_sum_aten_f32": ([_vp, _i64, _i64, _i64, _i64, _int, _int, _vp, _vp], _int),
    "hg_stream_copy": ([_vp, _vp, _i64, _vp], _int),
    "hg_version": ([], ctypes.c_char_p),
}

_lock = threading.Lock()
_lib = None


class HipError(RuntimeError):
    """A C-ABI entry point returned a non-zero hipError_t."""

    def __init__(self, fn: str, code: int):
        super().__init__(f"{fn} failed with hipError_t {code}")
        self.code = code


def lib() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`"
                    " (the MI355X kernels have no CPU fallback)")
            handle = ctypes.CDLL(LIB_PATH)
            for name, (argtypes, restype) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.argtypes = argtypes
                fn.restype = restype
            _lib = handle
    return _lib


_tune = None


def tune() -> ctypes.CDLL:
    """The kernel-variant / timing-loop library (include/sks_homography_tune.h) used by
    tools/ and tests; not part of the product path."""
    global _tune
    if _tune is None:
        lib()  # the product library first (the tune library links it)
        if not os.path.exists(TUNE_LIB_PATH):
            raise ImportError(f"{TUNE_LIB_PATH} not built: run build()")
        _tune = ctypes.CDLL(TUNE_LIB_PATH)
    return _tune


class DeviceBatch(ctypes.Structure):
    """hg_device_batch (include/sks_homography_multi.h)."""
    _fields_ = [("device", ctypes.c_int), ("src", ctypes.c_void_p), ("tar", ctypes.c_void_p),
                ("H", ctypes.c_void_p), ("n", ctypes.c_int64), ("stream", ctypes.c_void_p)]


MULTI_SIGNATURES = {
    "hg_shard_range": ([_i64, _int, _int, ctypes.POINTER(_i64), ctypes.POINTER(_i64)], _int),
    "hg_solve_multi": ([_int, _int, ctypes.POINTER(DeviceBatch), _int, _int, _int], _int),
    "hg_sync_multi": ([ctypes.POINTER(DeviceBatch), _int], _int),
    "hg_comm_init_all": ([_int, ctypes.POINTER(_int), ctypes.POINTER(_vp)], _int),
    "hg_comm_destroy": ([_int, ctypes.POINTER(_vp)], _int),
    "hg_gather_multi": ([ctypes.POINTER(DeviceBatch), _int, _int, _int, _vp, ctypes.POINTER(_vp)],
                        _int),
}
_multi = None


def multi() -> ctypes.CDLL:
    """The multi-GPU C ABI (include/sks_homography_multi.h; links librccl)."""
    global _multi
    if _multi is None:
        lib()  # the product library first (the multi library links it)
        if not os.path.exists(MULTI_LIB_PATH):
            raise ImportError(f"{MULTI_LIB_PATH} not built: run build()")
        m = ctypes.CDLL(MULTI_LIB_PATH)
        for name, (args, res) in MULTI_SIGNATURES.items():
            fn = getattr(m, name)
            fn.argtypes, fn.restype = args, res
        _multi = m
    return _multi


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise HipError(name, rc)


def version() -> str:
    return lib().hg_version().decode()
