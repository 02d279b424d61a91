"""ctypes front-end for the CPU checkers built by oracle/build.sh.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.

* ``Oracle``    -- our C restatement (oracle/hg_oracle.c), parity pinned against
                   tests/golden/ (which came from the reference itself).
* ``RefOracle`` -- the reference's own ACA_SKS.cpp compiled by oracle/build.sh
                   (oracle/_ref/libsks_ref.so); present wherever it was built.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SKS_ORACLE_SO / SKS_REF_SO: alternative builds of the same checkers (the ASan/UBSan builds
# of tests/test_sanitizers.py)
ORACLE_SO = os.environ.get("SKS_ORACLE_SO", os.path.join(HERE, "_build", "libhg_oracle.so"))
REF_SO = os.environ.get("SKS_REF_SO", os.path.join(HERE, "_ref", "libsks_ref.so"))
# the same reference sources built for speed (-O3, AVX-512, FMA contraction, LTO): a CPU
# baseline for bench.py only, never a checker -- its outputs are not bit-exact
REF_NATIVE_SO = os.path.join(HERE, "_ref", "libsks_ref_native.so")


def cpu_has_avx512() -> bool:
    """The x86-64-v4 feature set REF_NATIVE_SO was built for (loading it elsewhere would
    fault on the first AVX-512 instruction)."""
    try:
        flags = open("/proc/cpuinfo").read()
    except OSError:
        return False
    return all(f" {f}" in flags for f in ("avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl"))

_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_i64 = ctypes.c_int64

ALGOS = {"aca": 0, "sks": 1, "ge": 2}


def _ptr(a: np.ndarray, ctype):
    assert a.flags["C_CONTIGUOUS"], "oracle buffers must be C-contiguous"
    return a.ctypes.data_as(ctype)


class Oracle:
    """C restatement of sks::runKernel_{ACA,SKS}[_double] and TensorACA_rect."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run oracle/build.sh")
        lib = ctypes.CDLL(path)
        for name, fp in (("oracle_aca_f32", _f32p), ("oracle_sks_f32", _f32p),
                         ("oracle_aca_f64", _f64p), ("oracle_sks_f64", _f64p),
                         ("oracle_ge_f32", _f32p), ("oracle_ge_f64", _f64p),
                         ("oracle_gpt_f64", _f64p)):
            fn = getattr(lib, name)
            fn.argtypes = [fp, fp, fp, _i64, ctypes.c_int, ctypes.c_int]
            fn.restype = ctypes.c_int
        lib.oracle_tensor_aca_rect_f32.argtypes = [_f32p, _f32p, _f32p, _i64,
                                                   ctypes.c_float, ctypes.c_float]
        lib.oracle_tensor_aca_rect_f32.restype = ctypes.c_int
        lib.oracle_fill_uniform_f32.argtypes = [_f32p, _i64, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_float, ctypes.c_float]
        lib.oracle_fill_uniform_f32.restype = ctypes.c_int
        lib.oracle_tensor_aca_rect_backward_f32.argtypes = [_f32p, _f32p, _f32p, _i64,
                                                            ctypes.c_float, ctypes.c_float,
                                                            _f32p, _f32p, _f32p]
        lib.oracle_tensor_aca_rect_backward_f32.restype = ctypes.c_int
        lib.oracle_aca_vanilla_backward_f32.argtypes = [_f32p, _f32p, _f32p, _i64, _f32p, _f32p]
        lib.oracle_aca_vanilla_backward_f64.argtypes = [_f64p, _f64p, _f64p, _i64, _f64p, _f64p]
        lib.oracle_tensor_aca_rect_rows_f32.argtypes = [_f32p, _f32p, _f32p, _i64, _f32p, _f32p]
        lib.oracle_tensor_aca_rect_rows_f32.restype = ctypes.c_int
        lib.oracle_tensor_aca_rect_rows_backward_f32.argtypes = [_f32p, _f32p, _f32p, _i64, _f32p,
                                                                 _f32p, _f32p, _f32p, _f32p, _f32p,
                                                                 _f32p, _f32p]
        lib.oracle_tensor_aca_rect_rows_backward_f32.restype = ctypes.c_int
        lib.oracle_fill_bits_u32.argtypes = [ctypes.c_void_p, _i64, ctypes.c_uint64, ctypes.c_uint64]
        lib.oracle_ransac_score_f32.argtypes = [_f32p, _i64, _f32p, _f32p, ctypes.c_uint32,
                                                ctypes.c_float, ctypes.c_void_p]
        lib.oracle_time_f32.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, _i64,
                                        ctypes.c_int, ctypes.c_int]
        lib.oracle_time_f32.restype = ctypes.c_double
        self.lib = lib

    def solve(self, algo: str, src: np.ndarray, tar: np.ndarray, normalize: bool = True,
              layout: str = "aos") -> np.ndarray:
        """Batch solve.  AoS: src/tar (n,8) -> H (n,9); SoA: (8,n) -> (9,n)."""
        dt = src.dtype
        assert dt in (np.float32, np.float64) and tar.dtype == dt
        soa = layout == "soa"
        src = np.ascontiguousarray(src)
        tar = np.ascontiguousarray(tar)
        n = src.shape[1] if soa else src.shape[0]
        H = np.empty((9, n) if soa else (n, 9), dtype=dt)
        suffix = "f32" if dt == np.float32 else "f64"
        fp = _f32p if dt == np.float32 else _f64p
        fn = getattr(self.lib, f"oracle_{algo}_{suffix}")
        fn(_ptr(src, fp), _ptr(tar, fp), _ptr(H, fp), n, 1 if soa else 0, 1 if normalize else 0)
        return H

    def tensor_aca_rect(self, src: np.ndarray, tar: np.ndarray, scale: float,
                        div: float) -> np.ndarray:
        src = np.ascontiguousarray(src, dtype=np.float32)
        tar = np.ascontiguousarray(tar, dtype=np.float32)
        B = tar.shape[0]
        H = np.empty((B, 3, 3), dtype=np.float32)
        self.lib.oracle_tensor_aca_rect_f32(_ptr(src, _f32p), _ptr(tar, _f32p), _ptr(H, _f32p),
                                            B, float(np.float32(scale)), float(np.float32(div)))
        return H

    def aca_vanilla_backward(self, src, tar, gH):
        """(dL/dsrc, dL/dtar), each (n,8), for ACA_vanilla (.py:322-382) given dL/dH (n,9):
        ATen autograd's gradients through its statements.  float32 or float64 (src's dtype)."""
        dt = np.float64 if np.asarray(src).dtype == np.float64 else np.float32
        fp = _f64p if dt == np.float64 else _f32p
        n = np.asarray(src).shape[0]
        src = np.ascontiguousarray(np.asarray(src, dt).reshape(n, 8))
        tar = np.ascontiguousarray(np.asarray(tar, dt).reshape(n, 8))
        gH = np.ascontiguousarray(np.asarray(gH, dt).reshape(n, 9))
        gs, gt = np.empty((n, 8), dt), np.empty((n, 8), dt)
        fn = (self.lib.oracle_aca_vanilla_backward_f64 if dt == np.float64
              else self.lib.oracle_aca_vanilla_backward_f32)
        fn(_ptr(src, fp), _ptr(tar, fp), _ptr(gH, fp), n, _ptr(gs, fp), _ptr(gt, fp))
        return gs, gt

    @staticmethod
    def _rows(x, B):
        """scale / div (any shape broadcastable to (B,3,1), leading size-1 dimensions beyond
        three dropped as the reference's column assignment drops them) as (B,3) float32."""
        a = np.asarray(x, np.float32)
        while a.ndim > 3 and a.shape[0] == 1:
            a = a[0]
        return np.ascontiguousarray(np.broadcast_to(a, (B, 3, 1)).reshape(B, 3))

    def tensor_aca_rect_rows(self, src, tar, scale, div) -> np.ndarray:
        """TensorACA with scale / div broadcast against the (B,3,1) columns (.py:301-302)."""
        src = np.ascontiguousarray(src, dtype=np.float32)
        tar = np.ascontiguousarray(tar, dtype=np.float32)
        B = tar.shape[0]
        sc, dv = self._rows(scale, B), self._rows(div, B)
        H = np.empty((B, 3, 3), dtype=np.float32)
        self.lib.oracle_tensor_aca_rect_rows_f32(_ptr(src, _f32p), _ptr(tar, _f32p),
                                                 _ptr(H, _f32p), B, _ptr(sc, _f32p),
                                                 _ptr(dv, _f32p))
        return H

    def tensor_aca_rect_rows_backward(self, src, tar, gH, scale, div):
        """(grad_src, grad_tar, dscale per (problem, row) (B,3), ddiv (B,3), dscale per
        problem (B) as three-row sums, ddiv (B))."""
        src = np.ascontiguousarray(src, dtype=np.float32)
        tar = np.ascontiguousarray(tar, dtype=np.float32)
        gH = np.ascontiguousarray(gH, dtype=np.float32)
        B = tar.shape[0]
        sc, dv = self._rows(scale, B), self._rows(div, B)
        gs, gt = np.empty((B, 3, 4), np.float32), np.empty((B, 3, 4), np.float32)
        gsr, gdr = np.empty((B, 3), np.float32), np.empty((B, 3), np.float32)
        gss, gds = np.empty(B, np.float32), np.empty(B, np.float32)
        self.lib.oracle_tensor_aca_rect_rows_backward_f32(
            _ptr(src, _f32p), _ptr(tar, _f32p), _ptr(gH, _f32p), B, _ptr(sc, _f32p),
            _ptr(dv, _f32p), _ptr(gs, _f32p), _ptr(gt, _f32p), _ptr(gsr, _f32p), _ptr(gdr, _f32p),
            _ptr(gss, _f32p), _ptr(gds, _f32p))
        return gs, gt, gsr, gdr, gss, gds

    def tensor_aca_rect_backward(self, src, tar, gH, scale: float, div: float):
        """Returns (grad_src (B,3,4), grad_tar (B,3,4), per-problem (B,2) [dscale, ddiv])."""
        src = np.ascontiguousarray(src, dtype=np.float32)
        tar = np.ascontiguousarray(tar, dtype=np.float32)
        gH = np.ascontiguousarray(gH, dtype=np.float32)
        B = tar.shape[0]
        gs = np.empty((B, 3, 4), np.float32)
        gt = np.empty((B, 3, 4), np.float32)
        gsd = np.empty((B, 2), np.float32)
        self.lib.oracle_tensor_aca_rect_backward_f32(
            _ptr(src, _f32p), _ptr(tar, _f32p), _ptr(gH, _f32p), B, float(np.float32(scale)),
            float(np.float32(div)), _ptr(gs, _f32p), _ptr(gt, _f32p), _ptr(gsd, _f32p))
        return gs, gt, gsd

    def fill_bits(self, count: int, seed: int, offset: int = 0) -> np.ndarray:
        out = np.empty(count, dtype=np.uint32)
        self.lib.oracle_fill_bits_u32(out.ctypes.data, count, seed, offset)
        return out

    def ransac_score(self, H, pool_src, pool_tar, thresh: float) -> np.ndarray:
        H = np.ascontiguousarray(H, dtype=np.float32).reshape(-1, 9)
        ps = np.ascontiguousarray(pool_src, dtype=np.float32)
        pt = np.ascontiguousarray(pool_tar, dtype=np.float32)
        counts = np.empty(H.shape[0], dtype=np.uint32)
        self.lib.oracle_ransac_score_f32(_ptr(H, _f32p), H.shape[0], _ptr(ps, _f32p),
                                         _ptr(pt, _f32p), ps.shape[0], float(np.float32(thresh)),
                                         counts.ctypes.data)
        return counts

    def sample_problems(self, pool_src, pool_tar, idx):
        """Gather like get_rand_list (GPU_Runtime Test.cu:52-78): rows of 4 indices,
        each reduced modulo the pool size -> (n,8) src, (n,8) tar."""
        idx = np.asarray(idx).astype(np.uint32) % np.uint32(pool_src.shape[0])
        return (pool_src[idx].reshape(-1, 8).astype(np.float32),
                pool_tar[idx].reshape(-1, 8).astype(np.float32))

    def fill_uniform(self, count: int, seed: int, offset: int = 0, lo: float = 0.0,
                     hi: float = 1024.0) -> np.ndarray:
        out = np.empty(count, dtype=np.float32)
        self.lib.oracle_fill_uniform_f32(_ptr(out, _f32p), count, seed, offset, lo, hi)
        return out

    def time_batch(self, algo: str, src, tar, H, threads: int, reps: int) -> float:
        return self.lib.oracle_time_f32(ALGOS[algo], _ptr(src, _f32p), _ptr(tar, _f32p),
                                        _ptr(H, _f32p), src.shape[0], threads, reps)


def rect_grad_batch(o: "Oracle", B: int, seed: int):
    """A deterministic TensorACA batch for the large gradient fixtures (no stored arrays):
    128 x 128 rectangles at corners in [10, 30), targets offset by [0, 32), dL/dH in [-1, 1),
    all drawn from fill_uniform's counter streams and assembled with float32 additions.
    Returns (src_h, tar_h, gH): (B,3,4), (B,3,4), (B,3,3) float32."""
    corner = o.fill_uniform(2 * B, seed, 0, 10.0, 30.0).reshape(B, 2)
    off = o.fill_uniform(8 * B, seed, 2 * B, 0.0, 32.0).reshape(B, 4, 2)
    gH = o.fill_uniform(9 * B, seed, 10 * B, -1.0, 1.0).reshape(B, 3, 3)
    rect = np.array([[0, 0], [128, 0], [0, 128], [128, 128]], np.float32)
    src = corner[:, None, :] + rect[None]
    tar = src + off
    ones = np.ones((B, 1, 4), np.float32)
    src_h = np.ascontiguousarray(np.concatenate([src.transpose(0, 2, 1), ones], 1))
    tar_h = np.ascontiguousarray(np.concatenate([tar.transpose(0, 2, 1), ones], 1))
    return src_h, tar_h, np.ascontiguousarray(gH)


class RefOracle:
    """The reference's own solver bodies (oracle/_ref/libsks_ref.so)."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing (reference not built here)")
        lib = ctypes.CDLL(path)
        lib.ref_batch_f32.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, _i64]
        lib.ref_batch_f64.argtypes = [ctypes.c_int, _f64p, _f64p, _f64p, _i64]
        lib.ref_time_f32.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, _i64, ctypes.c_int,
                                     ctypes.c_int]
        lib.ref_time_f32.restype = ctypes.c_double
        lib.ref_time_repeat_f32.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, _i64]
        lib.ref_time_repeat_f32.restype = ctypes.c_double
        lib.ref_time_repeat_f64.argtypes = [ctypes.c_int, _f64p, _f64p, _f64p, _i64]
        lib.ref_time_repeat_f64.restype = ctypes.c_double
        lib.ref_time_pinned_f32.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, _i64,
                                            ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        lib.ref_time_pinned_f32.restype = ctypes.c_double
        self.lib = lib

    @staticmethod
    def available(path: str = REF_SO) -> bool:
        return os.path.exists(path)

    def solve(self, algo: str, src: np.ndarray, tar: np.ndarray) -> np.ndarray:
        src = np.ascontiguousarray(src)
        tar = np.ascontiguousarray(tar)
        n = src.shape[0]
        H = np.empty((n, 9), dtype=src.dtype)
        if src.dtype == np.float32:
            self.lib.ref_batch_f32(ALGOS[algo], _ptr(src, _f32p), _ptr(tar, _f32p),
                                   _ptr(H, _f32p), n)
        else:
            self.lib.ref_batch_f64(ALGOS[algo], _ptr(src, _f64p), _ptr(tar, _f64p),
                                   _ptr(H, _f64p), n)
        return H

    def time_batch(self, algo: str, src, tar, H, threads: int, reps: int) -> float:
        return self.lib.ref_time_f32(ALGOS[algo], _ptr(src, _f32p), _ptr(tar, _f32p),
                                     _ptr(H, _f32p), src.shape[0], threads, reps)

    def time_repeat(self, algo: str, src8, tar8, iters: int) -> float:
        """One 4-point set solved `iters` times on one core (main.cpp:87-114); float32 or
        float64 by the inputs' dtype.  Wall seconds."""
        if np.asarray(src8).dtype == np.float64:
            src8 = np.ascontiguousarray(src8, np.float64)
            tar8 = np.ascontiguousarray(tar8, np.float64)
            H9 = np.empty(9, dtype=np.float64)
            return self.lib.ref_time_repeat_f64(ALGOS[algo], _ptr(src8, _f64p), _ptr(tar8, _f64p),
                                                _ptr(H9, _f64p), iters)
        H9 = np.empty(9, dtype=np.float32)
        return self.lib.ref_time_repeat_f32(ALGOS[algo], _ptr(src8, _f32p), _ptr(tar8, _f32p),
                                            _ptr(H9, _f32p), iters)

    def time_pinned(self, algo: str, src, tar, cpus, reps: int, H=None) -> float:
        """The streaming batch on len(cpus) threads, thread k pinned to logical CPU cpus[k],
        each first-touching its own slice (NUMA-local pages); wall seconds of `reps` passes.
        With H given, the results are copied there afterwards (untimed)."""
        cpu_arr = (ctypes.c_int * len(cpus))(*cpus)
        hp = _ptr(H, _f32p) if H is not None else None
        return self.lib.ref_time_pinned_f32(ALGOS[algo], _ptr(src, _f32p), _ptr(tar, _f32p), hp,
                                            src.shape[0], ctypes.cast(cpu_arr, ctypes.c_void_p),
                                            len(cpus), reps)


REF_CU_SO = os.environ.get("SKS_REF_CU_SO", os.path.join(HERE, "_ref", "libsks_ref_cu.so"))


class RefCuOracle:
    """The statements of cal_Homo_ACA / _SKS / _GE / _GPT (lines 81-507 of "GPU_Runtime
    Test.cu") compiled by hipcc behind a prepended HIP header (oracle/build.sh,
    oracle/ref_cu_driver.hip; -ffp-contract=off) and launched as the reference's host code
    launches them.  A STAND-IN build (nvcc and the CUDA headers are absent): a cross-check of
    statement-order IEEE evaluation, not the reference's own build's output.  SoA binary64,
    unnormalised (GE/GPT: H[8] = 1).  Runs on the GPU (a checker: tests only)."""

    ALGO = {"aca": 0, "sks": 1, "ge": 2, "gpt": 3}

    def __init__(self, path: str = REF_CU_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing (reference CUDA kernels not built here)")
        lib = ctypes.CDLL(path)
        lib.refcu_solve_f64.argtypes = [ctypes.c_int, _f64p, _f64p, _f64p, ctypes.c_int]
        lib.refcu_solve_f64.restype = ctypes.c_int
        self.lib = lib

    @staticmethod
    def available(path: str = REF_CU_SO) -> bool:
        return os.path.exists(path)

    def solve(self, algo: str, src: np.ndarray, tar: np.ndarray) -> np.ndarray:
        """src/tar (8, n) float64 -> H (9, n) float64."""
        src = np.ascontiguousarray(src, np.float64)
        tar = np.ascontiguousarray(tar, np.float64)
        n = src.shape[1]
        H = np.empty((9, n), np.float64)
        rc = self.lib.refcu_solve_f64(self.ALGO[algo], _ptr(src, _f64p), _ptr(tar, _f64p),
                                      _ptr(H, _f64p), n)
        if rc != 0:
            raise RuntimeError(f"refcu_solve_f64({algo}) failed with hipError_t {rc}")
        return H


def same_bits(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Elementwise bit equality with every NaN equal to every NaN (payloads differ
    between x86 and CDNA: x86 propagates an operand's payload, the GPU may return
    the canonical quiet NaN)."""
    a = np.asarray(a)
    b = np.asarray(b)
    ui = np.uint32 if a.dtype == np.float32 else np.uint64
    eq = a.view(ui) == b.view(ui)
    return eq | (np.isnan(a) & np.isnan(b))
