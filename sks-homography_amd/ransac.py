"""RANSAC on the solver: hypothesis sampling, the fused
gather + closed-form solve, and inlier scoring -- all on the device.

The reference stops at timing random 4-point hypotheses: cuRAND indices, the
get_rand_list gather and the solver kernel (GPU_Runtime Test.cu:1443-1451, :52-78,
:81-151), the "sampling number" use case of its Table 8.  This module runs that
pipeline, adds the scoring step it implies, and returns the best hypothesis.
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple

import torch

from . import _lib
from .ops import _gpu_device, _guard, _require_device, _stream


_strtof_fn = None


def _strtof(tokens):
    """Decimal strings -> binary32 the way the reference's sscanf("%f") converts them (C
    strtof: one correct rounding).  numpy's str -> float32 goes through binary64 first, and
    that double rounding gives the other neighbour for a decimal just above a binary32
    midpoint (e.g. 1.00000005960464477539062500000001 -> 1.0 instead of 1 + 2^-23)."""
    global _strtof_fn
    import ctypes
    import ctypes.util

    import numpy as np

    if _strtof_fn is None:
        fn = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6").strtof
        fn.restype = ctypes.c_float
        fn.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
        _strtof_fn = fn
    return np.array([_strtof_fn(t.encode(), None) for t in tokens], dtype=np.float32)


def read_points(filename: str):
    """The reference's correspondence-file reader (CPU_Runtime Test/utils.cpp:6-21; the GPU
    harness's copy at GPU_Runtime Test.cu:31-46): the first line holds the count N, then N
    lines "x1 y1 x2 y2" (source point, target point), each value parsed as sscanf's "%f"
    does.  Returns (pool_src, pool_tar), each an (N,2) float32 numpy array, ready for
    sample_solve / score / ransac (orig_pts_wall.txt is the reference's own file)."""
    import numpy as np

    with open(filename) as f:
        head = f.readline().split()
        if not head:
            raise ValueError(f"{filename}: empty file (expected the point count first)")
        count = int(head[0])
        tokens = []
        for i in range(count):
            vals = f.readline().split()[:4]
            if len(vals) < 4:
                raise ValueError(f"{filename}: line {i + 2} has fewer than 4 values")
            tokens += vals
    a = _strtof(tokens).reshape(count, 4)
    return np.ascontiguousarray(a[:, 0:2]), np.ascontiguousarray(a[:, 2:4])


def fill_bits(count: int, seed: int, offset: int = 0, device="cuda") -> torch.Tensor:
    """Counter-based uint32 draws (held in an int32 tensor), bit-identical to the
    host regeneration."""
    if count < 0:
        raise ValueError(f"count must be >= 0, got {count}")
    dev = _gpu_device(device)
    out = torch.empty(count, dtype=torch.int32, device=dev)
    with _guard(dev):
        _lib.call("hg_fill_bits_u32", out.data_ptr(), count, seed, offset, _stream(dev))
    return out


def _pool(pool: torch.Tensor) -> torch.Tensor:
    if pool.dim() != 2 or pool.shape[1] != 2:
        raise ValueError(f"pool must be (npool,2), got {tuple(pool.shape)}")
    return pool.to(torch.float32).contiguous()


def sample_solve(pool_src: torch.Tensor, pool_tar: torch.Tensor, idx: torch.Tensor,
                 algo: str = "aca", normalize: bool = True) -> torch.Tensor:
    """H of each row of ``idx`` ((n,4) int32/uint32; entries reduced modulo the pool
    size like get_rand_list, .cu:56-59) gathered from (npool,2) pools.  (n,9)."""
    dev = _require_device(pool_src, pool_tar, idx)
    if idx.dim() != 2 or idx.shape[1] != 4 or idx.dtype not in (torch.int32, torch.uint32):
        raise ValueError("idx must be an (n,4) int32/uint32 tensor")
    if algo not in ("aca", "sks"):
        raise ValueError(f"algo must be 'aca' or 'sks', got {algo!r}")
    ps, pt, idx = _pool(pool_src), _pool(pool_tar), idx.contiguous()
    n = idx.shape[0]
    out = torch.empty((n, 9), dtype=torch.float32, device=dev)
    with _guard(dev):
        _lib.call("hg_sample_solve_f32", ps.data_ptr(), pt.data_ptr(), ps.shape[0],
                  idx.data_ptr(), out.data_ptr(), n, 0 if algo == "aca" else 1,
                  1 if normalize else 0, _stream(dev))
    return out


def sample_solve_seeded(pool_src: torch.Tensor, pool_tar: torch.Tensor, n: int, seed: int,
                        offset: int = 0, algo: str = "aca", normalize: bool = True) -> torch.Tensor:
    """``n`` hypotheses drawn AND solved in one launch: bit for bit
    ``sample_solve(pool_src, pool_tar, fill_bits(4 * n, seed, offset).view(n, 4))``, with the
    draws made in the kernel instead of read from an index array.  (n,9)."""
    dev = _require_device(pool_src, pool_tar)
    if algo not in ("aca", "sks"):
        raise ValueError(f"algo must be 'aca' or 'sks', got {algo!r}")
    if n < 0:
        raise ValueError(f"n must be >= 0, got {n}")
    ps, pt = _pool(pool_src), _pool(pool_tar)
    out = torch.empty((n, 9), dtype=torch.float32, device=dev)
    with _guard(dev):
        _lib.call("hg_sample_solve_seeded_f32", ps.data_ptr(), pt.data_ptr(), ps.shape[0],
                  seed, offset, out.data_ptr(), n, 0 if algo == "aca" else 1,
                  1 if normalize else 0, _stream(dev))
    return out


def score(H: torch.Tensor, pool_src: torch.Tensor, pool_tar: torch.Tensor,
          thresh: float) -> torch.Tensor:
    """Inlier count of every hypothesis H (n,9) over the pool: points whose
    reprojection error is at most ``thresh`` (division-free test, see
    include/sks_homography.h).  Returns (n,) int32."""
    dev = _require_device(H, pool_src, pool_tar)
    H = H.reshape(-1, 9).to(torch.float32).contiguous()
    ps, pt = _pool(pool_src), _pool(pool_tar)
    counts = torch.empty(H.shape[0], dtype=torch.int32, device=dev)
    with _guard(dev):
        _lib.call("hg_ransac_score_f32", H.data_ptr(), H.shape[0], ps.data_ptr(), pt.data_ptr(),
                  ps.shape[0], float(thresh), counts.data_ptr(), _stream(dev))
    return counts


# ---- the reference's Table-8 pipeline in its own formats (GPU_Runtime Test.cu:1443-1451) ----
_ALGO_IDS = {"aca": 0, "sks": 1, "ge": 2, "gpt": 3}


def rand_mrg32k3a(count: int, seed: int = 11, device="cuda") -> torch.Tensor:
    """``count`` MRG32K3A words, as curandGenerate fills the reference's index list
    (.cu:1443-1446, seed 11): the hand-written generator, uint32 values in an int32 tensor.
    The words equal rocRAND's host-API MRG32K3A words on gfx950 bit for bit (their order is
    rocRAND's gfx950 launch layout, hg_mrg32k3a.hpp kOrderLog2); equality with cuRAND's
    words, which the reference's CUDA harness draws, is unpinned (no cuRAND here).
    Asynchronous on the current stream, like every op here."""
    if count < 0:
        raise ValueError(f"count must be >= 0, got {count}")
    dev = _gpu_device(device)
    out = torch.empty(count, dtype=torch.int32, device=dev)
    with _guard(dev):
        _lib.call("hg_rand_mrg32k3a_u32", out.data_ptr(), count, seed, _stream(dev))
    return out


def _point_pool(pool: torch.Tensor) -> torch.Tensor:
    if pool.dim() != 2 or pool.shape[1] != 2 or pool.dtype != torch.float64:
        raise ValueError(f"pool must be an (npool,2) float64 tensor (Point2d), got "
                         f"{tuple(pool.shape)} {pool.dtype}")
    return pool.contiguous()


def _rand_list(rl: torch.Tensor) -> torch.Tensor:
    if rl.dim() != 2 or rl.shape[0] != 4 or rl.dtype not in (torch.int32, torch.uint32):
        raise ValueError("rand_list must be a (4,n) int32/uint32 tensor (word k of hypothesis "
                         "id at [k, id], as get_rand_list reads it)")
    return rl.contiguous()


def get_rand_list(rand_list: torch.Tensor, pool_src: torch.Tensor, pool_tar: torch.Tensor):
    """The reference's get_rand_list (.cu:52-78): (4,n) words and two (npool,2) float64
    point pools -> (d_src, d_tar), each (8,n) float64 SoA, ready for solve(..., layout="soa")."""
    dev = _require_device(rand_list, pool_src, pool_tar)
    rl, ps, pt = _rand_list(rand_list), _point_pool(pool_src), _point_pool(pool_tar)
    if ps.shape[0] != pt.shape[0] or ps.shape[0] == 0:
        raise ValueError("pool_src and pool_tar must hold the same, non-zero number of points")
    n = rl.shape[1]
    d_src = torch.empty((8, n), dtype=torch.float64, device=dev)
    d_tar = torch.empty((8, n), dtype=torch.float64, device=dev)
    with _guard(dev):
        _lib.call("hg_get_rand_list_f64", rl.data_ptr(), ps.shape[0], ps.data_ptr(), pt.data_ptr(),
                  d_src.data_ptr(), d_tar.data_ptr(), n, _stream(dev))
    return d_src, d_tar


def gather_solve(pool_src: torch.Tensor, pool_tar: torch.Tensor, rand_list: torch.Tensor,
                 algo: str = "aca", normalize: bool = False) -> torch.Tensor:
    """get_rand_list fused with cal_Homo_{ACA,SKS,GE,GPT} (.cu:52-78 + :81-507): (9,n)
    float64 SoA H, bit for bit ``solve(algo, *get_rand_list(...), normalize, layout="soa")``
    without the (8,n) rows in memory.  Unnormalised by default, like the reference kernels."""
    dev = _require_device(rand_list, pool_src, pool_tar)
    if algo not in _ALGO_IDS:
        raise ValueError(f"algo must be one of {sorted(_ALGO_IDS)}, got {algo!r}")
    rl, ps, pt = _rand_list(rand_list), _point_pool(pool_src), _point_pool(pool_tar)
    if ps.shape[0] != pt.shape[0] or ps.shape[0] == 0:
        raise ValueError("pool_src and pool_tar must hold the same, non-zero number of points")
    n = rl.shape[1]
    H = torch.empty((9, n), dtype=torch.float64, device=dev)
    with _guard(dev):
        _lib.call("hg_gather_solve_f64", _ALGO_IDS[algo], ps.data_ptr(), pt.data_ptr(), ps.shape[0],
                  rl.data_ptr(), H.data_ptr(), n, 1 if normalize else 0, _stream(dev))
    return H


def rand_gather_solve(pool_src: torch.Tensor, pool_tar: torch.Tensor, n: int, seed: int = 11,
                      algo: str = "aca", normalize: bool = False) -> torch.Tensor:
    """The whole Table-8 flow in one launch (.cu:1443-1451 + :52-78 + :81-507): (9,n) float64
    SoA H, bit for bit ``gather_solve(pool_src, pool_tar, rand_mrg32k3a(4*n, seed).view(4, n),
    algo, normalize)``, with the MRG32K3A words made in registers."""
    dev = _require_device(pool_src, pool_tar)
    if algo not in _ALGO_IDS:
        raise ValueError(f"algo must be one of {sorted(_ALGO_IDS)}, got {algo!r}")
    if n < 0:
        raise ValueError(f"n must be >= 0, got {n}")
    ps, pt = _point_pool(pool_src), _point_pool(pool_tar)
    if ps.shape[0] != pt.shape[0] or ps.shape[0] == 0:
        raise ValueError("pool_src and pool_tar must hold the same, non-zero number of points")
    H = torch.empty((9, n), dtype=torch.float64, device=dev)
    with _guard(dev):
        _lib.call("hg_rand_gather_solve_f64", _ALGO_IDS[algo], ps.data_ptr(), pt.data_ptr(),
                  ps.shape[0], seed, H.data_ptr(), n, 1 if normalize else 0, _stream(dev))
    return H


def mrg32k3a_state(seed: int, subsequence: int = 0, offset: int = 0) -> tuple:
    """The engine state curand_init / rocrand_init(seed, subsequence, offset) sets up, as
    (x1[n-3], x1[n-2], x1[n-1], x2[n-3], x2[n-2], x2[n-1]) (host computation)."""
    st = (ctypes.c_uint32 * 6)()
    _lib.call("hg_mrg32k3a_state", seed, subsequence, offset, st)
    return tuple(st)


class RansacResult(NamedTuple):
    H: torch.Tensor          # (9,) best hypothesis (normalised)
    inliers: int             # its inlier count
    index: int               # which hypothesis won
    counts: torch.Tensor     # (n,) inlier count of every hypothesis


def ransac(pool_src: torch.Tensor, pool_tar: torch.Tensor, hypotheses: int, thresh: float,
           seed: int = 11, algo: str = "aca") -> RansacResult:
    """Draws ``hypotheses`` random 4-point samples and solves them (one fused launch),
    scores them all and returns the best (ties: lowest index)."""
    _require_device(pool_src, pool_tar)
    if hypotheses < 1:
        raise ValueError(f"ransac needs at least one hypothesis, got {hypotheses}")
    H = sample_solve_seeded(pool_src, pool_tar, hypotheses, seed, 0, algo=algo, normalize=True)
    counts = score(H, pool_src, pool_tar, thresh)
    best = int((counts == counts.max()).nonzero()[0].item())
    return RansacResult(H[best].clone(), int(counts[best].item()), best, counts)
