"""Independent restatements of the counter-based input streams, for the tests only.

``hg_fill_uniform_f32`` (GPU, hg_kernels.hip) and ``oracle_fill_uniform_f32`` (C,
oracle/hg_oracle.c) generate every bench and parity input: value i of stream (seed,
offset) is

    r = splitmix64(seed * 0xD1B54A32D192ED03 + offset + i)      (mod 2**64)
    u = (r >> 40) * 2**-24                                       (exact in binary32)
    x = lo + (hi - lo) * u                                       (binary32, each op rounded)

Restated here twice, with no code shared with either implementation: in Python integers
(``uniform_f32_pyint``, the definition read literally; slow) and vectorised in numpy uint64
arithmetic (``uniform_f32``, wrapping multiplies; fast).  numpy's float32 scalar and array
operations round each + and * to binary32 (IEEE 754), as the C and HIP code do with
contraction off.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
K_UNIFORM = 0xD1B54A32D192ED03


def splitmix64(z: int) -> int:
    """splitmix64's finaliser (Steele, Lea & Flood, OOPSLA 2014), in Python integers."""
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def uniform_f32_pyint(count: int, seed: int, offset: int, lo: float = 0.0,
                      hi: float = 1024.0) -> np.ndarray:
    lo32, hi32 = np.float32(lo), np.float32(hi)
    span = np.float32(hi32 - lo32)
    base = (seed * K_UNIFORM) & M64
    out = np.empty(count, np.float32)
    for i in range(count):
        r = splitmix64((base + offset + i) & M64)
        u = np.float32(r >> 40) * np.float32(2.0 ** -24)  # exact: r >> 40 < 2**24
        out[i] = lo32 + np.float32(span * u)
    return out


def _splitmix64_np(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniform_f32(count: int, seed: int, offset: int, lo: float = 0.0,
                hi: float = 1024.0) -> np.ndarray:
    lo32, hi32 = np.float32(lo), np.float32(hi)
    span = np.float32(hi32 - lo32)
    start = np.uint64(((seed * K_UNIFORM) + offset) & M64)
    with np.errstate(over="ignore"):
        ctr = start + np.arange(count, dtype=np.uint64)  # wraps mod 2**64 like the C
    r = _splitmix64_np(ctr)
    u = (r >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    return (lo32 + (span * u).astype(np.float32)).astype(np.float32)
