"""Independent restatement of the MRG32K3A word stream of the reference's Table-8 draws
(GPU_Runtime Test.cu:1443-1446: curandCreateGenerator(MRG32K3A), seed 11, curandGenerate of
4*N words).  Test infrastructure only: nothing under sks-homography_amd/ imports it.

What is restated, and from where:
  * the recurrence -- L'Ecuyer, "Good parameters and implementations for combined multiple
    recursive random number generators", Operations Research 47(1), 1999: two order-3
    recurrences mod m1 = 2^32 - 209 and m2 = 2^32 - 22853,
        x1[n] = (1403580 x1[n-2] - 810728 x1[n-3]) mod m1
        x2[n] = (527612 x2[n-1] - 1370589 x2[n-3]) mod m2
        z[n]  = (x1[n] - x2[n]) mod m1, reported in [1, m1] (0 -> m1);
  * subsequences 2^76 steps apart (the jump A^(2^76) is computed here by modular matrix
    powers, not read from any table);
  * the seeding and the 32-bit output conversion of rocRAND's MRG32K3A engine, as its
    public device header in this image states them (rocrand/rocrand_mrg32k3a.h: seed(),
    mod_mul_m1/_m2, rocrand()), including its 64-bit wrap-around for large seeds;
  * the host-API word order, measured against rocrand_generate on the MI355X box
    (tools/mrg_dump.py -> tests/golden/mrg32k3a_rocrand.npz): word i comes from
    subsequence i mod 131072 at position i div 131072.

What stays unpinned: cuRAND's own seeding of the state from the 64-bit seed, its uint
conversion and its host-API ordering are not fixed by anything in this image (no cuRAND,
no documentation), so these words are rocRAND's, not necessarily cuRAND's.
"""
from __future__ import annotations

import numpy as np

M1 = 4294967087
M2 = 4294944443
A12 = 1403580
A13N = 810728
A21 = 527612
A23N = 1370589
UINT_NORM = 1.000000048661607  # (2^32 - 1) / (m1 - 1), the header's double literal
SUBSEQ_LOG2 = 76
ORDER_SUBSEQUENCES = 131072  # the host API's word order (measured, see the docstring)
_U64 = (1 << 64) - 1

# one step of each component as a 3x3 matrix on (x[n-3], x[n-2], x[n-1])
A1 = ((0, 1, 0), (0, 0, 1), ((M1 - A13N) % M1, A12, 0))
A2 = ((0, 1, 0), (0, 0, 1), ((M2 - A23N) % M2, 0, A21))


def mat_mul(a, b, m):
    return tuple(tuple(sum(a[i][k] * b[k][j] for k in range(3)) % m for j in range(3))
                 for i in range(3))


def mat_vec(a, x, m):
    return tuple(sum(a[i][k] * x[k] for k in range(3)) % m for i in range(3))


def mat_pow(a, e, m):
    r = ((1, 0, 0), (0, 1, 0), (0, 0, 1))
    while e:
        if e & 1:
            r = mat_mul(r, a, m)
        a = mat_mul(a, a, m)
        e >>= 1
    return r


def _mod_m(p, m, c, twice):
    """The header's partial reduction of a 64-bit value: c*(p>>32) + low, once or twice,
    then one conditional subtraction (not a full reduction for every 64-bit p)."""
    p &= _U64
    p = (c * (p >> 32) + (p & 0xFFFFFFFF)) & _U64
    if twice:
        p = (c * (p >> 32) + (p & 0xFFFFFFFF)) & _U64
    return p - m if p >= m else p


def _mod_mul(i, j, m, c, twice):
    """mod_mul_m1/_m2(i, j) with the header's 64-bit integer semantics."""
    hi, lo = i // 131072, i % 131072
    t1 = (_mod_m((hi * j) & _U64, m, c, twice) * 131072) & _U64
    t2 = _mod_m((lo * j) & _U64, m, c, twice)
    return _mod_m((t1 + t2) & _U64, m, c, twice)


def seed_state(seed: int):
    """(g1, g2) of a freshly seeded engine, before any step (truncated to uint32 as the
    header's state words are)."""
    seed &= _U64
    if seed == 0:
        seed = 12345
    x = (seed & 0xFFFFFFFF) ^ 0x55555555
    y = ((seed >> 32) ^ 0xAAAAAAAA) & 0xFFFFFFFF
    m1 = lambda i: _mod_mul(i, seed, M1, 209, False) & 0xFFFFFFFF  # noqa: E731
    m2 = lambda i: _mod_mul(i, seed, M2, 22853, True) & 0xFFFFFFFF  # noqa: E731
    return (m1(x), m1(y), m1(x)), (m2(y), m2(x), m2(y))


def state_at(seed: int, subsequence: int = 0, offset: int = 0):
    g1, g2 = seed_state(seed)
    e = (subsequence << SUBSEQ_LOG2) + offset
    return mat_vec(mat_pow(A1, e, M1), g1, M1), mat_vec(mat_pow(A2, e, M2), g2, M2)


def to_uint(z: int) -> int:
    """rocrand(): (z - 1) * UINT_NORM in binary64, truncated."""
    return int(float(z - 1) * UINT_NORM)


def words_python(seed: int, subsequence: int, offset: int, count: int) -> list[int]:
    """count consecutive words of one subsequence, pure Python integers."""
    g1, g2 = state_at(seed, subsequence, offset)
    out = []
    for _ in range(count):
        p1 = (A12 * g1[1] - A13N * g1[0]) % M1
        p2 = (A21 * g2[2] - A23N * g2[0]) % M2
        g1, g2 = (g1[1], g1[2], p1), (g2[1], g2[2], p2)
        out.append(to_uint(p1 - p2 if p1 > p2 else p1 - p2 + M1))
    return out


def _mat_vec_np(a, x, m):
    """a (3x3 Python ints < m) times every column of x (3, n) uint64 < m, mod m: each product
    is below 2^64 and is reduced before the three are added."""
    mm = np.uint64(m)
    return np.stack([((np.uint64(a[i][0]) * x[0]) % mm + (np.uint64(a[i][1]) * x[1]) % mm
                      + (np.uint64(a[i][2]) * x[2]) % mm) % mm for i in range(3)])


def subsequence_starts(seed: int, count: int, first: int = 0):
    """(g1, g2) uint64 arrays (3, count) of subsequences first .. first+count-1 at offset 0,
    by doubling: starts[h .. 2h) = J^h starts[0 .. h) with J = A^(2^76)."""
    s1, s2 = state_at(seed, first, 0)
    g1 = np.array(s1, np.uint64).reshape(3, 1)
    g2 = np.array(s2, np.uint64).reshape(3, 1)
    j1, j2 = mat_pow(A1, 1 << SUBSEQ_LOG2, M1), mat_pow(A2, 1 << SUBSEQ_LOG2, M2)
    while g1.shape[1] < count:
        g1 = np.concatenate([g1, _mat_vec_np(j1, g1, M1)], axis=1)
        g2 = np.concatenate([g2, _mat_vec_np(j2, g2, M2)], axis=1)
        j1, j2 = mat_mul(j1, j1, M1), mat_mul(j2, j2, M2)
    return g1[:, :count].copy(), g2[:, :count].copy()


def step_words(g1, g2):
    """One step of every column (in place); returns the words (uint32).  All products are
    below 2^53, so uint64 arithmetic is exact."""
    p1 = (np.uint64(A12) * g1[1] + np.uint64(A13N) * (np.uint64(M1) - g1[0])) % np.uint64(M1)
    p2 = (np.uint64(A21) * g2[2] + np.uint64(A23N) * (np.uint64(M2) - g2[0])) % np.uint64(M2)
    g1[0], g1[1], g1[2] = g1[1].copy(), g1[2].copy(), p1
    g2[0], g2[1], g2[2] = g2[1].copy(), g2[2].copy(), p2
    z = np.where(p1 > p2, p1 - p2, p1 + np.uint64(M1) - p2)
    return ((z - np.uint64(1)).astype(np.float64) * UINT_NORM).astype(np.uint64).astype(np.uint32)


def generate(seed: int, count: int, subsequences: int = ORDER_SUBSEQUENCES) -> np.ndarray:
    """The host API's count words: word i from subsequence i % S at position i // S."""
    out = np.empty(count, np.uint32)
    if count == 0:
        return out
    cols = min(count, subsequences)
    g1, g2 = subsequence_starts(seed, cols)
    pos = 0
    while pos * subsequences < count:
        w = step_words(g1, g2)
        base = pos * subsequences
        k = min(cols, count - base)
        out[base:base + k] = w[:k]
        pos += 1
    return out
