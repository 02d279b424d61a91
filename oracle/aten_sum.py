"""ATen-CPU's float32 sum order, restated in numpy (TEST INFRASTRUCTURE ONLY: imported by
tests/ and never by the product package).

Why it exists.  The reference gets TensorACA_rect's scale / div gradients from ATen autograd
(PyTorch Codes/Modules_Runtime_Test.py:301-302 under .backward()): a (1,)-shaped scale or div
-- what adjust() returns (.py:33-35) -- receives sum_to_size((B,3,1) per-(problem,row) terms,
(1,)), a full reduction of 3B contiguous floats; a (3,1)-shaped one receives the (B,3) terms
summed down each column.  Which float32 additions ATen makes there is the algorithm this file
restates.  It lives in the reference's third-party dependency, PyTorch (torch 2.10.0 here,
not part of /root/reference):

  * aten/src/ATen/native/cpu/SumKernel.cpp  -- cascade_sum: a contiguous inner reduction goes
    to vectorized_inner_sum (Vectorized<float>: W = 8 lanes -- measured: ATen runs the sum
    kernel's 8-lane build under CPU capability AVX512 too, tests/test_aten_sum_order.py),
    whose row_sum treats the vectors as a (-1, 4) array summed by multi_row_sum, a 4-level cascade with level step 2^max(4, CeilLog2(n)/4); the leftover
    vectors join column 0, the columns fold 0 += 1, += 2, += 3, the scalar tail and then the
    lanes fold into a 0-initialised float.  A strided column (the (3,1) case) takes
    scalar_outer_sum -> row_sum with one lane: the same cascade with W = 1.  The output is
    zero-filled first and the result ADDED to it (CastStoreAccumulate): 0 + s.
  * aten/src/ATen/TensorIteratorReduce.cpp -- parallel_reduce: below GRAIN_SIZE = 32768
    elements or with one thread, serially; a single-output reduction above it takes
    two_pass_reduction: at::parallel_for splits [0, m) into min(T, ceil(m/32768)) chunks of
    ceil(m/chunks) (ParallelOpenMP.h invoke_parallel), each chunk's serial sum lands in a
    zeroed buffer of T = at::get_num_threads() slots, and the buffer is then summed serially
    the same way.  A column reduction ((3,1)) splits over columns (parallel_dim_reduction),
    so its order does not depend on T.

Pinned, not assumed: tests/test_aten_sum_order.py compares aten_sum / aten_column_sums with
torch.sum on this container's CPU bit for bit over sizes 0 .. 4.2 M, every chunking regime,
several thread counts, and the fixtures in
tests/golden/torch_rect_grad_large.npz record ATen autograd's own gradients with the T and W
they were made with.
"""
from __future__ import annotations

import numpy as np

GRAIN_SIZE = 32768  # at::internal::GRAIN_SIZE
NUM_LEVELS = 4      # multi_row_sum's num_levels
ILP = 4             # row_sum's ilp_factor


def ceil_log2(x: int) -> int:
    """ATen's utils::CeilLog2: 1 for x <= 2, else floor(log2(x - 1)) + 1."""
    return 1 if x <= 2 else int(x - 1).bit_length()


def level_power(n: int) -> int:
    return max(4, ceil_log2(n) // NUM_LEVELS)


def multi_row_sum(R: np.ndarray) -> np.ndarray:
    """multi_row_sum over the n rows of R (n, S): S independent float32 cascades.  Row i is
    added into acc[0]; after each full block of `step` rows acc[j] += acc[j-1], acc[j-1] = 0
    for j = 1.. while i is a multiple of step^(j+1); the remaining rows go into acc[0]; the
    result is ((acc0 + acc1) + acc2) + acc3.  Vectorised over blocks: every addition below
    is the float32 addition ATen makes, in its order."""
    n, S = R.shape
    lp = level_power(n)
    step = 1 << lp
    f32 = np.float32
    nb = n // step                       # full level-0 blocks
    # level 0: each block's sum from 0, row by row
    b = np.zeros((nb, S), f32)
    if nb:
        blk = R[: nb * step].reshape(nb, step, S)
        for j in range(step):
            b += blk[:, j]
    # level 1: block sums, flushed every `step` blocks
    n1 = nb // step
    s1 = np.zeros((n1, S), f32)
    for j in range(step):
        if n1:
            s1 += b[: n1 * step].reshape(n1, step, S)[:, j]
    acc1 = np.zeros(S, f32)
    for r in b[n1 * step:]:
        acc1 += r
    # level 2: super-block sums, flushed every `step`
    n2 = n1 // step
    s2 = np.zeros((n2, S), f32)
    for j in range(step):
        if n2:
            s2 += s1[: n2 * step].reshape(n2, step, S)[:, j]
    acc2 = np.zeros(S, f32)
    for r in s1[n2 * step:]:
        acc2 += r
    # level 3: never flushed
    acc3 = np.zeros(S, f32)
    for r in s2:
        acc3 += r
    acc0 = np.zeros(S, f32)
    for r in R[nb * step:]:
        acc0 += r
    acc0 += acc1
    acc0 += acc2
    acc0 += acc3
    return acc0


def serial_sum(x: np.ndarray, lanes: int) -> np.float32:
    """One serial pass of cascade_sum over a contiguous run (vectorized_inner_sum with W =
    lanes when len(x) >= lanes, else row_sum's one-lane form), before the store's 0 + s."""
    x = np.ascontiguousarray(x, np.float32)
    m = x.shape[0]
    W = lanes if m >= lanes else 1
    V = m // W
    vec = x[: V * W].reshape(V, W)
    n = V // ILP
    p = multi_row_sum(vec[: n * ILP].reshape(n, ILP * W)).reshape(ILP, W)
    p0 = p[0].copy()
    for v in range(n * ILP, V):
        p0 += vec[v]
    for k in range(1, ILP):
        p0 += p[k]
    final = np.float32(0)
    for k in range(V * W, m):
        final = np.float32(final + x[k])
    for lane in range(W):
        final = np.float32(final + p0[lane])
    return final


@np.errstate(all="ignore")  # inf - inf and NaN propagate as in ATen
def aten_sum(x, lanes: int = 8, threads: int = 1) -> np.float32:
    """torch.sum of a contiguous float32 tensor (or sum_to_size to one element) on ATen-CPU
    with Vectorized<float>::size() = lanes and at::get_num_threads() = threads."""
    x = np.ascontiguousarray(x, np.float32).ravel()
    m = x.shape[0]
    zero = np.float32(0)
    if m < GRAIN_SIZE or threads == 1:
        return np.float32(zero + serial_sum(x, lanes))
    chunks = min(threads, -(-m // GRAIN_SIZE))
    size = -(-m // chunks)
    buf = np.zeros(threads, np.float32)
    for t in range(chunks):
        lo = t * size
        if lo < m:
            buf[t] = np.float32(zero + serial_sum(x[lo: min(m, lo + size)], lanes))
    return np.float32(zero + serial_sum(buf, lanes))


@np.errstate(all="ignore")
def aten_column_sums(x) -> np.ndarray:
    """(B, C) float32 with C < 4 summed over B as ATen sums a (B,C,1) tensor to (C,1): each
    column by row_sum with one lane (scalar_outer_sum), whatever the thread count."""
    x = np.asarray(x, np.float32)
    return np.array([np.float32(0) + serial_sum(np.ascontiguousarray(x[:, c]), 1)
                     for c in range(x.shape[1])], np.float32)
