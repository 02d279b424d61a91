// hg_reduce.hpp -- a float32 sum in ATen-CPU's order (hg_sum_aten_f32).
//
// The reference gets TensorACA_rect's batch-uniform scale / div gradients from ATen autograd
// (Modules_Runtime_Test.py:301-302 under .backward(); adjust() gives them shape (1,),
// .py:33-35): sum_to_size of the (B,3,1) per-(problem,row) terms.  This reproduces the
// float32 additions ATen's CPU sum makes there (SumKernel.cpp cascade_sum, TensorIterator-
// Reduce.cpp two_pass_reduction; restated and pinned against torch.sum by oracle/aten_sum.py
// and tests/test_aten_sum_order.py).  One run of m floats is summed as:
//   * chunks: with T threads and m >= 32768, min(T, ceil(m/32768)) chunks of ceil(m/chunks),
//     each summed serially into a zeroed T-slot buffer, which is then summed serially;
//   * serially: W lanes (1 when the run is shorter than W) x 4 columns = 4W independent
//     streams, stream (k, l) taking elements (4i + k) W + l, i < n = (m/W)/4, in a 4-level
//     cascade with level step 2^lp, lp = max(4, CeilLog2(n)/4): blocks of `step` elements
//     summed from 0, their sums accumulated and flushed every step blocks (a "super-block"),
//     those flushed every step super-blocks, the last level never; then the leftover vectors
//     join column 0, the columns fold into column 0, and the scalar tail and the W lanes add
//     into a 0-initialised float; the stored value is 0 + that.
// On the device the cascade's levels become launches: L1 sums each super-block of every stream
// (one block per super-block, one thread per block of a stream), L2 each group of `step`
// super-block sums, L3 one block per run finishes
// the streams and folds them (thread 0), L4 sums the chunk buffer.  Partial results are
// written in place over elements their own thread has finished reading: x is scratch.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hg {

constexpr int64_t kAtenGrain = 32768;  // at::internal::GRAIN_SIZE
constexpr int kAtenMaxLanes = 16;      // 4 * lanes streams fit one wave
constexpr int kAtenMaxThreads = 1024;  // the chunk buffer's slots

__host__ __device__ inline int aten_ceil_log2(int64_t x) {
    if (x <= 2) return 1;
    int b = 0;
    for (uint64_t v = (uint64_t)(x - 1); v; v >>= 1) ++b;
    return b;
}

__host__ __device__ inline int aten_level_power(int64_t n) {
    const int c = aten_ceil_log2(n) / 4;
    return c > 4 ? c : 4;
}

// The runs: row r's elements are x[r * row_stride + e * es], e < m; each row is `chunks`
// runs of `chunk` elements (the last one shorter).
struct AtenSum {
    float* x;
    int64_t row_stride, es, m, chunk;
    int chunks, lanes;
};

// One run's shape, the same on host and device.
struct AtenRun {
    float* base;     // element 0 of the run
    int64_t es, len;
    int W, S;        // lanes, streams (4W)
    int64_t V, n;    // vectors, rows of each stream
    int lp;
    int64_t step, nb, g1, r1, g2, k2;  // step, full blocks, full super-blocks, blocks of the
                                       // partial one, full level-2 groups, super-blocks past them

    __host__ __device__ AtenRun(const AtenSum& a, int run) {
        const int r = run / a.chunks, c = run % a.chunks;
        const int64_t lo = (int64_t)c * a.chunk;
        const int64_t hi = lo + a.chunk < a.m ? lo + a.chunk : a.m;
        es = a.es;
        base = a.x + r * a.row_stride + lo * a.es;
        len = hi > lo ? hi - lo : 0;
        W = len >= a.lanes ? a.lanes : 1;
        S = 4 * W;
        V = len / W;
        n = V / 4;
        lp = aten_level_power(n);
        step = (int64_t)1 << lp;
        nb = n / step;
        g1 = nb / step;
        r1 = nb - g1 * step;
        g2 = g1 / step;
        k2 = g1 - g2 * step;
    }

    // stream s's row i (s = k W + l: column k, lane l)
    __device__ __forceinline__ float* at(int64_t i, int s) const {
        const int k = s / W, l = s - k * W;
        return base + ((4 * i + k) * W + l) * es;
    }
    __device__ __forceinline__ float* flat(int64_t e) const { return base + e * es; }
};

// L1: block (g, run) sums super-block g of every stream of the run: thread task (b, s) --
// block b of stream s, `step` rows from 0, all loads issued together -- lands in LDS, then
// thread s adds the super-block's block sums from 0 and writes the sum over the super-block's
// row 0; g == g1 is the partial super-block's r1 blocks (acc1 when the cascade stops),
// written over its row 0 too.  A wave's load touches 128-B runs (32 streams x 4 B).
constexpr int kAtenL1Threads = 256;
constexpr int kAtenMaxStep = 64;  // lp <= 6: runs up to 2^27 rows of each stream

__global__ __launch_bounds__(kAtenL1Threads) void aten_sum_l1(AtenSum a) {
    __shared__ float bs[kAtenMaxStep * 4 * kAtenMaxLanes];
    const AtenRun R(a, blockIdx.y);
    const int64_t g = blockIdx.x;
    if (g > R.g1 || (g == R.g1 && R.r1 == 0)) return;  // block-uniform
    const int blocks = (int)(g < R.g1 ? R.step : R.r1);
    const int64_t i0 = g * R.step * R.step;
    const int step = (int)R.step;
    for (int task = threadIdx.x; task < blocks * R.S; task += kAtenL1Threads) {
        const int b = task / R.S, s = task - b * R.S;
        const int64_t ib = i0 + (int64_t)b * step;
        float acc0 = 0.f;
        for (int j = 0; j < step; j += 16) {  // step is a multiple of 16
            float v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = *R.at(ib + j + u, s);
#pragma unroll
            for (int u = 0; u < 16; ++u) acc0 = acc0 + v[u];
        }
        bs[b * R.S + s] = acc0;
    }
    __syncthreads();
    if (threadIdx.x >= R.S) return;
    const int s = threadIdx.x;
    float acc1 = 0.f;
    for (int b = 0; b < blocks; ++b) acc1 = acc1 + bs[b * R.S + s];
    *R.at(i0, s) = acc1;
}

// L2: thread (h, s) sums group h of `step` super-block sums from 0 (over the group's row 0);
// h == g2 sums the k2 full super-blocks past the last group (acc2 when the cascade stops),
// written over row 1 of the group's first super-block (row 0 holds that super-block's sum).
__global__ __launch_bounds__(256) void aten_sum_l2(AtenSum a) {
    const AtenRun R(a, blockIdx.y);
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int s = (int)(idx % R.S);
    const int64_t h = idx / R.S;
    if (h > R.g2 || (h == R.g2 && R.k2 == 0)) return;
    const int64_t cnt = h < R.g2 ? R.step : R.k2;
    const int64_t sb = R.step * R.step;  // rows per super-block
    const int64_t i0 = h * R.step * sb;
    float acc2 = 0.f;
    for (int64_t j = 0; j < cnt; j += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = j + u < cnt ? *R.at(i0 + (j + u) * sb, s) : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (j + u < cnt) acc2 = acc2 + v[u];
    }
    *R.at(h < R.g2 ? i0 : i0 + 1, s) = acc2;
}

// L3: block per run.  Thread s finishes stream s: acc3 over the level-2 sums, then
// ((acc0 + acc1) + acc2) + acc3 with acc0 the < step rows past the last block; thread 0 then
// adds the leftover vectors into column 0, folds the columns, and adds the scalar tail and
// the lanes into 0.  Unchunked: out[row] = 0 + sum.  Chunked: the run's sum is written over
// its element 0 for L4.
__global__ __launch_bounds__(64) void aten_sum_l3(AtenSum a, float* __restrict__ out) {
    __shared__ float p[4 * kAtenMaxLanes];
    const AtenRun R(a, blockIdx.x);
    const int s = threadIdx.x;
    if (s < R.S) {
        const int64_t sb = R.step * R.step;
        float acc3 = 0.f;
        for (int64_t h = 0; h < R.g2; h += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = h + u < R.g2 ? *R.at((h + u) * R.step * sb, s) : 0.f;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (h + u < R.g2) acc3 = acc3 + v[u];
        }
        const float acc2 = R.k2 > 0 ? *R.at(R.g2 * R.step * sb + 1, s) : 0.f;
        const float acc1 = R.r1 > 0 ? *R.at(R.g1 * sb, s) : 0.f;
        float acc0 = 0.f;
        for (int64_t i = R.nb * R.step; i < R.n; ++i) acc0 = acc0 + *R.at(i, s);
        p[s] = ((acc0 + acc1) + acc2) + acc3;
    }
    __syncthreads();
    if (s != 0) return;
    float final_acc = 0.f;
    for (int64_t e = R.V * R.W; e < R.len; ++e) final_acc = final_acc + *R.flat(e);
    for (int l = 0; l < R.W; ++l) {
        float p0 = p[l];
        for (int64_t v = 4 * R.n; v < R.V; ++v) p0 = p0 + *R.flat(v * R.W + l);
        p0 = p0 + p[R.W + l];
        p0 = p0 + p[2 * R.W + l];
        p0 = p0 + p[3 * R.W + l];
        final_acc = final_acc + p0;
    }
    const float stored = 0.f + final_acc;
    if (a.chunks == 1) {
        out[blockIdx.x] = stored;
    } else if (R.len > 0) {
        *R.flat(0) = stored;
    }
}

// L4 (chunked runs only): one thread per row sums the T-slot buffer -- the chunks' sums,
// then zeros -- serially, exactly as one L1-L3 pass would (the buffer is short: no block).
__global__ __launch_bounds__(64) void aten_sum_l4(AtenSum a, int threads, int lanes,
                                                  float* __restrict__ out) {
    if (threadIdx.x != 0) return;
    const int row = blockIdx.x;
    auto slot = [&](int64_t t) -> float {
        if (t >= a.chunks) return 0.f;
        const int64_t lo = t * a.chunk;
        return lo < a.m ? a.x[row * a.row_stride + lo * a.es] : 0.f;
    };
    const int m = threads;
    const int W = m >= lanes ? lanes : 1;
    const int V = m / W, n = V / 4;
    const int step = 1 << aten_level_power(n);
    float p[4 * kAtenMaxLanes];
    // n <= 256 rows here: the cascade's block stage at most; no flush above level 1 fires
    // before the tail (step^2 >= 256 rows), so acc1 is all that carries
    for (int s = 0; s < 4 * W; ++s) {
        const int k = s / W, l = s - k * W;
        const int nb = n / step;
        float acc1 = 0.f;
        for (int b = 0; b < nb; ++b) {
            float acc0 = 0.f;
            for (int j = 0; j < step; ++j) acc0 = acc0 + slot((4 * (b * step + j) + k) * W + l);
            acc1 = acc1 + acc0;
        }
        float acc0 = 0.f;
        for (int i = nb * step; i < n; ++i) acc0 = acc0 + slot((4 * i + k) * W + l);
        p[s] = ((acc0 + acc1) + 0.f) + 0.f;
    }
    float final_acc = 0.f;
    for (int e = V * W; e < m; ++e) final_acc = final_acc + slot(e);
    for (int l = 0; l < W; ++l) {
        float p0 = p[l];
        for (int v = 4 * n; v < V; ++v) p0 = p0 + slot(v * W + l);
        p0 = p0 + p[W + l];
        p0 = p0 + p[2 * W + l];
        p0 = p0 + p[3 * W + l];
        final_acc = final_acc + p0;
    }
    out[row] = 0.f + final_acc;
}

}  // namespace hg
