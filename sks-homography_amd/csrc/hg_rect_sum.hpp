// hg_rect_sum.hpp -- TensorACA_rect's backward with the batch-uniform scale / div gradients
// summed in ATen-CPU's order, the sum's first level fused into the backward kernel
// (hg_tensor_aca_rect_backward_sum_f32).  Included by hg_kernels.hip after hg_rect.hpp and
// hg_reduce.hpp.
//
// The two-launch form (hg_tensor_aca_rect_backward_terms_f32, then hg_sum_aten_f32 over the
// (2,B,3) terms) writes 24 B of terms per problem and reads them straight back in aten_sum_l1
// (≈ 95 us of an 804-us op at B = 16 M).  Here each workgroup owns a range of the
// cascade's level-0 blocks (hg_reduce.hpp: a block is `step` rows of S = 4W streams, one
// contiguous run of step * S floats of the terms): it computes the problems whose terms fall in
// that range, keeps the terms in LDS, and writes each block's S sums (from 0, row by row, the
// order aten_sum_l1 adds them in) over the block's first row in the scratch.  The range past the
// last full block of a run (the rows, vectors and scalars the cascade adds raw) is written raw.
// aten_sum_l1_blocks then folds each super-block's block sums exactly as aten_sum_l1 does, and
// aten_sum_l2 / l3 / l4 run unchanged: the bits are those of the two-launch form.
#pragma once

#include "hg_rect.hpp"
#include "hg_reduce.hpp"

namespace hg {

constexpr int kRectSumBudget = 4096;  // floats of each parameter's terms a workgroup stages (default)
constexpr int kRectSumThreads = 256;  // kWavesPerBlock waves
constexpr int64_t kRectSumMaxStep = 128;  // larger level steps (runs of > 2^31 rows): two launches
// LDS: the four waves' slabs (21 KiB) + 2 x max(budget, step S) floats (32 KiB at 4096 / step 128)

// Level-0 blocks per workgroup for a run, and its workgroups: ceil(nb / G) summing ones plus
// one for the raw remainder.  The same function on host (grid, LDS) and device.
__host__ __device__ inline int64_t rect_sum_group(const AtenRun& R, int budget) {
    const int64_t per = R.step * R.S;
    return per >= budget ? 1 : budget / per;
}
__host__ __device__ inline int64_t rect_sum_units(const AtenRun& R, int budget) {
    const int64_t G = rect_sum_group(R, budget);
    return (R.nb + G - 1) / G + 1;
}

// Grid (units, chunks): workgroup (u, c) serves run c of both rows of the (2, 3B) scratch
// a.x (row 0 dL/dscale's terms, row 1 dL/ddiv's; a.es == 1).  Every problem is computed by
// the workgroups whose float ranges hold one of its three terms and written (dL/dtar, dL/dsrc)
// by the one holding its first.  The waves take tiles of 64 problems from a 4-aligned start as
// tensor_aca_rect_backward_staged does -- tar and dL/dH slabs by LDS-DMA, dL/dtar and dL/dsrc
// leaving as contiguous slabs when the workgroup owns the whole tile, per lane at the range's
// edges -- and each lane puts the terms of its problem that fall in the range into LDS; then
// task (param, block, stream) sums its block's rows from 0 in order.  16-B aligned src / tar /
// grad_H / grad_src / grad_tar (the launcher checks).  The arithmetic is
// tensor_aca_rect_grad_rows<kAtenCpu>: the terms' bits are those of
// tensor_aca_rect_backward_staged<..., kSdTerms>.
// Measured at B = 16 M, T = 16 (tools/kbench_rect_sum.py, profiles/r06): a 4096-float budget
// 713 us for this kernel (2048: 746, 1024: 790; dL/dH per lane instead of by DMA +20 us);
// a variant with no workgroup-wide LDS -- each wave walking its own unit tile after tile and
// adding its streams in registers -- 808 us: one wave's tiles in series expose their latency.
template <bool WANT_SRC, bool NT>
__global__ __launch_bounds__(kRectSumThreads) void rect_backward_sum_l0(
    const float* __restrict__ src, const float* __restrict__ tar, const float* __restrict__ gH,
    int64_t B, const float* __restrict__ scale_p, const float* __restrict__ div_p,
    float* __restrict__ gsrc, float* __restrict__ gtar, AtenSum a, int budget) {
    constexpr int kTar = kWave * 48, kG = kWave * 36;
    __shared__ __attribute__((aligned(16))) char slab[kWavesPerBlock][kTar + kG];
    extern __shared__ float terms[];  // [2][F]: this workgroup's terms of each parameter
    const int c = blockIdx.y;
    const AtenRun R(a, c);
    const int64_t G = rect_sum_group(R, budget);
    const int64_t sums = (R.nb + G - 1) / G;
    const int64_t u = blockIdx.x;
    if (u > sums) return;  // workgroup-uniform
    const bool raw = u == sums;
    const int64_t blockf = R.step * R.S;  // floats of one level-0 block
    const int64_t F0 = raw ? R.nb * blockf : u * G * blockf;
    const int64_t F1 = raw ? R.len : (F0 + G * blockf < R.nb * blockf ? F0 + G * blockf : R.nb * blockf);
    if (F1 <= F0) return;
    const int64_t F = F1 - F0;
    const int64_t off = (int64_t)c * a.chunk;  // the run's first float in its row
    const int64_t g0 = off + F0, g1 = off + F1;
    const int64_t p0 = g0 / 3, p1 = (g1 + 2) / 3;
    const int64_t q0 = p0 & ~(int64_t)3;  // tiles start 4-aligned: dL/dH slabs 16-B aligned
    float* const row0 = a.x;
    float* const row1 = a.x + a.row_stride;
    const float scale = scale_p[0], div = div_p[0];
    const float sc[3] = {scale, scale, scale}, dv[3] = {div, div, div};
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    char* lds = slab[wave];
    const int64_t tiles = (p1 - q0 + kWave - 1) / kWave;
    for (int64_t t = wave; t < tiles; t += kWavesPerBlock) {
        const int64_t base = q0 + t * kWave;
        const int64_t p = base + lane;
        float tr[12], g[9], gt[12], mx, my;
        const bool full = base + kWave <= B;  // wave-uniform
        if (full) {
            mx = NT ? __builtin_nontemporal_load(src + p * 12 + 0) : src[p * 12 + 0];
            my = NT ? __builtin_nontemporal_load(src + p * 12 + 4) : src[p * 12 + 4];
            dma_slab_issue<kTar, NT>(reinterpret_cast<const char*>(tar + base * 12), lds, lane);
            dma_slab_issue<kG, NT>(reinterpret_cast<const char*>(gH + base * 9), lds + kTar, lane);
            dma_wait_sync();
            __builtin_memcpy(tr, lds + lane * 48, 48);
#pragma unroll
            for (int k = 0; k < 9; ++k) g[k] = reinterpret_cast<const float*>(lds + kTar)[lane * 9 + k];
        } else {
            const int64_t q = p < B ? p : B - 1;  // lanes past the batch compute a copy, write nothing
#pragma unroll
            for (int k = 0; k < 12; ++k) tr[k] = tar[q * 12 + k];
#pragma unroll
            for (int k = 0; k < 9; ++k) g[k] = gH[q * 9 + k];
            mx = src[q * 12 + 0];
            my = src[q * 12 + 4];
        }
        float gmx, gmy, gs, gd, gsr[3], gdr[3];
        tensor_aca_rect_grad_rows<kAtenCpu>(tr, mx, my, sc, dv, g, gt, gmx, gmy, gs, gd, gsr, gdr);
        const float gsv[12] = {gmx, 0.f, 0.f, 0.f, gmy, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        // the whole tile is this workgroup's: first terms 3 base ... 3 (base + 63) in range
        if (full && 3 * base >= g0 && 3 * (base + kWave - 1) < g1) {
            wave_lds_sync();  // the staging below reuses the input bytes
            store_rows_staged<12, NT>(reinterpret_cast<char*>(gtar + base * 12), gt, lds, lane);
            if constexpr (WANT_SRC)
                store_rows_staged<12, NT>(reinterpret_cast<char*>(gsrc + base * 12), gsv, lds, lane);
        } else {
            if (p < B && 3 * p >= g0 && 3 * p < g1) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    u32x4 w;
                    __builtin_memcpy(&w, gt + 4 * q, 16);
                    st16<NT>(reinterpret_cast<char*>(gtar + p * 12 + 4 * q), w);
                    if constexpr (WANT_SRC) {
                        __builtin_memcpy(&w, gsv + 4 * q, 16);
                        st16<NT>(reinterpret_cast<char*>(gsrc + p * 12 + 4 * q), w);
                    }
                }
            }
            wave_lds_sync();  // this tile's slab reads are done before the next tile's DMA
        }
        if (p < B) {
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const int64_t e = 3 * p + r;
                if (e < g0 || e >= g1) continue;
                if (raw) {  // the cascade adds these one by one: the scratch holds them as they are
                    row0[e] = gsr[r];
                    row1[e] = gdr[r];
                } else {
                    terms[e - g0] = gsr[r];
                    terms[F + (e - g0)] = gdr[r];
                }
            }
        }
    }
    if (raw) return;
    __syncthreads();
    // task (param, b, s): block b of stream s, its `step` rows summed from 0 in order, written
    // over the block's first row (row (u G + b) step of the run)
    const int64_t nblk = F / blockf;
    const int64_t tasks = 2 * nblk * R.S;
    for (int64_t t = threadIdx.x; t < tasks; t += kRectSumThreads) {
        const int param = (int)(t / (nblk * R.S));
        const int64_t rem = t - param * nblk * R.S;
        const int64_t b = rem / R.S;
        const int s = (int)(rem - b * R.S);
        const float* v = terms + param * F + b * blockf + s;
        float acc0 = 0.f;
        for (int64_t j = 0; j < R.step; ++j) acc0 = acc0 + v[j * R.S];
        const int64_t i = (u * G + b) * R.step;
        (param ? row1 : row0)[off + 4 * i * R.W + s] = acc0;
    }
}

// aten_sum_l1 over block sums already in place (rect_backward_sum_l0): thread s of block
// (g, run) adds super-block g's block sums of stream s from 0 -- row b * step of the
// super-block holds block b's -- and writes the result over the super-block's row 0.
__global__ __launch_bounds__(64) void aten_sum_l1_blocks(AtenSum a) {
    const AtenRun R(a, blockIdx.y);
    const int64_t g = blockIdx.x;
    if (g > R.g1 || (g == R.g1 && R.r1 == 0)) return;  // block-uniform
    const int s = threadIdx.x;
    if (s >= R.S) return;
    const int64_t blocks = g < R.g1 ? R.step : R.r1;
    const int64_t i0 = g * R.step * R.step;
    float acc1 = 0.f;
    for (int64_t b = 0; b < blocks; b += 8) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = b + q < blocks ? *R.at(i0 + (b + q) * R.step, s) : 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (b + q < blocks) acc1 = acc1 + v[q];
    }
    *R.at(i0, s) = acc1;
}

}  // namespace hg
