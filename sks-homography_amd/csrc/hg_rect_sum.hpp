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

constexpr int kRectSumBudget = 4096;  // floats of each parameter's terms a workgroup stages
constexpr int kRectSumThreads = 256;

// Level-0 blocks per workgroup for a run, and its workgroups: ceil(nb / G) summing ones plus
// one for the raw remainder.  The same function on host (grid, LDS) and device.
__host__ __device__ inline int64_t rect_sum_group(const AtenRun& R) {
    const int64_t per = R.step * R.S;
    return per >= kRectSumBudget ? 1 : kRectSumBudget / per;
}
__host__ __device__ inline int64_t rect_sum_units(const AtenRun& R) {
    const int64_t G = rect_sum_group(R);
    return (R.nb + G - 1) / G + 1;
}

// Grid (units, chunks): workgroup (u, c) serves run c of both rows of the (2, 3B) scratch
// a.x (row 0 dL/dscale's terms, row 1 dL/ddiv's; a.es == 1).  Every problem is computed by
// the workgroups whose float ranges hold one of its three terms and written (dL/dtar, dL/dsrc)
// by the one holding its first.  16-B aligned src / tar / grad_src / grad_tar (the launcher
// checks).  The arithmetic is tensor_aca_rect_grad_rows<kAtenCpu>: the terms' bits are those of
// tensor_aca_rect_backward_staged<..., kSdTerms>.
template <bool WANT_SRC, bool NT>
__global__ __launch_bounds__(kRectSumThreads) void rect_backward_sum_l0(
    const float* __restrict__ src, const float* __restrict__ tar, const float* __restrict__ gH,
    const float* __restrict__ scale_p, const float* __restrict__ div_p,
    float* __restrict__ gsrc, float* __restrict__ gtar, AtenSum a) {
    extern __shared__ float terms[];  // [2][F]: this workgroup's terms of each parameter
    const int c = blockIdx.y;
    const AtenRun R(a, c);
    const int64_t G = rect_sum_group(R);
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
    float* const row0 = a.x;
    float* const row1 = a.x + a.row_stride;
    const float scale = scale_p[0], div = div_p[0];
    const float sc[3] = {scale, scale, scale}, dv[3] = {div, div, div};
    for (int64_t p = p0 + threadIdx.x; p < p1; p += kRectSumThreads) {
        float tr[12], g[9], gt[12];
        load_row8<float, NT>(tar + p * 12, *reinterpret_cast<float(*)[8]>(tr));
        {
            const u32x4 w = ld16<NT>(reinterpret_cast<const char*>(tar + p * 12 + 8));
            __builtin_memcpy(tr + 8, &w, 16);
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) g[k] = NT ? __builtin_nontemporal_load(gH + p * 9 + k) : gH[p * 9 + k];
        const float mx = NT ? __builtin_nontemporal_load(src + p * 12) : src[p * 12];
        const float my = NT ? __builtin_nontemporal_load(src + p * 12 + 4) : src[p * 12 + 4];
        float gmx, gmy, gs, gd, gsr[3], gdr[3];
        tensor_aca_rect_grad_rows<kAtenCpu>(tr, mx, my, sc, dv, g, gt, gmx, gmy, gs, gd, gsr, gdr);
        if (3 * p >= g0) {  // this workgroup holds the problem's first term: its gradients
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                u32x4 w;
                __builtin_memcpy(&w, gt + 4 * q, 16);
                st16<NT>(reinterpret_cast<char*>(gtar + p * 12 + 4 * q), w);
            }
            if constexpr (WANT_SRC) {
                const float z[12] = {gmx, 0.f, 0.f, 0.f, gmy, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    u32x4 w;
                    __builtin_memcpy(&w, z + 4 * q, 16);
                    st16<NT>(reinterpret_cast<char*>(gsrc + p * 12 + 4 * q), w);
                }
            }
        }
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
