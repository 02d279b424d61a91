// hg_rect.hpp -- TensorACA kernels (rect (B,3,4) form, compact corner+offsets form,
// and their backward passes).  Included by hg_kernels.hip
// (the C ABI) and hg_tune.hip (the variant sweep).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "hg_aos.hpp"
#include "hg_solvers.hpp"

namespace hg {

// ---------------------------------------------------------------------------
// TensorACA rect: src/tar (B,3,4) f32, H (B,3,3) f32, unnormalised.
// A wave owns 64*P problems.  Full tiles (VEC: 16-B aligned tensors): the wave's
// contiguous tar slab (64*P*48 B) lands in LDS by LDS-DMA, each lane then reads its
// 48-B record with three ds_read_b128; M's x and y come from src with two dword
// loads per lane (offsets 0 and 16 of the 48-B src record) issued before the DMA
// wait.  H is written through the LDS-staged 16-B store.  Ragged/unaligned tiles
// use per-lane loads and stores.
// ORDER: kAtenCpu or kAtenRocm, whose evaluation of the statements to follow (hg_solvers.hpp).
template <int P, bool VEC, bool SCALAR_ARGS, bool SQUARE = false, bool NT = true, int ORDER = kAtenCpu>
__global__ __launch_bounds__(kBlock) void tensor_aca_rect_kernel(
    const float* __restrict__ src, const float* __restrict__ tar, float* __restrict__ H,
    int64_t B, const float* __restrict__ scale_p, const float* __restrict__ div_p,
    float scale_v, float div_v) {
    constexpr int kTile = kWave * P;
    constexpr int kSlab = kTile * 48;
    constexpr int kLds = kSlab > kTile * 36 ? kSlab : kTile * 36;
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][VEC ? kLds : 16];

    const float scale = SCALAR_ARGS ? scale_v : scale_p[0];
    const float div = SCALAR_ARGS ? div_v : div_p[0];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kTile;
    if (base >= B) return;
    const bool full = VEC && base + kTile <= B;
    char* lds = smem[wave];

    float h[P][9];
    if (full) {
        float mx[P], my[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int64_t p = base + j * kWave + lane;
            mx[j] = NT ? __builtin_nontemporal_load(src + p * 12 + 0) : src[p * 12 + 0];
            my[j] = NT ? __builtin_nontemporal_load(src + p * 12 + 4) : src[p * 12 + 4];
        }
        const char* const g[1] = {reinterpret_cast<const char*>(tar + base * 12)};
        char* const l[1] = {lds};
        slabs_to_lds<kSlab, 1, true, NT>(g, l, lane);
#pragma unroll
        for (int j = 0; j < P; ++j) {
            float tr[12];
            __builtin_memcpy(tr, lds + (j * kWave + lane) * 48, 48);
            tensor_aca_rect_solve<SQUARE, ORDER>(tr, mx[j], my[j], scale, div, h[j]);
        }
        wave_lds_sync();
        store_rows9_staged<float, P, NT>(reinterpret_cast<char*>(H + base * 9), h, lds, lane);
        return;
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int64_t p = base + j * kWave + lane;
        if (p < B) {
            float tr[12];
#pragma unroll
            for (int k = 0; k < 12; ++k) tr[k] = tar[p * 12 + k];
            tensor_aca_rect_solve<SQUARE, ORDER>(tr, src[p * 12 + 0], src[p * 12 + 4], scale, div, h[j]);
#pragma unroll
            for (int k = 0; k < 9; ++k) H[p * 9 + k] = h[j][k];
        }
    }
}

// ---------------------------------------------------------------------------
// TensorACA rect backward: one lane per problem, grid-stride.  Writes dL/dtar
// (B,3,4), optionally dL/dsrc (B,3,4: only [0][0] and [1][0] are non-zero) and, by SD,
// dL/dscale and dL/ddiv as
//   kSdSums  -- a (2,B) array of per-problem sums (the three row terms from +0, ATen's
//               reduction to a (B,1,1) operand: hg_tensor_aca_rect_backward_f32's contract), or
//   kSdTerms -- the (problem, row) terms as a (2,B,3) array, each half in the order of the
//               (B,3,1) tensor ATen autograd sums to the (1,) parameter (hg_sum_aten_f32;
//               hg_tensor_aca_rect_backward_terms_f32).
enum : int { kSdNone = 0, kSdSums = 1, kSdTerms = 2 };

template <int SD>
__device__ __forceinline__ void store_sd(float* __restrict__ gsd, int64_t B, int64_t p,
                                         const float (&gsr)[3], const float (&gdr)[3], float gs,
                                         float gd) {
    if constexpr (SD == kSdSums) {
        gsd[p] = gs;
        gsd[B + p] = gd;
    } else if constexpr (SD == kSdTerms) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            gsd[3 * p + r] = gsr[r];
            gsd[3 * B + 3 * p + r] = gdr[r];
        }
    }
}

// A wave's 64 rows of 3 floats (lane l's v) as ONE contiguous 768-B run at `out` (16-B
// aligned): ds_write_b32 at an odd dword stride (conflict-free), then lanes 0..47 store 16 B.
template <bool NT>
__device__ __forceinline__ void store_terms3_staged(char* __restrict__ out, const float (&v)[3],
                                                    char* lds, int lane) {
    float* st = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int r = 0; r < 3; ++r) st[lane * 3 + r] = v[r];
    wave_lds_sync();
    if (lane < 48) st16<NT>(out + 16 * lane, *reinterpret_cast<const u32x4*>(lds + 16 * lane));
    wave_lds_sync();
}

template <bool WANT_SRC, int SD, int ORDER = kAtenCpu>
__global__ __launch_bounds__(kBlock) void tensor_aca_rect_backward_kernel(
    const float* __restrict__ src, const float* __restrict__ tar, const float* __restrict__ gH,
    int64_t B, const float* __restrict__ scale_p, const float* __restrict__ div_p,
    float* __restrict__ gsrc, float* __restrict__ gtar, float* __restrict__ gsd) {
    const float scale = scale_p[0], div = div_p[0];
    const float sc[3] = {scale, scale, scale}, dv[3] = {div, div, div};
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < B; p += stride) {
        float tr[12], g[9], gt[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) tr[k] = tar[p * 12 + k];
#pragma unroll
        for (int k = 0; k < 9; ++k) g[k] = gH[p * 9 + k];
        float gmx, gmy, gs, gd, gsr[3], gdr[3];
        tensor_aca_rect_grad_rows<ORDER>(tr, src[p * 12 + 0], src[p * 12 + 4], sc, dv, g, gt, gmx,
                                         gmy, gs, gd, gsr, gdr);
#pragma unroll
        for (int k = 0; k < 12; ++k) gtar[p * 12 + k] = gt[k];
        if constexpr (WANT_SRC) {
#pragma unroll
            for (int k = 0; k < 12; ++k) gsrc[p * 12 + k] = k == 0 ? gmx : (k == 4 ? gmy : 0.f);
        }
        store_sd<SD>(gsd, B, p, gsr, gdr, gs, gd);
    }
}

// ---------------------------------------------------------------------------
// TensorACA rect with scale / div broadcast as the reference composition broadcasts them
// (.py:301-302: torch.mul(div, X) and scale * h_temp against (B,3,1) columns): value (b, r)
// of each is p[b * sb + r * sr], element strides, 0 along a broadcast dimension -- a (B,1,1)
// tensor gives one value per problem, (3,1) one per row, (B,3,1) one per (problem, row).
// One lane per problem, grid-stride; the arithmetic of tensor_aca_rect_solve_rows.
struct RectBcast {
    const float* scale;
    int64_t ssb, ssr;
    const float* div;
    int64_t dsb, dsr;
};

__device__ __forceinline__ void rect_bcast_load(const RectBcast& a, int64_t p, float (&sc)[3],
                                                float (&dv)[3]) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        sc[r] = a.scale[p * a.ssb + r * a.ssr];
        dv[r] = a.div[p * a.dsb + r * a.dsr];
    }
}

template <int ORDER = kAtenCpu>
__global__ __launch_bounds__(kBlock) void tensor_aca_rect_bcast_kernel(
    const float* __restrict__ src, const float* __restrict__ tar, float* __restrict__ H, int64_t B,
    RectBcast a) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < B; p += stride) {
        float tr[12], sc[3], dv[3], h[9];
#pragma unroll
        for (int k = 0; k < 12; ++k) tr[k] = tar[p * 12 + k];
        rect_bcast_load(a, p, sc, dv);
        tensor_aca_rect_solve_rows<false, ORDER>(tr, src[p * 12 + 0], src[p * 12 + 4], sc, dv, h);
#pragma unroll
        for (int k = 0; k < 9; ++k) H[p * 9 + k] = h[k];
    }
}

// The same, staged like tensor_aca_rect_kernel<1, true, ...> (16-B aligned src / tar / H): the
// wave's tar slab by LDS-DMA, M's x and y with two dword loads, scale / div per (problem, row)
// through RectBcast, H through the staged 16-B store; a ragged last wave takes the per-lane
// code.  Same arithmetic, same bits.
template <bool NT, int ORDER = kAtenCpu>
__global__ __launch_bounds__(kBlock) void tensor_aca_rect_bcast_staged(
    const float* __restrict__ src, const float* __restrict__ tar, float* __restrict__ H, int64_t B,
    RectBcast a) {
    constexpr int kSlab = kWave * 48;  // >= the 36-B rows H stages
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][kSlab];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kWave;
    if (base >= B) return;
    const int64_t p = base + lane;
    char* lds = smem[wave];
    float h[1][9], sc[3], dv[3];
    if (base + kWave <= B) {
        const float mx = NT ? __builtin_nontemporal_load(src + p * 12 + 0) : src[p * 12 + 0];
        const float my = NT ? __builtin_nontemporal_load(src + p * 12 + 4) : src[p * 12 + 4];
        rect_bcast_load(a, p, sc, dv);
        const char* const g[1] = {reinterpret_cast<const char*>(tar + base * 12)};
        char* const l[1] = {lds};
        slabs_to_lds<kSlab, 1, true, NT>(g, l, lane);
        float tr[12];
        __builtin_memcpy(tr, lds + lane * 48, 48);
        tensor_aca_rect_solve_rows<false, ORDER>(tr, mx, my, sc, dv, h[0]);
        wave_lds_sync();
        store_rows9_staged<float, 1, NT>(reinterpret_cast<char*>(H + base * 9), h, lds, lane);
        return;
    }
    if (p >= B) return;
    float tr[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) tr[k] = tar[p * 12 + k];
    rect_bcast_load(a, p, sc, dv);
    tensor_aca_rect_solve_rows<false, ORDER>(tr, src[p * 12 + 0], src[p * 12 + 4], sc, dv, h[0]);
#pragma unroll
    for (int k = 0; k < 9; ++k) H[p * 9 + k] = h[0][k];
}

// Its backward: dL/dtar, optionally dL/dsrc, and per parameter (mode *_rows) the problem's
// three-row sum ((B): gs[p] = ((0 + t0) + t1) + t2, ATen's reduction to a (B,1,1) shape; mode
// 0), each row's share as (3,B) rows (gs[r * B + p]; mode 1) or as the (B,3) terms in the
// order ATen sums them to a batch-uniform shape (gs[3 p + r]; mode 2); the caller reduces
// them to the parameter's shape.
template <int ORDER = kAtenCpu>
__global__ __launch_bounds__(kBlock) void tensor_aca_rect_bcast_backward_kernel(
    const float* __restrict__ src, const float* __restrict__ tar, const float* __restrict__ gH,
    int64_t B, RectBcast a, float* __restrict__ gsrc, float* __restrict__ gtar,
    float* __restrict__ gsc, int sc_rows, float* __restrict__ gdv, int dv_rows) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < B; p += stride) {
        float tr[12], g[9], gt[12], sc[3], dv[3], gsr[3], gdr[3];
#pragma unroll
        for (int k = 0; k < 12; ++k) tr[k] = tar[p * 12 + k];
#pragma unroll
        for (int k = 0; k < 9; ++k) g[k] = gH[p * 9 + k];
        rect_bcast_load(a, p, sc, dv);
        float gmx, gmy, gscale, gdiv;
        tensor_aca_rect_grad_rows<ORDER>(tr, src[p * 12 + 0], src[p * 12 + 4], sc, dv, g, gt, gmx, gmy,
                                  gscale, gdiv, gsr, gdr);
#pragma unroll
        for (int k = 0; k < 12; ++k) gtar[p * 12 + k] = gt[k];
        if (gsrc) {
#pragma unroll
            for (int k = 0; k < 12; ++k) gsrc[p * 12 + k] = k == 0 ? gmx : (k == 4 ? gmy : 0.f);
        }
        if (gsc) {
            if (sc_rows == 1) {
#pragma unroll
                for (int r = 0; r < 3; ++r) gsc[r * B + p] = gsr[r];
            } else if (sc_rows == 2) {
#pragma unroll
                for (int r = 0; r < 3; ++r) gsc[3 * p + r] = gsr[r];
            } else {
                gsc[p] = gscale;
            }
        }
        if (gdv) {
            if (dv_rows == 1) {
#pragma unroll
                for (int r = 0; r < 3; ++r) gdv[r * B + p] = gdr[r];
            } else if (dv_rows == 2) {
#pragma unroll
                for (int r = 0; r < 3; ++r) gdv[3 * p + r] = gdr[r];
            } else {
                gdv[p] = gdiv;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Compact TensorACA: corner (B,2) + offsets (B,4,2) -> H (B,3,3) = 8 + 32 + 36 B per
// problem instead of the (B,3,4) tensors' 48 + 48 + 36.  Full tiles: both slabs by
// LDS-DMA (P = 1: 512 B of corners + 2 KiB of offsets per wave), staged 16-B H stores.
template <int P, bool VEC, bool SQUARE, bool NT = true>
__global__ __launch_bounds__(kBlock) void tensor_aca_offsets_kernel(
    const float* __restrict__ corner, const float* __restrict__ offsets, float* __restrict__ H,
    int64_t B, float w, float h) {
    constexpr int kTile = kWave * P;
    constexpr int kCorner = kTile * 8, kOff = kTile * 32;
    constexpr int kLds = kCorner + kOff > kTile * 36 ? kCorner + kOff : kTile * 36;
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][VEC ? kLds : 16];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kTile;
    if (base >= B) return;
    const float div = w / h;
    char* lds = smem[wave];
    float hm[P][9];
    if (VEC && base + kTile <= B) {
        dma_slab_issue<kCorner, NT>(reinterpret_cast<const char*>(corner + base * 2), lds, lane);
        dma_slab_issue<kOff, NT>(reinterpret_cast<const char*>(offsets + base * 8),
                                   lds + kCorner, lane);
        dma_wait_sync();
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int row = j * kWave + lane;
            float c[2], off[8], tr[12];
            __builtin_memcpy(c, lds + row * 8, 8);
            __builtin_memcpy(off, lds + kCorner + row * 32, 32);
            rect_target_from_offsets(c[0], c[1], w, h, off, tr);
            tensor_aca_rect_solve<SQUARE>(tr, c[0], c[1], w, div, hm[j]);
        }
        wave_lds_sync();
        store_rows9_staged<float, P, NT>(reinterpret_cast<char*>(H + base * 9), hm, lds, lane);
        return;
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int64_t p = base + j * kWave + lane;
        if (p < B) {
            float off[8], tr[12];
#pragma unroll
            for (int k = 0; k < 8; ++k) off[k] = offsets[p * 8 + k];
            const float mx = corner[p * 2], my = corner[p * 2 + 1];
            rect_target_from_offsets(mx, my, w, h, off, tr);
            tensor_aca_rect_solve<SQUARE>(tr, mx, my, w, div, hm[j]);
#pragma unroll
            for (int k = 0; k < 9; ++k) H[p * 9 + k] = hm[j][k];
        }
    }
}

// Backward of the compact form: dL/doffsets (B,4,2) and optionally dL/dcorner (B,2).
template <bool WANT_CORNER>
__global__ __launch_bounds__(kBlock) void tensor_aca_offsets_backward_kernel(
    const float* __restrict__ corner, const float* __restrict__ offsets,
    const float* __restrict__ gH, int64_t B, float w, float h, float* __restrict__ g_off,
    float* __restrict__ g_corner) {
    const float div = w / h;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < B; p += stride) {
        float off[8], tr[12], g[9], gt[12];
#pragma unroll
        for (int k = 0; k < 8; ++k) off[k] = offsets[p * 8 + k];
#pragma unroll
        for (int k = 0; k < 9; ++k) g[k] = gH[p * 9 + k];
        const float mx = corner[p * 2], my = corner[p * 2 + 1];
        rect_target_from_offsets(mx, my, w, h, off, tr);
        float gmx, gmy, gsc, gdv;
        tensor_aca_rect_grad(tr, mx, my, w, div, g, gt, gmx, gmy, gsc, gdv);
        // tar[0][j] = x_j + off[j].x, tar[1][j] = y_j + off[j].y
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            g_off[p * 8 + 2 * j] = gt[j];
            g_off[p * 8 + 2 * j + 1] = gt[4 + j];
        }
        if constexpr (WANT_CORNER) {
            g_corner[p * 2] = gmx + (((gt[0] + gt[1]) + gt[2]) + gt[3]);
            g_corner[p * 2 + 1] = gmy + (((gt[4] + gt[5]) + gt[6]) + gt[7]);
        }
    }
}

// Staged forms of the two backward kernels (full 64-problem wave tiles, 16-B aligned
// tensors): the tile's input slabs land in LDS by LDS-DMA, each lane reads its records
// there, and the gradient rows leave as contiguous slabs (store_rows_staged) instead
// of 48-B / 32-B per-lane strided accesses.  The ragged tail takes the per-lane code.
// Same arithmetic (tensor_aca_rect_grad), same bits.
// NOSOLVE (tune only): the same loads and stores with the gradients replaced by a copy of the
// loaded values -- the memory pattern's own ceiling.
template <bool WANT_SRC, int SD, bool NT, int ORDER = kAtenCpu, bool NOSOLVE = false>
__global__ __launch_bounds__(kBlock) void tensor_aca_rect_backward_staged(
    const float* __restrict__ src, const float* __restrict__ tar, const float* __restrict__ gH,
    int64_t B, const float* __restrict__ scale_p, const float* __restrict__ div_p,
    float* __restrict__ gsrc, float* __restrict__ gtar, float* __restrict__ gsd) {
    constexpr int kTar = kWave * 48, kG = kWave * 36;
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][kTar + kG];
    const float scale = scale_p[0], div = div_p[0];
    const float sc[3] = {scale, scale, scale}, dv[3] = {div, div, div};
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kWave;
    if (base >= B) return;
    const int64_t p = base + lane;
    char* lds = smem[wave];
    if (base + kWave <= B) {
        const float mx = NT ? __builtin_nontemporal_load(src + p * 12 + 0) : src[p * 12 + 0];
        const float my = NT ? __builtin_nontemporal_load(src + p * 12 + 4) : src[p * 12 + 4];
        dma_slab_issue<kTar, NT>(reinterpret_cast<const char*>(tar + base * 12), lds, lane);
        dma_slab_issue<kG, NT>(reinterpret_cast<const char*>(gH + base * 9), lds + kTar, lane);
        dma_wait_sync();
        float tr[12], g[9], gt[12];
        __builtin_memcpy(tr, lds + lane * 48, 48);
#pragma unroll
        for (int k = 0; k < 9; ++k) g[k] = reinterpret_cast<const float*>(lds + kTar)[lane * 9 + k];
        float gmx, gmy, gs, gd, gsr[3], gdr[3];
        if constexpr (NOSOLVE) {
#pragma unroll
            for (int q = 0; q < 12; ++q) gt[q] = tr[q] + g[q % 9];
            gmx = mx + g[0];
            gmy = my + g[1];
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                gsr[r] = tr[r] * g[r];
                gdr[r] = tr[r + 4] * g[r + 3];
            }
            gs = gsr[0];
            gd = gdr[0];
        } else {
            tensor_aca_rect_grad_rows<ORDER>(tr, mx, my, sc, dv, g, gt, gmx, gmy, gs, gd, gsr, gdr);
        }
        wave_lds_sync();  // the staging below reuses the input bytes
        store_rows_staged<12, NT>(reinterpret_cast<char*>(gtar + base * 12), gt, lds, lane);
        if constexpr (WANT_SRC) {
            float gs[12];
#pragma unroll
            for (int k = 0; k < 12; ++k) gs[k] = k == 0 ? gmx : (k == 4 ? gmy : 0.f);
            store_rows_staged<12, NT>(reinterpret_cast<char*>(gsrc + base * 12), gs, lds, lane);
        }
        if constexpr (SD == kSdSums) {
            store_sd<SD>(gsd, B, p, gsr, gdr, gs, gd);  // lane-consecutive 4-B stores
        } else if constexpr (SD == kSdTerms) {
            // the wave's 64 x 3 terms of each parameter are one contiguous 768-B run:
            // staged, then 48 lanes store 16 B each (the second run is 16-B aligned when 3B
            // is a multiple of 4)
            store_terms3_staged<NT>(reinterpret_cast<char*>(gsd + 3 * base), gsr, lds, lane);
            if (((3 * B) & 3) == 0) {
                store_terms3_staged<NT>(reinterpret_cast<char*>(gsd + 3 * B + 3 * base), gdr, lds,
                                        lane);
            } else {
#pragma unroll
                for (int r = 0; r < 3; ++r) gsd[3 * B + 3 * p + r] = gdr[r];
            }
        }
        return;
    }
    if (p < B) {
        float tr[12], g[9], gt[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) tr[k] = tar[p * 12 + k];
#pragma unroll
        for (int k = 0; k < 9; ++k) g[k] = gH[p * 9 + k];
        float gmx, gmy, gs, gd, gsr[3], gdr[3];
        tensor_aca_rect_grad_rows<ORDER>(tr, src[p * 12 + 0], src[p * 12 + 4], sc, dv, g, gt, gmx,
                                         gmy, gs, gd, gsr, gdr);
#pragma unroll
        for (int k = 0; k < 12; ++k) gtar[p * 12 + k] = gt[k];
        if constexpr (WANT_SRC) {
#pragma unroll
            for (int k = 0; k < 12; ++k) gsrc[p * 12 + k] = k == 0 ? gmx : (k == 4 ? gmy : 0.f);
        }
        store_sd<SD>(gsd, B, p, gsr, gdr, gs, gd);
    }
}

template <bool WANT_CORNER, bool NT>
__global__ __launch_bounds__(kBlock) void tensor_aca_offsets_backward_staged(
    const float* __restrict__ corner, const float* __restrict__ offsets,
    const float* __restrict__ gH, int64_t B, float w, float h, float* __restrict__ g_off,
    float* __restrict__ g_corner) {
    constexpr int kC = kWave * 8, kO = kWave * 32, kG = kWave * 36;
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][kC + kO + kG];
    const float div = w / h;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kWave;
    if (base >= B) return;
    const int64_t p = base + lane;
    char* lds = smem[wave];
    float off[8], tr[12], g[9], gt[12], mx, my;
    const bool full = base + kWave <= B;
    if (full) {
        dma_slab_issue<kC, NT>(reinterpret_cast<const char*>(corner + base * 2), lds, lane);
        dma_slab_issue<kO, NT>(reinterpret_cast<const char*>(offsets + base * 8), lds + kC, lane);
        dma_slab_issue<kG, NT>(reinterpret_cast<const char*>(gH + base * 9), lds + kC + kO, lane);
        dma_wait_sync();
        float c[2];
        __builtin_memcpy(c, lds + lane * 8, 8);
        __builtin_memcpy(off, lds + kC + lane * 32, 32);
#pragma unroll
        for (int k = 0; k < 9; ++k)
            g[k] = reinterpret_cast<const float*>(lds + kC + kO)[lane * 9 + k];
        mx = c[0];
        my = c[1];
        wave_lds_sync();
    } else {
        if (p >= B) return;
#pragma unroll
        for (int k = 0; k < 8; ++k) off[k] = offsets[p * 8 + k];
#pragma unroll
        for (int k = 0; k < 9; ++k) g[k] = gH[p * 9 + k];
        mx = corner[p * 2];
        my = corner[p * 2 + 1];
    }
    rect_target_from_offsets(mx, my, w, h, off, tr);
    float gmx, gmy, gsc, gdv;
    tensor_aca_rect_grad(tr, mx, my, w, div, g, gt, gmx, gmy, gsc, gdv);
    // tar[0][j] = x_j + off[j].x, tar[1][j] = y_j + off[j].y
    float go[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        go[2 * j] = gt[j];
        go[2 * j + 1] = gt[4 + j];
    }
    float gc[2] = {gmx + (((gt[0] + gt[1]) + gt[2]) + gt[3]),
                   gmy + (((gt[4] + gt[5]) + gt[6]) + gt[7])};
    if (full) {
        store_rows_staged<8, NT>(reinterpret_cast<char*>(g_off + base * 8), go, lds, lane);
        if constexpr (WANT_CORNER) {
            // 8-B rows: 512 B slab, written straight (lane-consecutive 8-B stores)
            __builtin_memcpy(g_corner + p * 2, gc, 8);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) g_off[p * 8 + k] = go[k];
    if constexpr (WANT_CORNER) {
        g_corner[p * 2] = gc[0];
        g_corner[p * 2 + 1] = gc[1];
    }
}

// ---------------------------------------------------------------------------
// ACA_vanilla backward (aca_vanilla_grad): src, tar (B,4,2), dL/dH (B,3,3) -> dL/dsrc,
// dL/dtar (B,4,2), either optional.  One lane per problem, grid-stride; 100 B read and up
// to 64 B written per problem.
template <typename T>
__global__ __launch_bounds__(kBlock) void aca_vanilla_backward_kernel(
    const T* __restrict__ src, const T* __restrict__ tar, const T* __restrict__ gH, int64_t B,
    T* __restrict__ gsrc, T* __restrict__ gtar) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < B; p += stride) {
        T s[8], t[8], g[9], gs[8], gt[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s[k] = src[p * 8 + k];
            t[k] = tar[p * 8 + k];
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) g[k] = gH[p * 9 + k];
        aca_vanilla_grad(s, t, g, gs, gt);
        if (gsrc) {
#pragma unroll
            for (int k = 0; k < 8; ++k) gsrc[p * 8 + k] = gs[k];
        }
        if (gtar) {
#pragma unroll
            for (int k = 0; k < 8; ++k) gtar[p * 8 + k] = gt[k];
        }
    }
}

// Its staged binary32 form (16-B aligned tensors): a wave's 64 problems -- src and tar
// slabs of 2 KiB, the dL/dH slab of 2304 B -- land in LDS by LDS-DMA, and the gradient rows
// leave as contiguous 2-KiB slabs (store_rows_staged); a ragged last wave takes the
// per-lane code.  Same arithmetic, same bits.
template <bool WANT_SRC, bool WANT_TAR, bool NT>
__global__ __launch_bounds__(kBlock) void aca_vanilla_backward_staged(
    const float* __restrict__ src, const float* __restrict__ tar, const float* __restrict__ gH,
    int64_t B, float* __restrict__ gsrc, float* __restrict__ gtar) {
    constexpr int kS = kWave * 32, kG = kWave * 36;
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][2 * kS + kG];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kWave;
    if (base >= B) return;
    const int64_t p = base + lane;
    char* lds = smem[wave];
    float s[8], t[8], g[9], gs[8], gt[8];
    const bool full = base + kWave <= B;
    if (full) {
        dma_slab_issue<kS, NT>(reinterpret_cast<const char*>(src + base * 8), lds, lane);
        dma_slab_issue<kS, NT>(reinterpret_cast<const char*>(tar + base * 8), lds + kS, lane);
        dma_slab_issue<kG, NT>(reinterpret_cast<const char*>(gH + base * 9), lds + 2 * kS, lane);
        dma_wait_sync();
        __builtin_memcpy(s, lds + lane * 32, 32);
        __builtin_memcpy(t, lds + kS + lane * 32, 32);
#pragma unroll
        for (int k = 0; k < 9; ++k) g[k] = reinterpret_cast<const float*>(lds + 2 * kS)[lane * 9 + k];
        wave_lds_sync();  // the staging below reuses the input bytes
    } else {
        if (p >= B) return;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s[k] = src[p * 8 + k];
            t[k] = tar[p * 8 + k];
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) g[k] = gH[p * 9 + k];
    }
    aca_vanilla_grad(s, t, g, gs, gt);
    if (full) {
        if constexpr (WANT_SRC) store_rows_staged<8, NT>(reinterpret_cast<char*>(gsrc + base * 8), gs, lds, lane);
        if constexpr (WANT_TAR) store_rows_staged<8, NT>(reinterpret_cast<char*>(gtar + base * 8), gt, lds, lane);
        return;
    }
    if constexpr (WANT_SRC) {
#pragma unroll
        for (int k = 0; k < 8; ++k) gsrc[p * 8 + k] = gs[k];
    }
    if constexpr (WANT_TAR) {
#pragma unroll
        for (int k = 0; k < 8; ++k) gtar[p * 8 + k] = gt[k];
    }
}

}  // namespace hg
