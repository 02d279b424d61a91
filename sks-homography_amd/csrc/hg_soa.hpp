// hg_soa.hpp -- SoA streaming solver (the reference GPU layout,
// GPU_Runtime Test.cu:87-95 / :141-149: src/tar (8,n), H (9,n)).
//
// A lane owns G groups of V = 16/sizeof(T) consecutive problems and moves each of a
// group's 8 + 8 input and 9 output components as ONE 16-B access, so every
// wave-instruction touches 1 KiB contiguous of one component row.  Needs n % V == 0
// and 16-B aligned bases (else solve_generic runs).  Block b covers groups
// [b*256*G, (b+1)*256*G); PERSIST loops blocks over that range grid-stride.
#pragma once
#include "hg_aos.hpp"

namespace hg {

template <int ALGO, bool NORM, typename T, int G, bool PERSIST, bool NT = true>
__global__ __launch_bounds__(kBlock) void solve_soa_vec(const T* __restrict__ src,
                                                        const T* __restrict__ tar,
                                                        T* __restrict__ H, int64_t n) {
    constexpr int V = 16 / sizeof(T);
    const int64_t groups = n / V;
    const int64_t chunks = (groups + (int64_t)kBlock * G - 1) / ((int64_t)kBlock * G);
    for (int64_t c = blockIdx.x; c < chunks; c += PERSIST ? gridDim.x : chunks) {
        const int64_t q0 = c * kBlock * G + threadIdx.x;
        T s[G][8][V], t[G][8][V];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int64_t q = q0 + (int64_t)g * kBlock;
            if (q < groups) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    u32x4 a = ld16<NT>(src + (int64_t)k * n + q * V);
                    u32x4 b = ld16<NT>(tar + (int64_t)k * n + q * V);
                    __builtin_memcpy(s[g][k], &a, 16);
                    __builtin_memcpy(t[g][k], &b, 16);
                }
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int64_t q = q0 + (int64_t)g * kBlock;
            if (q >= groups) continue;
            T h[V][9];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                T sv[8], tv[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) { sv[k] = s[g][k][v]; tv[k] = t[g][k][v]; }
                solve<ALGO, NORM>(sv, tv, h[v]);
            }
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                T o[V];
#pragma unroll
                for (int v = 0; v < V; ++v) o[v] = h[v][k];
                u32x4 w;
                __builtin_memcpy(&w, o, 16);
                st16<NT>(H + (int64_t)k * n + q * V, w);
            }
        }
    }
}

// Experiment (hg_tune.hip): the AoS kernel's tile form for SoA -- a wave's 64*V problems
// are 16 component-row slabs of 1 KiB each, all landed in LDS by LDS-DMA behind one
// wait, then read per lane from LDS; H rows leave as 1 KiB lane-consecutive stores.
// Needs n % V == 0 and 16-B aligned bases.  The ragged last tile goes per lane.
template <int ALGO, bool NORM, typename T, bool NT>
__global__ __launch_bounds__(kBlock) void solve_soa_dma(const T* __restrict__ src,
                                                        const T* __restrict__ tar,
                                                        T* __restrict__ H, int64_t n) {
    constexpr int V = 16 / sizeof(T);
    constexpr int kTile = kWave * V;
    constexpr int kRow = kWave * 16;
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][16 * kRow];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kTile;
    if (base >= n) return;
    char* lds = smem[wave];
    if (base + kTile <= n) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            dma_slab_issue<kRow, NT>(reinterpret_cast<const char*>(src + (int64_t)k * n + base),
                                     lds + k * kRow, lane);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            dma_slab_issue<kRow, NT>(reinterpret_cast<const char*>(tar + (int64_t)k * n + base),
                                     lds + (8 + k) * kRow, lane);
        dma_wait_sync();
        T s[8][V], t[8][V];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            __builtin_memcpy(s[k], lds + k * kRow + lane * 16, 16);
            __builtin_memcpy(t[k], lds + (8 + k) * kRow + lane * 16, 16);
        }
        T h[V][9];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            T sv[8], tv[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) { sv[k] = s[k][v]; tv[k] = t[k][v]; }
            solve<ALGO, NORM>(sv, tv, h[v]);
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            T o[V];
#pragma unroll
            for (int v = 0; v < V; ++v) o[v] = h[v][k];
            u32x4 w;
            __builtin_memcpy(&w, o, 16);
            st16<NT>(H + (int64_t)k * n + base + lane * V, w);
        }
        return;
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int64_t p = base + lane * V + v;
        if (p < n) {
            T sv[8], tv[8], h[9];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                sv[k] = src[(int64_t)k * n + p];
                tv[k] = tar[(int64_t)k * n + p];
            }
            solve<ALGO, NORM>(sv, tv, h);
#pragma unroll
            for (int k = 0; k < 9; ++k) H[(int64_t)k * n + p] = h[k];
        }
    }
}

// Narrow-access form: a lane owns V = W/sizeof(T) consecutive problems and moves each
// component row with ONE W-byte access (W = 4 / 8), so a wave-instruction touches 64*W
// contiguous bytes of a row.  Fewer live VGPRs than the 16-B form (inputs 16*V dwords'
// worth), hence more waves in flight per SIMD.  n % V == 0 and W-aligned bases.
template <int W, bool NT>
__device__ __forceinline__ void ldw(const void* p, void* dst) {
    if constexpr (W == 4) {
        const unsigned v = NT ? __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(p))
                              : *reinterpret_cast<const unsigned*>(p);
        __builtin_memcpy(dst, &v, 4);
    } else {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 v = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p))
                           : *reinterpret_cast<const u32x2*>(p);
        __builtin_memcpy(dst, &v, 8);
    }
}

template <int W, bool NT>
__device__ __forceinline__ void stw(void* p, const void* src) {
    if constexpr (W == 4) {
        unsigned v;
        __builtin_memcpy(&v, src, 4);
        if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<unsigned*>(p));
        else *reinterpret_cast<unsigned*>(p) = v;
    } else {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        u32x2 v;
        __builtin_memcpy(&v, src, 8);
        if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x2*>(p));
        else *reinterpret_cast<u32x2*>(p) = v;
    }
}

template <int ALGO, bool NORM, typename T, int W, bool NT = true>
__global__ __launch_bounds__(kBlock) void solve_soa_narrow(const T* __restrict__ src,
                                                           const T* __restrict__ tar,
                                                           T* __restrict__ H, int64_t n) {
    constexpr int V = W / sizeof(T);
    static_assert(V >= 1 && V * sizeof(T) == W, "W must be a multiple of sizeof(T)");
    const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q >= n / V) return;
    T s[8][V], t[8][V];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        ldw<W, NT>(src + (int64_t)k * n + q * V, s[k]);
        ldw<W, NT>(tar + (int64_t)k * n + q * V, t[k]);
    }
    T h[V][9];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        T sv[8], tv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { sv[k] = s[k][v]; tv[k] = t[k][v]; }
        solve<ALGO, NORM>(sv, tv, h[v]);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        T o[V];
#pragma unroll
        for (int v = 0; v < V; ++v) o[v] = h[v][k];
        stw<W, NT>(H + (int64_t)k * n + q * V, o);
    }
}

// Block-contiguous row segments: a block of WAVES waves owns a tile of
// SEG bytes of EVERY component row (SEG / sizeof(T) consecutive problems).  The tile's 16
// input-row segments land in LDS by LDS-DMA -- the waves share the 1-KiB pieces -- behind
// one wait and one barrier; each thread then solves SEG / sizeof(T) / (64 WAVES) problems
// (problem j = thread + k * 64 WAVES) reading its components from LDS, and every H row
// segment leaves as SEG contiguous bytes (lane-consecutive stores).  So each row is touched
// in SEG-byte runs instead of the narrow kernel's 512-B wave accesses.  XCD: the blocks one
// XCD runs (the hardware deals block b to XCD b % 8) take one contiguous range of tiles.
// NOSOLVE: the same traffic with H = a copy of the inputs (the pattern's own ceiling).
// One tile per block; 16-B aligned bases; the ragged last tile goes per thread.
template <int ALGO, bool NORM, typename T, int SEG, int WAVES, bool XCD, bool NOSOLVE,
          bool NT = true>
__global__ __launch_bounds__(64 * WAVES) void solve_soa_seg(const T* __restrict__ src,
                                                            const T* __restrict__ tar,
                                                            T* __restrict__ H, int64_t n) {
    constexpr int kThreads = kWave * WAVES;
    constexpr int kTile = SEG / (int)sizeof(T);
    constexpr int kPer = kTile / kThreads;
    constexpr int kPieces = SEG / (16 * kWave);
    static_assert(kTile % kThreads == 0 && SEG % (16 * kWave) == 0, "whole pieces, whole problems");
    __shared__ __attribute__((aligned(16))) char lds[16 * SEG];
    int64_t b = blockIdx.x;
    if constexpr (XCD) {
        const uint32_t G = gridDim.x, per = G / 8, rem = G % 8;
        const uint32_t x = blockIdx.x % 8, k = blockIdx.x / 8;
        b = (int64_t)(x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + k;
    }
    const int64_t base = b * kTile;
    if (base >= n) return;
    if (base + kTile > n) {  // the ragged last tile: per thread, straight from HBM
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int64_t p = base + threadIdx.x + k * kThreads;
            if (p >= n) continue;
            T s[8], t[8], h[9];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                s[r] = src[(int64_t)r * n + p];
                t[r] = tar[(int64_t)r * n + p];
            }
            if constexpr (NOSOLVE) {
#pragma unroll
                for (int r = 0; r < 8; ++r) h[r] = s[r] + t[r];
                h[8] = t[0];
            } else {
                solve<ALGO, NORM>(s, t, h);
            }
#pragma unroll
            for (int r = 0; r < 9; ++r) H[(int64_t)r * n + p] = h[r];
        }
        return;
    }
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
#pragma unroll
    for (int p = wave; p < 16 * kPieces; p += WAVES) {
        const int r = p / kPieces, c = p % kPieces;
        const T* row = (r < 8 ? src + (int64_t)r * n : tar + (int64_t)(r - 8) * n) + base;
        __builtin_amdgcn_global_load_lds(
            (gbl_ptr_t)(reinterpret_cast<const char*>(row) + 16 * (c * kWave + lane)),
            (lds_ptr_t)(lds + r * SEG + 16 * c * kWave), 16, 0, NT ? 2 : 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int j = threadIdx.x + k * kThreads;
        T s[8], t[8], h[9];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            s[r] = reinterpret_cast<const T*>(lds + r * SEG)[j];
            t[r] = reinterpret_cast<const T*>(lds + (8 + r) * SEG)[j];
        }
        if constexpr (NOSOLVE) {
#pragma unroll
            for (int r = 0; r < 8; ++r) h[r] = s[r] + t[r];
            h[8] = t[0];
        } else {
            solve<ALGO, NORM>(s, t, h);
        }
#pragma unroll
        for (int r = 0; r < 9; ++r) {
            T* dst = H + (int64_t)r * n + base + j;
            if constexpr (NT) __builtin_nontemporal_store(h[r], dst);
            else *dst = h[r];
        }
    }
}

template <int G, bool PERSIST>
inline int64_t soa_grid(int64_t groups, int per_cu = 8) {
    const int64_t chunks = (groups + (int64_t)kBlock * G - 1) / ((int64_t)kBlock * G);
    if (PERSIST) return chunks < 256LL * per_cu ? chunks : 256LL * per_cu;
    return chunks > 0 ? chunks : 1;
}

}  // namespace hg
