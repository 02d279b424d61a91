// hg_aos.hpp -- the AoS streaming solver kernel (the headline path) and its
// memory helpers.  One template covers the shipped configuration and the variants
// tools/kbench.py sweeps (hg_tune.hip); see DESIGN.md "Kernel variants".
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hg_solvers.hpp"

namespace hg {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

// AoS kernel option bits (template parameter FL)
enum : int {
    kNtLoad = 1,     // non-temporal (streaming) global loads
    kNtStore = 2,    // non-temporal global stores
    kLdsLoad = 4,    // stage inputs through LDS: each load instruction reads 1 KiB contiguous
    kDirectSt = 8,   // store H rows per lane (9 x 4-B stores) instead of LDS-staged 16-B stores
    kPersist = 16,   // persistent grid: blocks loop over tiles
    kLdsDma = 32,    // with kLdsLoad: global_load_lds_dwordx4 (LDS-DMA, no VGPR staging)
    kXcdMap = 64,    // one-shot grid: each XCD's blocks take one contiguous range of tiles
    kStSc1 = 128,    // staged H stores as buffer stores with sc1 (| nt with kNtStore); tune only
    kLdSc0 = 256,    // LDS-DMA input loads with sc0 added to their cache policy; tune only
    kLdSc1 = 512,    // ... with sc1 added; tune only
    kSlabMajor = 1024,  // issue all of src's DMA pieces, then all of tar's (not interleaved); tune only
    kNoSolve = 2048,    // same loads and stores, no solver: H row = src row + tar[0] (the memory
                        // pattern's own ceiling); tune only
};

// The solve of one problem, or -- with kNoSolve -- a copy with the same traffic and a
// dependence on every loaded value (tune-only yardstick).
template <int ALGO, bool NORM, int FL, typename T>
__device__ __forceinline__ void tile_solve(const T (&s)[8], const T (&t)[8], T (&h)[9]) {
    if constexpr ((FL & kNoSolve) != 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = s[k] + t[k];
        h[8] = t[0];
    } else {
        solve<ALGO, NORM>(s, t, h);
    }
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) const void* gbl_ptr_t;

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const void* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
}

template <bool NT>
__device__ __forceinline__ void st16(void* p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else *reinterpret_cast<u32x4*>(p) = v;
}

// Read 8 T's (one problem's point row) with 16-B loads.
template <typename T, bool NT>
__device__ __forceinline__ void load_row8(const T* p, T (&v)[8]) {
    constexpr int kChunks = 8 * sizeof(T) / 16;
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
        u32x4 w = ld16<NT>(reinterpret_cast<const char*>(p) + 16 * c);
        __builtin_memcpy(reinterpret_cast<char*>(v) + 16 * c, &w, 16);
    }
}

// splitmix64 finaliser: the counter-based generator shared (bit for bit) with the
// host-side regeneration in oracle/hg_oracle.c.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Copies NS contiguous slabs of kBytes each (a multiple of 1 KiB) from global
// memory into this wave's LDS, every wave-instruction moving 1 KiB (64 lanes x 16 B);
// all loads of all slabs are issued before the single wait.  DMA: global_load_lds
// _dwordx4 (no VGPR round trip); else global_load_dwordx4 + ds_write_b128.
// Ends with the slabs visible to every lane of the wave.
// AUXX: extra cache-policy bits for the DMA (gfx950: sc0 = 1, nt = 2, sc1 = 16); SLAB_MAJOR:
// issue slab 0's pieces, then slab 1's, instead of interleaving them piece by piece.
template <int kBytes, int NS, bool DMA, bool NT, int AUXX = 0, bool SLAB_MAJOR = false>
__device__ __forceinline__ void slabs_to_lds(const char* const (&g)[NS], char* const (&l)[NS],
                                             int lane) {
    static_assert(kBytes % (16 * kWave) == 0, "slab must be whole 1 KiB pieces");
    constexpr int kPieces = kBytes / (16 * kWave);
    constexpr int kAux = (NT ? 2 : 0) | AUXX;
    if constexpr (DMA) {
        if constexpr (SLAB_MAJOR) {
#pragma unroll
            for (int s = 0; s < NS; ++s)
#pragma unroll
                for (int c = 0; c < kPieces; ++c)
                    __builtin_amdgcn_global_load_lds((gbl_ptr_t)(g[s] + 16 * (c * kWave + lane)),
                                                     (lds_ptr_t)(l[s] + 16 * c * kWave), 16, 0, kAux);
        } else {
#pragma unroll
            for (int c = 0; c < kPieces; ++c)
#pragma unroll
                for (int s = 0; s < NS; ++s)
                    __builtin_amdgcn_global_load_lds((gbl_ptr_t)(g[s] + 16 * (c * kWave + lane)),
                                                     (lds_ptr_t)(l[s] + 16 * c * kWave), 16, 0, kAux);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        u32x4 v[NS][kPieces];
#pragma unroll
        for (int c = 0; c < kPieces; ++c)
#pragma unroll
            for (int s = 0; s < NS; ++s) v[s][c] = ld16<NT>(g[s] + 16 * (c * kWave + lane));
#pragma unroll
        for (int c = 0; c < kPieces; ++c)
#pragma unroll
            for (int s = 0; s < NS; ++s)
                *reinterpret_cast<u32x4*>(l[s] + 16 * (c * kWave + lane)) = v[s][c];
    }
    wave_lds_sync();
}

// Issue-only LDS-DMA of one kBytes slab (no wait): for slabs of different sizes,
// issue each, then call dma_wait_sync() once.  A last piece under 1 KiB is issued by
// the lanes it covers only.
template <int kBytes, bool NT>
__device__ __forceinline__ void dma_slab_issue(const char* __restrict__ g, char* l, int lane) {
    static_assert(kBytes % 16 == 0, "slab must be whole 16-B granules");
    constexpr int kWhole = kBytes / (16 * kWave), kTail = (kBytes % (16 * kWave)) / 16;
#pragma unroll
    for (int c = 0; c < kWhole; ++c)
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)(g + 16 * (c * kWave + lane)),
                                         (lds_ptr_t)(l + 16 * c * kWave), 16, 0, NT ? 2 : 0);
    if constexpr (kTail > 0) {
        if (lane < kTail)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(g + 16 * (kWhole * kWave + lane)),
                                             (lds_ptr_t)(l + 16 * kWhole * kWave), 16, 0,
                                             NT ? 2 : 0);
    }
}

// The same issue through inline asm (cdna_hip_programming.md section 5.7): hipcc then
// does not see LDS writes in flight, so it inserts no `s_waitcnt vmcnt(0)` before
// later ds_reads -- the caller's counted `s_waitcnt vmcnt(N)` alone orders them.
// Needed to keep a next tile's DMA in flight while the current tile is read.
template <int kBytes, bool NT>
__device__ __forceinline__ void dma_slab_issue_asm(const char* __restrict__ g, char* l, int lane) {
    static_assert(kBytes % (16 * kWave) == 0, "slab must be whole 1 KiB pieces");
    const uint32_t lbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)l);
#pragma unroll
    for (int c = 0; c < kBytes / (16 * kWave); ++c) {
        const char* gp = g + 16 * (c * kWave + lane);
        uint32_t keep;
        if constexpr (NT)
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(gp), "s"(lbase + 1024u * c) : "memory");
        else
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(gp), "s"(lbase + 1024u * c) : "memory");
    }
}

__device__ __forceinline__ void dma_wait_sync() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_lds_sync();
}

// Writes a wave's 64*P rows of 9 T (36/72-B rows, not 16-B aligned per lane) to
// the contiguous slab `out`: rows are staged in LDS at a 9-element stride (odd dword
// stride: conflict-free ds_write_b32), then every lane stores consecutive 16-B chunks.
// This wave's 64 rows of kFloats floats (row l = lane l's `v`) leave as ONE contiguous
// slab: 16-B ds_writes of each row into LDS, then lane-consecutive 16-B global stores.
// kFloats % 4 == 0 (32-B and 48-B rows: the backward's gradient records).
template <int kFloats, bool NT>
__device__ __forceinline__ void store_rows_staged(char* __restrict__ out, const float (&v)[kFloats],
                                                  char* lds, int lane) {
    static_assert(kFloats % 4 == 0, "rows of whole 16-B granules");
#pragma unroll
    for (int c = 0; c < kFloats / 4; ++c)
        __builtin_memcpy(lds + (lane * kFloats + 4 * c) * 4, &v[4 * c], 16);
    wave_lds_sync();
    constexpr int kChunks = kWave * kFloats / 4;
#pragma unroll
    for (int c = 0; c < kChunks / kWave; ++c) {
        const int chunk = c * kWave + lane;
        st16<NT>(out + 16 * chunk, *reinterpret_cast<const u32x4*>(lds + 16 * chunk));
    }
    wave_lds_sync();
}

template <typename T, int P, bool NT, bool SC1 = false>
__device__ __forceinline__ void store_rows9_staged(char* __restrict__ out, const T (&h)[P][9],
                                                   char* lds, int lane) {
    T* st = reinterpret_cast<T*>(lds);
#pragma unroll
    for (int j = 0; j < P; ++j)
#pragma unroll
        for (int k = 0; k < 9; ++k) st[(j * kWave + lane) * 9 + k] = h[j][k];
    wave_lds_sync();
    constexpr int kChunks = kWave * P * 9 * (int)sizeof(T) / 16;  // 144*P*sizeof(T)/4
    constexpr int kIters = (kChunks + kWave - 1) / kWave;
#pragma unroll
    for (int c = 0; c < kIters; ++c) {
        const int chunk = c * kWave + lane;
        if (kChunks % kWave == 0 || chunk < kChunks) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(lds + 16 * chunk);
            if constexpr (SC1) {
                const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, kChunks * 16, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, 16 * chunk, 0, NT ? 18 : 16);
            } else {
                st16<NT>(out + 16 * chunk, v);
            }
        }
    }
    wave_lds_sync();  // the caller may rewrite the staging bytes next
}

template <typename T, int P, int FL>
struct AosSmem {
    static constexpr int kTile = kWave * P;                     // problems per wave
    static constexpr int kOutBytes = kTile * 9 * (int)sizeof(T);
    static constexpr int kInBytes = (FL & kLdsLoad) ? 2 * kTile * 8 * (int)sizeof(T) : 0;
    static constexpr int kBytes = (FL & kDirectSt) && !(FL & kLdsLoad) ? 16
                                  : (kInBytes > kOutBytes ? kInBytes : kOutBytes);
};

// One wave solves problems [base, base + 64*P): lane l owns base + j*64 + l.
template <int ALGO, bool NORM, typename T, int P, int FL>
__device__ __forceinline__ void aos_wave_tile(const T* __restrict__ src, const T* __restrict__ tar,
                                              T* __restrict__ H, int64_t n, int64_t base,
                                              char* lds, int lane) {
    constexpr bool NTL = FL & kNtLoad, NTS = FL & kNtStore;
    constexpr int kTile = kWave * P;
    const bool full = base + kTile <= n;

    T h[P][9];
    if ((FL & kLdsLoad) && full) {
        // each instruction: 64 lanes x 16 B contiguous; slab = kTile rows of 8 T
        constexpr int kSlab = kTile * 8 * (int)sizeof(T);   // bytes per operand
        const char* gs = reinterpret_cast<const char*>(src + base * 8);
        const char* gt = reinterpret_cast<const char*>(tar + base * 8);
        const char* const gsrc[2] = {gs, gt};
        char* const lsrc[2] = {lds, lds + kSlab};
        constexpr int kAuxx = ((FL & kLdSc0) ? 1 : 0) | ((FL & kLdSc1) ? 16 : 0);
        slabs_to_lds<kSlab, 2, (FL & kLdsDma) != 0, NTL, kAuxx, (FL & kSlabMajor) != 0>(gsrc, lsrc,
                                                                                         lane);
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int row = j * kWave + lane;
            T s[8], t[8];
            __builtin_memcpy(s, lds + row * 8 * sizeof(T), 8 * sizeof(T));
            __builtin_memcpy(t, lds + kSlab + row * 8 * sizeof(T), 8 * sizeof(T));
            tile_solve<ALGO, NORM, FL>(s, t, h[j]);
        }
        wave_lds_sync();  // the output staging below reuses these bytes
    } else {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int64_t p = base + j * kWave + lane;
            T s[8], t[8];
            if (full || p < n) {
                load_row8<T, NTL>(src + p * 8, s);
                load_row8<T, NTL>(tar + p * 8, t);
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) s[k] = t[k] = T(0);
            }
            tile_solve<ALGO, NORM, FL>(s, t, h[j]);
        }
    }

    bool staged = false;
    if constexpr (!(FL & kDirectSt)) {
      if (full) {
        staged = true;
        store_rows9_staged<T, P, NTS, (FL & kStSc1) != 0>(reinterpret_cast<char*>(H + base * 9), h,
                                                          lds, lane);
      }
    }
    if (!staged) {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int64_t p = base + j * kWave + lane;
            if (full || p < n) {
#pragma unroll
                for (int k = 0; k < 9; ++k) {
                    if constexpr (NTS) __builtin_nontemporal_store(h[j][k], H + p * 9 + k);
                    else H[p * 9 + k] = h[j][k];
                }
            }
        }
    }
}

// AoS vector kernel: src/tar (n,8), H (n,9); all three 16-B aligned.
// Block b's wave w owns tile (4b + w) (or loops over tiles with kPersist).
template <int ALGO, bool NORM, typename T, int P, int FL>
__global__ __launch_bounds__(kBlock) void solve_aos(const T* __restrict__ src,
                                                    const T* __restrict__ tar,
                                                    T* __restrict__ H, int64_t n) {
    using S = AosSmem<T, P, FL>;
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][S::kBytes];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t tiles = (n + S::kTile - 1) / S::kTile;
    if constexpr (FL & kPersist) {
        for (int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + wave; t < tiles;
             t += (int64_t)gridDim.x * kWavesPerBlock)
            aos_wave_tile<ALGO, NORM, T, P, FL>(src, tar, H, n, t * S::kTile, smem[wave], lane);
    } else {
        int64_t b = blockIdx.x;
        if constexpr (FL & kXcdMap) {
            // blocks are dispatched to the 8 XCDs round-robin (b % 8); renumber so that
            // XCD x's blocks cover one contiguous slice of the batch
            const uint32_t G = gridDim.x, per = G / 8, rem = G % 8;
            const uint32_t x = blockIdx.x % 8, k = blockIdx.x / 8;
            b = (int64_t)(x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + k;
        }
        const int64_t t = b * kWavesPerBlock + wave;
        if (t < tiles)
            aos_wave_tile<ALGO, NORM, T, P, FL>(src, tar, H, n, t * S::kTile, smem[wave], lane);
    }
}

// Pipelined AoS kernel (experiment, hg_tune.hip): each wave walks TPW consecutive
// full tiles with a 2-deep LDS ring -- the LDS-DMA of tile i+1 is in flight while
// tile i is solved and stored; a counted `s_waitcnt vmcnt(N)` (N = the next tile's
// DMA instructions) retires tile i only.  The ragged tail tile takes the per-lane path.
template <int ALGO, bool NORM, int P, int TPW>
__global__ __launch_bounds__(kBlock) void solve_aos_pipe(const float* __restrict__ src,
                                                         const float* __restrict__ tar,
                                                         float* __restrict__ H, int64_t n) {
    constexpr int kTile = kWave * P;
    constexpr int kSlab = kTile * 32;               // bytes per operand per tile
    constexpr int kPieces = kSlab / (16 * kWave);   // DMA instructions per operand
    constexpr int kBuf = 2 * kSlab;
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][2 * kBuf];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t full_tiles = n / kTile;
    const int64_t t0 = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * TPW;
    char* ring = smem[wave];
    auto issue = [&](int64_t t, char* buf) {
        dma_slab_issue_asm<kSlab, true>(reinterpret_cast<const char*>(src + t * kTile * 8), buf,
                                        lane);
        dma_slab_issue_asm<kSlab, true>(reinterpret_cast<const char*>(tar + t * kTile * 8),
                                        buf + kSlab, lane);
    };
    const int64_t cnt = full_tiles - t0 < TPW ? full_tiles - t0 : TPW;
    if (cnt > 0) {
        issue(t0, ring);
        for (int i = 0; i < cnt; ++i) {
            char* cur = ring + (i & 1) * kBuf;
            if (i + 1 < cnt) {
                issue(t0 + i + 1, ring + ((i + 1) & 1) * kBuf);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kPieces) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            wave_lds_sync();
            float h[P][9];
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int row = j * kWave + lane;
                float s[8], t[8];
                __builtin_memcpy(s, cur + row * 32, 32);
                __builtin_memcpy(t, cur + kSlab + row * 32, 32);
                solve<ALGO, NORM>(s, t, h[j]);
            }
            wave_lds_sync();
            store_rows9_staged<float, P, true>(reinterpret_cast<char*>(H + (t0 + i) * kTile * 9),
                                               h, cur, lane);
        }
    }
    // the ragged tail tile belongs to the wave whose range holds tile index full_tiles
    if (n % kTile && t0 <= full_tiles && full_tiles < t0 + TPW)
        aos_wave_tile<ALGO, NORM, float, P, kNtLoad | kNtStore | kDirectSt>(
            src, tar, H, n, full_tiles * kTile, ring, lane);
}

// Grid for solve_aos: one block per 4 tiles, or a persistent grid of `per_cu`
// blocks on each of the 256 CUs.
template <typename T, int P, int FL>
inline int64_t aos_grid(int64_t n, int per_cu = 8) {
    const int64_t tile = (int64_t)kWave * P;
    const int64_t blocks = ((n + tile - 1) / tile + kWavesPerBlock - 1) / kWavesPerBlock;
    if constexpr (FL & kPersist) {
        const int64_t cap = 256LL * per_cu;
        return blocks < cap ? blocks : cap;
    }
    return blocks;
}

}  // namespace hg
