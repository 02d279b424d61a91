// hg_ransac.hpp -- RANSAC kernels: counter draws, the fused sampler +
// solver (global-gather and LDS-pool forms), the inlier scorers, and the sampler's host
// launcher.  Included by hg_ransac.hip (the C ABI) and hg_tune.hip (variant sweeps).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <utility>
#include <vector>

#include "hg_aos.hpp"
#include "hg_launch.hpp"
#include "hg_solvers.hpp"
#include "sks_homography.h"

#pragma clang fp contract(off)

namespace hg {

constexpr uint64_t kBitsMul = 0xA0761D6478BD642Full;

typedef int i32x2 __attribute__((ext_vector_type(2)));

// Word w of stream S = seed * kBitsMul is one half of the splitmix64 finaliser of counter
// S + w/2: the high 32 bits for even w, the low 32 for odd w -- one 64-bit hash per two
// draws (each finaliser costs six quarter-rate 32-bit multiplies; taking both halves
// halved the seeded sampler's hashing, tools/kbench_sample.py).  Restated in
// oracle/hg_oracle.c.
__device__ __forceinline__ uint32_t word_half(uint64_t z, bool lo) {
    return lo ? (uint32_t)z : (uint32_t)(z >> 32);
}

// out[i] = word(offset + i).  Thread t owns the hash of counter S + (offset >> 1) + t, i.e.
// words 2j, 2j + 1 of the stream; the pair lands in out[2t - (offset & 1)] and the next.
static __global__ __launch_bounds__(kBlock) void fill_bits_kernel(uint32_t* __restrict__ out,
                                                           int64_t count, uint64_t seed,
                                                           uint64_t offset) {
    const uint64_t base = seed * kBitsMul + (offset >> 1);
    const int64_t odd = (int64_t)(offset & 1);
    const int64_t pairs = (count + odd + 1) >> 1;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const bool vec = odd == 0 && (reinterpret_cast<uintptr_t>(out) & 7u) == 0;
    for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < pairs; t += stride) {
        const uint64_t z = mix64(base + (uint64_t)t);
        const int64_t i = 2 * t - odd;  // out index of word 2j (may be -1 when odd)
        if (vec && i + 1 < count) {
            *reinterpret_cast<uint2*>(out + i) = make_uint2(word_half(z, false), word_half(z, true));
        } else {
            if (i >= 0 && i < count) out[i] = word_half(z, false);
            if (i + 1 < count) out[i + 1] = word_half(z, true);
        }
    }
}

// How a lane's two paired hypotheses divide (PAIR; 0 = one hypothesis at a time): both
// solve as the halves of packed f32x2 values, and their divisions either split into two
// scalar expansions (kPairScalarDiv, the round-2 form, tune only) or run as one expansion
// whose FMA steps are packed too (kPairPacked, shipped; div_rn in hg_solvers.hpp).
constexpr int kPairScalarDiv = 1;
constexpr int kPairPacked = 2;

// Where a hypothesis' four draws come from.
constexpr int kDrawsIndexed = 0;  // row p of the (n,4) index array
constexpr int kDrawsPaired = 1;   // seeded: fill_bits' stream generated in place (shipped)
constexpr int kDrawsSingle = 2;   // seeded, tune only: one hash per draw (the earlier stream)
constexpr int kDrawsCheap = 3;    // tune ablation only: multiply-free scrambles of p (not a stream)

// The 4 draws of hypothesis p: row p of the (n,4) index array, or -- seeded -- the same
// four words generated in place: words offset + 4p ... + 3 of the stream, i.e. out[4p ..
// 4p+3] of fill_bits_kernel (so a seeded launch equals fill_bits + an indexed one, bit for
// bit, without the 16 B per hypothesis of index traffic).  bits_base = S + (offset >> 1);
// an odd offset shifts the four words across three hashes (a wave-uniform branch).
template <int DRAWS>
__device__ __forceinline__ u32x4 draws4(const uint4* idx, uint64_t bits_base, bool odd, int64_t p) {
    if constexpr (DRAWS == kDrawsPaired) {
        const uint64_t b = bits_base + 2 * (uint64_t)p;
        const uint64_t z0 = mix64(b), z1 = mix64(b + 1);
        if (!odd)
            return u32x4{word_half(z0, false), word_half(z0, true), word_half(z1, false),
                         word_half(z1, true)};
        const uint64_t z2 = mix64(b + 2);
        return u32x4{word_half(z0, true), word_half(z1, false), word_half(z1, true),
                     word_half(z2, false)};
    } else if constexpr (DRAWS == kDrawsCheap) {
        const uint32_t x = (uint32_t)p ^ (uint32_t)bits_base;
        const uint32_t a = x ^ (x << 13), b = a ^ (a >> 17), c = b ^ (b << 5);
        return u32x4{a, b, c, c ^ (c >> 11)};
    } else if constexpr (DRAWS == kDrawsSingle) {
        const uint64_t b = bits_base + 4 * (uint64_t)p;
        return u32x4{(uint32_t)(mix64(b) >> 32), (uint32_t)(mix64(b + 1) >> 32),
                     (uint32_t)(mix64(b + 2) >> 32), (uint32_t)(mix64(b + 3) >> 32)};
    } else {
        return ld16<true>(reinterpret_cast<const char*>(idx + p));
    }
}

// Fused sampler + solver.  A wave owns 64*P hypotheses: its 16-B index rows arrive by
// LDS-DMA (P = 2: 2 KiB), each lane gathers its 4 correspondences from the pool
// (npool x 8 B per side: L2/L1-resident), solves, and the H rows leave through the
// LDS-staged 16-B stores.  Index r of a row selects pool[r % npool], as get_rand_list
// does (.cu:56-59, modulo bias and duplicates included).
template <int ALGO, bool NORM, int P, int DRAWS = kDrawsIndexed, int PAIR = 0>
__global__ __launch_bounds__(kBlock) void sample_solve_kernel(
    const float2* __restrict__ pool_src, const float2* __restrict__ pool_tar, uint32_t npool,
    const uint4* __restrict__ idx, float* __restrict__ H, int64_t n, uint64_t bits_base = 0,
    uint32_t bits_odd = 0) {
    constexpr int kTile = kWave * P;
    constexpr int kIdx = kTile * 16;
    constexpr int kLds = kIdx > kTile * 36 ? kIdx : kTile * 36;
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][kLds];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kTile;
    if (base >= n) return;
    char* lds = smem[wave];
    const bool full = base + kTile <= n;
    uint4 r[P];
    if constexpr (DRAWS != kDrawsIndexed) {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const u32x4 d = draws4<DRAWS>(nullptr, bits_base, bits_odd != 0, base + j * kWave + lane);
            r[j] = make_uint4(d[0], d[1], d[2], d[3]);
        }
    } else if (full) {
        dma_slab_issue<kIdx, true>(reinterpret_cast<const char*>(idx + base), lds, lane);
        dma_wait_sync();
#pragma unroll
        for (int j = 0; j < P; ++j) r[j] = *reinterpret_cast<const uint4*>(lds + (j * kWave + lane) * 16);
        wave_lds_sync();
    } else {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int64_t p = base + j * kWave + lane;
            r[j] = p < n ? idx[p] : make_uint4(0, 0, 0, 0);
        }
    }
    float h[P][9];
    if constexpr (PAIR) {  // as sample_solve_lds_kernel's PAIR: packed f32x2 pairs
        static_assert(P % 2 == 0, "paired solve takes hypotheses two at a time");
#pragma unroll
        for (int j = 0; j < P; j += 2) {
            f32x2 s[8], t[8], hp[9];
            const uint32_t ra[4] = {r[j].x, r[j].y, r[j].z, r[j].w};
            const uint32_t rb[4] = {r[j + 1].x, r[j + 1].y, r[j + 1].z, r[j + 1].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t ia = ra[k] % npool, ib = rb[k] % npool;
                const float2 as = pool_src[ia], at = pool_tar[ia];
                const float2 bs = pool_src[ib], bt = pool_tar[ib];
                s[2 * k] = f32x2{as.x, bs.x}; s[2 * k + 1] = f32x2{as.y, bs.y};
                t[2 * k] = f32x2{at.x, bt.x}; t[2 * k + 1] = f32x2{at.y, bt.y};
            }
            solve<ALGO, NORM, PAIR == kPairPacked>(s, t, hp);
#pragma unroll
            for (int k = 0; k < 9; ++k) { h[j][k] = hp[k].x; h[j + 1][k] = hp[k].y; }
        }
    } else {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const uint32_t id[4] = {r[j].x % npool, r[j].y % npool, r[j].z % npool, r[j].w % npool};
            float s[8], t[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float2 a = pool_src[id[k]], b = pool_tar[id[k]];
                s[2 * k] = a.x; s[2 * k + 1] = a.y;
                t[2 * k] = b.x; t[2 * k + 1] = b.y;
            }
            solve<ALGO, NORM>(s, t, h[j]);
        }
    }
    if (full) {
        store_rows9_staged<float, P, true>(reinterpret_cast<char*>(H + base * 9), h, lds, lane);
        return;
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int64_t p = base + j * kWave + lane;
        if (p < n) {
#pragma unroll
            for (int k = 0; k < 9; ++k) H[p * 9 + k] = h[j][k];
        }
    }
}

// r mod d for every 32-bit r and d >= 1 with one high and one low 32-bit multiply:
// division by an invariant integer in the round-up form with a 33-bit multiplier
// (Granlund & Montgomery, PLDI 1994; Robison, ARITH 2005): for d = 2^l + x (0 < x < 2^l),
// M = floor(2^(33+l) / d) + 1 exceeds 2^32, so with m = M - 2^32 and hi = umulhi(r, m),
// floor(r M / 2^(33+l)) = (((r - hi) >> 1) + hi) >> l exactly for every r < 2^32
// (M d - 2^(33+l) <= d < 2^(l+1)).  Powers of two use m = 0 and shift l - 1; d = 1
// and d = 2 share m = 0, shift 0, and the min() clamps d = 1's remainder to 0 (a no-op
// for every other d).  Host side packs (shift << 32) | m.
__device__ __forceinline__ uint32_t fastmod_u32(uint32_t r, uint64_t packed, uint32_t d) {
    const uint32_t m = (uint32_t)packed, sh = (uint32_t)(packed >> 32);
    const uint32_t hi = __umulhi(r, m);
    const uint32_t q = (((r - hi) >> 1) + hi) >> sh;
    const uint32_t rem = r - q * d;
    return rem < d - 1 ? rem : d - 1;
}

inline uint64_t fastmod_magic(uint32_t d) {
    if (d <= 2) return 0;
    const uint32_t l = 31u - (uint32_t)__builtin_clz(d);
    if ((d & (d - 1)) == 0) return (uint64_t)(l - 1) << 32;
    const unsigned __int128 M = (((unsigned __int128)1) << (33 + l)) / d + 1;
    return ((uint64_t)l << 32) | (uint64_t)(uint32_t)(M - ((unsigned __int128)1 << 32));
}

// The alternative measured against it (tools/kbench_sample.py): Lemire, Kaser & Kurz,
// "Faster remainder by direct computation" (2019) -- M = floor((2^64 - 1) / d) + 1,
// r mod d = umulhi64(M r mod 2^64, d): five multiplies, a shorter dependency chain.
__device__ __forceinline__ uint32_t fastmod64_u32(uint32_t r, uint64_t M, uint32_t d) {
    return (uint32_t)__umul64hi(M * (uint64_t)r, (uint64_t)d);
}

inline uint64_t fastmod64_magic(uint32_t d) { return ~0ull / d + 1; }

// A third exact form, all full-rate binary64 (tools/kbench_sample.py): with u = the
// smallest double >= 1/d, q = trunc(RN(r u)) is floor(r/d) or one more (r u >= r/d, and
// the two roundings add < 2^-19 for r < 2^32), r - q d is exact in one FMA (every value
// an integer < 2^33), and a negative remainder takes d back.  Host side: the bits of u.
// Valid for d < 2^31 (the remainder passes through int32): the LDS pools are < 10^4.
__device__ __forceinline__ uint32_t fmod_f64_u32(uint32_t r, uint64_t inv_bits, uint32_t d) {
    const double x = (double)r;
    const double q = __builtin_trunc(x * __builtin_bit_cast(double, inv_bits));
    const int32_t rem = (int32_t)__builtin_fma(-q, (double)d, x);
    return (uint32_t)(rem < 0 ? rem + (int32_t)d : rem);
}

inline uint64_t fmod_f64_magic(uint32_t d) {
    double u = 1.0 / (double)d;
    if (__builtin_fma(u, (double)d, -1.0) < 0.0) u = __builtin_nextafter(u, 2.0);
    uint64_t bits;
    __builtin_memcpy(&bits, &u, sizeof bits);
    return bits;
}

// The binary64 form without a correction (round 6; the Table-8 kernel's mrg::step_index):
// q = trunc(RN(r u + u/2)) is floor(r/d) exactly -- (r + 1/2)/d lies 1/(2d) from every
// integer, the product errs by < 2^-19/d -- so r - q d (one exact FMA) is the remainder, for
// every d < 2^32.  Same magic as fmod_f64_u32.
__device__ __forceinline__ uint32_t fmod_f64_exact_u32(uint32_t r, uint64_t inv_bits, uint32_t d) {
    const double w = (double)r, u = __builtin_bit_cast(double, inv_bits);
    const double q = __builtin_trunc(__builtin_fma(w, u, 0.5 * u));
    return (uint32_t)__builtin_fma(-q, (double)d, w);
}

// Remainder forms: 0 fastmod_u32 (shipped), 1 fastmod64_u32, 2 fmod_f64_u32, 4
// fmod_f64_exact_u32; 3 (tune ablation only, wrong indices) r & 1023 clamped to the pool -- the
// loop without a remainder.
template <int RED>
__device__ __forceinline__ uint32_t reduce_index(uint32_t r, uint64_t magic, uint32_t d) {
    if constexpr (RED == 1) return fastmod64_u32(r, magic, d);
    else if constexpr (RED == 2) return fmod_f64_u32(r, magic, d);
    else if constexpr (RED == 4) return fmod_f64_exact_u32(r, magic, d);
    else if constexpr (RED == 3) return (r & 1023u) < d ? (r & 1023u) : 0u;
    else return fastmod_u32(r, magic, d);
}

template <int RED>
inline uint64_t reduce_magic(uint32_t d) {
    if constexpr (RED == 1) return fastmod64_magic(d);
    else if constexpr (RED == 2 || RED == 4) return fmod_f64_magic(d);
    else return fastmod_magic(d);
}

// The same sampler with the pool staged in LDS once per block: {x, y, u, v} 16-B
// records, so a hypothesis gathers with 4 ds_read_b128 instead of 8 scattered global
// loads through the texture path (the bound of sample_solve_kernel: 47 G hyp/s, 30 % of
// HBM).  Persistent grid sized to the resident blocks; each wave walks its tiles with
// the next tile's index rows already in flight (per-lane 16-B loads, lane-consecutive),
// and the H rows leave through the LDS-staged 16-B stores.  Requires the pool plus the
// staging to fit the block's LDS (checked on the host).
// PAIR (P even): hypotheses j and j+1 of a lane are solved together as the two halves of
// packed f32x2 values, so each v_pk_mul_f32 / v_pk_add_f32 does the same IEEE operation
// for both (the values of two scalar solves; only a NaN's sign may differ, since a packed
// subtraction is an add with a negate modifier); the divisions stay scalar per half.
// STP (tune only): the H stores' cache policy -- 0 non-temporal (shipped), 1 default,
// 2 sc1 buffer stores, 3 sc1|nt buffer stores.
template <int ALGO, bool NORM, int P, int PF = 1, int WPB = kWavesPerBlock,
          int DRAWS = kDrawsIndexed, int RED = 0, int PAIR = 0, int STP = 0>
__global__ __launch_bounds__(WPB * kWave) void sample_solve_lds_kernel(
    const float2* __restrict__ pool_src, const float2* __restrict__ pool_tar, uint32_t npool,
    uint64_t magic, const uint4* __restrict__ idx, float* __restrict__ H, int64_t n,
    uint64_t bits_base = 0, uint32_t bits_odd = 0) {
    constexpr int kTile = kWave * P;
    constexpr int kStage = kTile * 36;
    extern __shared__ __attribute__((aligned(16))) char dyn[];
    float4* pool = reinterpret_cast<float4*>(dyn);
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    char* stage = dyn + (size_t)npool * 16 + (size_t)wave * kStage;
    for (uint32_t i = threadIdx.x; i < npool; i += WPB * kWave) {
        const float2 a = pool_src[i], b = pool_tar[i];
        pool[i] = make_float4(a.x, a.y, b.x, b.y);
    }
    __syncthreads();

    const int64_t tiles = (n + kTile - 1) / kTile;
    const int64_t stride = (int64_t)gridDim.x * WPB;
    int64_t t = (int64_t)blockIdx.x * WPB + wave;
    auto load = [&](int64_t tile, u32x4 (&r)[P]) {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int64_t p = tile * kTile + j * kWave + lane;
            // generated draws need no bound: past n they feed rows that are never stored
            r[j] = (DRAWS != kDrawsIndexed || p < n) ? draws4<DRAWS>(idx, bits_base, bits_odd != 0, p)
                                                     : u32x4{0, 0, 0, 0};
        }
    };
    // index rows of the next PF tiles stay in flight while this tile is solved; PF = 0
    // makes each tile's draws where they are used (nothing to hide when they are computed)
    static_assert(PF >= 0 && PF <= 2, "prefetch depth 0, 1 or 2");
    u32x4 cur[P], ahead[P]{};
    if (PF > 0 && t < tiles) load(t, cur);
    if (PF == 2 && t + stride < tiles) load(t + stride, ahead);
    for (; t < tiles; t += stride) {
        u32x4 nxt[P]{};
        if constexpr (PF == 0) load(t, cur);
        else if (t + PF * stride < tiles) load(t + PF * stride, nxt);
        float h[P][9];
        if constexpr (PAIR) {
            static_assert(P % 2 == 0, "paired solve takes hypotheses two at a time");
#pragma unroll
            for (int j = 0; j < P; j += 2) {
                f32x2 s[8], tt[8], hp[9];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float4 a = pool[reduce_index<RED>(cur[j][k], magic, npool)];
                    const float4 b = pool[reduce_index<RED>(cur[j + 1][k], magic, npool)];
                    s[2 * k] = f32x2{a.x, b.x}; s[2 * k + 1] = f32x2{a.y, b.y};
                    tt[2 * k] = f32x2{a.z, b.z}; tt[2 * k + 1] = f32x2{a.w, b.w};
                }
                solve<ALGO, NORM, PAIR == kPairPacked>(s, tt, hp);
#pragma unroll
                for (int k = 0; k < 9; ++k) { h[j][k] = hp[k].x; h[j + 1][k] = hp[k].y; }
            }
        } else {
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const uint32_t id[4] = {reduce_index<RED>(cur[j].x, magic, npool),
                                        reduce_index<RED>(cur[j].y, magic, npool),
                                        reduce_index<RED>(cur[j].z, magic, npool),
                                        reduce_index<RED>(cur[j].w, magic, npool)};
                float s[8], tt[8];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float4 q = pool[id[k]];
                    s[2 * k] = q.x; s[2 * k + 1] = q.y;
                    tt[2 * k] = q.z; tt[2 * k + 1] = q.w;
                }
                solve<ALGO, NORM>(s, tt, h[j]);
            }
        }
        const int64_t base = t * kTile;
        if (base + kTile <= n) {
            store_rows9_staged<float, P, STP == 0 || STP == 3, STP >= 2>(
                reinterpret_cast<char*>(H + base * 9), h, stage, lane);
        } else {
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int64_t p = base + j * kWave + lane;
                if (p < n) {
#pragma unroll
                    for (int k = 0; k < 9; ++k) H[p * 9 + k] = h[j][k];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < P; ++j) {
            if constexpr (PF == 2) {
                cur[j] = ahead[j];
                ahead[j] = nxt[j];
            } else if constexpr (PF == 1) {
                cur[j] = nxt[j];
            }
        }
    }
}

// LDS bytes of sample_solve_lds_kernel<P, *, WPB> for a pool of npool points.
template <int P, int WPB = kWavesPerBlock>
constexpr size_t sample_lds_bytes(uint32_t npool) {
    return (size_t)npool * 16 + (size_t)WPB * kWave * P * 36;
}
constexpr size_t kSampleLdsMax = 64 * 1024;      // per-block dynamic LDS without opt-in
constexpr size_t kSampleLdsOptIn = 160 * 1024;   // gfx950: a workgroup may take the whole LDS

// Allows `kernel` more than 64 KiB of dynamic LDS on the current device.  Remembered per
// (device, kernel): the kernels of one signature share a function type, so a static per
// template instantiation would opt in only the first of them.
// static_lds: the kernel's own __shared__ bytes, which count against the same 160 KiB.
inline bool lds_opt_in(const void* kernel, size_t static_lds = 0) {
    static std::mutex mu;
    static std::vector<std::pair<int, const void*>> done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    std::lock_guard<std::mutex> lock(mu);
    for (const auto& e : done)
        if (e.first == dev && e.second == kernel) return true;
    if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(kSampleLdsOptIn - static_lds)) != hipSuccess)
        return false;
    done.emplace_back(dev, kernel);
    return true;
}
template <typename K>
inline bool lds_opt_in(K kernel, size_t static_lds = 0) {
    return lds_opt_in(reinterpret_cast<const void*>(kernel), static_lds);
}

// Variant sweep helper: the LDS-pool sampler with WPB waves per block (tools/kbench_sample.py).
template <int P, int WPB>
inline int launch_sample_wide(const float2* ps, const float2* pt, uint32_t npool,
                              const uint4* ix, float* H, int64_t n, int algo, bool norm,
                              hipStream_t s, int cus) {
    const size_t lds = sample_lds_bytes<P, WPB>(npool);
    if (lds > kSampleLdsOptIn) return (int)hipErrorInvalidValue;
    const int64_t tiles = (n + (int64_t)kWave * P - 1) / ((int64_t)kWave * P);
    const int64_t want = (tiles + WPB - 1) / WPB;
    int64_t per_cu = (int64_t)kSampleLdsOptIn / (int64_t)lds;
    per_cu = per_cu < 1 ? 1 : (per_cu > 8 ? 8 : per_cu);
    const int64_t cap = per_cu * cus;
    const unsigned g = (unsigned)(want < cap ? want : cap);
    const uint64_t magic = fastmod_magic(npool);
#define HG_SW(A, N)                                                                            \
    do {                                                                                       \
        auto k = sample_solve_lds_kernel<A, N, P, 1, WPB>;                                     \
        if (lds > kSampleLdsMax && !lds_opt_in(k)) return (int)hipErrorInvalidValue;           \
        rc = launch(k, g, WPB * kWave, lds, s, ps, pt, npool, magic, ix, H, n, 0, 0);          \
    } while (0)
    int rc;
    if (algo == 0) { if (norm) HG_SW(kACA, true); else HG_SW(kACA, false); }
    else { if (norm) HG_SW(kSKS, true); else HG_SW(kSKS, false); }
#undef HG_SW
    return rc;
}

// Inlier test of one (hypothesis, correspondence) pair, division-free:
//   (x', y', w') = H (x, y, 1),  inlier <=> w' != 0 and
//   (x' - u w')^2 + (y' - v w')^2 <= t^2 w'^2        [== |(x'/w', y'/w') - (u, v)|^2 <= t^2]
// with this exact FMA placement (restated in oracle/hg_oracle.c).
__device__ __forceinline__ bool is_inlier(const float (&h)[9], float4 q, float t2) {
    const float xs = __builtin_fmaf(h[0], q.x, __builtin_fmaf(h[1], q.y, h[2]));
    const float ys = __builtin_fmaf(h[3], q.x, __builtin_fmaf(h[4], q.y, h[5]));
    const float ws = __builtin_fmaf(h[6], q.x, __builtin_fmaf(h[7], q.y, h[8]));
    const float ex = __builtin_fmaf(-q.z, ws, xs);
    const float ey = __builtin_fmaf(-q.w, ws, ys);
    const float e2 = __builtin_fmaf(ex, ex, ey * ey);
    const float lim = t2 * (ws * ws);
    return (e2 <= lim) & (ws != 0.f);
}

// One lane per hypothesis; the block streams the pool through LDS in chunks of
// kChunk points {x, y, u, v} (every lane reads the same point: an LDS broadcast).
constexpr int kScoreChunk = 2048;  // 32 KiB of LDS per block

static __global__ __launch_bounds__(kBlock) void ransac_score_kernel(
    const float* __restrict__ H, int64_t n, const float2* __restrict__ pool_src,
    const float2* __restrict__ pool_tar, uint32_t npool, float t2, uint32_t* __restrict__ counts) {
    __shared__ __attribute__((aligned(16))) float4 pts[kScoreChunk];
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    float h[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) h[k] = p < n ? H[p * 9 + k] : 0.f;
    uint32_t cnt = 0;
    for (uint32_t c0 = 0; c0 < npool; c0 += kScoreChunk) {
        const uint32_t m = npool - c0 < (uint32_t)kScoreChunk ? npool - c0 : kScoreChunk;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += kBlock) {
            const float2 a = pool_src[c0 + i], b = pool_tar[c0 + i];
            pts[i] = make_float4(a.x, a.y, b.x, b.y);
        }
        __syncthreads();
        uint32_t i = 0;
        for (; i + 4 <= m; i += 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) cnt += is_inlier(h, pts[i + u], t2) ? 1u : 0u;
        }
        for (; i < m; ++i) cnt += is_inlier(h, pts[i], t2) ? 1u : 0u;
    }
    if (p < n) counts[p] = cnt;
}

// Two hypotheses per lane, evaluated as packed pairs (v_pk_fma_f32 / v_pk_mul_f32:
// one instruction serves both), every LDS point read shared by both.  Same per-pair
// arithmetic (and bits) as is_inlier.
template <int UNROLL>
__global__ __launch_bounds__(kBlock) void ransac_score2_kernel(
    const float* __restrict__ H, int64_t n, const float2* __restrict__ pool_src,
    const float2* __restrict__ pool_tar, uint32_t npool, float t2, uint32_t* __restrict__ counts) {
    __shared__ __attribute__((aligned(16))) float4 pts[kScoreChunk];
    // lane owns hypotheses p0 = 2*gid and p0 + 1 (adjacent rows: one 72-B read)
    const int64_t p0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 2;
    f32x2 h[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        h[k].x = p0 < n ? H[p0 * 9 + k] : 0.f;
        h[k].y = p0 + 1 < n ? H[(p0 + 1) * 9 + k] : 0.f;
    }
    const f32x2 t2v = {t2, t2};
    i32x2 cnt = {0, 0};
    for (uint32_t c0 = 0; c0 < npool; c0 += kScoreChunk) {
        const uint32_t m = npool - c0 < (uint32_t)kScoreChunk ? npool - c0 : kScoreChunk;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += kBlock) {
            const float2 a = pool_src[c0 + i], b = pool_tar[c0 + i];
            pts[i] = make_float4(a.x, a.y, b.x, b.y);
        }
        __syncthreads();
        auto pair = [&](float4 q) {
            const f32x2 x = {q.x, q.x}, y = {q.y, q.y}, nu = {-q.z, -q.z}, nv = {-q.w, -q.w};
            const f32x2 xs = __builtin_elementwise_fma(h[0], x, __builtin_elementwise_fma(h[1], y, h[2]));
            const f32x2 ys = __builtin_elementwise_fma(h[3], x, __builtin_elementwise_fma(h[4], y, h[5]));
            const f32x2 ws = __builtin_elementwise_fma(h[6], x, __builtin_elementwise_fma(h[7], y, h[8]));
            const f32x2 ex = __builtin_elementwise_fma(nu, ws, xs);
            const f32x2 ey = __builtin_elementwise_fma(nv, ws, ys);
            const f32x2 e2 = __builtin_elementwise_fma(ex, ex, ey * ey);
            const f32x2 lim = t2v * (ws * ws);
            const f32x2 zero = {0.f, 0.f};
            cnt -= (e2 <= lim) & (ws != zero);   // vector compares yield -1 / 0
        };
        uint32_t i = 0;
        for (; i + UNROLL <= m; i += UNROLL) {
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) pair(pts[i + u]);
        }
        for (; i < m; ++i) pair(pts[i]);
    }
    if (p0 < n) counts[p0] = (uint32_t)cnt.x;
    if (p0 + 1 < n) counts[p0 + 1] = (uint32_t)cnt.y;
}

// Pool points through the scalar unit instead of LDS: every lane of a wave needs the
// same point, so the loads are wave-uniform -- s_load into SGPRs that the packed VALU
// ops read directly.  No LDS (occupancy is then set by VGPRs alone), no block barriers,
// no chunking; the pool (16 B per pair) streams through the scalar cache / L2.
template <int UNROLL>
__global__ __launch_bounds__(kBlock) void ransac_score_sgpr_kernel(
    const float* __restrict__ H, int64_t n, const float2* __restrict__ pool_src,
    const float2* __restrict__ pool_tar, uint32_t npool, float t2, uint32_t* __restrict__ counts) {
    const int64_t p0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 2;
    f32x2 h[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        h[k].x = p0 < n ? H[p0 * 9 + k] : 0.f;
        h[k].y = p0 + 1 < n ? H[(p0 + 1) * 9 + k] : 0.f;
    }
    const f32x2 t2v = {t2, t2};
    i32x2 cnt = {0, 0};
    auto pair = [&](float2 a, float2 b) {
        const f32x2 x = {a.x, a.x}, y = {a.y, a.y}, nu = {-b.x, -b.x}, nv = {-b.y, -b.y};
        const f32x2 xs = __builtin_elementwise_fma(h[0], x, __builtin_elementwise_fma(h[1], y, h[2]));
        const f32x2 ys = __builtin_elementwise_fma(h[3], x, __builtin_elementwise_fma(h[4], y, h[5]));
        const f32x2 ws = __builtin_elementwise_fma(h[6], x, __builtin_elementwise_fma(h[7], y, h[8]));
        const f32x2 ex = __builtin_elementwise_fma(nu, ws, xs);
        const f32x2 ey = __builtin_elementwise_fma(nv, ws, ys);
        const f32x2 e2 = __builtin_elementwise_fma(ex, ex, ey * ey);
        const f32x2 lim = t2v * (ws * ws);
        const f32x2 zero = {0.f, 0.f};
        cnt -= (e2 <= lim) & (ws != zero);
    };
    uint32_t i = 0;
    for (; i + UNROLL <= npool; i += UNROLL) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) pair(pool_src[i + u], pool_tar[i + u]);
    }
    for (; i < npool; ++i) pair(pool_src[i], pool_tar[i]);
    if (p0 < n) counts[p0] = (uint32_t)cnt.x;
    if (p0 + 1 < n) counts[p0 + 1] = (uint32_t)cnt.y;
}

// Compute units of the current device (queried once per device).
inline int cu_count() {
    constexpr int kMaxDevices = 64;
    static std::atomic<int> cache[kMaxDevices] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
    int v = cache[dev].load(std::memory_order_relaxed);
    if (v == 0) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        cache[dev].store(v, std::memory_order_relaxed);
    }
    return v;
}

// variant -1 = shipped choice; 0 = global-gather kernel (P = 2); 1 / 2 = LDS-pool kernel
// P = 1 / 2; 3 = LDS-pool P = 2 with the index rows two tiles ahead; 4 = LDS-pool P = 2
// with the 64-bit remainder (fastmod64_u32); 5 = LDS-pool P = 2, the two hypotheses of a
// lane solved as packed f32x2 pairs (shipped); 6 = 5 with the pairs' divisions split into
// scalar expansions (the round-2 form, kPairScalarDiv).  The LDS forms fall back to 0 when
// the pool does not fit.
inline int launch_sample_solve(int variant, const float2* ps, const float2* pt, uint32_t npool,
                        const uint4* ix, float* H, int64_t n, int algo, bool norm, hipStream_t s) {
    constexpr int kShippedP = 2;
    const bool pf2 = variant == 3;
    const bool mod64 = variant == 4;
    const bool pair = variant == 5 || variant == 6 || variant == -1;  // shipped: P = 2 packed pairs
    const bool split_div = variant == 6;
    int use_p = variant == -1 ? kShippedP : (pf2 || mod64 || pair ? 2 : variant);
    const size_t lds = use_p == 1 ? sample_lds_bytes<1>(npool) : sample_lds_bytes<2>(npool);
    if (use_p > 0 && lds > kSampleLdsMax) use_p = 0;
    if (use_p == 0) {
        constexpr int P = 2;
        const int64_t blocks = (n + (int64_t)kBlock * P - 1) / ((int64_t)kBlock * P);
        if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
        const unsigned g = (unsigned)blocks;
#define HG_SS(A, N, PR)                                                                          \
    launch(sample_solve_kernel<A, N, P, kDrawsIndexed, PR>, g, kBlock, 0, s, ps, pt, npool, ix, H, n, \
           0, 0)
        if (pair && split_div) {
            if (algo == 0) return norm ? HG_SS(kACA, true, kPairScalarDiv) : HG_SS(kACA, false, kPairScalarDiv);
            return norm ? HG_SS(kSKS, true, kPairScalarDiv) : HG_SS(kSKS, false, kPairScalarDiv);
        }
        if (pair) {
            if (algo == 0) return norm ? HG_SS(kACA, true, kPairPacked) : HG_SS(kACA, false, kPairPacked);
            return norm ? HG_SS(kSKS, true, kPairPacked) : HG_SS(kSKS, false, kPairPacked);
        }
        if (algo == 0) return norm ? HG_SS(kACA, true, 0) : HG_SS(kACA, false, 0);
        return norm ? HG_SS(kSKS, true, 0) : HG_SS(kSKS, false, 0);
#undef HG_SS
    }
    // persistent: as many blocks as fit at once (LDS-limited), never more than the tiles
    const int64_t tiles = (n + (int64_t)kWave * use_p - 1) / ((int64_t)kWave * use_p);
    const int64_t want = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    int64_t per_cu = (int64_t)(160 * 1024) / (int64_t)lds;
    per_cu = per_cu < 1 ? 1 : (per_cu > 8 ? 8 : per_cu);
    const int64_t cap = per_cu * cu_count();
    const unsigned g = (unsigned)(want < cap ? want : cap);
    const uint64_t magic = mod64 ? fastmod64_magic(npool) : fastmod_magic(npool);
#define HG_SL(PP, A, N)                                                                      \
    launch(sample_solve_lds_kernel<A, N, PP>, g, kBlock, lds, s, ps, pt, npool, magic, ix, H, n, \
           0, 0)
    if (use_p == 1) {
        if (algo == 0) return norm ? HG_SL(1, kACA, true) : HG_SL(1, kACA, false);
        return norm ? HG_SL(1, kSKS, true) : HG_SL(1, kSKS, false);
    }
    if (mod64) {
#define HG_SL64(A, N)                                                                            \
    launch(sample_solve_lds_kernel<A, N, 2, 1, kWavesPerBlock, kDrawsIndexed, true>, g, kBlock, lds, \
           s, ps, pt, npool, magic, ix, H, n, 0, 0)
        if (algo == 0) return norm ? HG_SL64(kACA, true) : HG_SL64(kACA, false);
        return norm ? HG_SL64(kSKS, true) : HG_SL64(kSKS, false);
#undef HG_SL64
    }
    if (pair) {
#define HG_SLP(A, N, PR)                                                                         \
    launch(sample_solve_lds_kernel<A, N, 2, 1, kWavesPerBlock, kDrawsIndexed, 0, PR>, g, kBlock, \
           lds, s, ps, pt, npool, magic, ix, H, n, 0, 0)
        if (split_div) {
            if (algo == 0) return norm ? HG_SLP(kACA, true, kPairScalarDiv) : HG_SLP(kACA, false, kPairScalarDiv);
            return norm ? HG_SLP(kSKS, true, kPairScalarDiv) : HG_SLP(kSKS, false, kPairScalarDiv);
        }
        if (algo == 0) return norm ? HG_SLP(kACA, true, kPairPacked) : HG_SLP(kACA, false, kPairPacked);
        return norm ? HG_SLP(kSKS, true, kPairPacked) : HG_SLP(kSKS, false, kPairPacked);
#undef HG_SLP
    }
    if (!pf2) {
        if (algo == 0) return norm ? HG_SL(2, kACA, true) : HG_SL(2, kACA, false);
        return norm ? HG_SL(2, kSKS, true) : HG_SL(2, kSKS, false);
    }
#define HG_SL2(A, N)                                                                              \
    launch(sample_solve_lds_kernel<A, N, 2, 2>, g, kBlock, lds, s, ps, pt, npool, magic, ix, H, n, 0, \
           0)
    if (algo == 0) return norm ? HG_SL2(kACA, true) : HG_SL2(kACA, false);
    return norm ? HG_SL2(kSKS, true) : HG_SL2(kSKS, false);
#undef HG_SL2
#undef HG_SL
}

// The seeded sampler's launcher: the LDS-pool kernel with P problems per lane and WPB waves
// per block sharing one pool copy (LDS opt-in past 64 KiB), persistent grid, while the pool
// plus staging fit the CU's 160 KiB, else the global-gather form.  The draws are made in
// the kernel from word `offset` of stream seed * kBitsMul (draws4); PF = 0 makes each
// tile's draws where they are used (nothing to hide when the draws are computed).  The
// shipped shapes are launch_sample_seeded_shipped's; every parameter is open for the
// variant sweep (hg_tune_sample_seeded).
template <int P = 1, int WPB = 16, int DRAWS = kDrawsPaired, int RED = 0, int PF = 0,
          int PAIR = 0, int STP = 0>
inline int launch_sample_seeded(const float2* ps, const float2* pt, uint32_t npool,
                                uint64_t seed, uint64_t offset, float* H, int64_t n, int algo,
                                bool norm, hipStream_t s) {
    const uint64_t bits_base = DRAWS == kDrawsSingle ? seed * kBitsMul + offset
                                                     : seed * kBitsMul + (offset >> 1);
    const uint32_t odd = DRAWS == kDrawsSingle ? 0u : (uint32_t)(offset & 1);
    const size_t lds = sample_lds_bytes<P, WPB>(npool);
    if (lds > kSampleLdsOptIn) {
        constexpr int PG = 2;
        const int64_t blocks = (n + (int64_t)kBlock * PG - 1) / ((int64_t)kBlock * PG);
        if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
        const unsigned g = (unsigned)blocks;
#define HG_SG(A, N)                                                                          \
    launch(sample_solve_kernel<A, N, PG, DRAWS, PAIR>, g, kBlock, 0, s, ps, pt, npool, nullptr, H, \
           n, bits_base, odd)
        if (algo == 0) return norm ? HG_SG(kACA, true) : HG_SG(kACA, false);
        return norm ? HG_SG(kSKS, true) : HG_SG(kSKS, false);
#undef HG_SG
    }
    // persistent: as many blocks as fit at once (LDS-limited), never more than the tiles
    const int64_t tiles = (n + (int64_t)kWave * P - 1) / ((int64_t)kWave * P);
    const int64_t want = (tiles + WPB - 1) / WPB;
    int64_t per_cu = (int64_t)kSampleLdsOptIn / (int64_t)lds;
    per_cu = per_cu < 1 ? 1 : (per_cu > 8 ? 8 : per_cu);
    const int64_t cap = per_cu * cu_count();
    const unsigned g = (unsigned)(want < cap ? want : cap);
    const uint64_t magic = reduce_magic<RED>(npool);
#define HG_SD(A, N)                                                                         \
    do {                                                                                    \
        auto k = sample_solve_lds_kernel<A, N, P, PF, WPB, DRAWS, RED, PAIR, STP>;          \
        if (lds > kSampleLdsMax && !lds_opt_in(k)) return (int)hipErrorInvalidValue;        \
        rc = launch(k, g, WPB * kWave, lds, s, ps, pt, npool, magic, nullptr, H, n, bits_base, \
                    odd);                                                                   \
    } while (0)
    int rc;
    if (algo == 0) { if (norm) HG_SD(kACA, true); else HG_SD(kACA, false); }
    else { if (norm) HG_SD(kSKS, true); else HG_SD(kSKS, false); }
#undef HG_SD
    return rc;
}

// The shipped seeded shapes, all solving two hypotheses per lane as packed f32x2 pairs --
// the arithmetic of the indexed sampler and of both global-gather fallbacks, so a seeded
// launch equals fill_bits + an indexed one to the last bit, NaN signs included (packed and
// scalar solves agree on every value but not always on a NaN's sign).  8 waves per block;
// ACA from kSeededPairMinN hypotheses 4 (fewer resident waves, fewer concurrent write
// streams: the launch is within ~10 % of the write-only HBM ceiling there).  16 M: ACA
// 109-114 vs 118-126 us for the round-1 P = 1 scalar form, SKS 131-133 vs 147-155; at 1 M
// ACA pays ~5 % against that form (tools/kbench_sample.py, profiles/r02/kbench_pair*).
constexpr int64_t kSeededPairMinN = int64_t(1) << 22;
inline int launch_sample_seeded_shipped(const float2* ps, const float2* pt, uint32_t npool,
                                        uint64_t seed, uint64_t offset, float* H, int64_t n,
                                        int algo, bool norm, hipStream_t s) {
    // ACA from 4 M: the binary64 remainder without a correction (RED 4, fmod_f64_exact_u32; same
    // indices): 149.8 -> 137.8 VALU per 64 hypotheses (profiles/r06/pmc_table8_r06v.json); its
    // time is within the sweeps' spread (round 6)
    if (algo == 0 && n >= kSeededPairMinN)
        return launch_sample_seeded<2, 4, kDrawsPaired, 4, 0, kPairPacked>(ps, pt, npool, seed,
                                                                            offset, H, n, algo, norm, s);
    return launch_sample_seeded<2, 8, kDrawsPaired, 0, 0, kPairPacked>(ps, pt, npool, seed, offset,
                                                                        H, n, algo, norm, s);
}

// Four hypotheses per lane (two packed pairs): each scalar-loaded point feeds twice
// the arithmetic, half the waves.
template <int UNROLL>
__global__ __launch_bounds__(kBlock) void ransac_score_sgpr4_kernel(
    const float* __restrict__ H, int64_t n, const float2* __restrict__ pool_src,
    const float2* __restrict__ pool_tar, uint32_t npool, float t2, uint32_t* __restrict__ counts) {
    const int64_t p0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    f32x2 h[2][9];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int64_t a = p0 + 2 * q, b = a + 1;
            h[q][k].x = a < n ? H[a * 9 + k] : 0.f;
            h[q][k].y = b < n ? H[b * 9 + k] : 0.f;
        }
    const f32x2 t2v = {t2, t2};
    i32x2 cnt[2] = {{0, 0}, {0, 0}};
    auto pair = [&](float2 a, float2 b) {
        const f32x2 x = {a.x, a.x}, y = {a.y, a.y}, nu = {-b.x, -b.x}, nv = {-b.y, -b.y};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const f32x2 xs = __builtin_elementwise_fma(h[q][0], x, __builtin_elementwise_fma(h[q][1], y, h[q][2]));
            const f32x2 ys = __builtin_elementwise_fma(h[q][3], x, __builtin_elementwise_fma(h[q][4], y, h[q][5]));
            const f32x2 ws = __builtin_elementwise_fma(h[q][6], x, __builtin_elementwise_fma(h[q][7], y, h[q][8]));
            const f32x2 ex = __builtin_elementwise_fma(nu, ws, xs);
            const f32x2 ey = __builtin_elementwise_fma(nv, ws, ys);
            const f32x2 e2 = __builtin_elementwise_fma(ex, ex, ey * ey);
            const f32x2 lim = t2v * (ws * ws);
            const f32x2 zero = {0.f, 0.f};
            cnt[q] -= (e2 <= lim) & (ws != zero);
        }
    };
    uint32_t i = 0;
    for (; i + UNROLL <= npool; i += UNROLL) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) pair(pool_src[i + u], pool_tar[i + u]);
    }
    for (; i < npool; ++i) pair(pool_src[i], pool_tar[i]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int64_t a = p0 + 2 * q;
        if (a < n) counts[a] = (uint32_t)cnt[q].x;
        if (a + 1 < n) counts[a + 1] = (uint32_t)cnt[q].y;
    }
}

}  // namespace hg
