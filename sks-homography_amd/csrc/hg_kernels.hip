// hg_kernels.hip -- batched ACA / SKS / TensorACA kernels for MI355X (gfx950) and
// the C ABI (include/sks_homography.h).
//
// Headline data path (AoS f32, hg_aos.hpp): a wave owns a tile of 64*P problems
// (P = 2: 8 KiB of src + tar).
//   load   : the tile's src and tar slabs are contiguous, so they land in the wave's
//            LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction,
//            non-temporal), no VGPR round trip,
//   compute: each lane reads its problems' 32-B rows from LDS and runs the closed
//            form in VGPRs (hg_solvers.hpp; no FMA contraction, IEEE division),
//   store  : H rows are 36 B -- not 16-B aligned per lane -- so the wave stages its
//            rows in LDS and writes its contiguous H slab as 16-B non-temporal
//            stores, lane-consecutive (fully coalesced).
// Bytes per problem (f32): 64 read + 36 written = 100 B at ~1-1.7 FLOP/B: the bound
// is HBM bandwidth, not VALU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "hg_aos.hpp"
#include "hg_launch.hpp"
#include "hg_rect.hpp"
#include "hg_reduce.hpp"
#include "hg_rect_sum.hpp"
#include "hg_soa.hpp"
#include "hg_solvers.hpp"
#include "sks_homography.h"

namespace hg {

// ---------------------------------------------------------------------------
// Generic kernel: any alignment, AoS or SoA (the reference GPU layout,
// GPU_Runtime Test.cu:87-95 / :141-149).  One problem per lane, grid-stride.
// SoA accesses are naturally coalesced (lane-consecutive addresses per component).
template <int ALGO, bool NORM, typename T, bool SOA>
__global__ __launch_bounds__(kBlock) void solve_generic(const T* __restrict__ src,
                                                        const T* __restrict__ tar,
                                                        T* __restrict__ H, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n; p += stride) {
        T s[8], t[8], h[9];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s[k] = SOA ? src[(int64_t)k * n + p] : src[p * 8 + k];
            t[k] = SOA ? tar[(int64_t)k * n + p] : tar[p * 8 + k];
        }
        solve<ALGO, NORM>(s, t, h);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            if (SOA) H[(int64_t)k * n + p] = h[k];
            else H[p * 9 + k] = h[k];
        }
    }
}

// Many small batches in one launch (hg_solve_grouped_*): up to kGroupMax batches ride in
// the kernel arguments; block b of the grid belongs to the batch whose block range holds
// it (a wave-uniform search over the block prefix sums), and within it one lane solves
// one problem exactly as solve_generic does.  Small batches are bound by the per-launch
// cost (argument staging, ~1 us of the ~2.7 us a launch costs back to back, §6 of
// DESIGN.md), so one launch for a group replaces one per batch.
constexpr int kGroupMax = 32;
template <typename T>
struct GroupArgs {
    const T* src[kGroupMax];
    const T* tar[kGroupMax];
    T* H[kGroupMax];
    int64_t n[kGroupMax];
    uint32_t first_block[kGroupMax + 1];  // prefix sums of each batch's block count
    int count;
};

template <int ALGO, bool NORM, typename T, bool SOA>
__global__ __launch_bounds__(kBlock) void solve_grouped(GroupArgs<T> g) {
    const uint32_t blk = blockIdx.x;
    int b = 0;
    while (b + 1 < g.count && g.first_block[b + 1] <= blk) ++b;  // uniform: scalar loop
    const int64_t n = g.n[b];
    const int64_t p = (int64_t)(blk - g.first_block[b]) * kBlock + threadIdx.x;
    if (p >= n) return;
    const T* __restrict__ src = g.src[b];
    const T* __restrict__ tar = g.tar[b];
    T* __restrict__ H = g.H[b];
    T s[8], t[8], h[9];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        s[k] = SOA ? src[(int64_t)k * n + p] : src[p * 8 + k];
        t[k] = SOA ? tar[(int64_t)k * n + p] : tar[p * 8 + k];
    }
    solve<ALGO, NORM>(s, t, h);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        if (SOA) H[(int64_t)k * n + p] = h[k];
        else H[p * 9 + k] = h[k];
    }
}

// ---------------------------------------------------------------------------
// Counter-based uniform generator (bit-identical to oracle_fill_uniform_f32).

__global__ __launch_bounds__(kBlock) void fill_uniform_kernel(float* __restrict__ out,
                                                              int64_t count, uint64_t seed,
                                                              uint64_t offset, float lo,
                                                              float hi) {
    const float span = hi - lo;
    const uint64_t base = seed * 0xD1B54A32D192ED03ull + offset;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < count; i += stride) {
        const uint64_t r = mix64(base + (uint64_t)i);
        const float u = (float)(uint32_t)(r >> 40) * 5.9604644775390625e-08f;
        const float su = span * u;
        out[i] = lo + su;
    }
}

// One problem whose points travel in the kernel arguments (no H2D copy); one lane
// solves and writes H (9 values) straight to `H`, typically host memory mapped into the
// device address space -- the latency path of the single-problem sks:: calls.
template <typename T>
struct Quad {
    T src[8], tar[8];
};

template <int ALGO, bool NORM, typename T>
__global__ __launch_bounds__(kWave) void solve_one_kernel(Quad<T> q, T* __restrict__ H) {
    if (threadIdx.x != 0) return;
    T h[9];
    solve<ALGO, NORM>(q.src, q.tar, h);
#pragma unroll
    for (int k = 0; k < 9; ++k) H[k] = h[k];
}

// The same, then a completion word: H first, a system-scope fence, then *done = seq, so a
// host thread that sees seq in mapped memory also sees all of H (the sks:: host-pointer
// calls spin on it instead of waiting for the stream: hg_sks_api.cpp).
template <int ALGO, bool NORM, typename T>
__global__ __launch_bounds__(kWave) void solve_one_signal_kernel(Quad<T> q, T* __restrict__ H,
                                                                 uint32_t* done, uint32_t seq) {
    if (threadIdx.x != 0) return;
    T h[9];
    solve<ALGO, NORM>(q.src, q.tar, h);
#pragma unroll
    for (int k = 0; k < 9; ++k) H[k] = h[k];
    __threadfence_system();
    __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Deterministic row sums, in place (hg_sum_rows_f32).  Pass 1: block (c, r) sums chunk c
// = x[r][c*kSumChunk, (c+1)*kSumChunk) -- thread t adds elements c*kSumChunk + t + 256 i,
// i = 0, 1, ... in order (out-of-range elements count as +0), then the 256 sums fold by
// halving strides (v[t] += v[t + s], s = 128 ... 1) -- and writes the chunk's sum over the
// chunk's first element, which no other block reads.  Pass 2: one block per row folds
// the chunk sums the same way.  Fixed order, so the result is bit-reproducible (and
// restated in numpy by tests/test_gpu_parity.py).
constexpr int kSumChunk = kBlock * 16;

__device__ __forceinline__ float block_fold(float v, float* red) {
    red[threadIdx.x] = v;
    __syncthreads();
#pragma unroll
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + s];
        __syncthreads();
    }
    return red[0];
}

__global__ __launch_bounds__(kBlock) void sum_rows_pass1(float* __restrict__ x, int64_t cols) {
    __shared__ float red[kBlock];
    float* row = x + (int64_t)blockIdx.y * cols;
    const int64_t c0 = (int64_t)blockIdx.x * kSumChunk;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < kSumChunk / kBlock; ++i) {
        const int64_t e = c0 + threadIdx.x + (int64_t)i * kBlock;
        v = v + (e < cols ? row[e] : 0.f);
    }
    const float sum = block_fold(v, red);  // ends with every read of the chunk done
    if (threadIdx.x == 0) row[c0] = sum;
}

__global__ __launch_bounds__(kBlock) void sum_rows_pass2(const float* __restrict__ x, int64_t cols,
                                                         int64_t chunks, float* __restrict__ out) {
    __shared__ float red[kBlock];
    const float* row = x + (int64_t)blockIdx.x * cols;
    float v = 0.f;
    for (int64_t c = threadIdx.x; c < chunks; c += kBlock) v = v + row[c * kSumChunk];
    const float sum = block_fold(v, red);
    if (threadIdx.x == 0) out[blockIdx.x] = sum;
}

// Streaming copy, 16 B per lane per iteration (bandwidth yardstick).
__global__ __launch_bounds__(kBlock) void stream_copy_kernel(const u32x4* __restrict__ src,
                                                             u32x4* __restrict__ dst,
                                                             int64_t n16) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n16; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

}  // namespace hg

// ===========================================================================
// Host launchers
// ===========================================================================
namespace hg {

constexpr int kErrInvalid = (int)hipErrorInvalidValue;

// Shipped AoS configuration (chosen by tools/kbench.py sweeps, profiles/r01/):
// P problems per lane (2 f32 / 1 f64: an 8 KiB wave tile either way), inputs by
// LDS-DMA with the non-temporal policy, LDS-staged non-temporal 16-B H stores.
template <typename T>
constexpr int kAosP = sizeof(T) == 4 ? 2 : 1;
constexpr int kAosFlags = kNtLoad | kNtStore | kLdsLoad | kLdsDma;
// Batches whose bytes (in + out) fit the 256 MB Infinity Cache (MALL) with room to spare
// use the default cache policy instead: a caller that re-reads or just produced them
// (back-to-back launches, a pipeline) hits the MALL -- 7 % faster at 1-2 M f32 AoS, 11 %
// at 1 M f64 SoA; beyond it non-temporal wins (10 M: 154 vs 171 us).  Same arithmetic,
// same bits (tools/kbench.py, tools/kbench_soa_small.py).
constexpr int kAosCachedFlags = kLdsLoad | kLdsDma;
constexpr int64_t kMallResidentBytes = 200000000;
constexpr int kRectP = 1;  // TensorACA problems per lane (tools/kbench_rect.py, profiles/r01/kbench_rect.json)
// SoA: the narrow form (one problem per lane, element-wide row accesses; hg_soa.hpp
// solve_soa_narrow) everywhere -- 3-5 % ahead of the 16-B register and LDS-DMA forms at
// 10 M, 10-20 % ahead at N <= 10 K -- except MALL-resident binary64 batches of
// kSoaWideMinN problems and up, where the 16-B register form (kSoaG groups per lane)
// leads (tools/kbench_soa.py, tools/kbench_soa_small.py; profiles/r01/kbench_soa*.json).
constexpr int kSoaG = 1;
constexpr int64_t kSoaWideMinN = 32768;

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
template <int A>
inline bool aligned_to(const void* p) { return (reinterpret_cast<uintptr_t>(p) & (A - 1)) == 0; }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline unsigned generic_grid(int64_t n) {
    // Enough blocks to fill 256 CUs several times over, grid-stride beyond that.
    const int64_t want = ceil_div(n, kBlock);
    return (unsigned)(want < 8192 ? (want > 0 ? want : 1) : 8192);
}

// host = the buffers are host memory read and written over PCIe (hg_solve_host_*): the
// non-temporal hints are about HBM / MALL residency and buy nothing there, so host batches
// take the default policy -- which also keeps their 12 ms launches apart from the
// headline's in kernel traces.
template <int ALGO, bool NORM, typename T>
int launch_solver(const T* src, const T* tar, T* H, int64_t n, int layout, hipStream_t s,
                  bool host = false) {
    const bool cached = host || n <= kMallResidentBytes / (25 * (int64_t)sizeof(T));  // 25 values/problem
    if (layout == HG_LAYOUT_SOA) {
        constexpr int V = 16 / sizeof(T);
        const bool wide = sizeof(T) == 8 && n >= kSoaWideMinN && n % V == 0 && aligned16(src) &&
                          aligned16(tar) && aligned16(H);
        if (wide && ALGO == kGPT && !host) {
            // GPT-LU is VALU-bound (~1000 instructions a problem): two problems per lane in
            // 16-B registers with non-temporal access at every size from 32 K, 5 % ahead of
            // the narrow form at 10 M and level at 1 M (tools/kbench_gpt.py)
            const unsigned g = (unsigned)soa_grid<kSoaG, false>(n / V);
            return launch(solve_soa_vec<ALGO, NORM, T, kSoaG, false, true>, g, kBlock, 0, s, src,
                          tar, H, n);
        }
        if (wide && cached) {
            // binary64, MALL-resident, mid-size: the 16-B register form (8 % ahead at 100 K)
            const unsigned g = (unsigned)soa_grid<kSoaG, false>(n / V);
            return launch(solve_soa_vec<ALGO, NORM, T, kSoaG, false, false>, g, kBlock, 0, s, src,
                          tar, H, n);
        }
        if (aligned_to<sizeof(T)>(src) && aligned_to<sizeof(T)>(tar) && aligned_to<sizeof(T)>(H)) {
            // one problem per lane, one element-wide access per component row
            const int64_t blocks = ceil_div(n, kBlock);
            if (blocks > 0x7fffffffLL) return kErrInvalid;
            if (cached)
                return launch(solve_soa_narrow<ALGO, NORM, T, sizeof(T), false>, (unsigned)blocks,
                              kBlock, 0, s, src, tar, H, n);
            return launch(solve_soa_narrow<ALGO, NORM, T, sizeof(T), true>, (unsigned)blocks,
                          kBlock, 0, s, src, tar, H, n);
        }
        return launch(solve_generic<ALGO, NORM, T, true>, generic_grid(n), kBlock, 0, s, src, tar,
                      H, n);
    }
    if (aligned16(src) && aligned16(tar) && aligned16(H)) {
        constexpr int P = kAosP<T>;
        const int64_t blocks = aos_grid<T, P, kAosFlags>(n);
        if (blocks > 0x7fffffffLL) return kErrInvalid;
        if (cached)
            return launch(solve_aos<ALGO, NORM, T, P, kAosCachedFlags>, (unsigned)blocks, kBlock, 0,
                          s, src, tar, H, n);
        return launch(solve_aos<ALGO, NORM, T, P, kAosFlags>, (unsigned)blocks, kBlock, 0, s, src,
                      tar, H, n);
    }
    return launch(solve_generic<ALGO, NORM, T, false>, generic_grid(n), kBlock, 0, s, src, tar, H,
                  n);
}

template <int ALGO, typename T>
int dispatch(const T* src, const T* tar, T* H, int64_t n, int layout, int flags, void* stream,
             bool host = false) {
    if (n < 0) return kErrInvalid;
    if (layout != HG_LAYOUT_AOS && layout != HG_LAYOUT_SOA) return kErrInvalid;
    if (flags & ~HG_FLAG_NORMALIZE) return kErrInvalid;
    if (n == 0) return 0;
    if (!src || !tar || !H) return kErrInvalid;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (flags & HG_FLAG_NORMALIZE) return launch_solver<ALGO, true>(src, tar, H, n, layout, s, host);
    return launch_solver<ALGO, false>(src, tar, H, n, layout, s, host);
}

// Groups of batches: host arrays of device pointers and sizes, split into launches of at
// most kGroupMax batches (empty batches skipped).  Same validation as dispatch per batch.
template <int ALGO, bool NORM, typename T, bool SOA>
int launch_grouped_chunk(const GroupArgs<T>& g, hipStream_t s) {
    const uint32_t blocks = g.first_block[g.count];
    if (blocks == 0) return 0;
    return launch(solve_grouped<ALGO, NORM, T, SOA>, blocks, kBlock, 0, s, g);
}

template <typename T>
int dispatch_grouped(int algo, const T* const* src, const T* const* tar, T* const* H,
                     const int64_t* n, int count, int layout, int flags, void* stream) {
    const int max_algo = sizeof(T) == 8 ? kGPT : kGE;
    if (algo < kACA || algo > max_algo || count < 0) return kErrInvalid;
    if (layout != HG_LAYOUT_AOS && layout != HG_LAYOUT_SOA) return kErrInvalid;
    if (flags & ~HG_FLAG_NORMALIZE) return kErrInvalid;
    if (count == 0) return 0;
    if (!src || !tar || !H || !n) return kErrInvalid;
    for (int i = 0; i < count; ++i) {
        if (n[i] < 0) return kErrInvalid;
        if (n[i] > 0 && (!src[i] || !tar[i] || !H[i])) return kErrInvalid;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool norm = flags & HG_FLAG_NORMALIZE, soa = layout == HG_LAYOUT_SOA;
    GroupArgs<T> g{};
    auto flush = [&]() -> int {
        int rc = 0;
        if (g.count == 0) return 0;
#define HG_G(A)                                                                                   \
    rc = norm ? (soa ? launch_grouped_chunk<A, true, T, true>(g, s) : launch_grouped_chunk<A, true, T, false>(g, s)) \
              : (soa ? launch_grouped_chunk<A, false, T, true>(g, s) : launch_grouped_chunk<A, false, T, false>(g, s))
        switch (algo) {
            case kACA: HG_G(kACA); break;
            case kSKS: HG_G(kSKS); break;
            case kGE: HG_G(kGE); break;
            default:
                if constexpr (sizeof(T) == 8) { HG_G(kGPT); }
                break;
        }
#undef HG_G
        g = GroupArgs<T>{};
        return rc;
    };
    for (int i = 0; i < count; ++i) {
        if (n[i] == 0) continue;
        const int64_t nb = ceil_div(n[i], kBlock);
        if (nb > 0x7fffffffLL || (int64_t)g.first_block[g.count] + nb > 0x7fffffffLL) {
            if (g.count && (int64_t)g.first_block[g.count] + nb > 0x7fffffffLL) {
                if (int rc = flush()) return rc;
            }
            if (nb > 0x7fffffffLL) return kErrInvalid;
        }
        const int j = g.count++;
        g.src[j] = src[i];
        g.tar[j] = tar[i];
        g.H[j] = H[i];
        g.n[j] = n[i];
        g.first_block[j + 1] = g.first_block[j] + (uint32_t)nb;
        if (g.count == kGroupMax) {
            if (int rc = flush()) return rc;
        }
    }
    return flush();
}

// The square specialisation (ACA_rect.m:28) is taken only where the ratio is known on
// the host and is exactly 1, so dropping the multiply cannot change a bit.
inline bool is_unit_ratio(float div) { return div == 1.0f; }

template <bool SCALAR>
int launch_rect(const float* src, const float* tar, float* H, int64_t B, const float* sp,
                const float* dp, float sv, float dv, void* stream) {
    if (B < 0) return kErrInvalid;
    if (B == 0) return 0;
    if (!src || !tar || !H || (!SCALAR && (!sp || !dp))) return kErrInvalid;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    constexpr int P = kRectP;
    const int64_t blocks = ceil_div(B, (int64_t)kBlock * P);
    if (blocks > 0x7fffffffLL) return kErrInvalid;
    // 132 B actually move per problem (the whole 48-B src record is fetched); cache
    // policy by size as launch_solver (tools/kbench_rect.py: 1 M 23.2 -> 21.4 us cached,
    // 16 M 351 nt vs 397 cached)
    const bool cached = B * 132 <= kMallResidentBytes;
    const bool vec = aligned16(src) && aligned16(tar) && aligned16(H);
    const unsigned g = (unsigned)blocks;
#define HG_RECT(SQ, NT)                                                                       \
    launch(tensor_aca_rect_kernel<P, true, SCALAR, SQ, NT>, g, kBlock, 0, s, src, tar, H, B, sp, \
           dp, sv, dv)
    int rc;
    if (vec && SCALAR && is_unit_ratio(dv)) {
        rc = cached ? HG_RECT(true, false) : HG_RECT(true, true);
    } else if (vec) {
        rc = cached ? HG_RECT(false, false) : HG_RECT(false, true);
    } else {  // unaligned views: per-lane loads and stores
        rc = launch(tensor_aca_rect_kernel<P, false, SCALAR>, g, kBlock, 0, s, src, tar, H, B, sp,
                    dp, sv, dv);
    }
#undef HG_RECT
    return rc;
}

template <typename T>
int launch_one(int algo, const T* src, const T* tar, T* H, int flags, void* stream,
               uint32_t* done = nullptr, uint32_t seq = 0) {
    if (!src || !tar || !H || (flags & ~HG_FLAG_NORMALIZE)) return kErrInvalid;
    if (algo != kACA && algo != kSKS) return kErrInvalid;
    Quad<T> q;
    for (int k = 0; k < 8; ++k) {
        q.src[k] = src[k];
        q.tar[k] = tar[k];
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool norm = flags & HG_FLAG_NORMALIZE;
#define HG_ONE(A, N)                                                                         \
    (done ? launch(solve_one_signal_kernel<A, N, T>, 1, kWave, 0, s, q, H, done, seq)       \
          : launch(solve_one_kernel<A, N, T>, 1, kWave, 0, s, q, H))
    if (algo == kACA) return norm ? HG_ONE(kACA, true) : HG_ONE(kACA, false);
    return norm ? HG_ONE(kSKS, true) : HG_ONE(kSKS, false);
#undef HG_ONE
}

}  // namespace hg

// ===========================================================================
// C ABI (include/sks_homography.h)
// ===========================================================================
extern "C" {

int hg_aca_f32(const float* src, const float* tar, float* H, int64_t n, int layout, int flags,
               void* stream) {
    return hg::dispatch<hg::kACA>(src, tar, H, n, layout, flags, stream);
}

int hg_aca_f64(const double* src, const double* tar, double* H, int64_t n, int layout,
               int flags, void* stream) {
    return hg::dispatch<hg::kACA>(src, tar, H, n, layout, flags, stream);
}

int hg_sks_f32(const float* src, const float* tar, float* H, int64_t n, int layout, int flags,
               void* stream) {
    return hg::dispatch<hg::kSKS>(src, tar, H, n, layout, flags, stream);
}

int hg_sks_f64(const double* src, const double* tar, double* H, int64_t n, int layout,
               int flags, void* stream) {
    return hg::dispatch<hg::kSKS>(src, tar, H, n, layout, flags, stream);
}

int hg_ge_f32(const float* src, const float* tar, float* H, int64_t n, int layout, int flags,
              void* stream) {
    return hg::dispatch<hg::kGE>(src, tar, H, n, layout, flags, stream);
}

int hg_ge_f64(const double* src, const double* tar, double* H, int64_t n, int layout, int flags,
              void* stream) {
    return hg::dispatch<hg::kGE>(src, tar, H, n, layout, flags, stream);
}

int hg_gpt_f64(const double* src, const double* tar, double* H, int64_t n, int layout,
               int flags, void* stream) {
    return hg::dispatch<hg::kGPT>(src, tar, H, n, layout, flags, stream);
}

int hg_solve_grouped_f32(int algo, const float* const* src, const float* const* tar,
                         float* const* H, const int64_t* n, int count, int layout, int flags,
                         void* stream) {
    return hg::dispatch_grouped<float>(algo, src, tar, H, n, count, layout, flags, stream);
}

int hg_solve_grouped_f64(int algo, const double* const* src, const double* const* tar,
                         double* const* H, const int64_t* n, int count, int layout, int flags,
                         void* stream) {
    return hg::dispatch_grouped<double>(algo, src, tar, H, n, count, layout, flags, stream);
}

// Library-internal: the single-problem launch with a completion word (hg_sks_api.cpp).
int hg_internal_solve_one_signal_f32(int algo, const float* src, const float* tar, float* H,
                                     int flags, uint32_t* done, uint32_t seq, void* stream) {
    if (!done) return hg::kErrInvalid;
    return hg::launch_one(algo, src, tar, H, flags, stream, done, seq);
}
int hg_internal_solve_one_signal_f64(int algo, const double* src, const double* tar, double* H,
                                     int flags, uint32_t* done, uint32_t seq, void* stream) {
    if (!done) return hg::kErrInvalid;
    return hg::launch_one(algo, src, tar, H, flags, stream, done, seq);
}

// Library-internal (not in the public header): the solvers for buffers in host memory,
// reached from hg_solve_host_* (hg_host.cpp) with device-visible addresses.
int hg_internal_solve_host_f32(int algo, const float* src, const float* tar, float* H,
                               int64_t n, int layout, int flags, void* stream) {
    switch (algo) {
        case HG_ALGO_ACA: return hg::dispatch<hg::kACA>(src, tar, H, n, layout, flags, stream, true);
        case HG_ALGO_SKS: return hg::dispatch<hg::kSKS>(src, tar, H, n, layout, flags, stream, true);
        case HG_ALGO_GE: return hg::dispatch<hg::kGE>(src, tar, H, n, layout, flags, stream, true);
        default: return hg::kErrInvalid;
    }
}

int hg_internal_solve_host_f64(int algo, const double* src, const double* tar, double* H,
                               int64_t n, int layout, int flags, void* stream) {
    switch (algo) {
        case HG_ALGO_ACA: return hg::dispatch<hg::kACA>(src, tar, H, n, layout, flags, stream, true);
        case HG_ALGO_SKS: return hg::dispatch<hg::kSKS>(src, tar, H, n, layout, flags, stream, true);
        case HG_ALGO_GE: return hg::dispatch<hg::kGE>(src, tar, H, n, layout, flags, stream, true);
        case HG_ALGO_GPT: return hg::dispatch<hg::kGPT>(src, tar, H, n, layout, flags, stream, true);
        default: return hg::kErrInvalid;
    }
}

int hg_tensor_aca_rect_f32(const float* src, const float* tar, float* H, int64_t B,
                           const float* scale, const float* div, void* stream) {
    return hg::launch_rect<false>(src, tar, H, B, scale, div, 0.f, 0.f, stream);
}

int hg_tensor_aca_rect_f32_hostscalar(const float* src, const float* tar, float* H, int64_t B,
                                      float scale, float div, void* stream) {
    return hg::launch_rect<true>(src, tar, H, B, nullptr, nullptr, scale, div, stream);
}

extern "C++" {
namespace hg {
// The one-value backward: the staged form when every buffer is 16-B aligned
// (tools/kbench_bwd.py), cache policy by size as the forward; dL/dscale, dL/ddiv as (2,B)
// per-problem sums (kSdSums) or (2,B,3) terms (kSdTerms).
template <int ORDER, int SD>
int launch_rect_backward_sd(const float* src, const float* tar, const float* grad_H, int64_t B,
                            const float* scale, const float* div, float* grad_src,
                            float* grad_tar, float* grad_sd, hipStream_t s) {
    const bool ws = grad_src != nullptr;
    if (aligned16(src) && aligned16(tar) && aligned16(grad_H) && aligned16(grad_tar) &&
        (!ws || aligned16(grad_src)) && (SD != kSdTerms || aligned16(grad_sd))) {
        const unsigned g = (unsigned)ceil_div(B, kBlock);
        const bool nt = B * 232 > kMallResidentBytes;
#define HG_RB(A, NT)                                                                           \
    launch(tensor_aca_rect_backward_staged<A, SD, NT, ORDER>, g, kBlock, 0, s, src, tar, grad_H,  \
           B, scale, div, grad_src, grad_tar, grad_sd)
        if (nt) return ws ? HG_RB(true, true) : HG_RB(false, true);
        return ws ? HG_RB(true, false) : HG_RB(false, false);
#undef HG_RB
    }
    const unsigned g = generic_grid(B);
#define HG_RECT_BWD(A)                                                                        \
    launch(tensor_aca_rect_backward_kernel<A, SD, ORDER>, g, kBlock, 0, s, src, tar, grad_H, B, \
           scale, div, grad_src, grad_tar, grad_sd)
    return ws ? HG_RECT_BWD(true) : HG_RECT_BWD(false);
#undef HG_RECT_BWD
}

template <int ORDER, int SD>
int launch_rect_backward(const float* src, const float* tar, const float* grad_H, int64_t B,
                         const float* scale, const float* div, float* grad_src, float* grad_tar,
                         float* grad_sd, hipStream_t s) {
    if (!grad_sd)
        return launch_rect_backward_sd<ORDER, kSdNone>(src, tar, grad_H, B, scale, div, grad_src,
                                                       grad_tar, nullptr, s);
    return launch_rect_backward_sd<ORDER, SD>(src, tar, grad_H, B, scale, div, grad_src, grad_tar,
                                              grad_sd, s);
}

inline int rect_backward_args_ok(const float* src, const float* tar, const float* grad_H, int64_t B,
                                 const float* scale, const float* div, const float* grad_tar) {
    if (B < 0) return kErrInvalid;
    if (B == 0) return 0;
    if (!src || !tar || !grad_H || !scale || !div || !grad_tar) return kErrInvalid;
    return -1;  // go on
}
}  // namespace hg
}  // extern "C++"

int hg_tensor_aca_rect_backward_f32(const float* src, const float* tar, const float* grad_H,
                                    int64_t B, const float* scale, const float* div,
                                    float* grad_src, float* grad_tar, float* grad_scale_div,
                                    void* stream) {
    const int rc = hg::rect_backward_args_ok(src, tar, grad_H, B, scale, div, grad_tar);
    if (rc >= 0) return rc;
    return hg::launch_rect_backward<hg::kAtenCpu, hg::kSdSums>(
        src, tar, grad_H, B, scale, div, grad_src, grad_tar, grad_scale_div,
        reinterpret_cast<hipStream_t>(stream));
}

int hg_tensor_aca_rect_backward_terms_f32(const float* src, const float* tar, const float* grad_H,
                                          int64_t B, const float* scale, const float* div,
                                          float* grad_src, float* grad_tar, float* grad_terms,
                                          void* stream) {
    const int rc = hg::rect_backward_args_ok(src, tar, grad_H, B, scale, div, grad_tar);
    if (rc >= 0) return rc;
    return hg::launch_rect_backward<hg::kAtenCpu, hg::kSdTerms>(
        src, tar, grad_H, B, scale, div, grad_src, grad_tar, grad_terms,
        reinterpret_cast<hipStream_t>(stream));
}

int hg_tensor_aca_rect_bcast_f32(const float* src, const float* tar, float* H, int64_t B,
                                 const float* scale, int64_t scale_sb, int64_t scale_sr,
                                 const float* div, int64_t div_sb, int64_t div_sr, void* stream) {
    if (B < 0) return hg::kErrInvalid;
    if (B == 0) return 0;
    if (!src || !tar || !H || !scale || !div) return hg::kErrInvalid;
    const hg::RectBcast a{scale, scale_sb, scale_sr, div, div_sb, div_sr};
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (hg::aligned16(src) && hg::aligned16(tar) && hg::aligned16(H)) {
        const unsigned g = (unsigned)hg::ceil_div(B, hg::kBlock);
        if (B * 140 > hg::kMallResidentBytes)  // 132 B of (B,3,4) records and H + 8 B of scale / div
            return hg::launch(hg::tensor_aca_rect_bcast_staged<true>, g, hg::kBlock, 0, s, src, tar,
                              H, B, a);
        return hg::launch(hg::tensor_aca_rect_bcast_staged<false>, g, hg::kBlock, 0, s, src, tar, H,
                          B, a);
    }
    return hg::launch(hg::tensor_aca_rect_bcast_kernel<hg::kAtenCpu>, hg::generic_grid(B), hg::kBlock, 0, s, src,
                      tar, H, B, a);
}

int hg_tensor_aca_rect_bcast_backward_f32(const float* src, const float* tar, const float* grad_H,
                                          int64_t B, const float* scale, int64_t scale_sb,
                                          int64_t scale_sr, const float* div, int64_t div_sb,
                                          int64_t div_sr, float* grad_src, float* grad_tar,
                                          float* grad_scale, int scale_rows, float* grad_div,
                                          int div_rows, void* stream) {
    if (B < 0) return hg::kErrInvalid;
    if (B == 0) return 0;
    if (!src || !tar || !grad_H || !scale || !div || !grad_tar) return hg::kErrInvalid;
    if (scale_rows < 0 || scale_rows > 2 || div_rows < 0 || div_rows > 2) return hg::kErrInvalid;
    const hg::RectBcast a{scale, scale_sb, scale_sr, div, div_sb, div_sr};
    return hg::launch(hg::tensor_aca_rect_bcast_backward_kernel<hg::kAtenCpu>, hg::generic_grid(B), hg::kBlock,
                      0, reinterpret_cast<hipStream_t>(stream), src, tar, grad_H, B, a, grad_src,
                      grad_tar, grad_scale, scale_rows, grad_div, div_rows);
}

int hg_tensor_aca_rect_order_f32(const float* src, const float* tar, float* H, int64_t B,
                                 const float* scale, int64_t scale_sb, int64_t scale_sr,
                                 const float* div, int64_t div_sb, int64_t div_sr, int order,
                                 void* stream) {
    if (order == HG_ORDER_ATEN_CPU)
        return hg_tensor_aca_rect_bcast_f32(src, tar, H, B, scale, scale_sb, scale_sr, div, div_sb,
                                            div_sr, stream);
    if (order != HG_ORDER_ATEN_ROCM || B < 0) return hg::kErrInvalid;
    if (B == 0) return 0;
    if (!src || !tar || !H || !scale || !div) return hg::kErrInvalid;
    const hg::RectBcast a{scale, scale_sb, scale_sr, div, div_sb, div_sr};
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (hg::aligned16(src) && hg::aligned16(tar) && hg::aligned16(H)) {
        const unsigned g = (unsigned)hg::ceil_div(B, hg::kBlock);
        if (B * 140 > hg::kMallResidentBytes)
            return hg::launch(hg::tensor_aca_rect_bcast_staged<true, hg::kAtenRocm>, g, hg::kBlock, 0,
                              s, src, tar, H, B, a);
        return hg::launch(hg::tensor_aca_rect_bcast_staged<false, hg::kAtenRocm>, g, hg::kBlock, 0, s,
                          src, tar, H, B, a);
    }
    return hg::launch(hg::tensor_aca_rect_bcast_kernel<hg::kAtenRocm>, hg::generic_grid(B), hg::kBlock,
                      0, s, src, tar, H, B, a);
}

int hg_tensor_aca_rect_backward_order_f32(const float* src, const float* tar, const float* grad_H,
                                          int64_t B, const float* scale, int64_t scale_sb,
                                          int64_t scale_sr, const float* div, int64_t div_sb,
                                          int64_t div_sr, float* grad_src, float* grad_tar,
                                          float* grad_scale, int scale_rows, float* grad_div,
                                          int div_rows, int order, void* stream) {
    if (order == HG_ORDER_ATEN_CPU)
        return hg_tensor_aca_rect_bcast_backward_f32(src, tar, grad_H, B, scale, scale_sb, scale_sr,
                                                     div, div_sb, div_sr, grad_src, grad_tar,
                                                     grad_scale, scale_rows, grad_div, div_rows,
                                                     stream);
    if (order != HG_ORDER_ATEN_ROCM || B < 0) return hg::kErrInvalid;
    if (B == 0) return 0;
    if (!src || !tar || !grad_H || !scale || !div || !grad_tar) return hg::kErrInvalid;
    if (scale_rows < 0 || scale_rows > 2 || div_rows < 0 || div_rows > 2) return hg::kErrInvalid;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // one value each, with (B,3) terms side by side (or none): the one-value backward's staged
    // form, which writes them as one (2,B,3) buffer
    const bool uniform = !scale_sb && !scale_sr && !div_sb && !div_sr;
    const bool paired = (!grad_scale && !grad_div) ||
                        (grad_scale && grad_div == grad_scale + 3 * B && scale_rows == 2 &&
                         div_rows == 2);
    if (uniform && paired)
        return hg::launch_rect_backward<hg::kAtenRocm, hg::kSdTerms>(src, tar, grad_H, B, scale, div,
                                                                    grad_src, grad_tar, grad_scale, s);
    const hg::RectBcast a{scale, scale_sb, scale_sr, div, div_sb, div_sr};
    return hg::launch(hg::tensor_aca_rect_bcast_backward_kernel<hg::kAtenRocm>, hg::generic_grid(B),
                      hg::kBlock, 0, s, src, tar, grad_H, B, a, grad_src, grad_tar, grad_scale,
                      scale_rows, grad_div, div_rows);
}

int hg_tensor_aca_offsets_f32(const float* corner, const float* offsets, float* H, int64_t B,
                              float width, float height, void* stream) {
    if (B < 0) return hg::kErrInvalid;
    if (B == 0) return 0;
    if (!corner || !offsets || !H) return hg::kErrInvalid;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    constexpr int P = hg::kRectP;
    const int64_t blocks = hg::ceil_div(B, (int64_t)hg::kBlock * P);
    if (blocks > 0x7fffffffLL) return hg::kErrInvalid;
    const bool vec = hg::aligned16(corner) && hg::aligned16(offsets) && hg::aligned16(H);
    // width / height == 1 exactly iff the two are equal, finite and non-zero
    const bool square = width == height && width != 0.f && std::isfinite(width);
    const bool cached = B * 76 <= hg::kMallResidentBytes;  // policy by size, as launch_solver
#define HG_OFFSETS(V, SQ, NT)                                                                 \
    hg::launch(hg::tensor_aca_offsets_kernel<P, V, SQ, NT>, (unsigned)blocks, hg::kBlock, 0, s, \
               corner, offsets, H, B, width, height)
    if (vec && square) return cached ? HG_OFFSETS(true, true, false) : HG_OFFSETS(true, true, true);
    if (vec) return cached ? HG_OFFSETS(true, false, false) : HG_OFFSETS(true, false, true);
    return HG_OFFSETS(false, false, true);  // unaligned views: per-lane loads and stores
#undef HG_OFFSETS
}

int hg_tensor_aca_offsets_backward_f32(const float* corner, const float* offsets,
                                       const float* grad_H, int64_t B, float width,
                                       float height, float* grad_offsets, float* grad_corner,
                                       void* stream) {
    if (B < 0) return hg::kErrInvalid;
    if (B == 0) return 0;
    if (!corner || !offsets || !grad_H || !grad_offsets) return hg::kErrInvalid;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    using hg::aligned16;
    if (aligned16(corner) && aligned16(offsets) && aligned16(grad_H) && aligned16(grad_offsets) &&
        (reinterpret_cast<uintptr_t>(grad_corner) & 7u) == 0) {
        const unsigned g = (unsigned)hg::ceil_div(B, hg::kBlock);
        const bool nt = B * 116 > hg::kMallResidentBytes;
#define HG_OB(C, NT)                                                                          \
    hg::launch(hg::tensor_aca_offsets_backward_staged<C, NT>, g, hg::kBlock, 0, s, corner,      \
               offsets, grad_H, B, width, height, grad_offsets, grad_corner)
        if (grad_corner) return nt ? HG_OB(true, true) : HG_OB(true, false);
        return nt ? HG_OB(false, true) : HG_OB(false, false);
#undef HG_OB
    }
    const unsigned g = hg::generic_grid(B);
    if (grad_corner)
        return hg::launch(hg::tensor_aca_offsets_backward_kernel<true>, g, hg::kBlock, 0, s, corner,
                          offsets, grad_H, B, width, height, grad_offsets, grad_corner);
    return hg::launch(hg::tensor_aca_offsets_backward_kernel<false>, g, hg::kBlock, 0, s, corner,
                      offsets, grad_H, B, width, height, grad_offsets, nullptr);
}

int hg_aca_backward_f32(const float* src, const float* tar, const float* grad_H, int64_t n,
                        float* grad_src, float* grad_tar, void* stream) {
    if (n < 0) return hg::kErrInvalid;
    if (n == 0) return 0;
    if (!src || !tar || !grad_H || (!grad_src && !grad_tar)) return hg::kErrInvalid;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    using hg::aligned16;
    if (aligned16(src) && aligned16(tar) && aligned16(grad_H) &&
        (!grad_src || aligned16(grad_src)) && (!grad_tar || aligned16(grad_tar))) {
        const unsigned g = (unsigned)hg::ceil_div(n, hg::kBlock);
        const bool nt = n * 164 > hg::kMallResidentBytes;
#define HG_VB(S, T, NT)                                                                        \
    hg::launch(hg::aca_vanilla_backward_staged<S, T, NT>, g, hg::kBlock, 0, s, src, tar, grad_H, \
               n, grad_src, grad_tar)
        if (grad_src && grad_tar) return nt ? HG_VB(true, true, true) : HG_VB(true, true, false);
        if (grad_src) return nt ? HG_VB(true, false, true) : HG_VB(true, false, false);
        return nt ? HG_VB(false, true, true) : HG_VB(false, true, false);
#undef HG_VB
    }
    return hg::launch(hg::aca_vanilla_backward_kernel<float>, hg::generic_grid(n), hg::kBlock, 0,
                      s, src, tar, grad_H, n, grad_src, grad_tar);
}

int hg_aca_backward_f64(const double* src, const double* tar, const double* grad_H, int64_t n,
                        double* grad_src, double* grad_tar, void* stream) {
    if (n < 0) return hg::kErrInvalid;
    if (n == 0) return 0;
    if (!src || !tar || !grad_H || (!grad_src && !grad_tar)) return hg::kErrInvalid;
    return hg::launch(hg::aca_vanilla_backward_kernel<double>, hg::generic_grid(n), hg::kBlock, 0,
                      reinterpret_cast<hipStream_t>(stream), src, tar, grad_H, n, grad_src,
                      grad_tar);
}

int hg_fill_uniform_f32(float* out, int64_t count, uint64_t seed, uint64_t offset, float lo,
                        float hi, void* stream) {
    if (count < 0) return hg::kErrInvalid;
    if (count == 0) return 0;
    if (!out) return hg::kErrInvalid;
    return hg::launch(hg::fill_uniform_kernel, hg::generic_grid(count), hg::kBlock, 0,
                      reinterpret_cast<hipStream_t>(stream), out, count, seed, offset, lo, hi);
}

int hg_stream_copy(const void* src, void* dst, int64_t bytes, void* stream) {
    if (bytes < 0 || (bytes & 15)) return hg::kErrInvalid;
    if (bytes == 0) return 0;
    if (!src || !dst || !hg::aligned16(src) || !hg::aligned16(dst)) return hg::kErrInvalid;
    const int64_t n16 = bytes / 16;
    const int64_t want = hg::ceil_div(n16, hg::kBlock * 4);
    const unsigned g = (unsigned)(want < 16384 ? (want > 0 ? want : 1) : 16384);
    return hg::launch(hg::stream_copy_kernel, g, hg::kBlock, 0, reinterpret_cast<hipStream_t>(stream),
                      reinterpret_cast<const hg::u32x4*>(src), reinterpret_cast<hg::u32x4*>(dst),
                      n16);
}

int hg_solve_one_f32(int algo, const float* src, const float* tar, float* H, int flags,
                     void* stream) {
    return hg::launch_one<float>(algo, src, tar, H, flags, stream);
}

int hg_solve_one_f64(int algo, const double* src, const double* tar, double* H, int flags,
                     void* stream) {
    return hg::launch_one<double>(algo, src, tar, H, flags, stream);
}

int hg_sum_rows_f32(float* x, int64_t rows, int64_t cols, float* out, void* stream) {
    if (rows < 0 || cols < 0) return hg::kErrInvalid;
    if (rows == 0) return 0;
    if (!out || (cols > 0 && !x) || rows > 65535) return hg::kErrInvalid;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t chunks = hg::ceil_div(cols, hg::kSumChunk);
    if (chunks > 0x7fffffffLL) return hg::kErrInvalid;
    if (chunks > 0) {
        const int rc = hg::launch(hg::sum_rows_pass1, dim3((unsigned)chunks, (unsigned)rows),
                                  hg::kBlock, 0, s, x, cols);
        if (rc) return rc;
    }
    return hg::launch(hg::sum_rows_pass2, (unsigned)rows, hg::kBlock, 0, s, x, cols, chunks, out);
}

}  // extern "C"

namespace hg {
// ATen's setReduceConfig (ATen/native/hip/Reduce.cuh, torch 2.10) for the two iterators
// at::sum_to builds from a contiguous (B,3,1) float tensor: kind 0 -- one dimension of 3B
// reduced to one output; kind 1 (B >= 2) -- B reduced (stride 3) for each of 3 outputs.
// Restated in oracle/aten_rocm_sum.py's Config, which the fixture pins.
inline int64_t rocm_last_pow2(int64_t n) {
    if (n <= 1) return 1;
    int64_t p = 1;
    while (p <= n / 2) p <<= 1;
    return p;
}

inline RocmSum rocm_sum_config(const float* x, int64_t B, int kind, int num_mp, int max_tpm) {
    RocmSum a{};
    a.x = x;
    const bool fastest = kind == 0;
    int64_t dim0, dim1;
    if (fastest) {
        a.num_in = 3 * B;
        a.num_out = 1;
        a.in_stride = 1;
        a.out_stride = 0;
        dim0 = a.num_in;
        dim1 = 1;
        a.vec = dim0 >= 128;
        if (a.vec) dim0 /= 4;
    } else {
        a.num_in = B;
        a.num_out = 3;
        a.in_stride = 3;
        a.out_stride = 1;
        dim0 = 3;  // output vectors: 3 outputs give a vector size of 1
        dim1 = B;
        a.vec = 0;
    }
    const int64_t d0 = dim0 < kRocmSumThreads ? rocm_last_pow2(dim0) : kRocmSumThreads;
    const int64_t d1 = dim1 < kRocmSumThreads ? rocm_last_pow2(dim1) : kRocmSumThreads;
    int64_t bw = d0 < kWave ? d0 : kWave;
    const int64_t bh = d1 < kRocmSumThreads / bw ? d1 : kRocmSumThreads / bw;
    bw = d0 < kRocmSumThreads / bh ? d0 : kRocmSumThreads / bh;
    a.bw = (int)bw;
    a.bh = (int)bh;
    a.step_in = a.step_out = 1;
    auto split_in = [&](int64_t p) { const int64_t s0 = a.step_in; a.step_in *= p; return s0; };
    auto split_out = [&](int64_t p) { const int64_t s0 = a.step_out; a.step_out *= p; return s0; };
    if (fastest) a.in_mult[0] = split_in(bw);
    else a.out_mult[0] = split_out(bw);
    const int64_t thr = bh * 16 < 256 ? bh * 16 : 256;
    if (ceil_div(a.num_in, a.step_in) >= thr) a.in_mult[1] = split_in(bh);  // 256 CUs: no
    else a.out_mult[1] = split_out(bh);                                     // forced output split
    a.ctas = 1;
    const int64_t gx = ceil_div((int64_t)a.num_out, a.step_out);
    int tpm = max_tpm;
    if (gx != 1) tpm = fastest ? 512 : 256;  // ATen's `grid().x == grid().y == grid().z == 1`
    const int64_t target = (int64_t)num_mp * (tpm / (bw * bh));
    const int64_t vpt = ceil_div(a.num_in, a.step_in);
    if (a.in_mult[1] != 0 && vpt >= 256 && gx <= target) {
        const int64_t c1 = ceil_div(target, gx), c2 = ceil_div(vpt, (int64_t)16);
        const int64_t c3 = ceil_div(vpt, (int64_t)256);
        int64_t c = c1 < c2 ? c1 : c2;
        c = c > c3 ? c : c3;
        if (c > num_mp) c = num_mp < 128 ? (int64_t)num_mp * (c > 512 ? 4 : 2) : num_mp;
        else if (c > ceil_div((int64_t)num_mp, (int64_t)2)) c = ceil_div((int64_t)num_mp, (int64_t)2);
        else if (c < 16) c = 1;
        a.ctas = (int)c;
        if (c > 1) a.in_mult[2] = split_in(c);
    }
    return a;
}
}  // namespace hg

extern "C" {

int hg_sum_rocm_plan(int64_t B, int kind, int num_mp, int max_tpm, int64_t* plan) {
    if (B < 2 || (kind != HG_SUM_ROCM_FULL && kind != HG_SUM_ROCM_COLS) || num_mp < 1 ||
        max_tpm < 1 || !plan)
        return hg::kErrInvalid;
    const hg::RocmSum a = hg::rocm_sum_config(nullptr, B, kind, num_mp, max_tpm);
    const int64_t v[12] = {a.bw, a.bh, a.ctas, a.in_mult[0], a.in_mult[1], a.in_mult[2],
                           a.out_mult[0], a.out_mult[1], a.step_in, a.step_out, a.vec,
                           hg::ceil_div((int64_t)a.num_out, a.step_out)};
    for (int i = 0; i < 12; ++i) plan[i] = v[i];
    return 0;
}

int hg_sum_rocm_f32(const float* x, int64_t B, int kind, float* out, float* workspace,
                    void* stream) {
    if (B < 0 || (kind != HG_SUM_ROCM_FULL && kind != HG_SUM_ROCM_COLS) || !out)
        return hg::kErrInvalid;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int nout = kind == HG_SUM_ROCM_FULL ? 1 : 3;
    if (B == 0) return (int)hipMemsetAsync(out, 0, nout * sizeof(float), s);  // sums of nothing: +0
    if (!x) return hg::kErrInvalid;
    if (kind == HG_SUM_ROCM_COLS && B == 1)
        return hg::launch(hg::rocm_sum_single_kernel, 1u, 64u, 0, s, x, out);
    if (3 * B > 0x7fffffffLL) return hg::kErrInvalid;  // ATen splits beyond 32-bit indexing
    int dev = 0, num_mp = 0, max_tpm = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&num_mp, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipDeviceGetAttribute(&max_tpm, hipDeviceAttributeMaxThreadsPerMultiProcessor, dev) !=
            hipSuccess)
        return (int)hipErrorInvalidDevice;
    hg::RocmSum a = hg::rocm_sum_config(x, B, kind, num_mp, max_tpm);
    a.aligned = hg::aligned16(x);
    if (a.ctas > hg::kRocmSumMaxCtas) return hg::kErrInvalid;
    // CTA partials exist only for the one-output (FULL) reduction: the (3,1) form's output
    // split leaves one CTA per output (ATen's shape), and its partials would be indexed by
    // blockIdx.y past a 3-float output
    if (a.ctas > 1 && kind != HG_SUM_ROCM_FULL) return hg::kErrInvalid;
    const dim3 block((unsigned)a.bw, (unsigned)a.bh);
    const dim3 grid((unsigned)hg::ceil_div((int64_t)a.num_out, a.step_out), (unsigned)a.ctas);
    if (a.ctas == 1) return hg::launch(hg::rocm_sum_kernel, grid, block, 0, s, a, out);
    if (!workspace) return hg::kErrInvalid;
    const int rc = hg::launch(hg::rocm_sum_kernel, grid, block, 0, s, a, workspace);
    if (rc) return rc;
    return hg::launch(hg::rocm_sum_final_kernel, dim3(1), block, 0, s, a,
                      static_cast<const float*>(workspace), out);
}

}  // extern "C"

namespace hg {
// The ATen-order sum's runs of rows x m floats (hg_sum_aten_f32's chunking: min(T, ceil(m /
// 32768)) chunks of ceil(m / chunks) with T threads and m >= 32768, else one).
inline AtenSum aten_sum_of(float* x, int64_t m, int64_t row_stride, int64_t elem_stride,
                           int lanes, int threads) {
    const int64_t want = ceil_div(m, kAtenGrain);
    const int64_t chunks = threads > 1 && m >= kAtenGrain ? (want < threads ? want : threads) : 1;
    return AtenSum{x, row_stride, elem_stride, m, chunks > 1 ? ceil_div(m, chunks) : m,
                   (int)chunks, lanes};
}

// Levels 1 ... 4 of the sum over `rows` rows of a; `blocks_done`: level 0 already folded
// in place (rect_backward_sum_l0), so level 1 reads block sums (aten_sum_l1_blocks).
inline int aten_sum_launch(const AtenSum& a, int64_t rows, int threads, int lanes, float* out,
                           hipStream_t s, bool blocks_done) {
    const int64_t runs = rows * a.chunks;
    if (runs > 65535) return kErrInvalid;
    // The grids cover the largest extent over EVERY run: a shorter run (the last chunk) may
    // take a smaller level step and so have more super-blocks / level-2 groups than run 0.
    int64_t g1_max = -1, l2_max = 0, step_max = 0;
    for (int64_t run = 0; run < runs; ++run) {
        const AtenRun r(a, (int)run);
        if (r.step > kAtenMaxStep) return kErrInvalid;  // a run of > 2^35 rows per stream
        if (r.nb > 0 && r.g1 > g1_max) g1_max = r.g1;
        if (r.g1 > 0 && (r.g2 + 1) * r.S > l2_max) l2_max = (r.g2 + 1) * r.S;
        if (r.step * r.S > step_max) step_max = r.step * r.S;
    }
    if (g1_max >= 0) {
        const int64_t bx = g1_max + 1;  // one block per super-block (the last may be partial)
        if (bx > 0x7fffffffLL) return kErrInvalid;
        const int rc = blocks_done
                           ? launch(aten_sum_l1_blocks, dim3((unsigned)bx, (unsigned)runs), 64, 0, s, a)
                           : launch(aten_sum_l1, dim3((unsigned)bx, (unsigned)runs), kAtenL1Threads,
                                    (size_t)step_max * sizeof(float), s, a);
        if (rc) return rc;
    }
    if (l2_max > 0) {
        const int64_t bx = ceil_div(l2_max, (int64_t)256);
        if (bx > 0x7fffffffLL) return kErrInvalid;
        const int rc = launch(aten_sum_l2, dim3((unsigned)bx, (unsigned)runs), 256, 0, s, a);
        if (rc) return rc;
    }
    const int rc = launch(aten_sum_l3, (unsigned)runs, 64, 0, s, a, out);
    if (rc || a.chunks == 1) return rc;
    return launch(aten_sum_l4, (unsigned)rows, 64, 0, s, a, threads, lanes, out);
}

inline bool aten_sum_args_ok(int lanes, int threads) {
    return lanes >= 1 && lanes <= kAtenMaxLanes && threads >= 1 && threads <= kAtenMaxThreads &&
           (threads == 1 || lanes >= 4);
}
}  // namespace hg

extern "C" {

int hg_sum_aten_f32(float* x, int64_t rows, int64_t m, int64_t row_stride, int64_t elem_stride,
                    int lanes, int threads, float* out, void* stream) {
    if (rows < 0 || m < 0 || !hg::aten_sum_args_ok(lanes, threads)) return hg::kErrInvalid;
    if (rows == 0) return 0;
    if (!out || (m > 0 && !x)) return hg::kErrInvalid;
    const hg::AtenSum a = hg::aten_sum_of(x, m, row_stride, elem_stride, lanes, threads);
    return hg::aten_sum_launch(a, rows, threads, lanes, out, reinterpret_cast<hipStream_t>(stream),
                               false);
}

}  // extern "C"

namespace hg {
// The fused kernel's shape (hg_internal_rect_sum_config; tools/kbench_rect_sum.py): floats of
// each parameter's terms per workgroup.
inline int g_rect_sum_budget = kRectSumBudget;

// level0_only: the fused backward kernel alone (its block sums left in the workspace) -- for
// the bench's op-over-kernel figure (hg_internal_rect_backward_sum_l0).
inline int rect_backward_sum(const float* src, const float* tar, const float* grad_H, int64_t B,
                             const float* scale, const float* div, float* grad_src,
                             float* grad_tar, float* workspace, int lanes, int threads,
                             float* grad_sd, hipStream_t s, bool level0_only);
}  // namespace hg

extern "C" {

// Library-internal (tools/kbench_rect_sum.py): the fused kernel's unit -- floats of each
// parameter's terms a workgroup stages (512 ... 4096, a power of two); a value < 0 leaves it.
// prev[2] receives the settings before (prev[1]: 0, unused).
int hg_internal_rect_sum_config(int budget, int unused, int* prev) {
    (void)unused;
    if (prev) {
        prev[0] = hg::g_rect_sum_budget;
        prev[1] = 0;
    }
    if (budget >= 0 && (budget < 512 || budget > 4096 || (budget & (budget - 1)))) return hg::kErrInvalid;
    if (budget >= 0) hg::g_rect_sum_budget = budget;
    return 0;
}

// Library-internal (bench.py): rect_backward_sum_l0 alone, as hg_tensor_aca_rect_backward_sum_f32
// launches it (aligned tensors only).
int hg_internal_rect_backward_sum_l0(const float* src, const float* tar, const float* grad_H,
                                     int64_t B, const float* scale, const float* div,
                                     float* grad_src, float* grad_tar, float* workspace, int lanes,
                                     int threads, void* stream) {
    float dummy = 0.f;
    return hg::rect_backward_sum(src, tar, grad_H, B, scale, div, grad_src, grad_tar, workspace,
                                 lanes, threads, &dummy, reinterpret_cast<hipStream_t>(stream), true);
}

int hg_tensor_aca_rect_backward_sum_f32(const float* src, const float* tar, const float* grad_H,
                                        int64_t B, const float* scale, const float* div,
                                        float* grad_src, float* grad_tar, float* workspace,
                                        int lanes, int threads, float* grad_sd, void* stream) {
    return hg::rect_backward_sum(src, tar, grad_H, B, scale, div, grad_src, grad_tar, workspace,
                                 lanes, threads, grad_sd, reinterpret_cast<hipStream_t>(stream),
                                 false);
}

}  // extern "C"

namespace hg {
inline int rect_backward_sum(const float* src, const float* tar, const float* grad_H, int64_t B,
                             const float* scale, const float* div, float* grad_src,
                             float* grad_tar, float* workspace, int lanes, int threads,
                             float* grad_sd, hipStream_t s, bool level0_only) {
    if (B < 0 || !hg::aten_sum_args_ok(lanes, threads)) return hg::kErrInvalid;
    if (!grad_sd) return hg::kErrInvalid;
    if (B == 0) return (int)hipMemsetAsync(grad_sd, 0, 2 * sizeof(float), s);  // sums of nothing
    if (!src || !tar || !grad_H || !scale || !div || !grad_tar || !workspace) return hg::kErrInvalid;
    if (B > (int64_t)1 << 40) return hg::kErrInvalid;
    const int64_t m = 3 * B;
    const hg::AtenSum a = hg::aten_sum_of(workspace, m, m, 1, lanes, threads);
    bool fused = hg::aligned16(src) && hg::aligned16(tar) && hg::aligned16(grad_H) &&
                 hg::aligned16(grad_tar) && (!grad_src || hg::aligned16(grad_src));
    for (int c = 0; c < a.chunks && fused; ++c)
        fused = hg::AtenRun(a, c).step <= hg::kRectSumMaxStep;
    if (!fused) {  // the two-launch form: the same bits
        if (level0_only) return hg::kErrInvalid;
        int rc = hg::launch_rect_backward<hg::kAtenCpu, hg::kSdTerms>(
            src, tar, grad_H, B, scale, div, grad_src, grad_tar, workspace, s);
        if (rc) return rc;
        return hg::aten_sum_launch(a, 2, threads, lanes, grad_sd, s, false);
    }
    const int budget = g_rect_sum_budget;
    int64_t units = 0, lds_floats = 0;
    for (int c = 0; c < a.chunks; ++c) {
        const hg::AtenRun r(a, c);
        if (r.step > hg::kAtenMaxStep) return hg::kErrInvalid;
        units = std::max(units, hg::rect_sum_units(r, budget));
        lds_floats = std::max(lds_floats, hg::rect_sum_group(r, budget) * r.step * r.S);
    }
    if (units > 0x7fffffffLL) return hg::kErrInvalid;
    const size_t lds = 2 * (size_t)lds_floats * sizeof(float);  // <= 2 x 4096 floats (step 128)
    const dim3 grid((unsigned)units, (unsigned)a.chunks);
    const bool nt = B * 232 > hg::kMallResidentBytes;
#define HG_RS(W, NT)                                                                          \
    hg::launch(hg::rect_backward_sum_l0<W, NT>, grid, hg::kRectSumThreads, lds, s, src, tar, \
               grad_H, B, scale, div, grad_src, grad_tar, a, budget)
    const int rc = grad_src ? (nt ? HG_RS(true, true) : HG_RS(true, false))
                            : (nt ? HG_RS(false, true) : HG_RS(false, false));
#undef HG_RS
    if (rc || level0_only) return rc;
    return hg::aten_sum_launch(a, 2, threads, lanes, grad_sd, s, true);
}
}  // namespace hg

extern "C" {

const char* hg_version(void) { return "sks-homography-amd 0.3 (gfx950)"; }

}  // extern "C"
