// hg_tune.hip -- variant launcher for tools/kbench.py (not part of the C ABI header;
// declared in include/sks_homography_tune.h).  Every variant computes the same bits
// as the shipped kernel; only the memory schedule differs.
#include <hip/hip_runtime.h>
#include <rocrand/rocrand.h>

#include "hg_aos.hpp"
#include "hg_gather.hpp"
#include "hg_ransac.hpp"
#include "hg_rect.hpp"
#include "hg_soa.hpp"
#include "sks_homography.h"

namespace {

using namespace hg;

struct Variant {
    const char* name;
    int (*launch)(int algo, const float*, const float*, float*, int64_t, int, hipStream_t);
};

template <int P, int FL>
int launch_variant(int algo, const float* s, const float* t, float* H, int64_t n, int per_cu,
                   hipStream_t st) {
    const int64_t g = aos_grid<float, P, FL>(n, per_cu);
    if (algo == 0) solve_aos<kACA, true, float, P, FL><<<(unsigned)g, kBlock, 0, st>>>(s, t, H, n);
    else solve_aos<kSKS, true, float, P, FL><<<(unsigned)g, kBlock, 0, st>>>(s, t, H, n);
    return (int)hipGetLastError();
}

template <int P, int TPW>
int launch_pipe(int algo, const float* s, const float* t, float* H, int64_t n, int,
                hipStream_t st) {
    const int64_t tiles = (n + kWave * P - 1) / (kWave * P);
    const int64_t waves = (tiles + TPW - 1) / TPW;
    const unsigned g = (unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
    if (algo == 0) solve_aos_pipe<kACA, true, P, TPW><<<g, kBlock, 0, st>>>(s, t, H, n);
    else solve_aos_pipe<kSKS, true, P, TPW><<<g, kBlock, 0, st>>>(s, t, H, n);
    return (int)hipGetLastError();
}

const Variant kVariants[] = {
    {"P4 nt-ld nt-st stage (first version)", launch_variant<4, kNtLoad | kNtStore>},
    {"P4 plain", launch_variant<4, 0>},
    {"P4 nt-ld", launch_variant<4, kNtLoad>},
    {"P4 nt-st", launch_variant<4, kNtStore>},
    {"P8 nt-ld nt-st stage", launch_variant<8, kNtLoad | kNtStore>},
    {"P4 nt persist", launch_variant<4, kNtLoad | kNtStore | kPersist>},
    {"P4 nt lds-load", launch_variant<4, kNtLoad | kNtStore | kLdsLoad>},
    {"P8 nt lds-load", launch_variant<8, kNtLoad | kNtStore | kLdsLoad>},
    {"P4 nt direct-st", launch_variant<4, kNtLoad | kNtStore | kDirectSt>},
    {"P2 nt direct-st", launch_variant<2, kNtLoad | kNtStore | kDirectSt>},
    {"P1 nt direct-st", launch_variant<1, kNtLoad | kNtStore | kDirectSt>},
    {"P4 nt lds-load persist", launch_variant<4, kNtLoad | kNtStore | kLdsLoad | kPersist>},
    {"P4 plain lds-load", launch_variant<4, kLdsLoad>},
    {"P2 nt lds-load", launch_variant<2, kNtLoad | kNtStore | kLdsLoad>},
    {"P1 nt lds-load", launch_variant<1, kNtLoad | kNtStore | kLdsLoad>},
    {"P3 nt lds-load", launch_variant<3, kNtLoad | kNtStore | kLdsLoad>},
    {"P4 nt lds-dma", launch_variant<4, kNtLoad | kNtStore | kLdsLoad | kLdsDma>},
    {"P2 nt lds-dma", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma>},
    {"P4 lds-dma nt-st", launch_variant<4, kNtStore | kLdsLoad | kLdsDma>},
    {"P4 nt-ld lds-load plain-st", launch_variant<4, kNtLoad | kLdsLoad>},
    {"P2 nt stage", launch_variant<2, kNtLoad | kNtStore>},
    {"P2 nt lds-dma persist", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kPersist>},
    {"P1 nt lds-dma", launch_variant<1, kNtLoad | kNtStore | kLdsLoad | kLdsDma>},
    {"P2 lds-dma nt-ld plain-st", launch_variant<2, kNtLoad | kLdsLoad | kLdsDma>},
    {"P3 nt lds-dma", launch_variant<3, kNtLoad | kNtStore | kLdsLoad | kLdsDma>},
    {"P2 pipe x2 tiles/wave", launch_pipe<2, 2>},
    {"P2 pipe x4 tiles/wave", launch_pipe<2, 4>},
    {"P2 pipe x8 tiles/wave", launch_pipe<2, 8>},
    {"P1 pipe x4 tiles/wave", launch_pipe<1, 4>},
    {"P2 nt lds-dma xcd-contig", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kXcdMap>},
    {"P1 nt lds-dma xcd-contig", launch_variant<1, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kXcdMap>},
    {"P4 nt lds-dma xcd-contig", launch_variant<4, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kXcdMap>},
    {"P2 lds-dma plain (cached)", launch_variant<2, kLdsLoad | kLdsDma>},
    {"P2 nt lds-dma, sc1|nt buffer stores", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kStSc1>},
    {"P2 nt lds-dma, sc1 buffer stores", launch_variant<2, kNtLoad | kLdsLoad | kLdsDma | kStSc1>},
    // round 2: the input DMA's cache policy and issue order
    {"P2 nt lds-dma, loads sc0|nt", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kLdSc0>},
    {"P2 nt lds-dma, loads sc1|nt", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kLdSc1>},
    {"P2 nt lds-dma, loads sc0|sc1|nt", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kLdSc0 | kLdSc1>},
    {"P2 lds-dma, loads sc1, nt-st", launch_variant<2, kNtStore | kLdsLoad | kLdsDma | kLdSc1>},
    {"P2 nt lds-dma, slab-major issue", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kSlabMajor>},
    {"P4 nt lds-dma, slab-major issue", launch_variant<4, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kSlabMajor>},
    // the shipped kernel's memory pattern with the solver replaced by a copy (not bit-exact by design)
    {"P2 nt lds-dma, NO SOLVE (pattern ceiling)", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kNoSolve>},
};

// Streaming-copy variants for the bandwidth yardstick.
template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void copy_unrolled(const u32x4* __restrict__ src,
                                                        u32x4* __restrict__ dst, int64_t n16) {
    const int64_t base = (int64_t)blockIdx.x * kBlock * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * kBlock;
        if (i < n16) v[u] = ld16<NT>(src + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * kBlock;
        if (i < n16) st16<NT>(dst + i, v[u]);
    }
}

// LDS-DMA copy: each wave moves 8 KiB through LDS per iteration.
__global__ __launch_bounds__(kBlock) void copy_dma(const char* __restrict__ src,
                                                   char* __restrict__ dst, int64_t bytes) {
    constexpr int kSlab = 8192;
    __shared__ __attribute__((aligned(16))) char smem[kWavesPerBlock][kSlab];
    const int lane = threadIdx.x & 63, wave = threadIdx.x / 64;
    const int64_t slab = (int64_t)blockIdx.x * kWavesPerBlock + wave;
    if ((slab + 1) * kSlab > bytes) return;
    const char* const g[1] = {src + slab * kSlab};
    char* const l[1] = {smem[wave]};
    slabs_to_lds<kSlab, 1, true, true>(g, l, lane);
#pragma unroll
    for (int c = 0; c < kSlab / 1024; ++c)
        st16<true>(dst + slab * kSlab + 16 * (c * 64 + lane),
                   *reinterpret_cast<const u32x4*>(smem[wave] + 16 * (c * 64 + lane)));
}

template <typename T, int G, bool PERSIST, bool NT = true>
int launch_soa(int algo, const void* s, const void* t, void* H, int64_t n, int per_cu,
               hipStream_t st) {
    constexpr int V = 16 / sizeof(T);
    if (n % V) return (int)hipErrorInvalidValue;
    const unsigned g = (unsigned)soa_grid<G, PERSIST>(n / V, per_cu);
    const T* a = (const T*)s;
    const T* b = (const T*)t;
    T* h = (T*)H;
    if (algo == 0) solve_soa_vec<kACA, false, T, G, PERSIST, NT><<<g, kBlock, 0, st>>>(a, b, h, n);
    else if (algo == 1) solve_soa_vec<kSKS, false, T, G, PERSIST, NT><<<g, kBlock, 0, st>>>(a, b, h, n);
    else if constexpr (sizeof(T) == 8) {  // the baselines (tools/kbench_gpt.py)
        if (algo == 2) solve_soa_vec<kGE, false, T, G, PERSIST, NT><<<g, kBlock, 0, st>>>(a, b, h, n);
        else solve_soa_vec<kGPT, false, T, G, PERSIST, NT><<<g, kBlock, 0, st>>>(a, b, h, n);
    } else return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}

template <typename T>
int launch_soa_dma(int algo, const void* s, const void* t, void* H, int64_t n, int,
                   hipStream_t st) {
    constexpr int V = 16 / sizeof(T);
    if (n % V) return (int)hipErrorInvalidValue;
    const int64_t tile = (int64_t)kWave * V * kWavesPerBlock;
    const unsigned g = (unsigned)((n + tile - 1) / tile);
    const T* a = (const T*)s;
    const T* b = (const T*)t;
    T* h = (T*)H;
    if (algo == 0) solve_soa_dma<kACA, false, T, true><<<g, kBlock, 0, st>>>(a, b, h, n);
    else solve_soa_dma<kSKS, false, T, true><<<g, kBlock, 0, st>>>(a, b, h, n);
    return (int)hipGetLastError();
}

template <typename T, int W, bool NT = true>
int launch_soa_narrow(int algo, const void* s, const void* t, void* H, int64_t n, int,
                      hipStream_t st) {
    constexpr int V = W / sizeof(T);
    if (n % V) return (int)hipErrorInvalidValue;
    const unsigned g = (unsigned)((n / V + kBlock - 1) / kBlock);
    const T* a = (const T*)s;
    const T* b = (const T*)t;
    T* h = (T*)H;
    if (algo == 0) solve_soa_narrow<kACA, false, T, W, NT><<<g, kBlock, 0, st>>>(a, b, h, n);
    else if (algo == 1) solve_soa_narrow<kSKS, false, T, W, NT><<<g, kBlock, 0, st>>>(a, b, h, n);
    else if constexpr (sizeof(T) == 8) {
        if (algo == 2) solve_soa_narrow<kGE, false, T, W, NT><<<g, kBlock, 0, st>>>(a, b, h, n);
        else solve_soa_narrow<kGPT, false, T, W, NT><<<g, kBlock, 0, st>>>(a, b, h, n);
    } else return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}

template <typename T, int SEG, int WAVES, bool XCD, bool NOSOLVE>
int launch_soa_seg(int algo, const void* s, const void* t, void* H, int64_t n, int,
                   hipStream_t st) {
    constexpr int64_t kTile = SEG / (int)sizeof(T);
    const unsigned g = (unsigned)((n + kTile - 1) / kTile);
    const T* a = (const T*)s;
    const T* b = (const T*)t;
    T* h = (T*)H;
    if (algo == 0) solve_soa_seg<kACA, false, T, SEG, WAVES, XCD, NOSOLVE><<<g, 64 * WAVES, 0, st>>>(a, b, h, n);
    else solve_soa_seg<kSKS, false, T, SEG, WAVES, XCD, NOSOLVE><<<g, 64 * WAVES, 0, st>>>(a, b, h, n);
    return (int)hipGetLastError();
}

struct SoaVariant {
    const char* name;
    int (*launch)(int, const void*, const void*, void*, int64_t, int, hipStream_t);
};

const SoaVariant kSoaVariants[] = {
    {"f64 G1 one-shot (shipped)", launch_soa<double, 1, false>},
    {"f64 G2 one-shot", launch_soa<double, 2, false>},
    {"f64 G1 persist", launch_soa<double, 1, true>},
    {"f64 G2 persist", launch_soa<double, 2, true>},
    {"f32 G1 one-shot (shipped)", launch_soa<float, 1, false>},
    {"f32 G2 one-shot", launch_soa<float, 2, false>},
    {"f32 G1 persist", launch_soa<float, 1, true>},
    {"f64 G1 one-shot plain (cached) ld/st", launch_soa<double, 1, false, false>},
    {"f32 G1 one-shot plain (cached) ld/st", launch_soa<float, 1, false, false>},
    {"f64 LDS-DMA tile nt", launch_soa_dma<double>},
    {"f32 LDS-DMA tile nt", launch_soa_dma<float>},
    {"f32 narrow W4 (1 problem per lane)", launch_soa_narrow<float, 4>},
    {"f32 narrow W8 (2 problems per lane)", launch_soa_narrow<float, 8>},
    {"f64 narrow W8 (1 problem per lane)", launch_soa_narrow<double, 8>},
    {"f64 narrow W8 plain (cached) ld/st", launch_soa_narrow<double, 8, false>},
    {"f32 narrow W4 plain (cached) ld/st", launch_soa_narrow<float, 4, false>},
    // block-contiguous row segments (solve_soa_seg): SEG bytes of every row per block
    {"f64 seg 2K w1", launch_soa_seg<double, 2048, 1, false, false>},
    {"f64 seg 2K w2", launch_soa_seg<double, 2048, 2, false, false>},
    {"f64 seg 4K w1", launch_soa_seg<double, 4096, 1, false, false>},
    {"f64 seg 4K w2", launch_soa_seg<double, 4096, 2, false, false>},
    {"f64 seg 4K w4", launch_soa_seg<double, 4096, 4, false, false>},
    {"f64 seg 8K w2", launch_soa_seg<double, 8192, 2, false, false>},
    {"f64 seg 8K w4", launch_soa_seg<double, 8192, 4, false, false>},
    {"f64 seg 2K w1 xcd", launch_soa_seg<double, 2048, 1, true, false>},
    {"f64 seg 4K w2 xcd", launch_soa_seg<double, 4096, 2, true, false>},
    {"f64 seg 4K w4 xcd", launch_soa_seg<double, 4096, 4, true, false>},
    {"f64 seg 8K w4 xcd", launch_soa_seg<double, 8192, 4, true, false>},
    {"f64 seg 2K w1 nosolve", launch_soa_seg<double, 2048, 1, false, true>},
    {"f64 seg 4K w2 nosolve", launch_soa_seg<double, 4096, 2, false, true>},
    {"f64 seg 4K w4 nosolve", launch_soa_seg<double, 4096, 4, false, true>},
    {"f64 seg 8K w4 nosolve", launch_soa_seg<double, 8192, 4, false, true>},
    {"f64 seg 4K w4 xcd nosolve", launch_soa_seg<double, 4096, 4, true, true>},
    {"f32 seg 4K w2", launch_soa_seg<float, 4096, 2, false, false>},
    {"f32 seg 4K w4 xcd", launch_soa_seg<float, 4096, 4, true, false>},
};

// The HBM ceilings either side of a copy: read-only (every 16-B load folded into a
// per-lane XOR, one dword out per lane) and write-only (a constant).
template <int U>
__global__ __launch_bounds__(kBlock) void read_only(const u32x4* __restrict__ src,
                                                    uint32_t* __restrict__ sink, int64_t n16) {
    const int64_t base = (int64_t)blockIdx.x * kBlock * U + threadIdx.x;
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * kBlock;
        if (i < n16) {
            const u32x4 v = ld16<true>(src + i);
            acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
        }
    }
    sink[(int64_t)blockIdx.x * kBlock + threadIdx.x] = acc;
}

template <int U>
__global__ __launch_bounds__(kBlock) void write_only(u32x4* __restrict__ dst, int64_t n16) {
    const int64_t base = (int64_t)blockIdx.x * kBlock * U + threadIdx.x;
    const u32x4 v = {1u, 2u, 3u, 4u};
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * kBlock;
        if (i < n16) st16<true>(dst + i, v);
    }
}

// Row-stream probe (tools/soa_streams.py): RI input rows and RO output rows of row16
// 16-B chunks each, at a row pitch of pitch16 chunks; a lane reads chunk q of every input
// row (U chunks per lane, kBlock apart) and writes their XOR to chunk q of every output
// row -- the SoA solver's access pattern with the arithmetic taken out.
template <int RI, int RO, int U>
__global__ __launch_bounds__(kBlock) void row_streams(const u32x4* __restrict__ in,
                                                      u32x4* __restrict__ out, int64_t row16,
                                                      int64_t pitch16) {
    const int64_t base = (int64_t)blockIdx.x * kBlock * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t q = base + (int64_t)u * kBlock;
        if (q >= row16) break;
        u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < RI; ++k) acc ^= ld16<true>(in + k * pitch16 + q);
#pragma unroll
        for (int k = 0; k < RO; ++k) st16<true>(out + k * pitch16 + q, acc + (uint32_t)k);
    }
}

// Cache-policy probe (tools/hbm_policy.py): 16-B buffer stores / loads with explicit aux
// bits (gfx950: 1 = sc0, 2 = nt, 16 = sc1) over a 1 GB stream, U chunks per lane.
template <int AUX, int U>
__global__ __launch_bounds__(kBlock) void write_policy(char* __restrict__ dst, int64_t n16) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
    const int64_t base = (int64_t)blockIdx.x * kBlock * U + threadIdx.x;
    const u32x4 v = {1u, 2u, 3u, 4u};
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * kBlock;
        if (i < n16) __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, (int)(i * 16), 0, AUX);
    }
}

template <int AUX, int U>
__global__ __launch_bounds__(kBlock) void read_policy(const char* __restrict__ src,
                                                      uint32_t* __restrict__ sink, int64_t n16) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src), 0, 0x7fffffff,
                                                        0x00020000);
    const int64_t base = (int64_t)blockIdx.x * kBlock * U + threadIdx.x;
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * kBlock;
        if (i < n16) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(i * 16), 0, AUX);
            acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
        }
    }
    sink[(int64_t)blockIdx.x * kBlock + threadIdx.x] = acc;
}

__global__ void empty_kernel() {}
__global__ void store_one_kernel(uint32_t* p) {
    if (threadIdx.x == 0) p[0] = 1u;
}
// The same one-dword store under each cache policy (launch-floor probe: is the ~1.2 us a
// written kernel costs over an empty one the end-of-kernel L2 writeback of dirty lines?)
template <int POL>
__global__ void store_one_policy_kernel(uint32_t* p) {
    if (threadIdx.x != 0) return;
    const uint32_t v = 1u;
    if constexpr (POL == 0)
        asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 1)
        asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 2)
        asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    else
        __builtin_nontemporal_store(v, p);
}
__global__ void args_unused_kernel(const uint32_t*, uint32_t*) {}
// reads its kernel arguments (s_load from the kernarg segment) but touches no other memory
__global__ void args_read_kernel(uint64_t a, uint64_t b) {
    if (a == b + 12345u) __builtin_amdgcn_s_sleep(1);
}
__global__ void load_one_kernel(const uint32_t* p, uint32_t* never) {
    const uint32_t v = p[threadIdx.x];
    if (v == 0xdeadbeefu && threadIdx.x == 65) never[0] = v;  // never taken: no store
}
// one lane per problem, plain loads/stores (the latency probe's generic form)
template <int ALGO, bool NORM, typename T, bool SOA>
__global__ __launch_bounds__(kBlock) void solve_generic_t(const T* __restrict__ src,
                                                          const T* __restrict__ tar,
                                                          T* __restrict__ H, int64_t n) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
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

// q[i] = a[i] / b[i], two elements per lane as the halves of one f32x2 (div_rn): PK = true
// the packed expansion the samplers ship, false the compiler's two scalar divisions.
template <bool PK>
__global__ __launch_bounds__(kBlock) void div_pairs_kernel(const float* __restrict__ a,
                                                           const float* __restrict__ b,
                                                           float* __restrict__ q, int64_t pairs) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= pairs) return;
    const f32x2 x = {a[2 * i], a[2 * i + 1]}, y = {b[2 * i], b[2 * i + 1]};
    const f32x2 r = div_rn<PK>(x, y);
    q[2 * i] = r.x;
    q[2 * i + 1] = r.y;
}

}  // namespace

extern "C" {

/* q = a / b elementwise, n even, in pairs as the RANSAC samplers divide (packed != 0: the
 * shipped packed expansion; 0: the compiler's scalar divisions) -- the division's own test. */
int hg_tune_div_pairs(int packed, const float* a, const float* b, float* q, int64_t n,
                      void* stream) {
    if (n <= 0 || (n & 1) || !a || !b || !q) return (int)hipErrorInvalidValue;
    const int64_t pairs = n / 2;
    const unsigned g = (unsigned)((pairs + kBlock - 1) / kBlock);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (packed) div_pairs_kernel<true><<<g, kBlock, 0, st>>>(a, b, q, pairs);
    else div_pairs_kernel<false><<<g, kBlock, 0, st>>>(a, b, q, pairs);
    return (int)hipGetLastError();
}

int hg_tune_num_soa_variants(void) { return (int)(sizeof(kSoaVariants) / sizeof(kSoaVariants[0])); }

const char* hg_tune_soa_variant_name(int v) {
    return (v >= 0 && v < hg_tune_num_soa_variants()) ? kSoaVariants[v].name : nullptr;
}

/* SoA unnormalised (the reference GPU semantics); dtype follows the variant. */
int hg_tune_soa(int algo, int variant, const void* src, const void* tar, void* H, int64_t n,
                int per_cu, void* stream) {
    if (variant < 0 || variant >= hg_tune_num_soa_variants() || n <= 0) return (int)hipErrorInvalidValue;
    return kSoaVariants[variant].launch(algo, src, tar, H, n, per_cu > 0 ? per_cu : 8,
                                        reinterpret_cast<hipStream_t>(stream));
}

// variant 0: U=4 nt, 1: U=8 nt, 2: U=4 plain, 3: LDS-DMA (bytes % 32 KiB == 0),
// 4: read-only U=4 (dst receives bytes/64 B of XOR sinks), 5: write-only U=4 (src unused)
int hg_tune_copy(int variant, const void* src, void* dst, int64_t bytes, void* stream) {
    if (bytes <= 0 || (bytes & 15)) return (int)hipErrorInvalidValue;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t n16 = bytes / 16;
    const auto* s = reinterpret_cast<const u32x4*>(src);
    auto* d = reinterpret_cast<u32x4*>(dst);
    switch (variant) {
        case 0: copy_unrolled<4, true><<<(unsigned)((n16 + 1023) / 1024), kBlock, 0, st>>>(s, d, n16); break;
        case 1: copy_unrolled<8, true><<<(unsigned)((n16 + 2047) / 2048), kBlock, 0, st>>>(s, d, n16); break;
        case 2: copy_unrolled<4, false><<<(unsigned)((n16 + 1023) / 1024), kBlock, 0, st>>>(s, d, n16); break;
        case 3:
            if (bytes % 32768) return (int)hipErrorInvalidValue;
            copy_dma<<<(unsigned)(bytes / 32768), kBlock, 0, st>>>((const char*)src, (char*)dst, bytes);
            break;
        case 4: read_only<4><<<(unsigned)((n16 + 1023) / 1024), kBlock, 0, st>>>(s, reinterpret_cast<uint32_t*>(dst), n16); break;
        case 5: write_only<4><<<(unsigned)((n16 + 1023) / 1024), kBlock, 0, st>>>(d, n16); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int hg_tune_num_variants(void) { return (int)(sizeof(kVariants) / sizeof(kVariants[0])); }

const char* hg_tune_variant_name(int v) {
    return (v >= 0 && v < hg_tune_num_variants()) ? kVariants[v].name : nullptr;
}

int hg_tune_aos_f32(int algo, int variant, const float* src, const float* tar, float* H,
                    int64_t n, int per_cu, void* stream) {
    if (variant < 0 || variant >= hg_tune_num_variants() || n <= 0 || (algo != 0 && algo != 1))
        return (int)hipErrorInvalidValue;
    return kVariants[variant].launch(algo, src, tar, H, n, per_cu > 0 ? per_cu : 8,
                                     reinterpret_cast<hipStream_t>(stream));
}

// Cache-policy probe: variant 0-5 = stores with aux 0 / 1 / 2 / 3 / 16 / 18,
// 6-11 = loads with the same aux values (sink: one dword per lane into dst).  bytes < 2 GiB.
int hg_tune_policy(int variant, const void* src, void* dst, int64_t bytes, void* stream) {
    if (bytes <= 0 || (bytes & 15) || bytes >= 0x7fffffffLL) return (int)hipErrorInvalidValue;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t n16 = bytes / 16;
    const unsigned g = (unsigned)((n16 + 4 * kBlock - 1) / (4 * kBlock));
    char* d = reinterpret_cast<char*>(dst);
    const char* s = reinterpret_cast<const char*>(src);
    uint32_t* sink = reinterpret_cast<uint32_t*>(dst);
    switch (variant) {
        case 0: write_policy<0, 4><<<g, kBlock, 0, st>>>(d, n16); break;
        case 1: write_policy<1, 4><<<g, kBlock, 0, st>>>(d, n16); break;
        case 2: write_policy<2, 4><<<g, kBlock, 0, st>>>(d, n16); break;
        case 3: write_policy<3, 4><<<g, kBlock, 0, st>>>(d, n16); break;
        case 4: write_policy<16, 4><<<g, kBlock, 0, st>>>(d, n16); break;
        case 5: write_policy<18, 4><<<g, kBlock, 0, st>>>(d, n16); break;
        case 6: read_policy<0, 4><<<g, kBlock, 0, st>>>(s, sink, n16); break;
        case 7: read_policy<1, 4><<<g, kBlock, 0, st>>>(s, sink, n16); break;
        case 8: read_policy<2, 4><<<g, kBlock, 0, st>>>(s, sink, n16); break;
        case 9: read_policy<3, 4><<<g, kBlock, 0, st>>>(s, sink, n16); break;
        case 10: read_policy<16, 4><<<g, kBlock, 0, st>>>(s, sink, n16); break;
        case 11: read_policy<18, 4><<<g, kBlock, 0, st>>>(s, sink, n16); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

// The one-launch Table-8 kernel's H store pattern alone (no LDS, no barriers): block g owns
// C consecutive residue classes (mod 2^17) and walks their positions Q at a time, lane
// (qq, c) storing the 9 SoA rows of hypothesis g C + c + (q0 + qq) 2^17 (8-B nt stores).
// C = 256, Q = 4 is the shipped kernel's shape.
}  // extern "C"

template <int C>
__global__ __launch_bounds__(1024) void mrg_pattern_kernel(double* __restrict__ H, int64_t n) {
    constexpr int Q = 1024 / C;
    const int qq = threadIdx.x / C, c = threadIdx.x % C;
    const int64_t groups = ((n < (1 << 17) ? n : (1 << 17)) + C - 1) / C;
    for (int64_t g = blockIdx.x; g < groups; g += gridDim.x) {
        const int64_t h0 = g * C + c;
        const int64_t qn = (n - g * C + (1 << 17) - 1) >> 17;
        for (int64_t q0 = 0; q0 < qn; q0 += Q) {
            const int64_t h = h0 + ((q0 + qq) << 17);
            if (h < n) {
#pragma unroll
                for (int r = 0; r < 9; ++r) __builtin_nontemporal_store((double)(h + r), H + h + r * n);
            }
        }
    }
}

// the same 9 SoA rows written in hypothesis order (grid-stride, 8-B nt stores), and one row
// (W = 16: two hypotheses per lane, 16-B stores; NT: non-temporal or default policy)
template <int R, int W = 8, bool NT = true>
__global__ __launch_bounds__(1024) void seq_rows_kernel(double* __restrict__ H, int64_t n) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    constexpr int P = W / 8;
    for (int64_t h = ((int64_t)blockIdx.x * 1024 + threadIdx.x) * P; h < n;
         h += (int64_t)gridDim.x * 1024 * P) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if constexpr (W == 16) {
                const d2 v = {(double)(h + r), (double)(h + r + 1)};
                if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<d2*>(H + h + r * n));
                else *reinterpret_cast<d2*>(H + h + r * n) = v;
            } else {
                if constexpr (NT) __builtin_nontemporal_store((double)(h + r), H + h + r * n);
                else H[h + r * n] = (double)(h + r);
            }
        }
    }
}

extern "C" {

int hg_tune_mrg_pattern(int classes, double* H, int64_t n, void* stream) {
    if (n <= 0 || !H) return (int)hipErrorInvalidValue;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const unsigned grid = (unsigned)hg::cu_count();
    switch (classes) {
        case 0: seq_rows_kernel<9><<<grid * 8, 1024, 0, st>>>(H, n); break;    // 9 rows, h in order
        case 1: seq_rows_kernel<1><<<grid * 8, 1024, 0, st>>>(H, 9 * n); break;  // one row of 9 n
        case 2: seq_rows_kernel<1, 16, true><<<grid * 8, 1024, 0, st>>>(H, 9 * n); break;
        case 3: seq_rows_kernel<1, 8, false><<<grid * 8, 1024, 0, st>>>(H, 9 * n); break;
        case 4: seq_rows_kernel<1, 16, false><<<grid * 8, 1024, 0, st>>>(H, 9 * n); break;
        case 5: seq_rows_kernel<9, 16, true><<<grid * 8, 1024, 0, st>>>(H, n); break;
        case 6: seq_rows_kernel<9, 16, false><<<grid * 8, 1024, 0, st>>>(H, n); break;
        case 7: seq_rows_kernel<9, 8, false><<<grid * 8, 1024, 0, st>>>(H, n); break;
        case 64: mrg_pattern_kernel<64><<<grid, 1024, 0, st>>>(H, n); break;
        case 128: mrg_pattern_kernel<128><<<grid, 1024, 0, st>>>(H, n); break;
        case 256: mrg_pattern_kernel<256><<<grid, 1024, 0, st>>>(H, n); break;
        case 512: mrg_pattern_kernel<512><<<grid, 1024, 0, st>>>(H, n); break;
        case 1024: mrg_pattern_kernel<1024><<<grid, 1024, 0, st>>>(H, n); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

// Row-stream probe: variant -> (RI, RO, U); see row_streams.  in / out hold RI / RO rows
// of row_bytes at a pitch of pitch_bytes (both multiples of 16).
int hg_tune_streams(int variant, const void* in, void* out, int64_t row_bytes,
                    int64_t pitch_bytes, void* stream) {
    if (row_bytes <= 0 || (row_bytes & 15) || (pitch_bytes & 15) || pitch_bytes < row_bytes)
        return (int)hipErrorInvalidValue;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t r16 = row_bytes / 16, p16 = pitch_bytes / 16;
    const auto* s = reinterpret_cast<const u32x4*>(in);
    auto* d = reinterpret_cast<u32x4*>(out);
#define HG_RS(RI, RO, U)                                                                          \
    row_streams<RI, RO, U><<<(unsigned)((r16 + kBlock * U - 1) / (kBlock * U)), kBlock, 0, st>>>( \
        s, d, r16, p16)
    switch (variant) {
        case 0: HG_RS(16, 9, 1); break;   // SoA f32/f64 solver pattern
        case 1: HG_RS(16, 8, 1); break;
        case 2: HG_RS(8, 4, 1); break;
        case 3: HG_RS(4, 2, 1); break;
        case 4: HG_RS(2, 1, 1); break;
        case 5: HG_RS(16, 9, 4); break;   // 4 KiB per wave per row
        case 6: HG_RS(32, 16, 1); break;
        default: return (int)hipErrorInvalidValue;
    }
#undef HG_RS
    return (int)hipGetLastError();
}

// binary64 AoS sweep (tools/kbench_f64.py): 0 = P1 nt LDS-DMA (shipped), 1 = P2 nt LDS-DMA,
// 2 = P1 nt register-staged loads, 3 = P1 LDS-DMA default cache policy, 4 = variant 0's memory
// pattern with the solver replaced by a copy (kNoSolve; not bit-exact by design).
int hg_tune_aos_f64(int algo, int variant, const double* src, const double* tar, double* H,
                    int64_t n, void* stream) {
    if (n <= 0 || (algo != 0 && algo != 1)) return (int)hipErrorInvalidValue;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define HG_F64(P, FL)                                                                          \
    do {                                                                                       \
        const unsigned g = (unsigned)aos_grid<double, P, FL>(n);                               \
        if (algo == 0) solve_aos<kACA, true, double, P, FL><<<g, kBlock, 0, st>>>(src, tar, H, n); \
        else solve_aos<kSKS, true, double, P, FL><<<g, kBlock, 0, st>>>(src, tar, H, n);       \
    } while (0)
    switch (variant) {
        case 0: HG_F64(1, kNtLoad | kNtStore | kLdsLoad | kLdsDma); break;
        case 1: HG_F64(2, kNtLoad | kNtStore | kLdsLoad | kLdsDma); break;
        case 2: HG_F64(1, kNtLoad | kNtStore | kLdsLoad); break;
        case 3: HG_F64(1, kLdsLoad | kLdsDma); break;
        case 4: HG_F64(1, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kNoSolve); break;  // pattern only
        default: return (int)hipErrorInvalidValue;
    }
#undef HG_F64
    return (int)hipGetLastError();
}

// TensorACA tile sweep (tools/kbench_rect.py).  Variants 0-2: rect form (host scalars
// scale = a, div = b), P = 1 / 2 / 4 problems per lane; 3-5: compact form (src = corner,
// tar = offsets, a = width, b = height), P = 1 / 2 / 4.  16-B aligned inputs only.
int hg_tune_rect(int variant, const float* src, const float* tar, float* H, int64_t B, float a,
                 float b, void* stream) {
    if (B <= 0 || !src || !tar || !H) return (int)hipErrorInvalidValue;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const auto blocks = [B](int P) { return (unsigned)((B + (int64_t)kBlock * P - 1) / ((int64_t)kBlock * P)); };
    switch (variant) {
        case 0: tensor_aca_rect_kernel<1, true, true><<<blocks(1), kBlock, 0, st>>>(src, tar, H, B, nullptr, nullptr, a, b); break;
        case 1: tensor_aca_rect_kernel<2, true, true><<<blocks(2), kBlock, 0, st>>>(src, tar, H, B, nullptr, nullptr, a, b); break;
        case 2: tensor_aca_rect_kernel<4, true, true><<<blocks(4), kBlock, 0, st>>>(src, tar, H, B, nullptr, nullptr, a, b); break;
        case 3: tensor_aca_offsets_kernel<1, true, false><<<blocks(1), kBlock, 0, st>>>(src, tar, H, B, a, b); break;
        case 4: tensor_aca_offsets_kernel<2, true, false><<<blocks(2), kBlock, 0, st>>>(src, tar, H, B, a, b); break;
        case 5: tensor_aca_offsets_kernel<4, true, false><<<blocks(4), kBlock, 0, st>>>(src, tar, H, B, a, b); break;
        case 6: tensor_aca_rect_kernel<1, true, true, false, false><<<blocks(1), kBlock, 0, st>>>(src, tar, H, B, nullptr, nullptr, a, b); break;
        case 7: tensor_aca_offsets_kernel<1, true, false, false><<<blocks(1), kBlock, 0, st>>>(src, tar, H, B, a, b); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

// The TensorACA (B,3,4) backward with every gradient (dL/dsrc, dL/dtar and the (2,B,3) scale /
// div terms; 16-B aligned buffers, B a multiple of 64): variant 0 the shipped staged kernel
// (non-temporal), 1 its no-arithmetic twin -- the same loads and stores, the pattern's own
// ceiling (tools/kbench_bwd.py).
int hg_tune_rect_backward(int variant, const float* src, const float* tar, const float* gH,
                          int64_t B, const float* scale, const float* div, float* gsrc,
                          float* gtar, float* gterms, void* stream) {
    if (B <= 0 || (B & 63) || !src || !tar || !gH || !scale || !div || !gsrc || !gtar || !gterms)
        return (int)hipErrorInvalidValue;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const unsigned g = (unsigned)((B + kBlock - 1) / kBlock);
    switch (variant) {
        case 0: tensor_aca_rect_backward_staged<true, kSdTerms, true, kAtenCpu, false><<<g, kBlock, 0, st>>>(
                    src, tar, gH, B, scale, div, gsrc, gtar, gterms); break;
        case 1: tensor_aca_rect_backward_staged<true, kSdTerms, true, kAtenCpu, true><<<g, kBlock, 0, st>>>(
                    src, tar, gH, B, scale, div, gsrc, gtar, gterms); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

// cal_ACA's timing loop (GPU_Runtime Test.cu:1183-1200) in native code: `loops` back-to-
// back launches of the C-ABI solver from a C++ loop, bracketed by HIP events on
// `stream`.  Returns microseconds per launch, or -(hipError_t) on failure.  algo 0 ACA,
// 1 SKS; elem 4 (float) or 8 (double).
double hg_tune_launch_loop(int algo, int elem, const void* src, const void* tar, void* H,
                           int64_t n, int layout, int flags, int loops, void* stream) {
    if (algo < 0 || algo > 14 || (elem != 4 && elem != 8) || loops <= 0) return -1.0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    auto launch = [&]() -> int {
        if (algo == 2) {  // the floor: an empty kernel, raw launch, no checks
            empty_kernel<<<1, kWave, 0, st>>>();
            return 0;
        }
        if (algo >= 8 && algo <= 11) {  // one-dword store: sc0 sc1 / sc1 / sc0 sc1 nt / nt
            auto* h = static_cast<uint32_t*>(H);
            if (algo == 8) store_one_policy_kernel<0><<<1, kWave, 0, st>>>(h);
            if (algo == 9) store_one_policy_kernel<1><<<1, kWave, 0, st>>>(h);
            if (algo == 10) store_one_policy_kernel<2><<<1, kWave, 0, st>>>(h);
            if (algo == 11) store_one_policy_kernel<3><<<1, kWave, 0, st>>>(h);
            return 0;
        }
        if (algo == 13) {  // pointer arguments, never read
            args_unused_kernel<<<1, kWave, 0, st>>>(static_cast<const uint32_t*>(src),
                                                    static_cast<uint32_t*>(H));
            return 0;
        }
        if (algo == 14) {  // arguments read, no other memory access
            args_read_kernel<<<1, kWave, 0, st>>>((uint64_t)(uintptr_t)src, (uint64_t)n);
            return 0;
        }
        if (algo == 12) {  // one load per lane, no store
            load_one_kernel<<<1, kWave, 0, st>>>(static_cast<const uint32_t*>(src),
                                                 static_cast<uint32_t*>(H));
            return 0;
        }
        if (algo == 3) {  // the floor plus the error query every C-ABI call makes
            empty_kernel<<<1, kWave, 0, st>>>();
            return (int)hipGetLastError();
        }
        if (algo == 5 || algo == 6) {  // raw, non-temporal stores / one-dword kernel
            if (algo == 6) {
                store_one_kernel<<<1, kWave, 0, st>>>(static_cast<uint32_t*>(H));
                return 0;
            }
            const auto* s = static_cast<const double*>(src);
            const auto* t = static_cast<const double*>(tar);
            auto* h = static_cast<double*>(H);
            solve_soa_vec<kACA, false, double, 1, false, true>
                <<<(unsigned)soa_grid<1, false>(n / 2), kBlock, 0, st>>>(s, t, h, n);
            return 0;
        }
        if (algo == 7) {  // raw generic (one lane per problem, plain accesses)
            const auto* s = static_cast<const double*>(src);
            const auto* t = static_cast<const double*>(tar);
            auto* h = static_cast<double*>(H);
            solve_generic_t<kACA, false, double, true><<<(unsigned)((n + kBlock - 1) / kBlock), kBlock, 0, st>>>(s, t, h, n);
            return 0;
        }
        if (algo == 4) {  // the SoA f64 ACA kernel launched raw (no checks, no query)
            const auto* s = static_cast<const double*>(src);
            const auto* t = static_cast<const double*>(tar);
            auto* h = static_cast<double*>(H);
            solve_soa_vec<kACA, false, double, 1, false, false>
                <<<(unsigned)soa_grid<1, false>(n / 2), kBlock, 0, st>>>(s, t, h, n);
            return 0;
        }
        if (elem == 4) {
            const auto* s = static_cast<const float*>(src);
            const auto* t = static_cast<const float*>(tar);
            auto* h = static_cast<float*>(H);
            return algo == 0 ? hg_aca_f32(s, t, h, n, layout, flags, stream)
                             : hg_sks_f32(s, t, h, n, layout, flags, stream);
        }
        const auto* s = static_cast<const double*>(src);
        const auto* t = static_cast<const double*>(tar);
        auto* h = static_cast<double*>(H);
        return algo == 0 ? hg_aca_f64(s, t, h, n, layout, flags, stream)
                         : hg_sks_f64(s, t, h, n, layout, flags, stream);
    };
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return -1.0;
    if (hipEventCreate(&e1) != hipSuccess) return -1.0;
    int rc = 0;
    // warm as long as the timed run: after host-bound work the clocks need ~100 ms to ramp
    for (int i = 0; i < loops && rc == 0; ++i) rc = launch();
    if (rc == 0 && hipStreamSynchronize(st) != hipSuccess) rc = 1;
    float ms = 0.f;
    if (rc == 0) {
        (void)hipEventRecord(e0, st);
        for (int i = 0; i < loops && rc == 0; ++i) rc = launch();
        (void)hipEventRecord(e1, st);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc ? -(double)rc : (double)ms * 1e3 / loops;
}

// Sampler variants for tools/kbench_sample.py (0 global gather, 1 / 2 LDS pool P1 / P2;
// 8 the shipped packed pairs, 9 the same with the pairs' divisions split into scalar ones);
// same argument checks as hg_sample_solve_f32.
int hg_tune_sample(int variant, const float* pool_src, const float* pool_tar, uint32_t npool,
                   const uint32_t* idx, float* H, int64_t n, int algo, int flags, void* stream) {
    if (n <= 0 || npool == 0 || variant < 0 || variant > 9 || (algo != 0 && algo != 1))
        return (int)hipErrorInvalidValue;
    if (!pool_src || !pool_tar || !idx || !H || (reinterpret_cast<uintptr_t>(idx) & 15u) ||
        (reinterpret_cast<uintptr_t>(H) & 15u) || (reinterpret_cast<uintptr_t>(pool_src) & 7u) ||
        (reinterpret_cast<uintptr_t>(pool_tar) & 7u))
        return (int)hipErrorInvalidValue;
    const auto* ps = reinterpret_cast<const float2*>(pool_src);
    const auto* pt = reinterpret_cast<const float2*>(pool_tar);
    const auto* ix = reinterpret_cast<const uint4*>(idx);
    const bool norm = (flags & HG_FLAG_NORMALIZE) != 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (variant) {  // wider blocks: more waves share one LDS copy of the pool
        case 4: return hg::launch_sample_wide<1, 8>(ps, pt, npool, ix, H, n, algo, norm, st, hg::cu_count());
        case 5: return hg::launch_sample_wide<1, 16>(ps, pt, npool, ix, H, n, algo, norm, st, hg::cu_count());
        case 6: return hg::launch_sample_wide<2, 16>(ps, pt, npool, ix, H, n, algo, norm, st, hg::cu_count());
        case 7: return hg::launch_sample_solve(4, ps, pt, npool, ix, H, n, algo, norm, st);
        case 8: return hg::launch_sample_solve(5, ps, pt, npool, ix, H, n, algo, norm, st);
        case 9: return hg::launch_sample_solve(6, ps, pt, npool, ix, H, n, algo, norm, st);
        default: break;
    }
    return hg::launch_sample_solve(variant, reinterpret_cast<const float2*>(pool_src),
                                   reinterpret_cast<const float2*>(pool_tar), npool,
                                   reinterpret_cast<const uint4*>(idx), H, n, algo,
                                   (flags & HG_FLAG_NORMALIZE) != 0,
                                   reinterpret_cast<hipStream_t>(stream));
}

// Seeded sampler variants (tools/kbench_sample.py), (P, waves per block): 0 = shipped (2, 8);
// 1 = (2, 4); 2 = (1, 16); 3 = (2, 16); 4 = shipped shape with the 64-bit remainder;
// 5 / 6 = one hash per draw (the earlier stream, not fill_bits': compared by time only) at
// (2, 4) / (2, 8).
int hg_tune_sample_seeded(int variant, const float* pool_src, const float* pool_tar,
                          uint32_t npool, uint64_t seed, uint64_t offset, float* H, int64_t n,
                          int algo, int flags, void* stream) {
    if (n <= 0 || npool == 0 || !pool_src || !pool_tar || !H || (algo != 0 && algo != 1))
        return (int)hipErrorInvalidValue;
    const auto* ps = reinterpret_cast<const float2*>(pool_src);
    const auto* pt = reinterpret_cast<const float2*>(pool_tar);
    const bool norm = (flags & HG_FLAG_NORMALIZE) != 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    using namespace hg;
    switch (variant) {
        case 0: return launch_sample_seeded_shipped(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 13: return launch_sample_seeded<1, 16, kDrawsPaired, false, 0>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        // the remainder and the draws of the 4-wave packed-pair shape: 14 the binary64
        // remainder (exact); ablations, wrong bits, time only: 15 no remainder, 16 no hash,
        // 17 neither; 18 the 8-wave shape with the binary64 remainder
        case 14: return launch_sample_seeded<2, 4, kDrawsPaired, 2, 0, kPairPacked>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 15: return launch_sample_seeded<2, 4, kDrawsPaired, 3, 0, kPairPacked>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 16: return launch_sample_seeded<2, 4, kDrawsCheap, 0, 0, kPairPacked>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 17: return launch_sample_seeded<2, 4, kDrawsCheap, 3, 0, kPairPacked>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 18: return launch_sample_seeded<2, 8, kDrawsPaired, 2, 0, kPairPacked>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        // the 8-wave shape (SKS's shipped one) ablated the same way: 19 no remainder, 20 no
        // hash, 21 neither (wrong bits, time only)
        case 19: return launch_sample_seeded<2, 8, kDrawsPaired, 3, 0, kPairPacked>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 20: return launch_sample_seeded<2, 8, kDrawsCheap, 0, 0, kPairPacked>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 21: return launch_sample_seeded<2, 8, kDrawsCheap, 3, 0, kPairPacked>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 1: return launch_sample_seeded<2, 4, kDrawsPaired, false, 1>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 2: return launch_sample_seeded<1, 16, kDrawsPaired, false, 1>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 3: return launch_sample_seeded<2, 16, kDrawsPaired, false, 1>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 4: return launch_sample_seeded<2, 8, kDrawsPaired, true, 1>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 5: return launch_sample_seeded<2, 4, kDrawsSingle, false, 1>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 6: return launch_sample_seeded<2, 8, kDrawsSingle, false, 1>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 7: return launch_sample_seeded<2, 8, kDrawsPaired, false, 0>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 8: return launch_sample_seeded<2, 4, kDrawsPaired, false, 0>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 9: return launch_sample_seeded<2, 8, kDrawsPaired, false, 1>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        // two hypotheses per lane solved as packed f32x2 pairs, their divisions split into
        // scalar expansions (the round-2 forms; 10 and, from 4 M ACA hypotheses, 12 shipped then)
        case 10: return launch_sample_seeded<2, 8, kDrawsPaired, false, 0, kPairScalarDiv>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 11: return launch_sample_seeded<2, 16, kDrawsPaired, false, 0, kPairScalarDiv>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 12: return launch_sample_seeded<2, 4, kDrawsPaired, false, 0, kPairScalarDiv>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        // the shipped shapes with other H store policies (STP): 22-24 the 4-wave shape with
        // default, sc1, sc1|nt stores; 25-27 the 8-wave shape the same way
        case 22: return launch_sample_seeded<2, 4, kDrawsPaired, 0, 0, kPairPacked, 1>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 23: return launch_sample_seeded<2, 4, kDrawsPaired, 0, 0, kPairPacked, 2>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 24: return launch_sample_seeded<2, 4, kDrawsPaired, 0, 0, kPairPacked, 3>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 25: return launch_sample_seeded<2, 8, kDrawsPaired, 0, 0, kPairPacked, 1>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 26: return launch_sample_seeded<2, 8, kDrawsPaired, 0, 0, kPairPacked, 2>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 27: return launch_sample_seeded<2, 8, kDrawsPaired, 0, 0, kPairPacked, 3>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        // round 6: the packed-pair shape in 16-wave blocks, plain and with
        // the sc1 buffer stores (per-row resources in SGPRs), beside 22-27
        case 28: return launch_sample_seeded<2, 16, kDrawsPaired, 0, 0, kPairPacked, 0>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 29: return launch_sample_seeded<2, 16, kDrawsPaired, 0, 0, kPairPacked, 2>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 30: return launch_sample_seeded<2, 16, kDrawsPaired, 0, 0, kPairPacked, 3>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        // the binary64 remainder without a correction (fmod_f64_exact_u32) in the 4-, 8- and
        // 16-wave packed-pair shapes (same bits)
        case 31: return launch_sample_seeded<2, 4, kDrawsPaired, 4, 0, kPairPacked, 0>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 32: return launch_sample_seeded<2, 8, kDrawsPaired, 4, 0, kPairPacked, 0>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        case 33: return launch_sample_seeded<2, 16, kDrawsPaired, 4, 0, kPairPacked, 0>(ps, pt, npool, seed, offset, H, n, algo, norm, st);
        default: return (int)hipErrorInvalidValue;
    }
}

// Fused get_rand_list + cal_Homo_ACA/SKS (binary64, hg_gather.hpp) for tools/kbench_gather.py:
// 0 = pool in LDS (the shipped form for pools up to 5120 pairs; 1024-lane persistent blocks),
// 1 = the global-gather form, 2 = pool in LDS with 512-lane blocks (two blocks per CU when
// the pool fits 80 KiB), 3 = pool in LDS, 256-lane blocks, 4 / 5 / 6 = 0 / 2 / 3 with two
// hypotheses per lane (8-B word reads, 16-B H stores; n even), 7 = 0 with default-policy
// (not non-temporal) H stores.  Unnormalised.
int hg_tune_gather_solve_f64(int variant, int algo, const double* pool_src, const double* pool_tar,
                             uint32_t size, const uint32_t* rand_list, double* H, int64_t n,
                             void* stream) {
    if (n <= 0 || size == 0 || (algo != 0 && algo != 1) || variant < 0 || variant > 7)
        return (int)hipErrorInvalidValue;
    const bool plain_st = variant == 7;
    if (plain_st) variant = 0;
    const bool pair = variant >= 4;
    if (pair && ((n & 1) || (reinterpret_cast<uintptr_t>(H) & 15u) ||
                 (reinterpret_cast<uintptr_t>(rand_list) & 7u)))
        return (int)hipErrorInvalidValue;
    if (pair) variant = variant == 4 ? 0 : variant - 3;
    const auto* ps = reinterpret_cast<const double2*>(pool_src);
    const auto* pt = reinterpret_cast<const double2*>(pool_tar);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uint64_t magic = hg::fastmod_magic(size);
    const size_t lds = (size_t)size * 32;
    const int block = variant == 2 ? 512 : (variant == 3 ? 256 : 1024);
    const int64_t blocks = (n / (pair ? 2 : 1) + block - 1) / block;
    if (variant == 1) {
        auto k = algo == 0 ? hg::gather_solve_f64_kernel<hg::kACA, false, false>
                           : hg::gather_solve_f64_kernel<hg::kSKS, false, false>;
        return hg::launch(k, (unsigned)blocks, block, 0, s, rand_list, size, magic, ps, pt, H, n);
    }
    if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
    auto k = algo == 0 ? (pair ? hg::gather_solve_f64_kernel<hg::kACA, false, true, 2>
                               : (plain_st ? hg::gather_solve_f64_kernel<hg::kACA, false, true, 1, false>
                                           : hg::gather_solve_f64_kernel<hg::kACA, false, true>))
                       : (pair ? hg::gather_solve_f64_kernel<hg::kSKS, false, true, 2>
                               : (plain_st ? hg::gather_solve_f64_kernel<hg::kSKS, false, true, 1, false>
                                           : hg::gather_solve_f64_kernel<hg::kSKS, false, true>));
    if (lds > hg::kSampleLdsMax && !hg::lds_opt_in(k)) return (int)hipErrorInvalidValue;
    int64_t per_cu = (int64_t)(160 * 1024) / (int64_t)lds;
    const int64_t max_per_cu = 2048 / block;
    per_cu = per_cu < 1 ? 1 : (per_cu > max_per_cu ? max_per_cu : per_cu);
    const int64_t cap = per_cu * hg::cu_count();
    return hg::launch(k, (unsigned)(blocks < cap ? blocks : cap), block, lds, s, rand_list, size,
                      magic, ps, pt, H, n);
}

// Scorer variants for tools/kbench_score.py: 0 = one hypothesis per lane (unroll 4),
// 1 = two per lane packed (unroll 1), 2 = two per lane packed (unroll 4), 3 / 4 = two
// per lane packed, pool through scalar loads (unroll 4 / 8).
int hg_tune_score(int variant, const float* H, int64_t n, const float* pool_src,
                  const float* pool_tar, uint32_t npool, float thresh, uint32_t* counts,
                  void* stream) {
    if (n <= 0 || !H || !counts) return (int)hipErrorInvalidValue;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const float t2 = thresh * thresh;
    const auto* ps = reinterpret_cast<const float2*>(pool_src);
    const auto* pt = reinterpret_cast<const float2*>(pool_tar);
    const int64_t b1 = (n + hg::kBlock - 1) / hg::kBlock;
    const int64_t b2 = (n + 2 * hg::kBlock - 1) / (2 * hg::kBlock);
    switch (variant) {
        case 0: hg::ransac_score_kernel<<<(unsigned)b1, hg::kBlock, 0, s>>>(H, n, ps, pt, npool, t2, counts); break;
        case 1: hg::ransac_score2_kernel<1><<<(unsigned)b2, hg::kBlock, 0, s>>>(H, n, ps, pt, npool, t2, counts); break;
        case 2: hg::ransac_score2_kernel<4><<<(unsigned)b2, hg::kBlock, 0, s>>>(H, n, ps, pt, npool, t2, counts); break;
        case 3: hg::ransac_score_sgpr_kernel<4><<<(unsigned)b2, hg::kBlock, 0, s>>>(H, n, ps, pt, npool, t2, counts); break;
        case 4: hg::ransac_score_sgpr_kernel<8><<<(unsigned)b2, hg::kBlock, 0, s>>>(H, n, ps, pt, npool, t2, counts); break;
        case 5: hg::ransac_score_sgpr4_kernel<4><<<(unsigned)((n + 4 * hg::kBlock - 1) / (4 * hg::kBlock)), hg::kBlock, 0, s>>>(H, n, ps, pt, npool, t2, counts); break;
        case 6: hg::ransac_score_sgpr4_kernel<8><<<(unsigned)((n + 4 * hg::kBlock - 1) / (4 * hg::kBlock)), hg::kBlock, 0, s>>>(H, n, ps, pt, npool, t2, counts); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

// ---- MRG32K3A (round 3) ----
// rocRAND's own host API, the checker the hand-written generator is pinned against
// (tests/test_gpu_mrg32k3a.py) and the timing it replaced (tools/kbench_mrg.py): a fresh
// generator per call, as the reference harness creates one (GPU_Runtime Test.cu:1443-1446).
// Synchronous.  Statuses: ROCRAND_STATUS_ALLOCATION_FAILED -> hipErrorOutOfMemory, any
// other failure -> hipErrorLaunchFailure.
int hg_tune_rocrand_mrg32k3a_u32(uint32_t* out, int64_t count, uint64_t seed, void* stream) {
    if (count < 0 || (count > 0 && !out)) return (int)hipErrorInvalidValue;
    if (count == 0) return 0;
    rocrand_generator g = nullptr;
    rocrand_status st = rocrand_create_generator(&g, ROCRAND_RNG_PSEUDO_MRG32K3A);
    if (st == ROCRAND_STATUS_SUCCESS) st = rocrand_set_stream(g, reinterpret_cast<hipStream_t>(stream));
    if (st == ROCRAND_STATUS_SUCCESS) st = rocrand_set_seed(g, seed);
    if (st == ROCRAND_STATUS_SUCCESS) st = rocrand_generate(g, out, (size_t)count);
    const hipError_t sync = hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream));
    if (g) rocrand_destroy_generator(g);
    if (st == ROCRAND_STATUS_ALLOCATION_FAILED) return (int)hipErrorOutOfMemory;
    if (st != ROCRAND_STATUS_SUCCESS) return (int)hipErrorLaunchFailure;
    return (int)sync;
}

// The standalone generator with another split threshold (positions per thread).
// min_chunk >= 2^20 + 1 ... : ablations (wrong bits, timing only) at the shipped split --
// 2^20 + 1 no table jumps, 2^20 + 2 no engine steps, 2^20 + 3 neither; 2^20 + 4 the shipped
// kernel with non-temporal stores (same bits); 2^21 + c: non-temporal stores at split c.
int hg_tune_mrg_words(uint32_t* out, int64_t count, uint64_t seed, int64_t min_chunk,
                      void* stream) {
    if (count <= 0 || !out || min_chunk < 1) return (int)hipErrorInvalidValue;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (min_chunk > (1 << 21))
        return hg::launch_mrg_words<4>(out, count, seed, min_chunk - (1 << 21), s);
    const int64_t abl = min_chunk > (1 << 20) ? min_chunk - (1 << 20) : 0;
    switch (abl) {
        case 4: return hg::launch_mrg_words<4>(out, count, seed, hg::kMrgMinChunk, s);
        case 0: return hg::launch_mrg_words(out, count, seed, min_chunk, s);
        case 1: return hg::launch_mrg_words<1>(out, count, seed, hg::kMrgMinChunk, s);
        case 2: return hg::launch_mrg_words<2>(out, count, seed, hg::kMrgMinChunk, s);
        case 3: return hg::launch_mrg_words<3>(out, count, seed, hg::kMrgMinChunk, s);
        default: return (int)hipErrorInvalidValue;
    }
}

// Fused draws + gather + solve (unnormalised ACA / SKS): 0 = pool in global memory,
// 1 = pool in LDS beside the draws buffer (shipped when it fits); 2 ... 8 = the shipped
// form with parts removed (wrong bits, timing only: where the launch's time goes) --
// 2 no solve, 3 no table jumps at the engine starts, 4 no engine steps, 5 = 2 + 3,
// 6 = 2 + 4, 7 = 3 + 4, 8 = all three (the gather and the H stores alone).
}  // extern "C"

template <int ALGO>
static int rand_gather_variant(int variant, const double2* ps, const double2* pt, uint32_t size,
                               uint64_t seed, double* H, int64_t n, hipStream_t s) {
    using namespace hg;
    switch (variant) {
        case 0: return launch_rand_gather_solve<ALGO, false>(ps, pt, size, seed, H, n, s, 0);
        case 1: return launch_rand_gather_solve<ALGO, false>(ps, pt, size, seed, H, n, s, -1);
        case 2: return launch_rand_gather_solve<ALGO, false, kMrgAblNoSolve>(ps, pt, size, seed, H, n, s);
        case 3: return launch_rand_gather_solve<ALGO, false, kMrgAblNoStart>(ps, pt, size, seed, H, n, s);
        case 4: return launch_rand_gather_solve<ALGO, false, kMrgAblNoDraws>(ps, pt, size, seed, H, n, s);
        case 5: return launch_rand_gather_solve<ALGO, false, kMrgAblNoSolve | kMrgAblNoStart>(ps, pt, size, seed, H, n, s);
        case 6: return launch_rand_gather_solve<ALGO, false, kMrgAblNoSolve | kMrgAblNoDraws>(ps, pt, size, seed, H, n, s);
        case 7: return launch_rand_gather_solve<ALGO, false, kMrgAblNoStart | kMrgAblNoDraws>(ps, pt, size, seed, H, n, s);
        case 8:
            return launch_rand_gather_solve<ALGO, false, kMrgAblNoSolve | kMrgAblNoStart | kMrgAblNoDraws>(
                ps, pt, size, seed, H, n, s);
        case 9:  // the H stores alone (no draws, starts, pool reads or solve)
            return launch_rand_gather_solve<ALGO, false, kMrgAblNoSolve | kMrgAblNoStart | kMrgAblNoDraws |
                                                         kMrgAblNoGather>(ps, pt, size, seed, H, n, s);
        case 10:  // shipped + 16-B paired stores (bit-exact; n even, H 16-B aligned)
            return launch_rand_gather_solve<ALGO, false, kMrgSt16>(ps, pt, size, seed, H, n, s);
        case 12:  // 9 with the pool left in global memory (no 81 KB LDS copy: 2 blocks per CU)
            return launch_rand_gather_solve<ALGO, false, kMrgAblNoSolve | kMrgAblNoStart | kMrgAblNoDraws |
                                                         kMrgAblNoGather>(ps, pt, size, seed, H, n, s, 0);
        case 13:  // shipped with default-policy stores
            return launch_rand_gather_solve<ALGO, false, kMrgStDefault>(ps, pt, size, seed, H, n, s);
        case 14:  // shipped with default-policy 16-B paired stores
            return launch_rand_gather_solve<ALGO, false, kMrgSt16 | kMrgStDefault>(ps, pt, size, seed, H, n, s);
        case 11:  // 9 with 16-B paired stores
            return launch_rand_gather_solve<ALGO, false, kMrgAblNoSolve | kMrgAblNoStart | kMrgAblNoDraws |
                                                         kMrgAblNoGather | kMrgSt16>(ps, pt, size, seed, H, n, s);
        case 15:  // Q = 8 positions per chunk: two hypotheses per lane, half the barriers (bit-exact)
            return launch_rand_gather_solve<ALGO, false, kMrgAblNone, 8>(ps, pt, size, seed, H, n, s);
        case 16:  // Q = 4 forced (the round-3..4 shape)
            return launch_rand_gather_solve<ALGO, false, kMrgAblNone, 4>(ps, pt, size, seed, H, n, s);
        case 17:  // Q = 8 with no solve (the draws, gathers and stores of that shape)
            return launch_rand_gather_solve<ALGO, false, kMrgAblNoSolve, 8>(ps, pt, size, seed, H, n, s);
        case 18:  // Q = 8 in 768-lane blocks (168 VGPRs: no spill, 3 waves per SIMD)
            return launch_rand_gather_solve<ALGO, false, kMrgAblNone, 8, 768>(ps, pt, size, seed, H, n, s);
        case 19:  // Q = 8 in 512-lane blocks (2 waves per SIMD)
            return launch_rand_gather_solve<ALGO, false, kMrgAblNone, 8, 512>(ps, pt, size, seed, H, n, s);
        case 20:  // Q = 4 in 768-lane blocks
            return launch_rand_gather_solve<ALGO, false, kMrgAblNone, 4, 768>(ps, pt, size, seed, H, n, s);
        case 21:  // Q = 4, buffer stores (8 n < 2^32)
            return launch_rand_gather_solve<ALGO, false, kMrgStBuf, 4>(ps, pt, size, seed, H, n, s);
        case 22:  // Q = 8, buffer stores (8 n < 2^32)
            return launch_rand_gather_solve<ALGO, false, kMrgStBuf, 8>(ps, pt, size, seed, H, n, s);
        case 23:  // Q = 4, buffer stores, draws of the next chunk interleaved with the solves
            return launch_rand_gather_solve<ALGO, false, kMrgStBuf | kMrgInterleave, 4>(ps, pt, size, seed, H, n, s);
        case 24:  // Q = 8, the same
            return launch_rand_gather_solve<ALGO, false, kMrgStBuf | kMrgInterleave, 8>(ps, pt, size, seed, H, n, s);
        case 25:  // 21 with the engines writing pool indices (binary64 remainder)
            return launch_rand_gather_solve<ALGO, false, kMrgStBuf | kMrgIdxF64, 4>(ps, pt, size, seed, H, n, s);
        case 26:  // 23 with the same
            return launch_rand_gather_solve<ALGO, false, kMrgStBuf | kMrgInterleave | kMrgIdxF64, 4>(ps, pt, size, seed, H, n, s);
        case 27:  // Q = 8, buffer stores, pool indices from the engines
            return launch_rand_gather_solve<ALGO, false, kMrgStBuf | kMrgIdxF64, 8>(ps, pt, size, seed, H, n, s);
        default: return (int)hipErrorInvalidValue;
    }
}

extern "C" {

int hg_tune_rand_gather_solve_f64(int variant, int algo, const double* pool_src,
                                  const double* pool_tar, uint32_t size, uint64_t seed, double* H,
                                  int64_t n, void* stream) {
    if (n <= 0 || size == 0 || (algo != 0 && algo != 1) || variant < 0 || variant > 27)
        return (int)hipErrorInvalidValue;
    if ((variant == 10 || variant == 11 || variant == 14) && ((n & 1) || (reinterpret_cast<uintptr_t>(H) & 15)))
        return (int)hipErrorInvalidValue;
    if (variant >= 21 && variant <= 24 && n >= (int64_t)1 << 29) return (int)hipErrorInvalidValue;
    const auto* ps = reinterpret_cast<const double2*>(pool_src);
    const auto* pt = reinterpret_cast<const double2*>(pool_tar);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return algo == 0 ? rand_gather_variant<hg::kACA>(variant, ps, pt, size, seed, H, n, s)
                     : rand_gather_variant<hg::kSKS>(variant, ps, pt, size, seed, H, n, s);
}

}  // extern "C"

