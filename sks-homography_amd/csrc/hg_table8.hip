// hg_table8.hip -- the reference's Table-8 sampling pipeline in its own formats
// (GPU_Runtime Test.cu:1443-1451): MRG32K3A draws, get_rand_list (:52-78) and
// cal_Homo_* (:81-507), the last two also fused into one pass.  Kernels: hg_gather.hpp.
//
//   hg_rand_mrg32k3a_u32   curandCreateGenerator(MRG32K3A) + SetPseudoRandomGeneratorSeed
//                          + curandGenerate (.cu:1443-1446): hand-written (hg_mrg32k3a.hpp)
//   hg_rand_gather_solve_f64  all three fused: words made in registers, H (9,n)
//   hg_mrg32k3a_state      (host) the engine state of curand_init / rocrand_init
//   hg_get_rand_list_f64   get_rand_list itself: (4,n) words -> (8,n) src / tar rows
//   hg_gather_solve_f64    get_rand_list fused with cal_Homo_{ACA,SKS,GE,GPT}: (9,n) H
#include "hg_gather.hpp"

namespace {

constexpr int kInvalid = (int)hipErrorInvalidValue;
constexpr size_t kPoolLdsMax = 160 * 1024;  // gfx950: the whole LDS of a CU for one block

bool misaligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) != 0; }

template <int ALGO, bool NORM>
int launch_gather_solve(const uint32_t* rl, uint32_t size, const double2* ps, const double2* pt,
                        double* H, int64_t n, hipStream_t s) {
    constexpr int kGatherBlock = hg::gather_block<ALGO>();
    const uint64_t magic = hg::fastmod_magic(size);
    const size_t lds = (size_t)size * 32;
    const int64_t blocks = (n + kGatherBlock - 1) / kGatherBlock;
    if (lds <= kPoolLdsMax) {
        // persistent: as many blocks as are resident at once, each with one pool copy
        auto k = hg::gather_solve_f64_kernel<ALGO, NORM, true>;
        if (lds > hg::kSampleLdsMax && !hg::lds_opt_in(k)) return kInvalid;
        int64_t per_cu = (int64_t)kPoolLdsMax / (int64_t)(lds ? lds : 1);
        const int64_t max_per_cu = 2048 / kGatherBlock;  // 32 waves per CU
        per_cu = per_cu < 1 ? 1 : (per_cu > max_per_cu ? max_per_cu : per_cu);
        const int64_t cap = per_cu * hg::cu_count();
        const unsigned g = (unsigned)(blocks < cap ? blocks : cap);
        return hg::launch(k, g, kGatherBlock, lds, s, rl, size, magic, ps, pt, H, n);
    }
    if (blocks > 0x7fffffffLL) return kInvalid;
    return hg::launch(hg::gather_solve_f64_kernel<ALGO, NORM, false>, (unsigned)blocks,
                      kGatherBlock, 0, s, rl, size, magic, ps, pt, H, n);
}

}  // namespace

extern "C" {

int hg_rand_mrg32k3a_u32(uint32_t* out, int64_t count, uint64_t seed, void* stream) {
    if (count < 0) return kInvalid;
    if (count == 0) return 0;
    if (!out || misaligned(out, 4)) return kInvalid;
    return hg::launch_mrg_words(out, count, seed, hg::kMrgMinChunk,
                                reinterpret_cast<hipStream_t>(stream));
}

int hg_get_rand_list_f64(const uint32_t* rand_list, uint32_t size, const double* pool_src,
                         const double* pool_tar, double* d_src, double* d_tar, int64_t n,
                         void* stream) {
    if (n < 0 || size == 0) return kInvalid;
    if (n == 0) return 0;
    if (!rand_list || !pool_src || !pool_tar || !d_src || !d_tar) return kInvalid;
    if (misaligned(rand_list, 4) || misaligned(pool_src, 16) || misaligned(pool_tar, 16) ||
        misaligned(d_src, 8) || misaligned(d_tar, 8))
        return kInvalid;
    const int64_t blocks = (n + hg::kBlock - 1) / hg::kBlock;
    if (blocks > 0x7fffffffLL) return kInvalid;
    return hg::launch(hg::get_rand_list_kernel, (unsigned)blocks, hg::kBlock, 0,
                      reinterpret_cast<hipStream_t>(stream), rand_list, size,
                      hg::fastmod_magic(size), reinterpret_cast<const double2*>(pool_src),
                      reinterpret_cast<const double2*>(pool_tar), d_src, d_tar, n);
}

int hg_gather_solve_f64(int algo, const double* pool_src, const double* pool_tar, uint32_t size,
                        const uint32_t* rand_list, double* H, int64_t n, int flags, void* stream) {
    if (n < 0 || size == 0 || algo < HG_ALGO_ACA || algo > HG_ALGO_GPT ||
        (flags & ~HG_FLAG_NORMALIZE))
        return kInvalid;
    if (n == 0) return 0;
    if (!rand_list || !pool_src || !pool_tar || !H) return kInvalid;
    if (misaligned(rand_list, 4) || misaligned(pool_src, 16) || misaligned(pool_tar, 16) ||
        misaligned(H, 8))
        return kInvalid;
    const auto* ps = reinterpret_cast<const double2*>(pool_src);
    const auto* pt = reinterpret_cast<const double2*>(pool_tar);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool norm = (flags & HG_FLAG_NORMALIZE) != 0;
#define HG_GS(A)                                                                         \
    return norm ? launch_gather_solve<A, true>(rand_list, size, ps, pt, H, n, s)         \
                : launch_gather_solve<A, false>(rand_list, size, ps, pt, H, n, s)
    switch (algo) {
        case HG_ALGO_ACA: HG_GS(hg::kACA);
        case HG_ALGO_SKS: HG_GS(hg::kSKS);
        case HG_ALGO_GE: HG_GS(hg::kGE);
        default: HG_GS(hg::kGPT);
    }
#undef HG_GS
}

int hg_mrg32k3a_state(uint64_t seed, uint64_t subsequence, uint64_t offset, uint32_t* state) {
    if (!state) return kInvalid;
    namespace m = hg::mrg;
    m::Vec x1, x2;
    m::seed_state(seed, x1, x2);
    // (A^(2^76))^subsequence, then A^offset, by squaring
    m::Mat j1 = m::pow2<1>(m::kStep1, 76), j2 = m::pow2<2>(m::kStep2, 76);
    for (uint64_t e = subsequence; e; e >>= 1) {
        if (e & 1) {
            x1 = m::mat_vec<1>(j1, x1);
            x2 = m::mat_vec<2>(j2, x2);
        }
        j1 = m::mat_mul<1>(j1, j1);
        j2 = m::mat_mul<2>(j2, j2);
    }
    j1 = m::kStep1;
    j2 = m::kStep2;
    for (uint64_t e = offset; e; e >>= 1) {
        if (e & 1) {
            x1 = m::mat_vec<1>(j1, x1);
            x2 = m::mat_vec<2>(j2, x2);
        }
        j1 = m::mat_mul<1>(j1, j1);
        j2 = m::mat_mul<2>(j2, j2);
    }
    for (int k = 0; k < 3; ++k) {
        state[k] = x1.v[k];
        state[3 + k] = x2.v[k];
    }
    return 0;
}

int hg_rand_gather_solve_f64(int algo, const double* pool_src, const double* pool_tar,
                             uint32_t size, uint64_t seed, double* H, int64_t n, int flags,
                             void* stream) {
    if (n < 0 || size == 0 || algo < HG_ALGO_ACA || algo > HG_ALGO_GPT ||
        (flags & ~HG_FLAG_NORMALIZE) || n > (INT64_C(1) << 61))
        return kInvalid;
    if (n == 0) return 0;
    if (!pool_src || !pool_tar || !H) return kInvalid;
    if (misaligned(pool_src, 16) || misaligned(pool_tar, 16) || misaligned(H, 8)) return kInvalid;
    const auto* ps = reinterpret_cast<const double2*>(pool_src);
    const auto* pt = reinterpret_cast<const double2*>(pool_tar);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool norm = (flags & HG_FLAG_NORMALIZE) != 0;
    // H rows through buffer stores (row resources in SGPRs, one 32-bit lane offset: 16 VGPRs
    // fewer, 1-3 % faster at 10 M, tools/kbench_t8q.py) while a row's bytes fit 32 bits.  The
    // engines hand the solves pool indices, the remainder made in binary64 from the word's
    // binary64 value (kMrgIdxF64: 16 VALU fewer per 64 hypotheses; round 6)
    const bool buf = n < (INT64_C(1) << 29);
    constexpr int kBuf = hg::kMrgStBuf | hg::kMrgIdxF64, kFlat = hg::kMrgIdxF64;
#define HG_RGS(A)                                                                                \
    if (buf)                                                                                     \
        return norm ? hg::launch_rand_gather_solve<A, true, kBuf>(ps, pt, size, seed, H, n, s)   \
                    : hg::launch_rand_gather_solve<A, false, kBuf>(ps, pt, size, seed, H, n, s); \
    return norm ? hg::launch_rand_gather_solve<A, true, kFlat>(ps, pt, size, seed, H, n, s)      \
                : hg::launch_rand_gather_solve<A, false, kFlat>(ps, pt, size, seed, H, n, s)
    switch (algo) {
        case HG_ALGO_ACA: HG_RGS(hg::kACA);
        case HG_ALGO_SKS: HG_RGS(hg::kSKS);
        case HG_ALGO_GE: HG_RGS(hg::kGE);
        default: HG_RGS(hg::kGPT);
    }
#undef HG_RGS
}

}  // extern "C"
