// hg_ransac.hip -- RANSAC-style hypothesis generation and scoring on the solver
// (the reference's cuRAND + get_rand_list gather, GPU_Runtime
// Test.cu:52-78 / :1443-1451, fused with the closed-form solve, then inlier scoring).
//
//   hg_fill_bits_u32      counter-based 32-bit draws (4 per hypothesis)
//   hg_sample_solve_f32   idx (n,4) -> gather 4 correspondences from the pool -> H (n,9)
//   hg_sample_solve_seeded_f32   the same with the draws made in the kernel (no idx)
//   hg_ransac_score_f32   H (n,9) x pool (npool) -> inlier count per hypothesis
//
// The scorer is the one compute-bound kernel here: every (hypothesis, point) pair
// costs ~9 wave64 VALU instructions and no HBM traffic (the pool streams through the
// scalar cache, H sits in VGPRs), so its roofline is the FP32 VALU rate, not HBM.
// Kernels: hg_ransac.hpp.
#include "hg_ransac.hpp"

extern "C" {

int hg_fill_bits_u32(uint32_t* out, int64_t count, uint64_t seed, uint64_t offset, void* stream) {
    if (count < 0) return (int)hipErrorInvalidValue;
    if (count == 0) return 0;
    if (!out) return (int)hipErrorInvalidValue;
    const int64_t want = (count + hg::kBlock - 1) / hg::kBlock;
    const unsigned g = (unsigned)(want < 8192 ? want : 8192);
    return hg::launch(hg::fill_bits_kernel, g, hg::kBlock, 0, reinterpret_cast<hipStream_t>(stream),
                      out, count, seed, offset);
}

int hg_sample_solve_f32(const float* pool_src, const float* pool_tar, uint32_t npool,
                        const uint32_t* idx, float* H, int64_t n, int algo, int flags,
                        void* stream) {
    if (n < 0 || npool == 0 || (algo != 0 && algo != 1) || (flags & ~HG_FLAG_NORMALIZE))
        return (int)hipErrorInvalidValue;
    if (n == 0) return 0;
    if (!pool_src || !pool_tar || !idx || !H) return (int)hipErrorInvalidValue;
    if ((reinterpret_cast<uintptr_t>(idx) & 15u) || (reinterpret_cast<uintptr_t>(H) & 15u) ||
        (reinterpret_cast<uintptr_t>(pool_src) & 7u) || (reinterpret_cast<uintptr_t>(pool_tar) & 7u))
        return (int)hipErrorInvalidValue;
    return hg::launch_sample_solve(-1, reinterpret_cast<const float2*>(pool_src),
                                   reinterpret_cast<const float2*>(pool_tar), npool,
                                   reinterpret_cast<const uint4*>(idx), H, n, algo,
                                   (flags & HG_FLAG_NORMALIZE) != 0,
                                   reinterpret_cast<hipStream_t>(stream));
}

int hg_sample_solve_seeded_f32(const float* pool_src, const float* pool_tar, uint32_t npool,
                               uint64_t seed, uint64_t offset, float* H, int64_t n, int algo,
                               int flags, void* stream) {
    if (n < 0 || npool == 0 || (algo != 0 && algo != 1) || (flags & ~HG_FLAG_NORMALIZE))
        return (int)hipErrorInvalidValue;
    if (n == 0) return 0;
    if (!pool_src || !pool_tar || !H) return (int)hipErrorInvalidValue;
    if ((reinterpret_cast<uintptr_t>(H) & 15u) || (reinterpret_cast<uintptr_t>(pool_src) & 7u) ||
        (reinterpret_cast<uintptr_t>(pool_tar) & 7u))
        return (int)hipErrorInvalidValue;
    return hg::launch_sample_seeded_shipped(reinterpret_cast<const float2*>(pool_src),
                                    reinterpret_cast<const float2*>(pool_tar), npool,
                                    seed, offset, H, n, algo,
                                    (flags & HG_FLAG_NORMALIZE) != 0,
                                    reinterpret_cast<hipStream_t>(stream));
}

int hg_ransac_score_f32(const float* H, int64_t n, const float* pool_src, const float* pool_tar,
                        uint32_t npool, float thresh, uint32_t* counts, void* stream) {
    if (n < 0) return (int)hipErrorInvalidValue;
    if (n == 0) return 0;
    if (!H || !counts || (npool && (!pool_src || !pool_tar))) return (int)hipErrorInvalidValue;
    if ((reinterpret_cast<uintptr_t>(pool_src) & 7u) || (reinterpret_cast<uintptr_t>(pool_tar) & 7u))
        return (int)hipErrorInvalidValue;
    // shipped: two hypotheses per lane, packed, pool through scalar loads, unroll 8
    // (tools/kbench_score.py, profiles/r01/kbench_score.json)
    const int64_t blocks = (n + 2 * hg::kBlock - 1) / (2 * hg::kBlock);
    if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
    const float t2 = thresh * thresh;
    return hg::launch(hg::ransac_score_sgpr_kernel<8>, (unsigned)blocks, hg::kBlock, 0,
                      reinterpret_cast<hipStream_t>(stream), H, n,
                      reinterpret_cast<const float2*>(pool_src),
                      reinterpret_cast<const float2*>(pool_tar), npool, t2, counts);
}

}  // extern "C"
