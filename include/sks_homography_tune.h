/*
 * sks_homography_tune.h -- kernel-variant launchers and timing loops for tools/ and
 * bench.py (lib/libsks_homography_tune.so): the sweeps that picked each shipped
 * kernel's memory schedule, the HBM ceiling streams, and cal_ACA's launch loop
 * (GPU_Runtime Test.cu:1166-1206) in native code.  Not part of the drop-in boundary
 * (include/sks_homography.h); every solver variant produces the shipped kernel's bits.
 * Error reporting differs from the product library: these launchers return
 * hipGetLastError() after a <<<>>> launch, so an error left pending by an earlier HIP
 * call is reported (and consumed) here -- acceptable for measurement tools, which check
 * every call; the product's launches return only their own status (csrc/hg_launch.hpp).
 */
#ifndef SKS_HOMOGRAPHY_TUNE_H
#define SKS_HOMOGRAPHY_TUNE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int hg_tune_num_variants(void);
const char* hg_tune_variant_name(int variant);
/* AoS f32, normalised; algo 0 = ACA, 1 = SKS; per_cu = blocks per CU for persistent
 * variants (ignored otherwise). */
int hg_tune_aos_f32(int algo, int variant, const float* src, const float* tar, float* H,
                    int64_t n, int per_cu, void* stream);

/* Streaming-copy yardstick variants: 0 = 4x16 B/lane nt, 1 = 8x16 B/lane nt,
 * 2 = 4x16 B/lane plain, 3 = LDS-DMA 8 KiB per wave (bytes % 32 KiB == 0). */
int hg_tune_copy(int variant, const void* src, void* dst, int64_t bytes, void* stream);

/* SoA (reference GPU layout), unnormalised; each variant fixes its dtype.  algo: 0 ACA,
 * 1 SKS; binary64 variants of the 16-B register and narrow forms also 2 GE, 3 GPT-LU. */
int hg_tune_num_soa_variants(void);
const char* hg_tune_soa_variant_name(int variant);
int hg_tune_soa(int algo, int variant, const void* src, const void* tar, void* H, int64_t n,
                int per_cu, void* stream);

/* RANSAC scorer variants: 0 = one hypothesis per lane, 1/2 = two per lane packed
 * (inner unroll 1/4).  Same counts as hg_ransac_score_f32. */
/* TensorACA tile sweep: 0-2 rect form P = 1/2/4 (a = scale, b = div); 3-5 compact form
 * P = 1/2/4 (src = corner, tar = offsets, a = width, b = height). */
int hg_tune_rect(int variant, const float* src, const float* tar, float* H, int64_t B, float a,
                 float b, void* stream);

/* TensorACA (B,3,4) backward with every gradient (gsrc, gtar, gterms (2,B,3); 16-B aligned,
 * B % 64 == 0): 0 = the shipped staged kernel, 1 = its no-arithmetic twin (same loads and
 * stores: the memory pattern's ceiling). */
int hg_tune_rect_backward(int variant, const float* src, const float* tar, const float* gH,
                          int64_t B, const float* scale, const float* div, float* gsrc,
                          float* gtar, float* gterms, void* stream);

/* q = a / b elementwise (n even) in packed pairs as the RANSAC samplers divide: packed != 0
 * the shipped expansion (div_rn, hg_solvers.hpp), 0 the compiler's scalar divisions. */
int hg_tune_div_pairs(int packed, const float* a, const float* b, float* q, int64_t n,
                      void* stream);

/* Fused sampler variants: 0 global gather, 1 / 2 pool staged in LDS (P = 1 / 2), 3 P = 2 with
 * two-tile prefetch, 4-6 wider blocks, 7 P = 2 with the 64-bit remainder, 8 P = 2 solved as
 * packed f32x2 pairs (shipped), 9 the same with the pairs' divisions split into scalar ones. */
int hg_tune_sample(int variant, const float* pool_src, const float* pool_tar, uint32_t npool,
                   const uint32_t* idx, float* H, int64_t n, int algo, int flags, void* stream);

/* cal_ACA's launch loop in native code: `loops` back-to-back C-ABI launches, timed with
 * HIP events on `stream`; returns us per launch or -(hipError_t).  elem 4 / 8 bytes.
 * algo 0 ACA, 1 SKS; launch-floor probes: 2 empty kernel, 3 + hipGetLastError, 4 / 5 / 7
 * raw SoA f64 ACA kernels, 6 one-dword store, 8-11 one-dword store with sc0 sc1 / sc1 /
 * sc0 sc1 nt / nt, 12 one load per lane and no store, 13 pointer arguments never read, 14
 * arguments read and no other memory access. */
double hg_tune_launch_loop(int algo, int elem, const void* src, const void* tar, void* H,
                           int64_t n, int layout, int flags, int loops, void* stream);

/* Cache-policy probe over `bytes` (< 2 GiB): 0-5 buffer stores with aux 0 / sc0 / nt / sc0|nt /
 * sc1 / sc1|nt, 6-11 buffer loads with the same bits (one sink dword per lane into dst). */
int hg_tune_policy(int variant, const void* src, void* dst, int64_t bytes, void* stream);

/* The one-launch Table-8 kernel's H store pattern alone: blocks of 1024 lanes own `classes`
 * consecutive residue classes (64 ... 1024) and store 9 SoA rows per hypothesis. */
int hg_tune_mrg_pattern(int classes, double* H, int64_t n, void* stream);

/* Row-stream probe: RI input / RO output rows of row_bytes at pitch_bytes; variant 0 (16,9),
 * 1 (16,8), 2 (8,4), 3 (4,2), 4 (2,1), 5 (16,9) with 4 chunks per lane, 6 (32,16). */
int hg_tune_streams(int variant, const void* in, void* out, int64_t row_bytes,
                    int64_t pitch_bytes, void* stream);

/* Seeded fused sampler, (P, waves per block[, draws in place]): 0 shipped (packed pairs,
 * (2, 8); ACA from 4 M hypotheses (2, 4)), 13 (1, 16, in place) -- the round-1 shipped form,
 * 1 (2, 4), 2 (1, 16), 3 (2, 16), 4 (2, 8) with the 64-bit remainder, 5 / 6 one hash per draw
 * (a different stream) at (2, 4) / (2, 8), 7 (2, 8, in place), 8 (2, 4, in place), 9 (2, 8)
 * -- the previous shipped form; 10 / 11 / 12 (2, 8 / 16 / 4, in place) with the two
 * hypotheses of a lane solved as packed f32x2 pairs whose divisions split into scalar
 * expansions (10 and 12: the round-2 shipped forms; 0 packs the divisions' FMA steps too);
 * 14-18 the packed-division pairs with other remainders / ablations.  "In place": each
 * tile's draws made where they are used rather than one tile ahead. */
int hg_tune_sample_seeded(int variant, const float* pool_src, const float* pool_tar,
                          uint32_t npool, uint64_t seed, uint64_t offset, float* H, int64_t n,
                          int algo, int flags, void* stream);

/* binary64 AoS sweep: 0 P1 nt LDS-DMA (shipped), 1 P2 nt LDS-DMA, 2 P1 nt register-staged,
 * 3 P1 LDS-DMA default policy. */
int hg_tune_aos_f64(int algo, int variant, const double* src, const double* tar, double* H,
                    int64_t n, void* stream);

int hg_tune_score(int variant, const float* H, int64_t n, const float* pool_src,
                  const float* pool_tar, uint32_t npool, float thresh, uint32_t* counts,
                  void* stream);

/* The fused get_rand_list + cal_Homo_ACA/SKS kernel (hg_gather.hpp) in other shapes: 0 pool
 * in LDS, 1024-lane persistent blocks (shipped up to 5120 pairs); 1 global gather; 2 / 3 pool
 * in LDS with 512 / 256-lane blocks.  algo 0 ACA, 1 SKS; unnormalised (9,n) H. */
int hg_tune_gather_solve_f64(int variant, int algo, const double* pool_src, const double* pool_tar,
                             uint32_t size, const uint32_t* rand_list, double* H, int64_t n,
                             void* stream);

/* MRG32K3A (round 3).  rocRAND's own host API -- a fresh generator per call, as the reference
 * harness creates one (GPU_Runtime Test.cu:1443-1446) -- the checker the hand-written
 * generator is pinned against; synchronous.  ROCRAND_STATUS_ALLOCATION_FAILED ->
 * hipErrorOutOfMemory, any other failure -> hipErrorLaunchFailure. */
int hg_tune_rocrand_mrg32k3a_u32(uint32_t* out, int64_t count, uint64_t seed, void* stream);
/* hg_rand_mrg32k3a_u32 with another split threshold (positions per thread). */
int hg_tune_mrg_words(uint32_t* out, int64_t count, uint64_t seed, int64_t min_chunk,
                      void* stream);
/* Fused draws + gather + solve, unnormalised ACA (0) / SKS (1): variant 0 pool in global
 * memory, 1 pool in LDS beside the draws buffers (the shipped form when it fits); 2 ... 8 the
 * shipped form with the solve (2), the table jumps of the engine starts (3), the engine
 * steps (4) or combinations removed (5 = 2+3, 6 = 2+4, 7 = 3+4, 8 = all) -- wrong bits,
 * timing only. */
int hg_tune_rand_gather_solve_f64(int variant, int algo, const double* pool_src,
                                  const double* pool_tar, uint32_t size, uint64_t seed, double* H,
                                  int64_t n, void* stream);

#ifdef __cplusplus
}
#endif

#endif
