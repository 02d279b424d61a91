/*
 * sks_homography.h -- C ABI of the MI355X (gfx950) batched 4-point homography
 * solver.  Library: sks-homography_amd/lib/libsks_homography_amd.so
 *
 * Every entry point except hg_solve_host_* (host-resident batches, synchronous, below) and
 * hg_rand_mrg32k3a_u32 (rocRAND's generator: allocates once, synchronises, below):
 *   - takes DEVICE pointers the caller owns (the library allocates nothing),
 *   - enqueues its work on `stream` (a hipStream_t; NULL = the legacy default
 *     stream) and returns without synchronising,
 *   - returns 0 on success, otherwise a hipError_t code: hipErrorInvalidValue (1)
 *     for bad arguments (n < 0, NULL pointer with n > 0, unknown layout/flags),
 *     or the status of this call's own launch (hipLaunchKernel's return).  An error an
 *     earlier, unrelated HIP call left pending on the calling thread is neither returned
 *     nor cleared: it stays for its owner's hipGetLastError().  Per-problem numerics are
 *     never checked: a degenerate quad yields Inf/NaN exactly as the reference does
 *     (ACA_SKS.cpp:101 always returns 0),
 *   - is thread-safe (no global mutable state) and safe to capture in a hipGraph.
 *
 * A "problem" is 4 source + 4 target points ordered M, N, P, Q.
 *   HG_LAYOUT_AOS: src/tar are (n,8) {Mx,My,Nx,Ny,Px,Py,Qx,Qy} rows, H is (n,9)
 *                  row-major 3x3 -- the layout of the reference C++ API
 *                  (C++ Codes/modules/ACA_SKS.hpp:17-20, one problem per call).
 *   HG_LAYOUT_SOA: src/tar are (8,n), H is (9,n) -- the reference GPU layout
 *                  (C++ Codes/Runtime Test/GPU_Runtime Test/GPU_Runtime Test.cu:87-95,
 *                  :141-149).
 * HG_FLAG_NORMALIZE scales H so that H[8] == 1 exactly as ACA_SKS.cpp:94-98
 * (reciprocal of H[8], eight multiplies, H[8] := 1).  Without it H is returned up
 * to scale, as the reference CUDA kernels and the PyTorch formulations do.
 *
 * Results are bit-identical to the reference's C++ CPU path (no FMA contraction,
 * reference association order, IEEE division).
 */
#ifndef SKS_HOMOGRAPHY_H
#define SKS_HOMOGRAPHY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HG_LAYOUT_AOS 0
#define HG_LAYOUT_SOA 1
#define HG_FLAG_NORMALIZE 1
/* hg_solve_host_* only (new in 0.3): register the caller's pageable pages for the call
 * instead of staging them -- see hg_solve_host_f32. */
#define HG_FLAG_HOST_REGISTER 2

/* ACA, binary32.  Replaces sks::runKernel_ACA (C++ Codes/modules/ACA_SKS.cpp:24-102)
 * batched; with HG_LAYOUT_SOA and no flag it is the FP32 analogue of
 * cal_Homo_ACA (GPU_Runtime Test.cu:81-151). */
int hg_aca_f32(const float* src, const float* tar, float* H, int64_t n, int layout, int flags,
               void* stream);

/* ACA, binary64.  Replaces sks::runKernel_ACA_double (ACA_SKS.cpp:104-179); with
 * HG_LAYOUT_SOA and no flag it replaces cal_Homo_ACA (GPU_Runtime Test.cu:81-151). */
int hg_aca_f64(const double* src, const double* tar, double* H, int64_t n, int layout,
               int flags, void* stream);

/* SKS, binary32.  Replaces sks::runKernel_SKS (ACA_SKS.cpp:189-303). */
int hg_sks_f32(const float* src, const float* tar, float* H, int64_t n, int layout, int flags,
               void* stream);

/* SKS, binary64.  Replaces sks::runKernel_SKS_double (ACA_SKS.cpp:305-418); with
 * HG_LAYOUT_SOA and no flag it replaces cal_Homo_SKS (GPU_Runtime Test.cu:153-240). */
int hg_sks_f64(const double* src, const double* tar, double* H, int64_t n, int layout,
               int flags, void* stream);

/* RHO Gaussian elimination, binary32 -- the reference's comparison baseline
 * cv::runKernel_GE (C++ Codes/modules/GE.cpp:41-188; OpenCV rho.cpp hFuncRefC), batched
 * (SURVEY 8(f).4).  Its H[8] is 1 by construction; HG_FLAG_NORMALIZE is accepted and
 * changes no bits. */
int hg_ge_f32(const float* src, const float* tar, float* H, int64_t n, int layout, int flags,
              void* stream);

/* RHO Gaussian elimination, binary64 -- the reference GPU harness's cal_Homo_GE
 * (GPU_Runtime Test.cu:359-507: GE.cpp's statements in double), batched; Table 8's GE
 * row.  H[8] is 1 by construction. */
int hg_ge_f64(const double* src, const double* tar, double* H, int64_t n, int layout,
              int flags, void* stream);

/* 8x8 LU with partial pivoting, binary64 -- the reference GPU harness's
 * getPerspectiveTransform baseline cal_Homo_GPT (GPU_Runtime Test.cu:301-357, helpers
 * :242-300), batched.  H[8] is 1 by construction. */
int hg_gpt_f64(const double* src, const double* tar, double* H, int64_t n, int layout,
               int flags, void* stream);

/* TensorACA, rectangle -> quadrangle, binary32, unnormalised.  Replaces
 * TensorACA_rect(bs, src, tar, scale, div) (PyTorch Codes/Modules_Runtime_Test.py:286-309).
 * src, tar: (B,3,4) homogeneous point tensors (rows x, y, 1; columns M, N, P, Q);
 * only src[:,0,0] and src[:,1,0] are read.  H: (B,3,3).  scale = rectangle width,
 * div = width / height, both shared by the batch (.py:33-35); here they are DEVICE
 * pointers to one float each, as the reference keeps them in (1,)-shaped tensors. */
int hg_tensor_aca_rect_f32(const float* src, const float* tar, float* H, int64_t B,
                           const float* scale, const float* div, void* stream);

/* Same with host-side scalars. */
int hg_tensor_aca_rect_f32_hostscalar(const float* src, const float* tar, float* H, int64_t B,
                                      float scale, float div, void* stream);

/* Backward of hg_tensor_aca_rect_f32 (the gradients ATen autograd gives the
 * reference's composed TensorACA_rect, Modules_Runtime_Test.py:294-302).  grad_H:
 * (B,3,3) dL/dH.  Writes grad_tar (B,3,4); grad_src (B,3,4, only [0][0] and [1][0]
 * non-zero) when non-NULL; grad_scale_div (2,B) when non-NULL: [0][b] problem b's share
 * of dL/dscale, [1][b] its share of dL/ddiv, each the sum of the problem's three row terms
 * from +0 (((0 + t0) + t1) + t2, ATen-CPU's reduction to a (B,1,1) operand); their sum over
 * b is the batch-uniform gradient up to summation order.  scale, div: device pointers.
 * This layout is the one every version of the library has had under this name; the
 * (problem, row) terms for ATen's bit-exact batch sum are hg_tensor_aca_rect_backward_terms_f32. */
int hg_tensor_aca_rect_backward_f32(const float* src, const float* tar, const float* grad_H,
                                    int64_t B, const float* scale, const float* div,
                                    float* grad_src, float* grad_tar, float* grad_scale_div,
                                    void* stream);

/* The same backward with the (problem, row) terms instead of per-problem sums: grad_terms
 * (2,B,3) when non-NULL -- [0] the terms of dL/dscale, [1] those of dL/ddiv, each in the
 * order of the (B,3,1) tensor ATen autograd sums to the (1,) parameter.  Reduce each half
 * with hg_sum_aten_f32 (rows 1, m 3B) for ATen-CPU's bits, or hg_sum_rocm_f32 (FULL) for
 * torch-ROCm's.  New in 0.2 (hg_version). */
int hg_tensor_aca_rect_backward_terms_f32(const float* src, const float* tar, const float* grad_H,
                                          int64_t B, const float* scale, const float* div,
                                          float* grad_src, float* grad_tar, float* grad_terms,
                                          void* stream);

/* The all-gradient backward for a batch-uniform (one-value) scale / div, their gradients
 * summed in ATen-CPU's order: the bits of hg_tensor_aca_rect_backward_terms_f32 followed by
 * hg_sum_aten_f32(workspace, 2, 3B, 3B, 1, lanes, threads, grad_sd) -- grad_sd[0] = dL/dscale,
 * grad_sd[1] = dL/ddiv -- with the sum's first level folded into the backward kernel, so the
 * 24 B of terms a problem has are never written out and read back.
 * workspace: 6B floats of device scratch.  grad_src may be NULL (not wanted).  lanes and
 * threads as for hg_sum_aten_f32.  New in 0.3 (hg_version). */
int hg_tensor_aca_rect_backward_sum_f32(const float* src, const float* tar, const float* grad_H,
                                        int64_t B, const float* scale, const float* div,
                                        float* grad_src, float* grad_tar, float* workspace,
                                        int lanes, int threads, float* grad_sd, void* stream);

/* TensorACA with scale / div broadcast the way the reference composition broadcasts them
 * (Modules_Runtime_Test.py:301-302: torch.mul(div, X) and scale * h_temp, X and h_temp
 * (B,3,1)): any shape broadcastable to (B,3,1) -- one value, one per problem ((B,1,1)),
 * one per row ((3,1)), one per (problem, row) ((B,3,1)).  Value (b, r) is
 * scale[b * scale_sb + r * scale_sr] (element strides; 0 along a broadcast dimension), the
 * same for div.  Same arithmetic and bits as hg_tensor_aca_rect_f32 where the values agree.
 * One lane per problem (the batch-uniform entry points above keep the LDS-staged kernel). */
int hg_tensor_aca_rect_bcast_f32(const float* src, const float* tar, float* H, int64_t B,
                                 const float* scale, int64_t scale_sb, int64_t scale_sr,
                                 const float* div, int64_t div_sb, int64_t div_sr, void* stream);

/* Its backward: grad_tar (B,3,4), grad_src (B,3,4) when non-NULL, and per parameter, when
 * its pointer is non-NULL and by its *_rows mode: 0 -- each problem's three-row sum ((B):
 * ATen's reduction to a (B,1,1) parameter, final); 1 -- each row's share of dL/dparam(b, r)
 * as (3,B) rows, row r at [r * B]; 2 -- the same terms as (B,3), [3 b + r] (the order ATen
 * sums them to a batch-uniform parameter).  The caller sums modes 1 / 2 over the
 * parameter's broadcast dimensions in ATen's order (hg_sum_aten_f32: mode 1 rows 3,
 * lanes 1 for a (3,1) parameter; mode 2 rows 1 for a one-value parameter). */
int hg_tensor_aca_rect_bcast_backward_f32(const float* src, const float* tar, const float* grad_H,
                                          int64_t B, const float* scale, int64_t scale_sb,
                                          int64_t scale_sr, const float* div, int64_t div_sb,
                                          int64_t div_sr, float* grad_src, float* grad_tar,
                                          float* grad_scale, int scale_rows, float* grad_div,
                                          int div_rows, void* stream);

/* Whose evaluation of the reference's TensorACA_rect statements to reproduce, bit for bit.
 * HG_ORDER_ATEN_CPU: ATen on the CPU (what the fixtures pin, and what every other TensorACA
 * entry point follows).  HG_ORDER_ATEN_ROCM: torch-ROCm on the GPU -- the reference's default
 * run (Modules_Runtime_Test.py:393, device='cuda') -- which sums every 3-term reduction as
 * ((0 + t0) + t2) + t1 (the forward's torch.sum and the backward's sum_to_size over three
 * elements); cross products and element-wise ops are the same bits on both. */
#define HG_ORDER_ATEN_CPU 0
#define HG_ORDER_ATEN_ROCM 1

/* hg_tensor_aca_rect_bcast_f32 / its backward with the evaluation order `order`
 * (HG_ORDER_*); strides 0 / 0 give the batch-uniform (1,) scale / div.  HG_ORDER_ATEN_CPU
 * is exactly the bcast entry points.  The backward's per-parameter modes are theirs, and
 * modes 1 / 2 leave the batch sums to the caller: hg_sum_aten_f32 for ATen-CPU's order,
 * hg_sum_rocm_f32 on mode-2 (B,3) terms for the GPU run's (its reduction tree needs that
 * layout, for a (3,1) parameter too). */
int hg_tensor_aca_rect_order_f32(const float* src, const float* tar, float* H, int64_t B,
                                 const float* scale, int64_t scale_sb, int64_t scale_sr,
                                 const float* div, int64_t div_sb, int64_t div_sr, int order,
                                 void* stream);
int hg_tensor_aca_rect_backward_order_f32(const float* src, const float* tar, const float* grad_H,
                                          int64_t B, const float* scale, int64_t scale_sb,
                                          int64_t scale_sr, const float* div, int64_t div_sb,
                                          int64_t div_sr, float* grad_src, float* grad_tar,
                                          float* grad_scale, int scale_rows, float* grad_div,
                                          int div_rows, int order, void* stream);

/* Compact TensorACA for deep-homography nets: the source is the
 * axis-aligned width x height rectangle with top-left corner (B,2) -- getInput's shape,
 * Modules_Runtime_Test.py:9-16 -- and the target is source + offsets (B,4,2), the
 * 4-corner offsets a network predicts (getTar, .py:19-21).  Identical bits to
 * building the (B,3,4) tensors with float adds and calling hg_tensor_aca_rect_f32
 * with scale = width, div = width / height; moves 76 B per problem instead of 132. */
int hg_tensor_aca_offsets_f32(const float* corner, const float* offsets, float* H, int64_t B,
                              float width, float height, void* stream);

/* Backward of hg_tensor_aca_offsets_f32: grad_offsets (B,4,2); grad_corner (B,2) when
 * non-NULL. */
int hg_tensor_aca_offsets_backward_f32(const float* corner, const float* offsets,
                                       const float* grad_H, int64_t B, float width,
                                       float height, float* grad_offsets, float* grad_corner,
                                       void* stream);

/* Backward of the unnormalised general-quad ACA (ACA_vanilla, PyTorch Codes/
 * Modules_Runtime_Test.py:312-388, which ATen autograd differentiates w.r.t. src and tar):
 * src, tar (n,8) = (n,4,2) AoS, grad_H (n,9) -> grad_src, grad_tar (n,8), either may be
 * NULL (not both).  The gradients ATen autograd gives through the reference's statements,
 * bit for bit (operations in the autograd engine's order; hg_solvers.hpp aca_vanilla_grad).
 * 16-B aligned float buffers take the LDS-staged kernel. */
int hg_aca_backward_f32(const float* src, const float* tar, const float* grad_H, int64_t n,
                        float* grad_src, float* grad_tar, void* stream);
int hg_aca_backward_f64(const double* src, const double* tar, const double* grad_H, int64_t n,
                        double* grad_src, double* grad_tar, void* stream);

/* Synthetic input stream: out[i] = lo + (hi - lo) * u(i), u(i) = top 24 bits of
 * splitmix64(seed * 0xD1B54A32D192ED03 + offset + i) * 2^-24.  Counter based, so a
 * rank can generate its own shard (offset = first element) and a host can
 * regenerate any slice bit for bit.  Plays the role of the reference's cuRAND
 * draw + get_rand_list gather (GPU_Runtime Test.cu:1443-1451, :52-78). */
int hg_fill_uniform_f32(float* out, int64_t count, uint64_t seed, uint64_t offset, float lo,
                        float hi, void* stream);

/* Counter-based 32-bit draws: out[i] = word(offset + i), where word w is the high (w even)
 * or low (w odd) 32 bits of splitmix64(seed * 0xA0761D6478BD642F + w / 2) -- one 64-bit
 * finaliser per two draws.  The RANSAC sampler's index source (the reference draws with
 * cuRAND MRG32K3A, GPU_Runtime Test.cu:1443-1446).  out: 4-B aligned. */
int hg_fill_bits_u32(uint32_t* out, int64_t count, uint64_t seed, uint64_t offset,
                     void* stream);

/* Fused RANSAC-style hypothesis generator + solver (GPU_Runtime Test.cu:52-78 fused
 * with :81-151).  pool_src/pool_tar: (npool,2) correspondences (8-B aligned); idx:
 * (n,4) uint32 indices (16-B aligned), each reduced modulo npool like get_rand_list
 * (.cu:56-59).  Writes the gathered problem's H (AoS, (n,9), 16-B aligned); algo 0 =
 * ACA, 1 = SKS. */
int hg_sample_solve_f32(const float* pool_src, const float* pool_tar, uint32_t npool,
                        const uint32_t* idx, float* H, int64_t n, int algo, int flags,
                        void* stream);

/* The fused sampler with the draws made in the kernel: equals
 * hg_fill_bits_u32(idx, 4*n, seed, offset) followed by hg_sample_solve_f32(..., idx, ...),
 * bit for bit, without the (n,4) index array (cuRAND + get_rand_list + cal_Homo_ACA/SKS,
 * GPU_Runtime Test.cu:1443-1451, :52-78, :81-240, as one launch).  H: (n,9), 16-B
 * aligned; pools 8-B aligned. */
int hg_sample_solve_seeded_f32(const float* pool_src, const float* pool_tar, uint32_t npool,
                               uint64_t seed, uint64_t offset, float* H, int64_t n, int algo,
                               int flags, void* stream);

/* Inlier count per hypothesis: counts[h] = #{i : w' != 0 and
 * (x' - u w')^2 + (y' - v w')^2 <= thresh^2 w'^2}, (x',y',w') = H_h (x_i, y_i, 1),
 * (u_i, v_i) = pool_tar[i] -- the squared reprojection error against thresh, without
 * the division (exact FMA placement documented in csrc/hg_ransac.hip).  H: (n,9). */
int hg_ransac_score_f32(const float* H, int64_t n, const float* pool_src, const float* pool_tar,
                        uint32_t npool, float thresh, uint32_t* counts, void* stream);

/* ---- The reference's Table-8 sampling pipeline in its own formats (hg_table8.hip) ----
 * GPU_Runtime Test.cu:1443-1451: 4*n MRG32K3A words, get_rand_list, cal_ACA/cal_SKS.
 * rand_list is (4,n) uint32 -- word k of hypothesis id at rand_list[id + k*n], as
 * get_rand_list reads it (.cu:56-59) -- and each word selects pool[word % size] (modulo
 * bias and duplicates kept).  Pools are (size,2) binary64 {x, y} pairs (Point2d),
 * 16-B aligned. */

/* curandCreateGenerator(CURAND_RNG_PSEUDO_MRG32K3A) + curandSetPseudoRandomGeneratorSeed
 * + curandGenerate (.cu:1443-1446): `count` 32-bit MRG32K3A words into `out`, every call
 * starting the stream at `seed`, offset 0.  A hand-written generator (csrc/hg_mrg32k3a.hpp,
 * hg_gather.hpp::mrg_words_kernel): L'Ecuyer's recurrence with rocRAND's seeding, output
 * conversion and host-API word order (word i = position i / 2^17 of subsequence
 * i % 2^17), equal to rocrand_generate's words (tested); cuRAND's own seeding, conversion
 * and ordering are not available in this image, so equality with cuRAND is unpinned.
 * Asynchronous on `stream`, allocates nothing, graph-capturable (the host computes the
 * start states' jumps into the launch arguments). */
int hg_rand_mrg32k3a_u32(uint32_t* out, int64_t count, uint64_t seed, void* stream);

/* HOST function: the MRG32K3A engine state after seeding with `seed`, skipping
 * `subsequence` subsequences of 2^76 words and then `offset` words -- what
 * curand_init(seed, subsequence, offset, &state) / rocrand_init set up -- as
 * state[6] = {x1[n-3], x1[n-2], x1[n-1], x2[n-3], x2[n-2], x2[n-1]}.  The next word is then
 * made from these.  Returns 0, or hipErrorInvalidValue for a NULL state. */
int hg_mrg32k3a_state(uint64_t seed, uint64_t subsequence, uint64_t offset, uint32_t* state);

/* get_rand_list (.cu:52-78) itself: d_src / d_tar (8,n) binary64 rows, row 2k / 2k+1 =
 * x / y of the k-th selected point. */
int hg_get_rand_list_f64(const uint32_t* rand_list, uint32_t size, const double* pool_src,
                         const double* pool_tar, double* d_src, double* d_tar, int64_t n,
                         void* stream);

/* get_rand_list fused with cal_Homo_{ACA,SKS,GE,GPT} (.cu:52-78 + :81-507): H (9,n)
 * binary64 SoA, the bits of hg_get_rand_list_f64 followed by hg_<algo>_f64(...,
 * HG_LAYOUT_SOA, flags) without the (8,n) rows ever reaching memory.  algo: HG_ALGO_*;
 * flags 0 (the reference kernels' unnormalised H) or HG_FLAG_NORMALIZE. */
int hg_gather_solve_f64(int algo, const double* pool_src, const double* pool_tar, uint32_t size,
                        const uint32_t* rand_list, double* H, int64_t n, int flags, void* stream);

/* The whole Table-8 draw step fused too (.cu:1443-1451 + :52-78 + :81-507): the bits of
 * hg_rand_mrg32k3a_u32(words, 4*n, seed) followed by hg_gather_solve_f64(..., words, ...),
 * with the (4,n) words made in registers and never written to memory.  n <= 2^61. */
int hg_rand_gather_solve_f64(int algo, const double* pool_src, const double* pool_tar,
                             uint32_t size, uint64_t seed, double* H, int64_t n, int flags,
                             void* stream);

/* ONE problem, latency path: src[8] and tar[8] are read on the HOST and passed in the
 * kernel launch itself (no copy); H[9] is written by the device -- pass device memory,
 * or host memory mapped into the device address space (hipHostMalloc(...,
 * hipHostMallocMapped) and its hipHostGetDevicePointer) to skip the D2H copy too.
 * Asynchronous like every entry point: synchronise `stream` before reading H.  algo 0 =
 * ACA, 1 = SKS.  What sks::runKernel_* (ACA_SKS.cpp:24, :104, :189, :305) use for host
 * pointers (hg_sks_api.cpp). */
int hg_solve_one_f32(int algo, const float* src, const float* tar, float* H, int flags,
                     void* stream);
int hg_solve_one_f64(int algo, const double* src, const double* tar, double* H, int flags,
                     void* stream);

/* Solver ids of hg_solve_host_*. */
#define HG_ALGO_ACA 0
#define HG_ALGO_SKS 1
#define HG_ALGO_GE 2
#define HG_ALGO_GPT 3 /* binary64 only */

/* A batch whose src/tar/H live in HOST memory -- the reference C++ API's data placement
 * (ACA_SKS.hpp:17-20 take host arrays; CPU_Runtime Test/main.cpp:87-114), batched.  The
 * kernel of hg_<algo>_f32/_f64 solves it with the same bits:
 *  - pinned memory (hipHostMalloc, or the caller's own hipHostRegister with a device mapping)
 *    is read and written by the kernel in place over PCIe (zero-copy: both link directions
 *    busy at once, no device buffer);
 *  - pageable memory is copied, by host threads, through a ring of library-owned pinned
 *    stages (chunk k copied in while the kernel reads chunk k-1's stage, H copied out once
 *    its chunk is done).  The caller's pages are only ever touched by the CPU: the call
 *    leaves no GPU mapping of them behind (0.3);
 *  - with HG_FLAG_HOST_REGISTER, pageable memory is instead registered
 *    (hipHostRegisterMapped, whole pages, overlapping buffers merged) for the call and
 *    unregistered once no call uses it any more (concurrent calls on buffers that share
 *    pages share the library's registration, reference-counted; a call whose pages only
 *    partly overlap another's registration waits for it; a call fails
 *    (hipErrorHostMemoryAlreadyRegistered ...) if the caller itself holds a registration over
 *    part of those pages).  Zero-copy, but the driver keeps the pages mapped for the GPU
 *    after the unregistration: a later HIP copy of >= 2 MB into those heap pages, once reused,
 *    can fault.  Use it only on memory that is never handed back
 *    to the heap (e.g. a shared-memory mapping kept for the process's life).
 * Device or managed pointers are accepted too.
 * SYNCHRONOUS, unlike every other entry point: H is complete on return.  stream NULL =
 * hipStreamPerThread when any buffer is host memory, else the legacy default stream.
 * Same layouts, flags (plus HG_FLAG_HOST_REGISTER), validation and bits as hg_<algo>_*; algo
 * is an HG_ALGO_* id (HG_ALGO_GPT binary64 only).  hipErrorInvalidValue also when a buffer's
 * first and last bytes lie in different kinds of memory (e.g. a pinned block and pageable
 * memory after it).  Buffers must be the caller's own, whole: the call cannot see every
 * overrun. */
int hg_solve_host_f32(int algo, const float* src, const float* tar, float* H, int64_t n,
                      int layout, int flags, void* stream);
int hg_solve_host_f64(int algo, const double* src, const double* tar, double* H, int64_t n,
                      int layout, int flags, void* stream);

/* Many small batches in one launch: batch i is src[i], tar[i] -> H[i] with n[i] problems
 * (device pointers; the four arrays themselves are HOST arrays of `count` entries), every
 * batch in `layout` with `flags`, solved by `algo` (an HG_ALGO_* id; HG_ALGO_GPT binary64
 * only).  Up to 32 batches travel in one launch's arguments (more are split into further
 * launches on `stream`; empty batches are skipped).  The bits equal hg_<algo>_* on each
 * batch.  For callers with many small batches (e.g. a RANSAC per image pair), where one
 * launch per batch is bound by the ~2.7 us per-launch cost rather than by the work. */
int hg_solve_grouped_f32(int algo, const float* const* src, const float* const* tar,
                         float* const* H, const int64_t* n, int count, int layout, int flags,
                         void* stream);
int hg_solve_grouped_f64(int algo, const double* const* src, const double* const* tar,
                         double* const* H, const int64_t* n, int count, int layout, int flags,
                         void* stream);

/* Deterministic sums of the rows of x (rows, cols), row-major, into out[rows]: a fixed
 * two-level order (chunks of 4096 in order, folded by halving strides), so the bits do
 * not depend on timing.  x is OVERWRITTEN (used as the scratch for the chunk sums).
 * rows <= 65535.  A general deterministic row sum; the TensorACA gradient terms take
 * hg_sum_aten_f32 (ATen's own order) since round 4, when this stopped being their reduction. */
int hg_sum_rows_f32(float* x, int64_t rows, int64_t cols, float* out, void* stream);

/* Sums in ATen-CPU's float32 order (SumKernel.cpp cascade_sum under TensorIterator's
 * two-pass reduction; restated in oracle/aten_sum.py, pinned against torch.sum): row r of x
 * is x[r * row_stride + e * elem_stride], e < m, and out[r] receives the bits torch.sum of
 * that run gives on ATen-CPU with Vectorized<float>::size() == lanes (8: ATen's sum kernel
 * runs its 8-lane build on AVX2 and AVX-512 hosts alike) and at::get_num_threads() ==
 * threads.  lanes 1, threads 1 give the order of a strided column reduced to (C,1) (the
 * (3,1) parameter case).  1 <= lanes <= 16, 1 <= threads <= 1024, lanes >= 4 when
 * threads > 1; rows * min(threads, ceil(m / 32768)) <= 65535.  x is OVERWRITTEN (scratch).
 * Reduces the gradient terms of hg_tensor_aca_rect_backward_terms_f32 and *_bcast_*. */
int hg_sum_aten_f32(float* x, int64_t rows, int64_t m, int64_t row_stride, int64_t elem_stride,
                    int lanes, int threads, float* out, void* stream);

/* Sums in ATen-ROCm's float32 GPU order: torch.sum / at::sum_to of a contiguous (B,3,1)
 * float tensor x -- over {0,1} to out[1] (HG_SUM_ROCM_FULL: a (1,) parameter's gradient) or
 * over {0} to out[3] (HG_SUM_ROCM_COLS: a (3,1) one) -- with the bits torch-ROCm 2.10 gives
 * on the current device (its CU count and threads per CU pick the launch shape, as ATen's do;
 * restated in oracle/aten_rocm_sum.py, pinned against torch.sum on the MI355X).  How
 * torch-ROCm's autograd reduces TensorACA_rect's batch-uniform scale / div gradient terms
 * (HG_ORDER_ATEN_ROCM).  x is not modified; any alignment, summed in the order ATen gives an
 * aligned tensor (its fresh allocations are); workspace: HG_SUM_ROCM_WORKSPACE
 * device floats, needed when the sum spans several blocks (FULL from B ~ 43K; never COLS).
 * B = 0 writes +0. */
#define HG_SUM_ROCM_FULL 0
#define HG_SUM_ROCM_COLS 1
#define HG_SUM_ROCM_WORKSPACE 1024
int hg_sum_rocm_f32(const float* x, int64_t B, int kind, float* out, float* workspace,
                    void* stream);
/* The launch shape hg_sum_rocm_f32 takes for B >= 2 on a device with num_mp CUs and max_tpm
 * threads per CU (a host computation, no GPU): plan[12] = block x, block y, CTAs per output,
 * input splits x / y / CTA, output splits x / y, input step, output step, loads of 4, grid x.
 * For tests and tools (against oracle/aten_rocm_sum.py's Config). */
int hg_sum_rocm_plan(int64_t B, int kind, int num_mp, int max_tpm, int64_t* plan);

/* Device-to-device streaming copy (float4) used by bench.py as the measured
 * achievable-bandwidth yardstick.  bytes must be a multiple of 16. */
int hg_stream_copy(const void* src, void* dst, int64_t bytes, void* stream);

/* Library build/version string (static storage). */
const char* hg_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SKS_HOMOGRAPHY_H */
