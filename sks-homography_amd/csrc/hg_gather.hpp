// hg_gather.hpp -- the reference's own sampling pipeline in its own data formats
// (GPU_Runtime Test.cu:1443-1451): 4*N cuRAND MRG32K3A words laid out as FOUR ROWS of N
// (word k of hypothesis id at randList[id + k*N]), get_rand_list (:52-78) gathering
// Point2d (two binary64) source / target points into (8,N) SoA binary64 rows, then
// cal_Homo_* (:81-507) over them, unnormalised.  Round 1's sampler (hg_ransac.hpp) is the
// binary32 AoS form of the same pipeline; these kernels keep the reference's formats so
// Table 8's flow runs unchanged, with the gather and the solve fused into one pass.
#pragma once
#include "hg_mrg32k3a.hpp"
#include "hg_ransac.hpp"

#include <type_traits>

namespace hg {

// J^l and J^(256 h) for the subsequence jumps, evaluated by the compiler (internal linkage:
// each translation unit holds its own copy of the 61 KiB)
static __constant__ mrg::JumpTable kMrgJump = mrg::make_jump_table();
static constexpr mrg::PowTable kMrgPow = mrg::make_pow_table();

// J^l v for l < 256 (one table row per lane), as the binary64 engine state.  v: x1[3], x2[3].
__device__ __forceinline__ mrg::State mrg_apply_lo(uint32_t l, const uint32_t (&v)[6]) {
    const uint32_t* e = kMrgJump.lo[l];
    mrg::State st;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        st.x1[r] = (double)mrg::row_dot<1>(e + 3 * r, v[0], v[1], v[2]);
        st.x2[r] = (double)mrg::row_dot<2>(e + 9 + 3 * r, v[3], v[4], v[5]);
    }
    return st;
}

// Element t < 6 of (M v): row t % 3 of component t / 3 of the jump matrix entry e.
__device__ __forceinline__ uint32_t mrg_entry_dot(const uint32_t* e, int t, const uint32_t* v) {
    return t < 3 ? mrg::row_dot<1>(e + 3 * t, v[0], v[1], v[2])
                 : mrg::row_dot<2>(e + 9 + 3 * (t - 3), v[3], v[4], v[5]);
}

// The host API's `count` words: word i = position i >> 17 of subsequence i & (2^17 - 1).
// Block (x, j) owns subsequences 256 x .. 256 x + 255 and positions [j Q, j Q + Q): six lanes
// make the block's base J^(256 x) y[j] (y[j] = A^(j Q) x0), every lane then applies J^l for
// its own l < 256 and writes its positions -- lane-consecutive subsequences, so every store
// instruction covers 256 contiguous bytes.  Default-policy stores: the words are read again
// by the gather that follows, from the MALL when they fit.
// ABL (tune library only): 1 no table jumps (the lane starts from y[j]), 2 no engine steps
// (the words are the lane's index) -- wrong bits, timing only; 4 non-temporal stores (same bits)
template <int ABL = 0>
__global__ __launch_bounds__(kBlock) void mrg_words_kernel(uint32_t* __restrict__ out,
                                                           mrg::WordsArgs a) {
    static_assert(kBlock == mrg::kLo, "one table row per lane");
    __shared__ uint32_t base[6];
    const int j = blockIdx.y;
    if constexpr ((ABL & 1) == 0) {
        if (threadIdx.x < 6) base[threadIdx.x] = mrg_entry_dot(kMrgJump.hi[blockIdx.x], threadIdx.x, a.y[j].w);
        __syncthreads();
    }
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t cols = a.count < mrg::kOrder ? a.count : mrg::kOrder;
    if (s >= cols) return;
    const int64_t q_end_s = (a.count - s + mrg::kOrder - 1) >> mrg::kOrderLog2;
    const int64_t q = (int64_t)j * a.chunk;
    const int64_t q_end = q + a.chunk < q_end_s ? q + a.chunk : q_end_s;
    if (q >= q_end) return;
    mrg::State st;
    if constexpr ((ABL & 1) != 0) {
        st = mrg::unpack(a.y[j]);
        st.x1[0] += threadIdx.x;
    } else {
        const uint32_t v[6] = {base[0], base[1], base[2], base[3], base[4], base[5]};
        st = mrg_apply_lo(threadIdx.x, v);
    }
    // block-uniform base pointer (positions advance it), the lane's subsequence as offset
    uint32_t* o = out + (q << mrg::kOrderLog2) + (int64_t)blockIdx.x * kBlock;
    const uint32_t lane = threadIdx.x;
    const int64_t left = q_end - q;
    int64_t i = 0;
    if constexpr ((ABL & 2) != 0) {
        const uint32_t x = (uint32_t)__double2hiint(st.x1[0]) ^ lane;
        for (; i < left; ++i, o += mrg::kOrder) o[lane] = x + (uint32_t)i;
        return;
    }
    auto put = [&](uint32_t* p, uint32_t w) {
        if constexpr ((ABL & 4) != 0) __builtin_nontemporal_store(w, p);
        else *p = w;
    };
    for (; i + 3 <= left; i += 3, o += 3 * mrg::kOrder) {  // three steps: the state stays put
        put(o + lane, mrg::step<0>(st));
        put(o + mrg::kOrder + lane, mrg::step<1>(st));
        put(o + 2 * mrg::kOrder + lane, mrg::step<2>(st));
    }
    if (i < left) put(o + lane, mrg::step<0>(st));
    if (i + 1 < left) put(o + mrg::kOrder + lane, mrg::step<1>(st));
}

// One lane per hypothesis.  rand_list (4,n) uint32, pool_src / pool_tar (size,2) binary64
// (Point2d), d_src / d_tar (8,n): get_rand_list's own statement order (x, y of r1..r4).
// Exact r % size through fastmod_u32.
__global__ __launch_bounds__(kBlock) void get_rand_list_kernel(
    const uint32_t* __restrict__ rand_list, uint32_t size, uint64_t magic,
    const double2* __restrict__ pool_src, const double2* __restrict__ pool_tar,
    double* __restrict__ d_src, double* __restrict__ d_tar, int64_t n) {
    const int64_t id = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (id >= n) return;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t r = fastmod_u32(rand_list[id + k * n], magic, size);
        const double2 s = pool_src[r], t = pool_tar[r];
        __builtin_nontemporal_store(s.x, d_src + id + (2 * k) * n);
        __builtin_nontemporal_store(s.y, d_src + id + (2 * k + 1) * n);
        __builtin_nontemporal_store(t.x, d_tar + id + (2 * k) * n);
        __builtin_nontemporal_store(t.y, d_tar + id + (2 * k + 1) * n);
    }
}

// Fused get_rand_list + cal_Homo_*: each lane reads its 4 words (4 coalesced rows),
// gathers its 4 correspondences and solves in registers; the (8,n) intermediate rows
// never reach HBM, so a hypothesis moves 16 B in and 72 B out instead of 16 + 2*128 + 2*128
// + 72.  POOL_LDS: the block first copies the pool into LDS as 32-B {sx, sy, tx, ty}
// records and gathers from there (persistent grid, one pool copy per block); otherwise
// the gathers go to the pool in global memory (L2-resident for the reference's sizes).
// 1024-lane blocks (16 waves share one pool copy); GPT-LU's binary64 elimination needs more
// than the 128 VGPRs that allows, so it runs 512-lane blocks.
template <int ALGO>
constexpr int gather_block() { return ALGO == kGPT ? 512 : 1024; }

// V = 2 (tune): a lane owns two consecutive hypotheses, so its word reads are 8 B and its H
// stores 16 B per row (needs n even and 16-B aligned H).
// NTS (tune): non-temporal H stores (shipped) or default-policy ones.
template <int ALGO, bool NORM, bool POOL_LDS, int V = 1, bool NTS = true>
__global__ __launch_bounds__(gather_block<ALGO>()) void gather_solve_f64_kernel(
    const uint32_t* __restrict__ rand_list, uint32_t size, uint64_t magic,
    const double2* __restrict__ pool_src, const double2* __restrict__ pool_tar,
    double* __restrict__ H, int64_t n) {
    static_assert(V == 1 || V == 2, "one or two hypotheses per lane");
    extern __shared__ __attribute__((aligned(16))) char dyn[];
    double2* pool = reinterpret_cast<double2*>(dyn);  // [2 i] = src i, [2 i + 1] = tar i
    if constexpr (POOL_LDS) {
        for (uint32_t i = threadIdx.x; i < size; i += blockDim.x) {
            pool[2 * i] = pool_src[i];
            pool[2 * i + 1] = pool_tar[i];
        }
        __syncthreads();
    }
    auto gather = [&](uint32_t word, double2& a, double2& b) {
        const uint32_t r = fastmod_u32(word, magic, size);
        if constexpr (POOL_LDS) {
            a = pool[2 * r];
            b = pool[2 * r + 1];
        } else {
            a = pool_src[r];
            b = pool_tar[r];
        }
    };
    const int64_t m = n / V;  // lanes' units
    const int64_t stride = POOL_LDS ? (int64_t)gridDim.x * blockDim.x : m;
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < m; u += stride) {
        const int64_t id = u * V;
        double s[V][8], t[V][8], h[V][9];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t w[V];
            if constexpr (V == 1) {
                w[0] = __builtin_nontemporal_load(rand_list + id + k * n);
            } else {
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 x = __builtin_nontemporal_load(
                    reinterpret_cast<const u32x2*>(rand_list + id + k * n));
                w[0] = x[0];
                w[1] = x[1];
            }
#pragma unroll
            for (int v = 0; v < V; ++v) {
                double2 a, b;
                gather(w[v], a, b);
                s[v][2 * k] = a.x; s[v][2 * k + 1] = a.y;
                t[v][2 * k] = b.x; t[v][2 * k + 1] = b.y;
            }
        }
#pragma unroll
        for (int v = 0; v < V; ++v) solve<ALGO, NORM>(s[v], t[v], h[v]);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            if constexpr (V == 1) {
                if constexpr (NTS) __builtin_nontemporal_store(h[0][k], H + id + k * n);
                else H[id + k * n] = h[0][k];
            } else {
                typedef double f64x2 __attribute__((ext_vector_type(2)));
                const f64x2 o = {h[0][k], h[1][k]};
                __builtin_nontemporal_store(o, reinterpret_cast<f64x2*>(H + id + k * n));
            }
        }
    }
}

// The draws fused in too: the bits of mrg_words_kernel(4 n words) followed by
// gather_solve_f64_kernel, with no (4,n) word rows in memory.
//
// Word h + k n (row k of hypothesis h) is position (h + k n) >> 17 of subsequence
// (h + k n) & (2^17 - 1).  For the hypotheses h = h0 + q 2^17 of one residue class h0, row k
// therefore walks ONE subsequence, s_k = (h0 + b_k) mod 2^17, at consecutive positions
// q + a_k + carry_k (k n = a_k 2^17 + b_k, carry_k = h0 + b_k >= 2^17): one engine per
// (class, row), stepped once per hypothesis.  A block owns C = B/4 consecutive classes at a
// time (a group); lane (k, c) runs the engine of row k of class c (k is wave-uniform) and
// writes 4 words per chunk into LDS, then lane (qq, c) solves hypothesis h0_c + (q0 + qq)
// 2^17 from the 4 words of its class and position -- one hypothesis per lane per chunk, the
// next chunk's words made in the same pass (double buffer, one barrier per chunk).  H
// stores stay lane-consecutive in h.  Engine starts: with y[k][c] = A^(a_k + c) x0 from the
// host and base_k = (g C + b_k) mod 2^17, class c of row k starts at J^c (J^base_k y[k][0]),
// or at J^(c - w) y[k][1] past the wrap (c >= w = 2^17 - base_k), or at J^c (J^base_k y[k][1])
// when g C + b_k itself wrapped.  J^base_k y[k][.] is made
// once per group by 24 lanes (two table levels, through LDS, for a batch of the block's
// groups at once); each lane then applies one table row J^c per component.
// Block size: 1024 lanes (16 waves share one pool copy); RHO-GE and GPT-LU hold more than the
// 128 VGPRs that allows beside the engine's binary64 state, so they run 512-lane blocks.
template <int ALGO>
constexpr int mrg_gather_block() { return ALGO == kGPT || ALGO == kGE ? 512 : 1024; }

// Q: positions per chunk (a multiple of 4).  A lane makes Q words of its row per chunk and
// solves Q / 4 hypotheses from the chunk's words; the words buffer is [2][4][Q][classes].
template <int ALGO, int Q = 4, int KB = mrg_gather_block<ALGO>()>
constexpr size_t mrg_words_lds() { return (size_t)2 * 4 * Q * (KB / 4) * 4; }

constexpr int kMrgGroupBatch = 8;  // groups whose engine bases one pass makes
constexpr size_t kMrgStaticLds = 2 * kMrgGroupBatch * 24 * 4;

// Ablations (tune library only: wrong bits, timing only) and shape flags (same bits).  The
// shipped kernel is kMrgStBuf | kMrgIdxF64 (kMrgIdxF64 alone when 8 n >= 2^32; hg_table8.hip).
enum MrgAblation : int {
    kMrgAblNone = 0,
    kMrgAblNoSolve = 1,   // draws + gather, H = a cheap function of the gathered points
    kMrgAblNoStart = 2,   // engines start from the host states, no table jumps
    kMrgAblNoDraws = 4,   // no engine steps: the words are the lane's own index
    kMrgAblNoGather = 8,  // no pool reads: the points are the words themselves
    kMrgSt16 = 16,        // H rows stored as 16-B pairs of adjacent hypotheses (n even)
    kMrgStDefault = 32,   // H stores with the default cache policy instead of non-temporal
    kMrgStBuf = 64,       // H rows through buffer stores: a per-row resource in SGPRs and one
                          // 32-bit lane offset (8 n < 2^32), instead of nine 64-bit lane addresses
    kMrgInterleave = 128, // with kMrgStBuf: a chunk's gathers, then the NEXT chunk's draws, then
                          // its solves, in one basic block (the chunk loop unrolled by the three
                          // engine phases, the draws unconditional): the scheduler may overlap the
                          // independent draw and solve chains (same bits)
    kMrgIdxF64 = 256,     // the engines write pool indices, not words: mrg::step_index, the
                          // remainder in binary64 from the word's own binary64 value (same bits;
                          // `magic` carries fmod_f64_magic(size))
};

// the value of the other lane of an even/odd lane pair (DPP quad_perm [1, 0, 3, 2])
__device__ __forceinline__ double pair_swap(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0xB1, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0xB1, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
typedef double hg_dbl2 __attribute__((ext_vector_type(2)));

template <int ALGO, bool NORM, bool POOL_LDS, int ABL = kMrgAblNone, int Q = 4,
          int KB = mrg_gather_block<ALGO>()>
__global__ __launch_bounds__(KB) void mrg_gather_solve_f64_kernel(
    uint32_t size, uint64_t magic, const double2* __restrict__ pool_src,
    const double2* __restrict__ pool_tar, double* __restrict__ H, int64_t n,
    mrg::GatherArgs a) {
    static_assert(Q % 4 == 0 && Q >= 4, "whole hypotheses per lane per chunk");
    static_assert(KB % 256 == 0 && 24 * kMrgGroupBatch <= KB, "whole waves per row");
    constexpr int kB = KB;
    constexpr int kC = kB / 4;  // classes per group
    constexpr int kQ = Q;       // positions per chunk
    constexpr int kPer = Q / 4; // hypotheses a lane solves per chunk
    extern __shared__ __attribute__((aligned(16))) char dyn[];
    uint32_t* words = reinterpret_cast<uint32_t*>(dyn);  // [2][4][kQ][kC]
    double2* pool = reinterpret_cast<double2*>(dyn + mrg_words_lds<ALGO, Q, KB>());
    if constexpr (POOL_LDS) {
        for (uint32_t i = threadIdx.x; i < size; i += kB) {
            pool[2 * i] = pool_src[i];
            pool[2 * i + 1] = pool_tar[i];
        }
    }
    __shared__ uint32_t base_u[kMrgGroupBatch][24], base_v[kMrgGroupBatch][24];
    const double inv_d = __builtin_bit_cast(double, magic), half_inv_d = 0.5 * inv_d;  // kMrgIdxF64
    const double dd = (double)size;
    const int k = threadIdx.x / kC;  // engine row; also the solve's position in the chunk
    const int c = threadIdx.x % kC;
    const int64_t cols = n < mrg::kOrder ? n : mrg::kOrder;
    const int64_t groups = (cols + kC - 1) / kC;
    const int64_t stride = gridDim.x;
    for (int64_t g0 = blockIdx.x; g0 < groups; g0 += stride * kMrgGroupBatch) {
        // J^base_k y[k][0] of up to kMrgGroupBatch groups: lane (i, kk, t) makes element t
        // of group i, row kk -- first through the table's low level, then the high one
        const int bi = threadIdx.x / 24, br = threadIdx.x % 24, bk = br / 6, bt = br % 6;
        const int64_t bg = g0 + bi * stride;
        const bool bl = (ABL & kMrgAblNoStart) == 0 && threadIdx.x < 24 * kMrgGroupBatch && bg < groups;
        const int64_t braw = bg * kC + a.b[bl ? bk : 0];  // < 2^18
        const int bcarry = braw >= mrg::kOrder;
        const uint32_t bbase = (uint32_t)(braw & (mrg::kOrder - 1));
        if (bl)
            base_u[bi][br] = mrg_entry_dot(kMrgJump.lo[bbase & (mrg::kLo - 1)], bt, a.y[bk][bcarry].w);
        __syncthreads();
        if (bl)
            base_v[bi][br] = mrg_entry_dot(kMrgJump.hi[bbase >> mrg::kLoBits], bt, &base_u[bi][bk * 6]);
        __syncthreads();
    for (int gi = 0; gi < kMrgGroupBatch; ++gi) {
        const int64_t g = g0 + gi * stride;
        if (g >= groups) break;
        const int64_t h0 = g * kC + c;
        mrg::State st;
        if constexpr ((ABL & kMrgAblNoStart) != 0) {
            st = mrg::unpack(a.y[k][0]);
            st.x1[0] += c;
        } else {
            // the group's first class already wrapped (g C + b_k >= 2^17): every class of the
            // row is at position a_k + 1, and its base was made from y[k][1]
            const int64_t raw = g * kC + a.b[k];
            const uint32_t base = (uint32_t)(raw & (mrg::kOrder - 1));
            const uint32_t w = (uint32_t)mrg::kOrder - base;  // classes from w on wrapped
            if (raw >= mrg::kOrder || (uint32_t)c < w) {
                const uint32_t* bv = base_v[gi] + k * 6;
                const uint32_t v[6] = {bv[0], bv[1], bv[2], bv[3], bv[4], bv[5]};
                st = mrg_apply_lo((uint32_t)c, v);
            } else {
                st = mrg_apply_lo((uint32_t)c - w, a.y[k][1].w);
            }
        }
        // chunk m holds steps Q m .. Q m + Q - 1, in state slots (Q m + i) mod 3: one copy of
        // the Q steps per phase (Q m) mod 3 (a block-uniform branch), so no step moves the state
        auto gen = [&](int buf, int phase) {
            uint32_t* w = words + (buf * 4 + k) * kQ * kC + c;
            if constexpr ((ABL & kMrgAblNoDraws) != 0) {
                const uint32_t x = (uint32_t)threadIdx.x * 2654435761u + (uint32_t)phase;
#pragma unroll
                for (int i = 0; i < kQ; ++i) w[i * kC] = x ^ (uint32_t)i;
                return;
            }
            auto steps = [&](auto p) {
                constexpr int P = decltype(p)::value;
#pragma unroll
                for (int i = 0; i < kQ; ++i) {
                    if constexpr ((ABL & kMrgIdxF64) != 0) {
                        const int sl = (P + i) % 3;  // folds
                        w[i * kC] = sl == 0 ? mrg::step_index<0>(st, inv_d, half_inv_d, dd)
                                            : (sl == 1 ? mrg::step_index<1>(st, inv_d, half_inv_d, dd)
                                                       : mrg::step_index<2>(st, inv_d, half_inv_d, dd));
                    } else {
                        w[i * kC] = mrg::step_at(st, (P + i) % 3);  // folds
                    }
                }
            };
            if (phase == 0) steps(std::integral_constant<int, 0>());
            else if (phase == 1) steps(std::integral_constant<int, 1>());
            else steps(std::integral_constant<int, 2>());
        };
        // positions of the group's first class (the others have as many or one fewer)
        const int64_t qn = (n - g * kC + mrg::kOrder - 1) >> mrg::kOrderLog2;
        gen(0, 0);
        __syncthreads();
        if constexpr ((ABL & kMrgInterleave) != 0) {
            static_assert((ABL & kMrgStBuf) != 0 && (ABL & ~(kMrgInterleave | kMrgStBuf | kMrgIdxF64)) == 0,
                          "the interleaved chunk is the shipped one with buffer stores");
            int buf = 0;
            int64_t q0 = 0;
            auto chunk = [&](auto pn) {  // pn: the engine phase of the NEXT chunk
                constexpr int PN = decltype(pn)::value;
                double s[kPer][8], t[kPer][8];
#pragma unroll
                for (int j = 0; j < kPer; ++j) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const uint32_t w = words[((buf * 4 + r) * kQ + k + 4 * j) * kC + c];
                        const uint32_t ix = (ABL & kMrgIdxF64) != 0 ? w : fastmod_u32(w, magic, size);
                        double2 ps, pt;
                        if constexpr (POOL_LDS) {
                            ps = pool[2 * ix];
                            pt = pool[2 * ix + 1];
                        } else {
                            ps = pool_src[ix];
                            pt = pool_tar[ix];
                        }
                        s[j][2 * r] = ps.x; s[j][2 * r + 1] = ps.y;
                        t[j][2 * r] = pt.x; t[j][2 * r + 1] = pt.y;
                    }
                }
                {  // the next chunk's words (past a group's last chunk: drawn, never read)
                    uint32_t* w = words + ((buf ^ 1) * 4 + k) * kQ * kC + c;
#pragma unroll
                    for (int i = 0; i < kQ; ++i) {
                        if constexpr ((ABL & kMrgIdxF64) != 0) {
                            const int sl = (PN + i) % 3;
                            w[i * kC] = sl == 0 ? mrg::step_index<0>(st, inv_d, half_inv_d, dd)
                                                : (sl == 1 ? mrg::step_index<1>(st, inv_d, half_inv_d, dd)
                                                           : mrg::step_index<2>(st, inv_d, half_inv_d, dd));
                        } else {
                            w[i * kC] = mrg::step_at(st, (PN + i) % 3);
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < kPer; ++j) {
                    double hh[9];
                    solve<ALGO, NORM>(s[j], t[j], hh);
                    const int64_t h = h0 + ((q0 + k + 4 * j) << mrg::kOrderLog2);
                    if (h < n) {
                        const uint32_t off = (uint32_t)h * 8u;
#pragma unroll
                        for (int r = 0; r < 9; ++r) {
                            const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
                                H + (int64_t)r * n, 0, (int)(uint32_t)(n * 8), 0x00020000);
                            typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
                            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, hh[r]),
                                                                  rsrc, off, 0, 2);
                        }
                    }
                }
                __syncthreads();
                buf ^= 1;
                q0 += kQ;
            };
            // chunk m's words are in phase (Q m) mod 3: unrolled by three, every phase is static
            for (;;) {
                chunk(std::integral_constant<int, (1 * kQ) % 3>());
                if (q0 >= qn) break;
                chunk(std::integral_constant<int, (2 * kQ) % 3>());
                if (q0 >= qn) break;
                chunk(std::integral_constant<int, 0>());
                if (q0 >= qn) break;
            }
            continue;
        }
        int buf = 0, phase = 0;
        for (int64_t q0 = 0; q0 < qn; q0 += kQ, buf ^= 1) {
            phase = (phase + kQ) % 3;  // the phase of chunk q0 / Q + 1
            if (q0 + kQ < qn) gen(buf ^ 1, phase);
#pragma unroll
            for (int j = 0; j < kPer; ++j) {
            const int qq = k + 4 * j;  // this lane's position in the chunk
            const int64_t h = h0 + ((q0 + qq) << mrg::kOrderLog2);
            if ((ABL & kMrgSt16) != 0 || h < n) {
                double s[8], t[8], hh[9];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t w = words[((buf * 4 + r) * kQ + qq) * kC + c];
                    const uint32_t ix = (ABL & kMrgIdxF64) != 0 ? w : fastmod_u32(w, magic, size);
                    double2 ps, pt;
                    if constexpr ((ABL & kMrgAblNoGather) != 0) {
                        ps = double2((double)w, (double)(w >> 1));
                        pt = double2((double)(w >> 2), (double)(w >> 3));
                    } else if constexpr (POOL_LDS) {
                        ps = pool[2 * ix];
                        pt = pool[2 * ix + 1];
                    } else {
                        ps = pool_src[ix];
                        pt = pool_tar[ix];
                    }
                    s[2 * r] = ps.x; s[2 * r + 1] = ps.y;
                    t[2 * r] = pt.x; t[2 * r + 1] = pt.y;
                }
                if constexpr ((ABL & kMrgAblNoSolve) != 0) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) hh[r] = s[r] + t[7 - r];
                    hh[8] = s[0];
                } else {
                    solve<ALGO, NORM>(s, t, hh);
                }
                if constexpr ((ABL & kMrgSt16) != 0) {
                    // even lane: row r of (h, h + 1); odd lane: row r + 1 of (h - 1, h)
                    const int odd = threadIdx.x & 1;
                    const int64_t he = h - odd;
#pragma unroll
                    for (int r = 0; r < 8; r += 2) {
                        const double got = pair_swap(odd ? hh[r] : hh[r + 1]);
                        const hg_dbl2 v = odd ? hg_dbl2{got, hh[r + 1]} : hg_dbl2{hh[r], got};
                        hg_dbl2* p = reinterpret_cast<hg_dbl2*>(H + (r + odd) * n + he);
                        if (he < n) {
                            if constexpr ((ABL & kMrgStDefault) != 0) *p = v;
                            else __builtin_nontemporal_store(v, p);
                        }
                    }
                    if (h < n) {
                        if constexpr ((ABL & kMrgStDefault) != 0) H[h + 8 * n] = hh[8];
                        else __builtin_nontemporal_store(hh[8], H + h + 8 * n);
                    }
                } else if constexpr ((ABL & kMrgStBuf) != 0) {
                    const uint32_t off = (uint32_t)h * 8u;  // bytes into each row (8 n < 2^32)
#pragma unroll
                    for (int r = 0; r < 9; ++r) {
                        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(H + (int64_t)r * n, 0,
                                                                            (int)(uint32_t)(n * 8), 0x00020000);
                        typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, hh[r]),
                                                              rsrc, off, 0,
                                                              (ABL & kMrgStDefault) != 0 ? 0 : 2);
                    }
                } else if constexpr ((ABL & kMrgStDefault) != 0) {
#pragma unroll
                    for (int r = 0; r < 9; ++r) H[h + r * n] = hh[r];
                } else {
#pragma unroll
                    for (int r = 0; r < 9; ++r) __builtin_nontemporal_store(hh[r], H + h + r * n);
                }
            }
            }
            __syncthreads();
        }
    }
    }
}

// ---- host launchers ----

inline mrg::Packed mrg_seed_jump(uint64_t seed, uint64_t e) {  // A^e x0(seed)
    mrg::Vec x1, x2;
    mrg::seed_state(seed, x1, x2);
    return mrg::pack(mrg::host_jump(kMrgPow.p1, 1, e, x1), mrg::host_jump(kMrgPow.p2, 2, e, x2));
}

// Positions per thread below which the standalone generator stops splitting subsequences
// over more threads (each thread's start costs four 3x3 products mod m).
constexpr int64_t kMrgMinChunk = 64;

template <int ABL = 0>
inline int launch_mrg_words(uint32_t* out, int64_t count, uint64_t seed, int64_t min_chunk,
                            hipStream_t s) {
    mrg::WordsArgs a{};
    a.count = count;
    const int64_t positions = (count + mrg::kOrder - 1) >> mrg::kOrderLog2;
    int64_t chunks = positions / (min_chunk < 1 ? 1 : min_chunk);
    chunks = chunks < 1 ? 1 : (chunks > mrg::kWordsMaxChunks ? mrg::kWordsMaxChunks : chunks);
    a.chunk = (positions + chunks - 1) / chunks;
    chunks = (positions + a.chunk - 1) / a.chunk;
    mrg::Vec x1, x2;
    mrg::seed_state(seed, x1, x2);
    for (int64_t j = 0; j < chunks; ++j)
        a.y[j] = mrg::pack(mrg::host_jump(kMrgPow.p1, 1, (uint64_t)(j * a.chunk), x1),
                           mrg::host_jump(kMrgPow.p2, 2, (uint64_t)(j * a.chunk), x2));
    const int64_t cols = count < mrg::kOrder ? count : mrg::kOrder;
    const dim3 grid((unsigned)((cols + kBlock - 1) / kBlock), (unsigned)chunks);
    return launch(mrg_words_kernel<ABL>, grid, dim3(kBlock), 0, s, out, a);
}

// variant: -1 shipped (pool in LDS when it fits beside the draws buffer), 0 pool in global
// memory
template <int ALGO, bool NORM, int ABL = kMrgAblNone, int Q = 4, int KB = mrg_gather_block<ALGO>()>
inline int launch_rand_gather_solve(const double2* ps, const double2* pt, uint32_t size,
                                    uint64_t seed, double* H, int64_t n, hipStream_t s,
                                    int variant = -1) {
    constexpr int kB = KB;
    constexpr size_t kLdsMax = 160 * 1024;
    mrg::GatherArgs a{};
    mrg::Vec x1, x2;
    mrg::seed_state(seed, x1, x2);
    for (int k = 0; k < 4; ++k) {
        const uint64_t kn = (uint64_t)k * (uint64_t)n;
        a.b[k] = (uint32_t)(kn & (uint64_t)(mrg::kOrder - 1));
        const mrg::Vec y1 = mrg::host_jump(kMrgPow.p1, 1, kn >> mrg::kOrderLog2, x1);
        const mrg::Vec y2 = mrg::host_jump(kMrgPow.p2, 2, kn >> mrg::kOrderLog2, x2);
        a.y[k][0] = mrg::pack(y1, y2);
        a.y[k][1] = mrg::pack(mrg::host_jump(kMrgPow.p1, 1, 1, y1),
                              mrg::host_jump(kMrgPow.p2, 2, 1, y2));
    }
    const int64_t cols = n < mrg::kOrder ? n : mrg::kOrder;
    const int64_t groups = (cols + kB / 4 - 1) / (kB / 4);
    const uint64_t magic = (ABL & kMrgIdxF64) != 0 ? fmod_f64_magic(size) : fastmod_magic(size);
    const size_t words = mrg_words_lds<ALGO, Q, KB>();
    const bool pool_lds = variant != 0 && kMrgStaticLds + words + (size_t)size * 32 <= kLdsMax;
    const size_t lds = pool_lds ? words + (size_t)size * 32 : words;
    auto k = pool_lds ? mrg_gather_solve_f64_kernel<ALGO, NORM, true, ABL, Q, KB>
                      : mrg_gather_solve_f64_kernel<ALGO, NORM, false, ABL, Q, KB>;
    if (lds + kMrgStaticLds > kSampleLdsMax && !lds_opt_in(k, kMrgStaticLds))
        return (int)hipErrorInvalidValue;
    int64_t per_cu = (int64_t)(kLdsMax / (lds + kMrgStaticLds));
    const int64_t max_per_cu = 2048 / kB;  // 32 waves per CU
    per_cu = per_cu < 1 ? 1 : (per_cu > max_per_cu ? max_per_cu : per_cu);
    const int64_t cap = per_cu * cu_count();
    const unsigned grid = (unsigned)(groups < cap ? groups : cap);
    return launch(k, dim3(grid), dim3(kB), lds, s, size, magic, ps, pt, H, n, a);
}

}  // namespace hg
