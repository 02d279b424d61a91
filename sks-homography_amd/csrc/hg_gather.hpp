// hg_gather.hpp -- the reference's own sampling pipeline in its own data formats
// (GPU_Runtime Test.cu:1441-1451): 4*N cuRAND MRG32K3A words laid out as FOUR ROWS of N
// (word k of hypothesis id at randList[id + k*N]), get_rand_list (:52-78) gathering
// Point2d (two binary64) source / target points into (8,N) SoA binary64 rows, then
// cal_Homo_* (:81-507) over them, unnormalised.  Round 1's sampler (hg_ransac.hpp) is the
// binary32 AoS form of the same pipeline; these kernels keep the reference's formats so
// Table 8's flow runs unchanged, with the gather and the solve fused into one pass.
#pragma once
#include "hg_ransac.hpp"

namespace hg {

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

}  // namespace hg
