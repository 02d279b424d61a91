// hg_solvers.hpp -- per-lane closed-form 4-point solvers (device code, gfx950).
//
// One lane owns one problem; every intermediate lives in VGPRs (no LDS, no MFMA:
// ~100-170 scalar FLOPs per problem is not a contraction).  The association order
// of every expression is the reference's, and this header is compiled with FP
// contraction OFF (pragma below + -ffp-contract=off), so each product and sum is
// rounded on its own exactly as the reference's x86 SSE build rounds it.  That is
// what makes the GPU output bit-identical to sks::runKernel_* on the CPU.
#pragma once
#include <hip/hip_runtime.h>

#pragma clang fp contract(off)

namespace hg {

typedef float f32x2 __attribute__((ext_vector_type(2)));

// a / b, correctly rounded: the language's IEEE division.
template <bool PK, typename T>
__device__ __forceinline__ T div_rn(T a, T b) {
    return a / b;
}

// Two binary32 divisions carried as the halves of packed f32x2 values (the RANSAC
// samplers' paired hypotheses).  PK = false leaves them to the compiler, which splits
// them into two scalar expansions.  PK = true issues that same expansion -- v_div_scale
// of both operands, v_rcp, the three Newton-Raphson steps on the reciprocal and the
// quotient, v_div_fmas, v_div_fixup -- once per half for the non-packed instructions, and
// its six FMA / multiply steps once for both halves as v_pk_fma_f32 / v_pk_mul_f32 (22
// VALU instructions per pair of divisions -> 16).  The same instructions on the same
// operands, so the same bits as a / b, NaNs included.
template <bool PK>
__device__ __forceinline__ f32x2 div_rn(f32x2 a, f32x2 b) {
    if constexpr (!PK) {
        return a / b;
    } else {
        bool fx, fy, unused;
        const f32x2 den = {__builtin_amdgcn_div_scalef(a.x, b.x, false, &unused),
                           __builtin_amdgcn_div_scalef(a.y, b.y, false, &unused)};
        const f32x2 num = {__builtin_amdgcn_div_scalef(a.x, b.x, true, &fx),
                           __builtin_amdgcn_div_scalef(a.y, b.y, true, &fy)};
        const f32x2 r0 = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
        const f32x2 nden = -den, one = {1.0f, 1.0f};
        const f32x2 e0 = __builtin_elementwise_fma(nden, r0, one);
        const f32x2 r1 = __builtin_elementwise_fma(e0, r0, r0);
        const f32x2 q0 = num * r1;
        const f32x2 e1 = __builtin_elementwise_fma(nden, q0, num);
        const f32x2 q1 = __builtin_elementwise_fma(e1, r1, q0);
        const f32x2 e2 = __builtin_elementwise_fma(nden, q1, num);
        return f32x2{
            __builtin_amdgcn_div_fixupf(__builtin_amdgcn_div_fmasf(e2.x, r1.x, q1.x, fx), b.x, a.x),
            __builtin_amdgcn_div_fixupf(__builtin_amdgcn_div_fmasf(e2.y, r1.y, q1.y, fy), b.y, a.y)};
    }
}

// ACA: H = H_A2^-1 * H_C * H_A1 (C++ Codes/modules/ACA_SKS.cpp:24-82, 85 FLOPs).
// s, t = {Mx,My,Nx,Ny,Px,Py,Qx,Qy} of the source / target quad.
template <typename T>
__device__ __forceinline__ void aca_solve(const T (&s)[8], const T (&t)[8], T (&h)[9]) {
    // source-plane affine frame at M (ACA_SKS.cpp:28-32)
    const T sn_x = s[2] - s[0], sp_x = s[4] - s[0], sq_x = s[6] - s[0];
    const T sn_y = s[3] - s[1], sp_y = s[5] - s[1], sq_y = s[7] - s[1];
    const T det_s = sn_x * sp_y - sn_y * sp_x;
    const T qs_x = sp_y * sq_x - sp_x * sq_y;
    const T qs_y = sn_x * sq_y - sn_y * sq_x;
    // target-plane affine frame at M (:38-42)
    const T tn_x = t[2] - t[0], tp_x = t[4] - t[0], tq_x = t[6] - t[0];
    const T tn_y = t[3] - t[1], tp_y = t[5] - t[1], tq_y = t[7] - t[1];
    const T det_t = tn_x * tp_y - tn_y * tp_x;
    const T qt_x = tp_y * tq_x - tp_x * tq_y;
    const T qt_y = tn_x * tq_y - tn_y * tq_x;
    // core H_C (:49-54)
    const T r = det_s - qs_x - qs_y;
    const T c11 = qs_y * qt_x * r;
    const T c22 = qs_x * qt_y * r;
    const T c33 = qs_x * qs_y * (det_t - qt_x - qt_y);
    const T c31 = c11 - c33;
    const T c32 = c22 - c33;
    // H_A2^-1 * H_C, upper 2x2 (:61-66)
    const T m0 = t[0] * c33;
    const T m1 = t[1] * c33;
    const T a11 = t[2] * c11 - m0;
    const T a12 = t[4] * c22 - m0;
    const T a21 = t[3] * c11 - m1;
    const T a22 = t[5] * c22 - m1;
    // times H_A1 (:74-82)
    h[0] = a11 * sp_y - a12 * sn_y;
    h[1] = a12 * sn_x - a11 * sp_x;
    h[3] = a21 * sp_y - a22 * sn_y;
    h[4] = a22 * sn_x - a21 * sp_x;
    h[6] = c31 * sp_y - c32 * sn_y;
    h[7] = c32 * sn_x - c31 * sp_x;
    h[2] = m0 * det_s - h[0] * s[0] - h[1] * s[1];
    h[5] = m1 * det_s - h[3] * s[0] - h[4] * s[1];
    h[8] = c33 * det_s - h[6] * s[0] - h[7] * s[1];
}

// SKS: H = H_S2^-1 * H_K * H_S1 (ACA_SKS.cpp:189-293, 157 FLOPs, three IEEE
// divisions).  The reference's double literals (`0.5 *`, `1.0 /`) round to the
// same binary32 result as the binary32 operation used here.  PK: see div_rn.
template <bool PK = true, typename T>
__device__ __forceinline__ void sks_solve(const T (&s)[8], const T (&t)[8], T (&h)[9]) {
    const T half = T(0.5), one = T(1);
    // similarities from the M-N anchor pair (:192-206)
    const T o1x = half * (s[0] + s[2]), o1y = half * (s[1] + s[3]);
    const T e1x = o1x - s[0], e1y = s[1] - o1y;
    const T f1 = e1x * e1x + e1y * e1y;
    const T o2x = half * (t[0] + t[2]), o2y = half * (t[1] + t[3]);
    const T e2x = o2x - t[0], e2y = t[1] - o2y;
    const T f2 = e2x * e2x + e2y * e2y;
    // source P, Q in the canonical frame (:217-232)
    const T d3x = s[4] - o1x, d3y = s[5] - o1y;
    const T g3x = e1x * d3x - e1y * d3y;
    const T g3y = e1y * d3x + e1x * d3y;
    const T i3 = div_rn<PK>(one, g3y);
    const T k5x = i3 * g3x;
    const T k5y = i3 * f1;
    const T d5x = s[6] - o1x, d5y = s[7] - o1y;
    const T g5x = e1x * d5x - e1y * d5y;
    const T g5y = e1y * d5x + e1x * d5y;
    const T z7x = g3y * g5x - g3x * g5y;
    const T z7y = (g3y - g5y) * f1;
    const T z7w = g3y * g5y;
    // target P, Q (:238-253)
    const T d4x = t[4] - o2x, d4y = t[5] - o2y;
    const T g4x = e2x * d4x - e2y * d4y;
    const T g4y = e2y * d4x + e2x * d4y;
    const T i4 = div_rn<PK>(one, g4y);
    const T k6x = i4 * g4x;
    const T k6y = i4 * f2;
    const T d6x = t[6] - o2x, d6y = t[7] - o2y;
    const T g6x = e2x * d6x - e2y * d6y;
    const T g6y = e2y * d6x + e2x * d6y;
    const T z8x = g4y * g6x - g4x * g6y;
    const T z8y = (g4y - g6y) * f2;
    const T z8w = g4y * g6y;
    // kernel H_K parameters (:263-270)
    const T n1 = z7x * z8x - z7y * z8y;
    const T n2 = z7x * z8y - z7y * z8x;
    const T dd = z7x * z7x - z7y * z7y;
    const T sc = div_rn<PK>(z7w, dd * z8w);
    const T ka = n1 * sc;
    const T kb = n2 * sc;
    const T ku = k6x - ka * k5x - kb * k5y;
    const T kv = k6y - ka * k5y - kb * k5x;
    // H_L = H_S2^-1 * H_K, first two rows (:276-278)
    const T l0 = kb * o2x + ka * e2x;
    const T l1 = e2y + o2x * kv + ku * e2x;
    const T l2 = ka * o2x + kb * e2x;
    const T l3 = kb * o2y - ka * e2y;
    const T l4 = e2x + o2y * kv - ku * e2y;
    const T l5 = ka * o2y - kb * e2y;
    // H_S1 translation (:281-282)
    const T s13 = e1y * o1y - e1x * o1x;
    const T s23 = -e1y * o1x - e1x * o1y;
    // H = H_L * H_S1 (:285-293)
    h[0] = l0 * e1x + l1 * e1y;
    h[1] = l1 * e1x - l0 * e1y;
    h[2] = l2 * f1 + l0 * s13 + l1 * s23;
    h[3] = l3 * e1x + l4 * e1y;
    h[4] = l4 * e1x - l3 * e1y;
    h[5] = l5 * f1 + l3 * s13 + l4 * s23;
    h[6] = kb * e1x + kv * e1y;
    h[7] = kv * e1x - kb * e1y;
    h[8] = ka * f1 + kb * s13 + kv * s23;
}

// Last-element normalisation (ACA_SKS.cpp:94-98): one IEEE reciprocal-by-division,
// eight multiplies, H[8] := 1.
template <bool PK = true, typename T>
__device__ __forceinline__ void normalize_h(T (&h)[9]) {
    const T r = div_rn<PK>(T(1), h[8]);
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = h[i] * r;
    h[8] = T(1);
}

// RHO Gaussian elimination (the reference's comparison baseline cv::runKernel_GE,
// C++ Codes/modules/GE.cpp:41-188, itself OpenCV rho.cpp hFuncRefC; 221 FLOPs, four
// IEEE divisions, H[8] = 1 by construction).  Same operation order; the row-wise
// updates the reference writes out one statement per row are loops here (rows are
// independent, so the bits are the same).
template <typename T>
__device__ __forceinline__ void ge_solve(const T (&s)[8], const T (&t)[8], T (&h)[9]) {
    T xX[4], xY[4], yX[4], yY[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        xX[i] = s[2 * i] * t[2 * i];
        xY[i] = s[2 * i] * t[2 * i + 1];
        yX[i] = s[2 * i + 1] * t[2 * i];
        yY[i] = s[2 * i + 1] * t[2 * i + 1];
    }
    // q: the two source rows ("minor"), m: the three right-hand rows ("major"),
    // point P (index 2) is the pivot point the others are taken relative to
    T q[2][4], m[3][8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (i == 2) {
            q[0][2] = s[4]; q[1][2] = s[5];
            m[0][2] = -xX[2]; m[0][6] = -xY[2];
            m[1][2] = -yX[2]; m[1][6] = -yY[2];
            m[2][2] = t[4]; m[2][6] = t[5];
        } else {
            q[0][i] = s[2 * i] - s[4];
            q[1][i] = s[2 * i + 1] - s[5];
            m[0][i] = xX[2] - xX[i]; m[0][4 + i] = xY[2] - xY[i];
            m[1][i] = yX[2] - yX[i]; m[1][4 + i] = yY[2] - yY[i];
            m[2][i] = t[2 * i] - t[4]; m[2][4 + i] = t[2 * i + 1] - t[5];
        }
    }
    T a = q[0][0], b = q[0][1];
    q[1][1] = q[1][1] * a - q[1][0] * b;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        m[r][1] = m[r][1] * a - m[r][0] * b;
        m[r][5] = m[r][5] * a - m[r][4] * b;
    }
    b = q[0][3];
    q[1][3] = q[1][3] * a - q[1][0] * b;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        m[r][3] = m[r][3] * a - m[r][0] * b;
        m[r][7] = m[r][7] * a - m[r][4] * b;
    }
    a = q[1][1];
    b = q[1][3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        m[r][3] = m[r][3] * a - m[r][1] * b;
        m[r][7] = m[r][7] * a - m[r][5] * b;
    }
    b = q[1][0];
    q[0][0] = q[0][0] * a;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        m[r][0] = m[r][0] * a - m[r][1] * b;
        m[r][4] = m[r][4] * a - m[r][5] * b;
    }
    a = T(1) / q[0][0];
#pragma unroll
    for (int r = 0; r < 3; ++r) { m[r][0] = m[r][0] * a; m[r][4] = m[r][4] * a; }
    a = T(1) / q[1][1];
#pragma unroll
    for (int r = 0; r < 3; ++r) { m[r][1] = m[r][1] * a; m[r][5] = m[r][5] * a; }
    a = q[0][2];
    b = q[1][2];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        m[r][2] = m[r][2] - (m[r][0] * a + m[r][1] * b);
        m[r][6] = m[r][6] - (m[r][4] * a + m[r][5] * b);
    }
    a = m[0][7];
    m[1][7] = m[1][7] / a;
    m[2][7] = m[2][7] / a;
#pragma unroll
    for (int c = 0; c < 7; ++c) {
        m[1][c] = m[1][c] - m[0][c] * m[1][7];
        m[2][c] = m[2][c] - m[0][c] * m[2][7];
    }
    m[2][3] = m[2][3] / m[1][3];
#pragma unroll
    for (int c = 0; c < 8; ++c)
        if (c != 3) m[2][c] = m[2][c] - m[1][c] * m[2][3];
    h[0] = m[2][0]; h[1] = m[2][1]; h[2] = m[2][2];
    h[3] = m[2][4]; h[4] = m[2][5]; h[5] = m[2][6];
    h[6] = m[2][7]; h[7] = m[2][3]; h[8] = T(1);
}

// 8x8 LU with partial pivoting -- the reference GPU harness's getPerspectiveTransform
// baseline cal_Homo_GPT (GPU_Runtime Test.cu:301-357 with its helpers find_pivot,
// scaleIndex, eliminate, down_tri_solve, up_tri_solve, :242-300).  Crout form: row i
// right of the diagonal is divided by the pivot, the trailing rows are updated, L
// keeps the unscaled column.  The matrix lives in VGPRs: every loop is unrolled with
// compile-time indices and the row swap is a select per candidate row (a runtime row
// index would push the array to scratch, as the reference's local-memory a[64] is).
// The forward solve L y = b (down_tri_solve) is carried out as b is eliminated: row k's
// acc = b[k] - a[k][0]*y[0] - ... - a[k][k-1]*y[k-1] receives term j at step j, in the
// same order and from the same L entry (it travels with its row through later swaps),
// and y[k] = acc / a[k][k] once row k is pivoted -- the same roundings as the separate
// pass.  L is then dead after its own step, so a swap moves only columns i..7 and b.
// Steps 0-2 pick their pivot among rows i..3 only, which is exact for every input:
// rows 4..7 enter with a[r][0..2] = 0 and stay in {+-0, NaN} through those steps (their
// multipliers a[r][i] are in that set, so every product subtracted from them is too),
// and find_pivot never takes such a row (|a| is 0 or NaN: best < |a| is false for any
// best).  Rows 4..7 therefore keep their places through step 2.  Together 100 instead
// of 252 64-bit selects per problem, and 12 fewer pivot compares.
template <typename T>
__device__ __forceinline__ void gpt_solve(const T (&s)[8], const T (&t)[8], T (&h)[9]) {
    T a[8][8], b[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const T x = s[2 * i], y = s[2 * i + 1], u = t[2 * i], v = t[2 * i + 1];
        a[i][0] = x; a[i][1] = y; a[i][2] = T(1);
        a[i][3] = T(0); a[i][4] = T(0); a[i][5] = T(0);
        a[i][6] = -x * u; a[i][7] = -y * u;
        a[i + 4][0] = T(0); a[i + 4][1] = T(0); a[i + 4][2] = T(0);
        a[i + 4][3] = x; a[i + 4][4] = y; a[i + 4][5] = T(1);
        a[i + 4][6] = -x * v; a[i + 4][7] = -y * v;
        b[i] = u;
        b[i + 4] = v;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        // pivot: first row of max |a[r][i]|, r >= i (strict <, as find_pivot)
        T best = __builtin_fabs(a[i][i]);
        int p = i;
        constexpr int kRows = 8;
        const int last = i < 3 ? 4 : kRows;  // candidate rows i+1 .. last-1
#pragma unroll
        for (int r = i + 1; r < last; ++r) {
            const T c = __builtin_fabs(a[r][i]);
            if (best < c) { best = c; p = r; }
        }
#pragma unroll
        for (int r = i + 1; r < last; ++r) {
            const bool sw = p == r;
#pragma unroll
            for (int c = i; c < 8; ++c) {
                const T lo = a[i][c], hi = a[r][c];
                a[i][c] = sw ? hi : lo;
                a[r][c] = sw ? lo : hi;
            }
            const T lo = b[i], hi = b[r];
            b[i] = sw ? hi : lo;
            b[r] = sw ? lo : hi;
        }
        b[i] = b[i] / a[i][i];  // y[i]
#pragma unroll
        for (int c = i + 1; c < 8; ++c) a[i][c] = a[i][c] / a[i][i];
#pragma unroll
        for (int r = i + 1; r < 8; ++r) {
#pragma unroll
            for (int c = i + 1; c < 8; ++c) a[r][c] = a[r][c] - a[r][i] * a[i][c];
            b[r] = b[r] - a[r][i] * b[i];
        }
    }
#pragma unroll
    for (int k = 6; k >= 0; --k) {  // U x = y (unit diagonal), columns right to left
        T acc = b[k];
#pragma unroll
        for (int j = 7; j > k; --j) acc = acc - a[k][j] * b[j];
        b[k] = acc;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = b[k];
    h[8] = T(1);
}

enum Algo : int { kACA = 0, kSKS = 1, kGE = 2, kGPT = 3 };

// PK: how packed f32x2 pairs divide (div_rn); scalar T divides as the language does.
template <int ALGO, bool NORM, bool PK = true, typename T>
__device__ __forceinline__ void solve(const T (&s)[8], const T (&t)[8], T (&h)[9]) {
    if constexpr (ALGO == kACA) aca_solve(s, t, h);
    else if constexpr (ALGO == kSKS) sks_solve<PK>(s, t, h);
    else if constexpr (ALGO == kGE) ge_solve(s, t, h);
    else gpt_solve(s, t, h);
    if constexpr (NORM) normalize_h<PK>(h);
}

// TensorACA rectangle -> quad (PyTorch Codes/Modules_Runtime_Test.py:294-302),
// evaluated as ATen evaluates it: the cross product contracts one product per
// component into an FMA, the 3-term sum runs left to right from ATen's +0 accumulator
// (so three -0 terms sum to +0: the trailing "+ 0.f", exact for every other value),
// every other op rounds on its own.  tr = (3,4) target tensor rows {x, y, w} x cols {M, N, P, Q}.
// SQUARE: the square specialisation of ACA_rect.m:28 (ratio 1, 44 FLOPs) -- drops the
// multiply by div, which is exact when div == 1, so the bits are those of the general form.
// Row forms: scale and div per row r of H -- the reference composition broadcasts them
// against the (B,3,1) columns (.py:301-302), so a (B,1,1) tensor gives per-problem values
// and a (B,3,1) one per-row values; the batch-uniform forms below pass one value thrice.
//
// ORDER: whose evaluation of the statements to follow.  kAtenCpu (0): ATen-CPU's, above.
// kAtenRocm (1): torch-ROCm's on the GPU -- the reference's default run (.py:393,
// device='cuda') -- which differs only in its 3-term reductions: the forward's torch.sum and,
// in the backward, every sum_to_size over three elements run ((0 + t0) + t2) + t1 (measured:
// tools/rocm_grad_probe*.py, profiles/r04/rocm_grad_probe*.json); the cross products and the
// element-wise ops are the same bits on both devices.
constexpr int kAtenCpu = 0, kAtenRocm = 1;

// +0 + t as a real add.  With t = -x the IR holds fsub +0, x, and the gfx950 instruction
// selector folds that into a negate source modifier of the next add -- -0 for x = +0 where
// the subtraction gives +0 (seen as v_sub_f32 v, -x, y in tensor_aca_rect_grad_rows' sneg;
// tests/test_gpu_rect_rocm_order.py, tests/test_gpu_rect_bcast.py's signed-zero case).  The
// empty asm makes t opaque to that fold; it emits no instruction.
__device__ __forceinline__ float zero_plus(float t) {
    asm volatile("" : "+v"(t));
    return 0.f + t;
}

template <int ORDER>
__device__ __forceinline__ float sum3(float t0, float t1, float t2) {
    if constexpr (ORDER == kAtenRocm) return (zero_plus(t0) + t2) + t1;
    else return ((t0 + t1) + t2) + 0.f;  // left to right from ATen's +0 accumulator
}

// A (B,1,1) operand's three-row sum (sum_to_size): from +0 in the device's order (CPU:
// ((0 + t0) + t1) + t2, which the running sums from 0 gave until r03).
template <int ORDER>
__device__ __forceinline__ float rows3(float t0, float t1, float t2) {
    if constexpr (ORDER == kAtenRocm) return sum3<ORDER>(t0, t1, t2);
    else return (zero_plus(t0) + t1) + t2;
}

template <bool SQUARE = false, int ORDER = kAtenCpu>
__device__ __forceinline__ void tensor_aca_rect_solve_rows(const float (&tr)[12], float mx,
                                                           float my, const float (&scale)[3],
                                                           const float (&div)[3], float (&h)[9]) {
    const float ax = tr[5] - tr[4], ay = tr[6] - tr[4], az = tr[7] - tr[4];  // d[1]: MN, MP, MQ (y)
    const float bx = tr[1] - tr[0], by = tr[2] - tr[0], bz = tr[3] - tr[0];  // d[0]: MN, MP, MQ (x)
    const float c0 = __builtin_fmaf(ay, bz, -(az * by));
    const float c1 = __builtin_fmaf(az, bx, -(ax * bz));
    const float c2 = __builtin_fmaf(ax, by, -(ay * bx));
    const float sum = sum3<ORDER>(c0, c1, c2);  // torch.sum starts from +0
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const float b = sum * tr[4 * r];
        const float h0 = tr[4 * r + 1] * c0 - b;
        const float h1 = SQUARE ? tr[4 * r + 2] * c1 - b : div[r] * (tr[4 * r + 2] * c1 - b);
        h[3 * r + 0] = h0;
        h[3 * r + 1] = h1;
        h[3 * r + 2] = (scale[r] * b - mx * h0) - my * h1;
    }
}

template <bool SQUARE = false, int ORDER = kAtenCpu>
__device__ __forceinline__ void tensor_aca_rect_solve(const float (&tr)[12], float mx, float my,
                                                      float scale, float div, float (&h)[9]) {
    const float sc[3] = {scale, scale, scale}, dv[3] = {div, div, div};
    tensor_aca_rect_solve_rows<SQUARE, ORDER>(tr, mx, my, sc, dv, h);
}

// Compact deep-homography form: the source is the axis-aligned
// w x h rectangle at corner (mx, my) -- the shape getInput builds
// (Modules_Runtime_Test.py:9-16) -- and the network predicts the 4 corner offsets
// (getTar, .py:19-21).  Builds the (3,4) target tensor exactly as the reference's
// float ops do: N = M + (w,0), P = M + (0,h), Q = M + (w,h), tar = src + offset.
__device__ __forceinline__ void rect_target_from_offsets(float mx, float my, float w, float h,
                                                         const float (&off)[8],
                                                         float (&tr)[12]) {
    const float nx = mx + w, py = my + h;
    tr[0] = mx + off[0];
    tr[1] = nx + off[2];
    tr[2] = mx + off[4];
    tr[3] = nx + off[6];
    tr[4] = my + off[1];
    tr[5] = my + off[3];
    tr[6] = py + off[5];
    tr[7] = py + off[7];
    tr[8] = tr[9] = tr[10] = tr[11] = 1.f;
}

// Reverse-mode derivative of tensor_aca_rect_solve: the gradients ATen autograd gives
// through the reference's own statements (.py:296-302), op for op as the
// autograd graph evaluates them on the CPU (restated in oracle/hg_oracle.c, pinned by
// tests/golden/torch_rect_grad.npz):
//   * H is assembled in place from zeros, and column 2 reads columns 0 and 1 back: dL/dH's
//     columns 0 and 1 gain  -src * g2  and a zero-filled slice gradient (+0);
//   * dL/dh_temp accumulates in the order the graph delivers it: from scale*h_temp, then
//     from div's column, then from column 0;
//   * every reduction to a broadcast operand's shape (sum_to_size) and every sum with a
//     zero-filled slice gradient (slices of D, Q4, tar) ends in + 0 (ATen's accumulators
//     start from +0, so a sum of -0 terms gives +0);
//   * the cross product's backward is ATen's cross again (dL/da = b x gc, dL/db = gc x a),
//     one product per component contracted into an FMA like the forward.
// In: the forward's inputs and g = dL/dH (3x3).  Out: gt = dL/dtar (3,4); gmx/gmy = dL/d
// src[0][0], src[1][0] (an extension: the reference statements cannot differentiate src --
// autograd refuses the in-place H); gscale / gdiv = this problem's share of dL/dscale,
// dL/ddiv (three-row sums from +0, as sum_to_size gives a (B,1,1) parameter).
// Row form: per-row scale / div (as tensor_aca_rect_solve_rows), and each row's own share of
// dL/dscale[r], dL/ddiv[r] in gsr / gdr beside the per-problem sums gscale / gdiv.
// ORDER (see tensor_aca_rect_solve_rows): kAtenRocm runs every 3-term reduction the GPU's way.
template <int ORDER = kAtenCpu>
__device__ __forceinline__ void tensor_aca_rect_grad_rows(
    const float (&tr)[12], float mx, float my, const float (&scale)[3], const float (&div)[3],
    const float (&g)[9], float (&gt)[12], float& gmx, float& gmy, float& gscale, float& gdiv,
    float (&gsr)[3], float (&gdr)[3]) {
    const float ax = tr[5] - tr[4], ay = tr[6] - tr[4], az = tr[7] - tr[4];
    const float bx = tr[1] - tr[0], by = tr[2] - tr[0], bz = tr[3] - tr[0];
    const float c0 = __builtin_fmaf(ay, bz, -(az * by));
    const float c1 = __builtin_fmaf(az, bx, -(ax * bz));
    const float c2 = __builtin_fmaf(ax, by, -(ay * bx));
    const float sum = sum3<ORDER>(c0, c1, c2);  // torch.sum starts from +0
    float gh0[3], gy[3], ght[3], pmx[3], pmy[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const float b = sum * tr[4 * r];
        const float h0 = tr[4 * r + 1] * c0 - b;
        const float x = tr[4 * r + 2] * c1 - b;
        const float h1 = div[r] * x;
        const float g2 = g[3 * r + 2];
        gh0[r] = (g[3 * r + 0] - mx * g2) + 0.f;
        const float gh1 = (g[3 * r + 1] - my * g2) + 0.f;
        pmx[r] = -(g2 * h0);
        pmy[r] = -(g2 * h1);
        gsr[r] = g2 * b;
        gy[r] = div[r] * gh1;
        gdr[r] = gh1 * x;
        ght[r] = (scale[r] * g2 - gy[r]) - gh0[r];
    }
    // the per-problem sums over the rows (sum_to_size to (B,1,1))
    gmx = rows3<ORDER>(pmx[0], pmx[1], pmx[2]);
    gmy = rows3<ORDER>(pmy[0], pmy[1], pmy[2]);
    gscale = rows3<ORDER>(gsr[0], gsr[1], gsr[2]);
    gdiv = rows3<ORDER>(gdr[0], gdr[1], gdr[2]);
    // dL/dsum, dL/dQ4[0], dL/dQ4[1]: sums over the rows to the (B,1,1) shapes
    const float gS = sum3<ORDER>(ght[0] * tr[0], ght[1] * tr[4], ght[2] * tr[8]);
    const float s0 = sum3<ORDER>(gh0[0] * tr[1], gh0[1] * tr[5], gh0[2] * tr[9]);
    const float s1 = sum3<ORDER>(gy[0] * tr[2], gy[1] * tr[6], gy[2] * tr[10]);
    const float gc0 = (gS + s0) + 0.f, gc1 = (gS + s1) + 0.f, gc2 = gS + 0.f;
    // Q4 = a x b (a = D's y row, b = its x row): dL/da = b x gc, dL/db = gc x a
    float d[2][3];
    d[1][0] = __builtin_fmaf(by, gc2, -(bz * gc1)) + 0.f;
    d[1][1] = __builtin_fmaf(bz, gc0, -(bx * gc2)) + 0.f;
    d[1][2] = __builtin_fmaf(bx, gc1, -(by * gc0)) + 0.f;
    d[0][0] = __builtin_fmaf(gc1, az, -(gc2 * ay)) + 0.f;
    d[0][1] = __builtin_fmaf(gc2, ax, -(gc0 * az)) + 0.f;
    d[0][2] = __builtin_fmaf(gc0, ay, -(gc1 * ax)) + 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        // D = tar[:, :, 1:] - tar[:, :, 0:1]; D's w row has no gradient (+0)
        const float d0 = r < 2 ? d[r][0] : 0.f, d1 = r < 2 ? d[r][1] : 0.f;
        const float d2 = r < 2 ? d[r][2] : 0.f;
        const float sneg = sum3<ORDER>(-d0, -d1, -d2);
        gt[4 * r + 0] = (ght[r] * sum + sneg) + 0.f;
        gt[4 * r + 1] = (d0 + gh0[r] * c0) + 0.f;
        gt[4 * r + 2] = (d1 + gy[r] * c1) + 0.f;
        gt[4 * r + 3] = d2 + 0.f;
    }
}

// Reverse-mode derivative of ACA_vanilla (Modules_Runtime_Test.py:322-382): the gradients
// ATen autograd gives through its statements, op for op in the order the autograd engine
// runs them (restated independently in oracle/hg_oracle.c, pinned by
// tests/golden/torch_vanilla_grad.npz).  The engine runs the graph's nodes in reverse
// creation order, so a value used by several statements receives its gradient terms from
// its LAST use first, and they are summed in that order: H's copies (:373-381) first,
// then the statements from res_8 (:370) back to M1N1_X (:322).  Each statement's backward is
// ATen's: a - b gives (g, -g), a * b gives (g*b, g*a), (a*b)*c is two nodes.  The leaves'
// gradients gather their terms from zero-filled select gradients, hence the final + 0.
// In: s = src (4,2) = {Mx, My, Nx, Ny, Px, Py, Qx, Qy}, t = tar, g = dL/dH (3x3 row-major).
// Out: gs = dL/dsrc, gt = dL/dtar (same layout).  Every operation rounds on its own.
template <typename T>
__device__ __host__ __forceinline__ void aca_vanilla_grad(const T (&s)[8], const T (&t)[8],
                                                          const T (&g)[9], T (&gs)[8],
                                                          T (&gt)[8]) {
    const T s00 = s[0], s01 = s[1], s10 = s[2], s11 = s[3], s20 = s[4], s21 = s[5], s30 = s[6],
            s31 = s[7];
    const T t00 = t[0], t01 = t[1], t10 = t[2], t11 = t[3], t20 = t[4], t21 = t[5], t30 = t[6],
            t31 = t[7];
    // the forward's statements (:322-370), every intermediate kept
    const T M1N1_X = s10 - s00, M1N1_Y = s11 - s01, M1P1_X = s20 - s00, M1P1_Y = s21 - s01;
    const T M1Q1_X = s30 - s00, M1Q1_Y = s31 - s01;
    const T fA1 = M1N1_X * M1P1_Y - M1N1_Y * M1P1_X;
    const T Q3_x = M1P1_Y * M1Q1_X - M1P1_X * M1Q1_Y;
    const T Q3_y = M1N1_X * M1Q1_Y - M1N1_Y * M1Q1_X;
    const T M2N2_X = t10 - t00, M2N2_Y = t11 - t01, M2P2_X = t20 - t00, M2P2_Y = t21 - t01;
    const T M2Q2_X = t30 - t00, M2Q2_Y = t31 - t01;
    const T fA2 = M2N2_X * M2P2_Y - M2N2_Y * M2P2_X;
    const T Q4_x = M2P2_Y * M2Q2_X - M2P2_X * M2Q2_Y;
    const T Q4_y = M2N2_X * M2Q2_Y - M2N2_Y * M2Q2_X;
    const T tt1 = (fA1 - Q3_x) - Q3_y;
    const T P20 = Q3_y * Q4_x, C11 = P20 * tt1;
    const T P21 = Q3_x * Q4_y, C22 = P21 * tt1;
    const T P22 = Q3_x * Q3_y, E22 = (fA2 - Q4_x) - Q4_y, C33 = P22 * E22;
    const T C31 = C11 - C33, C32 = C22 - C33;
    const T tt3 = t00 * C33, tt4 = t01 * C33;
    const T H1_11 = t10 * C11 - tt3, H1_12 = t20 * C22 - tt3;
    const T H1_21 = t11 * C11 - tt4, H1_22 = t21 * C22 - tt4;
    const T res_0 = H1_11 * M1P1_Y - H1_12 * M1N1_Y;
    const T res_1 = H1_12 * M1N1_X - H1_11 * M1P1_X;
    const T res_3 = H1_21 * M1P1_Y - H1_22 * M1N1_Y;
    const T res_4 = H1_22 * M1N1_X - H1_21 * M1P1_X;
    const T res_6 = C31 * M1P1_Y - C32 * M1N1_Y;
    const T res_7 = C32 * M1N1_X - C31 * M1P1_X;
    // res_k: H's copy first, then its use in res_2 / res_5 / res_8 (:368-370)
    const T G8 = g[8], G5 = g[5], G2 = g[2];
    const T gr7 = g[7] + (-G8) * s01, gr6 = g[6] + (-G8) * s00;
    const T gr4 = g[4] + (-G5) * s01, gr3 = g[3] + (-G5) * s00;
    const T gr1 = g[1] + (-G2) * s01, gr0 = g[0] + (-G2) * s00;
    // res_8, res_5, res_2 (:370, :369, :368)
    T gs00 = (-G8) * res_6, gs01 = (-G8) * res_7;
    T gC33 = G8 * fA1, gfA1 = G8 * C33;
    gs01 = gs01 + (-G5) * res_4;
    gs00 = gs00 + (-G5) * res_3;
    T gtt4 = G5 * fA1;
    gfA1 = gfA1 + G5 * tt4;
    gs01 = gs01 + (-G2) * res_1;
    gs00 = gs00 + (-G2) * res_0;
    T gtt3 = G2 * fA1;
    gfA1 = gfA1 + G2 * tt3;
    // res_7, res_6, res_4, res_3, res_1, res_0 (:367 back to :362)
    T gC31 = (-gr7) * M1P1_X, gM1PX = (-gr7) * C31, gC32 = gr7 * M1N1_X, gM1NX = gr7 * C32;
    gC32 = gC32 + (-gr6) * M1N1_Y;
    T gM1NY = (-gr6) * C32;
    gC31 = gC31 + gr6 * M1P1_Y;
    T gM1PY = gr6 * C31;
    T gH21 = (-gr4) * M1P1_X;
    gM1PX = gM1PX + (-gr4) * H1_21;
    T gH22 = gr4 * M1N1_X;
    gM1NX = gM1NX + gr4 * H1_22;
    gH22 = gH22 + (-gr3) * M1N1_Y;
    gM1NY = gM1NY + (-gr3) * H1_22;
    gH21 = gH21 + gr3 * M1P1_Y;
    gM1PY = gM1PY + gr3 * H1_21;
    T gH11 = (-gr1) * M1P1_X;
    gM1PX = gM1PX + (-gr1) * H1_11;
    T gH12 = gr1 * M1N1_X;
    gM1NX = gM1NX + gr1 * H1_12;
    gH12 = gH12 + (-gr0) * M1N1_Y;
    gM1NY = gM1NY + (-gr0) * H1_12;
    gH11 = gH11 + gr0 * M1P1_Y;
    gM1PY = gM1PY + gr0 * H1_11;
    // H1_22, H1_21, H1_12, H1_11 (:360 back to :357)
    gtt4 = gtt4 - gH22;
    T gt21 = gH22 * C22, gC22 = gH22 * t21;
    gtt4 = gtt4 - gH21;
    T gt11 = gH21 * C11, gC11 = gH21 * t11;
    gtt3 = gtt3 - gH12;
    T gt20 = gH12 * C22;
    gC22 = gC22 + gH12 * t20;
    gtt3 = gtt3 - gH11;
    T gt10 = gH11 * C11;
    gC11 = gC11 + gH11 * t10;
    // tt4, tt3 (:356, :355), C32, C31 (:353, :352)
    T gt01 = gtt4 * C33;
    gC33 = gC33 + gtt4 * t01;
    T gt00 = gtt3 * C33;
    gC33 = gC33 + gtt3 * t00;
    gC22 = gC22 + gC32;
    gC33 = gC33 - gC32;
    gC11 = gC11 + gC31;
    gC33 = gC33 - gC31;
    // C33 = (Q3_x*Q3_y) * ((fA2 - Q4_x) - Q4_y), C22, C11, tt1 (:351 back to :348)
    const T gP22 = gC33 * E22, gE22 = gC33 * P22;
    T gQ4y = -gE22, gfA2 = gE22, gQ4x = -gE22;
    T gQ3x = gP22 * Q3_y, gQ3y = gP22 * Q3_x;
    const T gP21 = gC22 * tt1;
    T gtt1 = gC22 * P21;
    gQ3x = gQ3x + gP21 * Q4_y;
    gQ4y = gQ4y + gP21 * Q3_x;
    const T gP20 = gC11 * tt1;
    gtt1 = gtt1 + gC11 * P20;
    gQ3y = gQ3y + gP20 * Q4_x;
    gQ4x = gQ4x + gP20 * Q3_y;
    gQ3y = gQ3y - gtt1;
    gfA1 = gfA1 + gtt1;
    gQ3x = gQ3x - gtt1;
    // Q4_y, Q4_x, fA2 (:346 back to :344)
    T gM2NY = (-gQ4y) * M2Q2_X, gM2QX = (-gQ4y) * M2N2_Y, gM2NX = gQ4y * M2Q2_Y;
    T gM2QY = gQ4y * M2N2_X;
    T gM2PX = (-gQ4x) * M2Q2_Y;
    gM2QY = gM2QY + (-gQ4x) * M2P2_X;
    T gM2PY = gQ4x * M2Q2_X;
    gM2QX = gM2QX + gQ4x * M2P2_Y;
    gM2NY = gM2NY + (-gfA2) * M2P2_X;
    gM2PX = gM2PX + (-gfA2) * M2N2_Y;
    gM2NX = gM2NX + gfA2 * M2P2_Y;
    gM2PY = gM2PY + gfA2 * M2N2_X;
    // the target differences (:342 back to :335)
    const T gt31 = gM2QY;
    gt01 = gt01 - gM2QY;
    const T gt30 = gM2QX;
    gt00 = gt00 - gM2QX;
    gt21 = gt21 + gM2PY;
    gt01 = gt01 - gM2PY;
    gt20 = gt20 + gM2PX;
    gt00 = gt00 - gM2PX;
    gt11 = gt11 + gM2NY;
    gt01 = gt01 - gM2NY;
    gt10 = gt10 + gM2NX;
    gt00 = gt00 - gM2NX;
    // Q3_y, Q3_x, fA1 (:333 back to :331)
    gM1NY = gM1NY + (-gQ3y) * M1Q1_X;
    T gM1QX = (-gQ3y) * M1N1_Y;
    gM1NX = gM1NX + gQ3y * M1Q1_Y;
    T gM1QY = gQ3y * M1N1_X;
    gM1PX = gM1PX + (-gQ3x) * M1Q1_Y;
    gM1QY = gM1QY + (-gQ3x) * M1P1_X;
    gM1PY = gM1PY + gQ3x * M1Q1_X;
    gM1QX = gM1QX + gQ3x * M1P1_Y;
    gM1NY = gM1NY + (-gfA1) * M1P1_X;
    gM1PX = gM1PX + (-gfA1) * M1N1_Y;
    gM1NX = gM1NX + gfA1 * M1P1_Y;
    gM1PY = gM1PY + gfA1 * M1N1_X;
    // the source differences (:329 back to :322)
    gs01 = gs01 - gM1QY;
    gs00 = gs00 - gM1QX;
    gs01 = gs01 - gM1PY;
    gs00 = gs00 - gM1PX;
    gs01 = gs01 - gM1NY;
    gs00 = gs00 - gM1NX;
    gs[0] = gs00 + T(0); gs[1] = gs01 + T(0); gs[2] = gM1NX + T(0); gs[3] = gM1NY + T(0);
    gs[4] = gM1PX + T(0); gs[5] = gM1PY + T(0); gs[6] = gM1QX + T(0); gs[7] = gM1QY + T(0);
    gt[0] = gt00 + T(0); gt[1] = gt01 + T(0); gt[2] = gt10 + T(0); gt[3] = gt11 + T(0);
    gt[4] = gt20 + T(0); gt[5] = gt21 + T(0); gt[6] = gt30 + T(0); gt[7] = gt31 + T(0);
}

template <int ORDER = kAtenCpu>
__device__ __forceinline__ void tensor_aca_rect_grad(const float (&tr)[12], float mx, float my,
                                                     float scale, float div, const float (&g)[9],
                                                     float (&gt)[12], float& gmx, float& gmy,
                                                     float& gscale, float& gdiv) {
    const float sc[3] = {scale, scale, scale}, dv[3] = {div, div, div};
    float gsr[3], gdr[3];
    tensor_aca_rect_grad_rows<ORDER>(tr, mx, my, sc, dv, g, gt, gmx, gmy, gscale, gdiv, gsr, gdr);
}

}  // namespace hg
