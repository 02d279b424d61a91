// ref_cu_driver.hip -- host-side driver for the REFERENCE's own GPU kernels.
//
// TEST INFRASTRUCTURE ONLY (see oracle/hg_oracle.c header): never linked into the product.
// oracle/build.sh streams the kernel section of the reference's CUDA harness,
// "C++ Codes/Runtime Test/GPU_Runtime Test/GPU_Runtime Test.cu" lines 81-507 --
// cal_Homo_ACA (:81-151), cal_Homo_SKS (:153-240), the GPT-LU helpers and cal_Homo_GPT
// (:242-357) and cal_Homo_GE (:359-507), plain CUDA-dialect kernels with no header,
// library or OpenCV dependency -- straight from the file where it lies, followed by this
// text, into hipcc (gfx950, -ffp-contract=off: each + - * / rounded on its own in the
// reference's statement order, the convention the C++ reference is compiled under too).
// No reference text is stored in this repository; the kernels are not rewritten.  The rest
// of that file (OpenCV / cuRAND host code, the DLT/HO SVD kernels) is not compiled.
//
// refcu_solve_f64 runs one kernel exactly as the reference's host drivers launch it
// (cal_ACA, .cu:1177-1196: <<<ceil(N/32), 32>>>, SoA (8,N) in, (9,N) out, unnormalised;
// GPT/GE write H[8] = 1) on host arrays, copying in and out.  Returns 0 or a hipError_t.
#include <hip/hip_runtime.h>

#include <cstdint>

extern "C" int refcu_solve_f64(int algo, const double* src, const double* tar, double* H,
                               int n) {
    if (n <= 0) return n == 0 ? 0 : (int)hipErrorInvalidValue;
    if (algo < 0 || algo > 3) return (int)hipErrorInvalidValue;
    double *ds = nullptr, *dt = nullptr, *dh = nullptr;
    const size_t in = (size_t)n * 8 * sizeof(double), out = (size_t)n * 9 * sizeof(double);
    hipError_t e = hipMalloc(&ds, in);
    if (e == hipSuccess) e = hipMalloc(&dt, in);
    if (e == hipSuccess) e = hipMalloc(&dh, out);
    if (e == hipSuccess) e = hipMemcpy(ds, src, in, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dt, tar, in, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(dh, 0xff, out);
    if (e == hipSuccess) {
        const dim3 grid((unsigned)((n + 31) / 32)), block(32);
        switch (algo) {  // 0 ACA, 1 SKS, 2 GE, 3 GPT (HG_ALGO_* numbering)
            case 0: cal_Homo_ACA<<<grid, block>>>(ds, dt, dh, n); break;
            case 1: cal_Homo_SKS<<<grid, block>>>(ds, dt, dh, n); break;
            case 2: cal_Homo_GE<<<grid, block>>>(ds, dt, dh, n); break;
            default: cal_Homo_GPT<<<grid, block>>>(ds, dt, dh, n); break;
        }
        e = hipGetLastError();
        if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    if (e == hipSuccess) e = hipMemcpy(H, dh, out, hipMemcpyDeviceToHost);
    (void)hipFree(ds);
    (void)hipFree(dt);
    (void)hipFree(dh);
    return (int)e;
}
