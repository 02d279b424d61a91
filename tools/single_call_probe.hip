// Where a single sks::runKernel_ACA call on host pointers spends its ~7.6 us (tools only):
// the call itself, hipPointerGetAttributes on a host pointer (the call makes three), and an
// empty kernel launch + stream synchronize on a non-blocking stream.
//   hipcc --offload-arch=gfx950 -O2 -I include tools/single_call_probe.hip \
//       -L sks-homography_amd/lib -lsks_homography_amd -Wl,-rpath,$PWD/sks-homography_amd/lib
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#include "sks_aca_sks.hpp"

__global__ void empty_kernel() {}

template <typename F>
double us_per_call(F f, int reps) {
    for (int i = 0; i < 200; ++i) f();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) f();
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
    float s[8] = {0, 0, 200, 0, 50, 139, 181, 93}, t[8] = {10, 12, 220, 5, 40, 160, 190, 110}, h[9];
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 2;
    const int reps = 20000;
    const double call = us_per_call([&] { sks::runKernel_ACA(s, t, h); }, reps);
    const double attr = us_per_call([&] {
        hipPointerAttribute_t a;
        (void)hipPointerGetAttributes(&a, s);
    }, reps);
    const double launch_sync = us_per_call([&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
        (void)hipStreamSynchronize(st);
    }, reps);
    const double launch_only = us_per_call([&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st); }, reps);
    (void)hipStreamSynchronize(st);
    std::printf("{\"runKernel_ACA_host_us\": %.3f, \"pointer_attributes_us\": %.3f, "
                "\"empty_launch_sync_us\": %.3f, \"empty_launch_enqueue_us\": %.3f, \"h0\": %g}\n",
                call, attr, launch_sync, launch_only, h[0]);
    return 0;
}
