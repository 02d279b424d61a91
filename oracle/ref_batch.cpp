// ref_batch.cpp -- batch/timing shim around the REFERENCE's own solver bodies.
//
// TEST INFRASTRUCTURE ONLY (see oracle/hg_oracle.c header).  This file holds no
// solver arithmetic: it declares the four functions of the reference interface
// ("C++ Codes/modules/ACA_SKS.hpp:17-20") and links them from the reference source
// "C++ Codes/modules/ACA_SKS.cpp", compiled where it lies under /root/reference by
// oracle/build.sh into oracle/_ref/libsks_ref.so.  Outputs are the reference's
// normalised H (ACA_SKS.cpp:94-98).
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

namespace sks {
int runKernel_ACA(float* src, float* tar, float* result);
int runKernel_ACA_double(double* src, double* tar, double* result);
int runKernel_SKS(float* src, float* tar, float* result);
int runKernel_SKS_double(double* src, double* tar, double* result);
}  // namespace sks

namespace cv {
void runKernel_GE(float* src, float* tar, float* result);  // GE.cpp:43 (returns void)
}  // namespace cv

namespace {
int ge_adapter(float* s, float* t, float* h) {
    cv::runKernel_GE(s, t, h);
    return 0;
}
template <typename T, int (*F)(T*, T*, T*)>
void run_range(const T* src, const T* tar, T* H, int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i)
        F(const_cast<T*>(src + i * 8), const_cast<T*>(tar + i * 8), H + i * 9);
}

using Fn32 = int (*)(float*, float*, float*);
// algo 0 = ACA, 1 = SKS, 2 = GE (the reference's RHO-GE baseline, GE.cpp:43)
const Fn32 kF32[3] = {sks::runKernel_ACA, sks::runKernel_SKS, ge_adapter};

void range_f32(int algo, const float* src, const float* tar, float* H, int64_t lo, int64_t hi) {
    const Fn32 f = kF32[algo];
    for (int64_t i = lo; i < hi; ++i)
        f(const_cast<float*>(src + i * 8), const_cast<float*>(tar + i * 8), H + i * 9);
}
}  // namespace

extern "C" {

// AoS batch: src/tar (n,8), H (n,9).
int ref_batch_f32(int algo, const float* src, const float* tar, float* H, int64_t n) {
    if (algo < 0 || algo > 2) return 1;
    range_f32(algo, src, tar, H, 0, n);
    return 0;
}

int ref_batch_f64(int algo, const double* src, const double* tar, double* H, int64_t n) {
    if (algo == 0) run_range<double, sks::runKernel_ACA_double>(src, tar, H, 0, n);
    else if (algo == 1) run_range<double, sks::runKernel_SKS_double>(src, tar, H, 0, n);
    else return 1;
    return 0;
}

// Streaming batch timed over `threads` std::threads, `reps` passes; wall seconds.
double ref_time_f32(int algo, const float* src, const float* tar, float* H, int64_t n,
                    int threads, int reps) {
    if (threads < 1) threads = 1;
    if (algo < 0 || algo > 2) return -1.0;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int k = 0; k < threads; ++k) {
        int64_t lo = n * k / threads, hi = n * (k + 1) / threads;
        pool.emplace_back([=] {
            for (int r = 0; r < reps; ++r) range_f32(algo, src, tar, H, lo, hi);
        });
    }
    for (auto& t : pool) t.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// The reference's own CPU methodology (CPU_Runtime Test/main.cpp:87-92): one
// 4-point set solved `iters` times on one core.  Returns wall seconds.
double ref_time_repeat_f32(int algo, const float* src8, const float* tar8, float* H9,
                           int64_t iters) {
    if (algo < 0 || algo > 2) return -1.0;
    float s[8], t[8];
    for (int k = 0; k < 8; ++k) { s[k] = src8[k]; t[k] = tar8[k]; }
    const Fn32 f = kF32[algo];
    auto t0 = std::chrono::steady_clock::now();
    for (int64_t i = 0; i < iters; ++i) {
        f(s, t, H9);
        asm volatile("" ::"r"(H9) : "memory");
    }
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
}
