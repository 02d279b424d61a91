// ref_batch.cpp -- batch/timing shim around the REFERENCE's own solver bodies.
//
// TEST INFRASTRUCTURE ONLY (see oracle/hg_oracle.c header).  This file holds no
// solver arithmetic: it declares the four functions of the reference interface
// ("C++ Codes/modules/ACA_SKS.hpp:17-20") and links them from the reference source
// "C++ Codes/modules/ACA_SKS.cpp", compiled where it lies under /root/reference by
// oracle/build.sh into oracle/_ref/libsks_ref.so.  Outputs are the reference's
// normalised H (ACA_SKS.cpp:94-98).
#include <pthread.h>
#include <sched.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
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

// The streaming batch on `threads` threads, thread k pinned to logical CPU cpus[k] (one per
// physical core, chosen by the caller; cpus may be NULL for no pinning).  Each thread first
// copies its slice of src/tar into buffers it allocates itself, so under Linux's
// first-touch policy its pages sit on its own NUMA node, and writes H into its own buffer
// too; then all threads start together and make `reps` passes.  Returns the wall seconds
// from the common start to the last thread's end (setup excluded).  If H is not NULL each
// thread copies its H slice there afterwards (untimed), so the result can be checked.
double ref_time_pinned_f32(int algo, const float* src, const float* tar, float* H, int64_t n,
                           const int* cpus, int threads, int reps) {
    if (threads < 1 || reps < 1 || algo < 0 || algo > 2) return -1.0;
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<double> end(threads, 0.0);
    std::vector<std::thread> pool;
    std::chrono::steady_clock::time_point t0;
    for (int k = 0; k < threads; ++k) {
        const int64_t lo = n * k / threads, hi = n * (k + 1) / threads;
        pool.emplace_back([&, k, lo, hi] {
            if (cpus) {
                cpu_set_t set;
                CPU_ZERO(&set);
                CPU_SET(cpus[k], &set);
                (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
            }
            const int64_t m = hi - lo;
            std::vector<float> s(m * 8), t(m * 8), h(m * 9);  // first touch on this core
            if (m) {
                std::memcpy(s.data(), src + lo * 8, m * 32);
                std::memcpy(t.data(), tar + lo * 8, m * 32);
                std::memset(h.data(), 0, m * 36);
            }
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            for (int r = 0; r < reps; ++r) range_f32(algo, s.data(), t.data(), h.data(), 0, m);
            end[k] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (H && m) std::memcpy(H + lo * 9, h.data(), m * 36);
        });
    }
    while (ready.load() < threads) std::this_thread::yield();
    t0 = std::chrono::steady_clock::now();
    go.store(true, std::memory_order_release);
    for (auto& t : pool) t.join();
    double worst = 0;
    for (double e : end) worst = e > worst ? e : worst;
    return worst;
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

// The same for the binary64 functions (main.cpp:94-99, 109-114: runKernel_ACA_double and
// runKernel_SKS_double, Table 5's 0.0171 / 0.0256 us rows).  algo: 0 = ACA, 1 = SKS.
double ref_time_repeat_f64(int algo, const double* src8, const double* tar8, double* H9,
                           int64_t iters) {
    using Fn64 = int (*)(double*, double*, double*);
    if (algo < 0 || algo > 1) return -1.0;
    const Fn64 f = algo == 0 ? sks::runKernel_ACA_double : sks::runKernel_SKS_double;
    double s[8], t[8];
    for (int k = 0; k < 8; ++k) { s[k] = src8[k]; t[k] = tar8[k]; }
    auto t0 = std::chrono::steady_clock::now();
    for (int64_t i = 0; i < iters; ++i) {
        f(s, t, H9);
        asm volatile("" ::"r"(H9) : "memory");
    }
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
}
