// hg_sks_api.cpp -- the reference's sks:: C++ interface (ACA_SKS.hpp:17-20) on top
// of the C ABI.  Every call goes to the GPU; there is no CPU solver in the product.
#include <hip/hip_runtime_api.h>

#include <cstring>

#include "sks_aca_sks.hpp"

namespace {

bool is_device_pointer(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // unregistered host memory: clear the sticky error
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// Per-thread staging for one problem: device buffer [src 8 | tar 8 | H 9] and a
// pinned host mirror.  Allocated on first use, kept for the thread's lifetime.
template <typename T>
struct Scratch {
    T* dev = nullptr;
    T* host = nullptr;
    int device = -1;
    int ensure() {
        int cur = 0;
        hipError_t e = hipGetDevice(&cur);
        if (e != hipSuccess) return (int)e;
        if (dev && device == cur) return 0;
        if ((e = hipMalloc(&dev, 32 * sizeof(T))) != hipSuccess) return (int)e;
        if ((e = hipHostMalloc(&host, 32 * sizeof(T), hipHostMallocDefault)) != hipSuccess)
            return (int)e;
        device = cur;
        return 0;
    }
};

template <typename T>
Scratch<T>& scratch() {
    static thread_local Scratch<T> s;
    return s;
}

template <typename T>
using BatchFn = int (*)(const T*, const T*, T*, int64_t, int, int, void*);

template <typename T, BatchFn<T> F>
int solve_one(T* src, T* tar, T* result) {
    if (!src || !tar || !result) return (int)hipErrorInvalidValue;
    if (is_device_pointer(src) && is_device_pointer(tar) && is_device_pointer(result)) {
        int rc = F(src, tar, result, 1, HG_LAYOUT_AOS, HG_FLAG_NORMALIZE, nullptr);
        if (rc) return rc;
        return (int)hipStreamSynchronize(nullptr);
    }
    Scratch<T>& s = scratch<T>();
    int rc = s.ensure();
    if (rc) return rc;
    std::memcpy(s.host, src, 8 * sizeof(T));
    std::memcpy(s.host + 8, tar, 8 * sizeof(T));
    hipError_t e = hipMemcpyAsync(s.dev, s.host, 16 * sizeof(T), hipMemcpyHostToDevice, nullptr);
    if (e != hipSuccess) return (int)e;
    rc = F(s.dev, s.dev + 8, s.dev + 16, 1, HG_LAYOUT_AOS, HG_FLAG_NORMALIZE, nullptr);
    if (rc) return rc;
    e = hipMemcpyAsync(s.host + 16, s.dev + 16, 9 * sizeof(T), hipMemcpyDeviceToHost, nullptr);
    if (e != hipSuccess) return (int)e;
    if ((e = hipStreamSynchronize(nullptr)) != hipSuccess) return (int)e;
    std::memcpy(result, s.host + 16, 9 * sizeof(T));
    return 0;
}

}  // namespace

namespace sks {

int runKernel_ACA(float* src, float* tar, float* result) {
    return solve_one<float, hg_aca_f32>(src, tar, result);
}
int runKernel_ACA_double(double* src, double* tar, double* result) {
    return solve_one<double, hg_aca_f64>(src, tar, result);
}
int runKernel_SKS(float* src, float* tar, float* result) {
    return solve_one<float, hg_sks_f32>(src, tar, result);
}
int runKernel_SKS_double(double* src, double* tar, double* result) {
    return solve_one<double, hg_sks_f64>(src, tar, result);
}

int runKernel_ACA_batch(const float* src, const float* tar, float* result, int64_t n,
                        void* stream) {
    return hg_aca_f32(src, tar, result, n, HG_LAYOUT_AOS, HG_FLAG_NORMALIZE, stream);
}
int runKernel_ACA_double_batch(const double* src, const double* tar, double* result,
                               int64_t n, void* stream) {
    return hg_aca_f64(src, tar, result, n, HG_LAYOUT_AOS, HG_FLAG_NORMALIZE, stream);
}
int runKernel_SKS_batch(const float* src, const float* tar, float* result, int64_t n,
                        void* stream) {
    return hg_sks_f32(src, tar, result, n, HG_LAYOUT_AOS, HG_FLAG_NORMALIZE, stream);
}
int runKernel_SKS_double_batch(const double* src, const double* tar, double* result,
                               int64_t n, void* stream) {
    return hg_sks_f64(src, tar, result, n, HG_LAYOUT_AOS, HG_FLAG_NORMALIZE, stream);
}

}  // namespace sks
