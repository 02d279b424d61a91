// hg_sks_api.cpp -- the reference's sks:: C++ interface (ACA_SKS.hpp:17-20) on top
// of the C ABI.  Every call goes to the GPU; there is no CPU solver in the product.
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstring>
#include <mutex>
#include <vector>

#include "sks_aca_sks.hpp"

// Library-internal (hg_kernels.hip): one problem, then *done = seq after H (system scope).
extern "C" int hg_internal_solve_one_signal_f32(int, const float*, const float*, float*, int,
                                                uint32_t*, uint32_t, void*);
extern "C" int hg_internal_solve_one_signal_f64(int, const double*, const double*, double*, int,
                                                uint32_t*, uint32_t, void*);

namespace {

// Pointer probes.  On ROCm 7 hipPointerGetAttributes succeeds on unregistered host memory
// (type hipMemoryTypeUnregistered) and touches no error state, so an error the caller left
// pending stays pending (tools/probe_lasterror.cpp, tests/test_gpu_errors.py).  Runtimes
// that fail the probe instead (hipErrorInvalidValue) leave that error sticky: it is
// cleared here, because it is the probe's own, not the caller's.
bool is_device_pointer(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // the failed probe's own error (older runtimes)
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// Per-thread state for host-pointer calls: a non-blocking stream (threads never
// serialise on the legacy default stream) and host memory mapped into the device address
// space -- 16 values for H plus a completion word -- which the kernel writes directly.
// The points go in the kernel arguments, so a call is one launch, and the thread then
// spins on the completion word (the kernel stores it after H, system scope) instead of
// waiting on the stream: ~half the latency of a stream synchronisation.
//
// Slots (one per device a thread uses) come from a process-wide pool and go back to it when
// the thread exits; they are never freed.  So a thread's exit makes no HIP call (a HIP call
// from a thread-local destructor runs after the runtime's and any tool's own per-thread
// state may be gone -- under rocprofv3 it aborts the process), and the stream and mapped
// memory a call may still have in flight -- the kernel retires after it has stored the
// completion word -- stay valid: the next thread to take the slot orders its launch after
// that kernel on the same stream.
template <typename T>
struct Slot {
    static constexpr size_t kDoneOffset = 16 * sizeof(T);  // the completion word, after H
    T* host = nullptr;
    T* mapped = nullptr;
    hipStream_t stream = nullptr;
    uint32_t seq = 0;
    volatile uint32_t* done_host() { return reinterpret_cast<volatile uint32_t*>(reinterpret_cast<char*>(host) + kDoneOffset); }
    uint32_t* done_dev() { return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(mapped) + kDoneOffset); }
};

constexpr int kMaxDevices = 64;

template <typename T>
struct SlotPool {
    std::mutex mu;
    std::vector<Slot<T>*> idle[kMaxDevices];

    // A slot for `dev` on the calling thread's current device: an idle one, or a new one.
    int take(int dev, Slot<T>*& out) {
        {
            std::lock_guard<std::mutex> lock(mu);
            if (!idle[dev].empty()) {
                out = idle[dev].back();
                idle[dev].pop_back();
                return 0;
            }
        }
        auto* sl = new Slot<T>();
        hipError_t e = hipStreamCreateWithFlags(&sl->stream, hipStreamNonBlocking);
        if (e == hipSuccess)
            e = hipHostMalloc(reinterpret_cast<void**>(&sl->host), Slot<T>::kDoneOffset + 64,
                              hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) {
            *sl->done_host() = 0;
            e = hipHostGetDevicePointer(reinterpret_cast<void**>(&sl->mapped), sl->host, 0);
        }
        if (e != hipSuccess) {  // nothing half-made is kept
            if (sl->host) (void)hipHostFree(sl->host);
            if (sl->stream) (void)hipStreamDestroy(sl->stream);
            delete sl;
            return (int)e;
        }
        out = sl;
        return 0;
    }
    void give_back(int dev, Slot<T>* sl) {
        std::lock_guard<std::mutex> lock(mu);
        idle[dev].push_back(sl);
    }
};

template <typename T>
SlotPool<T>& slot_pool() {
    static SlotPool<T>* p = new SlotPool<T>();  // never destroyed: slots outlive every thread
    return *p;
}

template <typename T>
struct Scratch {
    Slot<T>* slot[kMaxDevices] = {};
    int cur_dev = -1;

    int ensure() {
        int dev = 0;
        const hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return (int)e;
        if (dev < 0 || dev >= kMaxDevices) return (int)hipErrorInvalidDevice;
        cur_dev = dev;
        if (slot[dev]) return 0;
        return slot_pool<T>().take(dev, slot[dev]);
    }
    Slot<T>& cur() { return *slot[cur_dev]; }
    ~Scratch() {  // no HIP call: the slots go back to the pool
        for (int d = 0; d < kMaxDevices; ++d)
            if (slot[d]) slot_pool<T>().give_back(d, slot[d]);
    }
};

template <typename T>
Scratch<T>& scratch() {
    static thread_local Scratch<T> s;
    return s;
}

template <typename T>
using BatchFn = int (*)(const T*, const T*, T*, int64_t, int, int, void*);
template <typename T>
using OneFn = int (*)(int, const T*, const T*, T*, int, uint32_t*, uint32_t, void*);

// Waits until the kernel has published H (*done == seq): a spin with pause, bounded; past
// the bound (a fault, a stalled device) the stream's own status decides.
template <typename T>
int wait_done(Slot<T>& sl, uint32_t seq) {
    auto seen = [&] { return __atomic_load_n(sl.done_host(), __ATOMIC_ACQUIRE) == seq; };
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; !seen(); ++i) {
        __builtin_ia32_pause();
        if ((i & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
            const hipError_t e = hipStreamSynchronize(sl.stream);
            if (e != hipSuccess) return (int)e;
            return seen() ? 0 : (int)hipErrorUnknown;
        }
    }
    return 0;
}

template <typename T, BatchFn<T> F, OneFn<T> ONE, int ALGO>
int solve_one(T* src, T* tar, T* result) {
    if (!src || !tar || !result) return (int)hipErrorInvalidValue;
    const bool ds = is_device_pointer(src), dt = is_device_pointer(tar);
    const bool dr = is_device_pointer(result);
    if (ds && dt && dr) {
        // device data may come from work the caller queued on the legacy default stream:
        // launching there keeps that order (a private stream would race it)
        int rc = F(src, tar, result, 1, HG_LAYOUT_AOS, HG_FLAG_NORMALIZE, nullptr);
        if (rc) return rc;
        return (int)hipStreamSynchronize(nullptr);
    }
    Scratch<T>& s = scratch<T>();
    int rc = s.ensure();
    if (rc) return rc;
    Slot<T>& sl = s.cur();
    const uint32_t seq = ++sl.seq ? sl.seq : ++sl.seq;  // never 0, the word's initial value
    if (ds || dt) {
        // mixed: stage device-resident inputs to the host first (rare)
        T in[16];
        hipError_t e = hipMemcpy(in, src, 8 * sizeof(T), hipMemcpyDefault);
        if (e == hipSuccess) e = hipMemcpy(in + 8, tar, 8 * sizeof(T), hipMemcpyDefault);
        if (e != hipSuccess) return (int)e;
        rc = ONE(ALGO, in, in + 8, sl.mapped, HG_FLAG_NORMALIZE, sl.done_dev(), seq, sl.stream);
    } else {
        rc = ONE(ALGO, src, tar, sl.mapped, HG_FLAG_NORMALIZE, sl.done_dev(), seq, sl.stream);
    }
    if (rc) return rc;
    if ((rc = wait_done<T>(sl, seq))) return rc;
    if (dr) return (int)hipMemcpy(result, sl.host, 9 * sizeof(T), hipMemcpyHostToDevice);
    std::memcpy(result, sl.host, 9 * sizeof(T));
    return 0;
}

// Batches: device-visible buffers (device, managed or pinned host memory) are solved
// asynchronously on `stream`; a batch with any pageable host buffer goes through
// hg_solve_host_* (staged through library-owned pinned memory, synchronous).
bool is_pageable(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // the failed probe's own error (older runtimes)
        return true;
    }
    return attr.type != hipMemoryTypeDevice && attr.type != hipMemoryTypeManaged &&
           attr.type != hipMemoryTypeHost;
}

template <typename T>
using HostFn = int (*)(int, const T*, const T*, T*, int64_t, int, int, void*);

template <typename T>
int solve_batch(BatchFn<T> dev, int algo, const T* src, const T* tar, T* result, int64_t n,
                void* stream) {
    if (n > 0 && src && tar && result &&
        (is_pageable(src) || is_pageable(tar) || is_pageable(result))) {
        HostFn<T> host;
        if constexpr (sizeof(T) == 4) host = hg_solve_host_f32;
        else host = hg_solve_host_f64;
        return host(algo, src, tar, result, n, HG_LAYOUT_AOS, HG_FLAG_NORMALIZE, stream);
    }
    return dev(src, tar, result, n, HG_LAYOUT_AOS, HG_FLAG_NORMALIZE, stream);
}

}  // namespace

namespace sks {

int runKernel_ACA(float* src, float* tar, float* result) {
    return solve_one<float, hg_aca_f32, hg_internal_solve_one_signal_f32, 0>(src, tar, result);
}
int runKernel_ACA_double(double* src, double* tar, double* result) {
    return solve_one<double, hg_aca_f64, hg_internal_solve_one_signal_f64, 0>(src, tar, result);
}
int runKernel_SKS(float* src, float* tar, float* result) {
    return solve_one<float, hg_sks_f32, hg_internal_solve_one_signal_f32, 1>(src, tar, result);
}
int runKernel_SKS_double(double* src, double* tar, double* result) {
    return solve_one<double, hg_sks_f64, hg_internal_solve_one_signal_f64, 1>(src, tar, result);
}

int runKernel_ACA_batch(const float* src, const float* tar, float* result, int64_t n,
                        void* stream) {
    return solve_batch<float>(hg_aca_f32, HG_ALGO_ACA, src, tar, result, n, stream);
}
int runKernel_ACA_double_batch(const double* src, const double* tar, double* result,
                               int64_t n, void* stream) {
    return solve_batch<double>(hg_aca_f64, HG_ALGO_ACA, src, tar, result, n, stream);
}
int runKernel_SKS_batch(const float* src, const float* tar, float* result, int64_t n,
                        void* stream) {
    return solve_batch<float>(hg_sks_f32, HG_ALGO_SKS, src, tar, result, n, stream);
}
int runKernel_SKS_double_batch(const double* src, const double* tar, double* result,
                               int64_t n, void* stream) {
    return solve_batch<double>(hg_sks_f64, HG_ALGO_SKS, src, tar, result, n, stream);
}

}  // namespace sks
