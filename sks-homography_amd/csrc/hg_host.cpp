// hg_host.cpp -- host-resident batches (hg_solve_host_f32/_f64): the kernels read src/tar
// straight out of host memory over PCIe and write H straight back (zero-copy), so both
// link directions carry traffic at once and no device buffer is needed.  Measured at 10 M
// f32 AoS (tools/host_probe.py, profiles/r01/host_probe.json): 12.0 ms pinned and 13.4 ms
// pageable, against 17.7 / 18.8 ms for H2D + solve + D2H on one stream; the H2D direction
// alone takes 11.7 ms, so the call runs at the PCIe read bound.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <unistd.h>
#include <vector>

#include "sks_homography.h"

namespace {

constexpr int kInvalid = (int)hipErrorInvalidValue;

// What a pointer is: device-visible already (device / managed memory, or host memory
// pinned with a device mapping), or pageable host memory that must be registered.
struct View {
    const void* host = nullptr;  // the caller's pointer
    size_t bytes = 0;
    void* dev = nullptr;         // device address once known
    bool in_host = true;         // host memory (pinned or pageable), read over PCIe
};

// Device address of [p, p + bytes) if the whole range is device-visible, nullptr if it is
// unregistered host memory; an error code if it is visible only in part.
int classify(View& v) {
    hipPointerAttribute_t a{}, b{};
    const char* first = static_cast<const char*>(v.host);
    const char* last = first + v.bytes - 1;
    const bool ka = hipPointerGetAttributes(&a, first) == hipSuccess;
    if (!ka) (void)hipGetLastError();  // unregistered host memory: clear the sticky error
    const bool kb = hipPointerGetAttributes(&b, last) == hipSuccess;
    if (!kb) (void)hipGetLastError();
    auto visible = [](bool known, const hipPointerAttribute_t& x) {
        return known && (x.type == hipMemoryTypeDevice || x.type == hipMemoryTypeManaged ||
                         x.type == hipMemoryTypeHost);
    };
    const bool va = visible(ka, a), vb = visible(kb, b);
    if (!va && !vb) {
        v.dev = nullptr;
        return 0;
    }
    if (va != vb || a.type != b.type) return kInvalid;  // straddles a mapped range's end
    if (a.type == hipMemoryTypeHost) {
        void *da = nullptr, *db = nullptr;
        hipError_t e = hipHostGetDevicePointer(&da, const_cast<char*>(first), 0);
        if (e == hipSuccess) e = hipHostGetDevicePointer(&db, const_cast<char*>(last), 0);
        if (e != hipSuccess) return (int)e;
        // one contiguous mapping, not two pinned blocks that happen to abut
        if (static_cast<char*>(db) - static_cast<char*>(da) != last - first) return kInvalid;
        v.dev = da;
    } else {
        v.dev = const_cast<void*>(v.host);  // device or managed memory: use as is
        v.in_host = false;
    }
    return 0;
}

// Registers the pages under the pageable views (overlapping or adjacent ranges merged,
// so buffers cut from one allocation share a registration) and fills in their device
// addresses.  The ranges registered are returned for hipHostUnregister.
int register_pageable(std::vector<View*>& pageable, std::vector<char*>& registered) {
    const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
    struct Range {
        uintptr_t lo, hi;
    };
    std::vector<Range> r;
    for (View* v : pageable) {
        const uintptr_t p = reinterpret_cast<uintptr_t>(v->host);
        r.push_back({p & ~(pg - 1), (p + v->bytes + pg - 1) & ~(pg - 1)});
    }
    std::sort(r.begin(), r.end(), [](const Range& a, const Range& b) { return a.lo < b.lo; });
    std::vector<Range> merged;
    for (const Range& x : r) {
        if (!merged.empty() && x.lo <= merged.back().hi)
            merged.back().hi = std::max(merged.back().hi, x.hi);
        else
            merged.push_back(x);
    }
    for (const Range& m : merged) {
        char* base = reinterpret_cast<char*>(m.lo);
        hipError_t e = hipHostRegister(base, m.hi - m.lo, hipHostRegisterMapped);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return (int)e;
        }
        registered.push_back(base);
        void* d = nullptr;
        if ((e = hipHostGetDevicePointer(&d, base, 0)) != hipSuccess) return (int)e;
        for (View* v : pageable) {
            const uintptr_t p = reinterpret_cast<uintptr_t>(v->host);
            if (p >= m.lo && p < m.hi) v->dev = static_cast<char*>(d) + (p - m.lo);
        }
    }
    return 0;
}

// One registration at a time: two calls sharing pageable pages must not unregister
// them under each other.  Calls on pinned or device memory never take it.
std::mutex& registration_mutex() {
    static std::mutex mu;
    return mu;
}

// The solvers with the host-memory cache policy (hg_kernels.hip, library-internal).
extern "C" int hg_internal_solve_host_f32(int, const float*, const float*, float*, int64_t, int,
                                          int, void*);
extern "C" int hg_internal_solve_host_f64(int, const double*, const double*, double*, int64_t,
                                          int, int, void*);

template <typename T>
int launch(int algo, const T* s, const T* t, T* h, int64_t n, int layout, int flags,
           void* stream, bool host) {
    if (host) {  // any buffer in host memory: the host-memory cache policy
        if constexpr (sizeof(T) == 4)
            return hg_internal_solve_host_f32(algo, s, t, h, n, layout, flags, stream);
        else
            return hg_internal_solve_host_f64(algo, s, t, h, n, layout, flags, stream);
    }
    if constexpr (sizeof(T) == 4) {  // all in device memory: the ordinary entry points
        switch (algo) {
            case HG_ALGO_ACA: return hg_aca_f32(s, t, h, n, layout, flags, stream);
            case HG_ALGO_SKS: return hg_sks_f32(s, t, h, n, layout, flags, stream);
            case HG_ALGO_GE: return hg_ge_f32(s, t, h, n, layout, flags, stream);
            default: return kInvalid;
        }
    } else {
        switch (algo) {
            case HG_ALGO_ACA: return hg_aca_f64(s, t, h, n, layout, flags, stream);
            case HG_ALGO_SKS: return hg_sks_f64(s, t, h, n, layout, flags, stream);
            case HG_ALGO_GE: return hg_ge_f64(s, t, h, n, layout, flags, stream);
            case HG_ALGO_GPT: return hg_gpt_f64(s, t, h, n, layout, flags, stream);
            default: return kInvalid;
        }
    }
}

template <typename T>
int solve_host(int algo, const T* src, const T* tar, T* H, int64_t n, int layout, int flags,
               void* stream) {
    const int max_algo = sizeof(T) == 8 ? HG_ALGO_GPT : HG_ALGO_GE;
    if (algo < HG_ALGO_ACA || algo > max_algo || n < 0) return kInvalid;
    if (layout != HG_LAYOUT_AOS && layout != HG_LAYOUT_SOA) return kInvalid;
    if (flags & ~HG_FLAG_NORMALIZE) return kInvalid;
    if (n == 0) return 0;
    if (!src || !tar || !H) return kInvalid;
    if (n > INT64_MAX / (9 * (int64_t)sizeof(T))) return kInvalid;
    View v[3] = {{src, (size_t)n * 8 * sizeof(T)},
                 {tar, (size_t)n * 8 * sizeof(T)},
                 {H, (size_t)n * 9 * sizeof(T)}};
    std::vector<View*> pageable;
    for (View& x : v) {
        const int rc = classify(x);
        if (rc) return rc;
        if (!x.dev) pageable.push_back(&x);
    }
    const bool all_device = !v[0].in_host && !v[1].in_host && !v[2].in_host;
    // Device-resident data may come from work queued on the legacy default stream, so
    // with no stream given it is solved there (a private stream would race it); host
    // data has no such producer and goes on the calling thread's own default stream.
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!s && !all_device) s = hipStreamPerThread;
    auto run = [&]() -> int {
        int rc = launch<T>(algo, static_cast<const T*>(v[0].dev), static_cast<const T*>(v[1].dev),
                           static_cast<T*>(v[2].dev), n, layout, flags, s, !all_device);
        const hipError_t e = hipStreamSynchronize(s);  // H is complete when the call returns
        return rc ? rc : (int)e;
    };
    if (pageable.empty()) return run();
    std::lock_guard<std::mutex> lock(registration_mutex());
    std::vector<char*> registered;
    int rc = register_pageable(pageable, registered);
    if (!rc) rc = run();
    for (char* base : registered) (void)hipHostUnregister(base);
    return rc;
}

}  // namespace

extern "C" {

int hg_solve_host_f32(int algo, const float* src, const float* tar, float* H, int64_t n,
                      int layout, int flags, void* stream) {
    return solve_host<float>(algo, src, tar, H, n, layout, flags, stream);
}

int hg_solve_host_f64(int algo, const double* src, const double* tar, double* H, int64_t n,
                      int layout, int flags, void* stream) {
    return solve_host<double>(algo, src, tar, H, n, layout, flags, stream);
}

}  // extern "C"
