// hg_host.cpp -- host-resident batches (hg_solve_host_f32/_f64): the kernels read src/tar
// straight out of host memory over PCIe and write H straight back (zero-copy), so both
// link directions carry traffic at once and no device buffer is needed.  Measured at 10 M
// f32 AoS (tools/host_probe.py, profiles/r01/host_probe.json): 12.0 ms pinned and 13.4 ms
// pageable, against 17.7 / 18.8 ms for H2D + solve + D2H on one stream; the H2D direction
// alone takes 11.7 ms, so the call runs at the PCIe read bound.  Batches whose pageable
// buffers fit kStageBytes are copied through library-owned pinned memory instead of being
// registered (cheaper than the registration below that size).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <unistd.h>
#include <vector>

#include "hg_host_ranges.hpp"
#include "sks_homography.h"

namespace {

namespace host = hg::host;

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
    // (ROCm 7 answers unregistered memory with success and type 0; an older runtime's failed
    // probe leaves its own sticky error, cleared here -- see hg_sks_api.cpp)
    const bool ka = hipPointerGetAttributes(&a, first) == hipSuccess;
    if (!ka) (void)hipGetLastError();
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

// Library-owned registrations of pageable host memory, shared between concurrent calls.
//
// Two calls may solve buffers that share pages (two threads, each with half of one numpy
// or torch allocation).  A page the library registered for call A reads as pinned memory
// (hipMemoryTypeHost) to call B, so B must not take it for user-pinned memory: B would
// launch on it unprotected while A unregisters it under B's kernel.  Instead every call
// classifies its buffers under the registry's mutex, treats a buffer that touches a
// library-owned range as pageable, and holds a reference on each registration it uses
// until its kernel has finished; the last reference unregisters.  A needed range that
// overlaps registrations without lying inside one waits until they are released.
// Consequence: two slices of one allocation run at once only when the split
// is page-aligned or one slice's pages lie inside the other's registration; slices that
// merely share an edge page (a split inside a page) take turns -- the second waits for the
// first to finish, and a waiting call can be passed by calls that share an existing
// registration.  Correctness never depends on which happens.
struct Registration {
    host::Range r;
    int refs;
};

// A record of every page range the library registered (the last kHistory of them), with its
// fate -- kept for fault diagnosis: a GPU fault on a host address can be matched against the
// ranges this library mapped and unmapped (hg_internal_host_registry_find).  Updated under the
// registry mutex.
constexpr size_t kHistory = 4096;
enum : int { kLive = 1, kReleased = 2, kReleaseFailed = 3 };
struct HistoryEntry {
    uint64_t lo = 0, hi = 0, seq = 0;
    int state = 0, err = 0;
};

struct Registry {
    std::mutex mu;
    std::condition_variable released;
    std::vector<Registration> regs;
    HistoryEntry history[kHistory];
    uint64_t registered = 0;         // registrations made so far (history[registered % kHistory])
    uint64_t unregister_failures = 0;
    int last_failure = 0;

    void note(uintptr_t lo, int state, int err) {
        for (uint64_t k = 0; k < kHistory && k < registered; ++k) {  // newest first
            HistoryEntry& h = history[(registered - 1 - k) % kHistory];
            if (h.lo == lo && h.state == kLive) {
                h.state = state;
                h.err = err;
                return;
            }
        }
    }

    std::vector<host::Range> ranges() const {
        std::vector<host::Range> out;
        out.reserve(regs.size());
        for (const Registration& x : regs) out.push_back(x.r);
        return out;
    }
    bool owns_any(const void* p, size_t bytes) const {
        const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
        const host::Range r{lo, lo + bytes};
        for (const Registration& x : regs)
            if (host::overlaps(r, x.r)) return true;
        return false;
    }
    // Drops one reference on each registration in `held` (their bases); the last one
    // unregisters.  Caller holds `mu`.
    void release(const std::vector<uintptr_t>& held) {
        for (uintptr_t base : held) {
            for (size_t j = 0; j < regs.size(); ++j) {
                if (regs[j].r.lo != base) continue;
                if (--regs[j].refs == 0) {
                    // a failed unregistration would leave a mapping of pages the caller is about
                    // to free or reuse: counted and recorded (hg_internal_host_registry_stats)
                    const hipError_t e = hipHostUnregister(reinterpret_cast<void*>(regs[j].r.lo));
                    if (e != hipSuccess) {
                        ++unregister_failures;
                        last_failure = (int)e;
                        (void)hipGetLastError();
                    }
                    note(regs[j].r.lo, e == hipSuccess ? kReleased : kReleaseFailed, (int)e);
                    regs.erase(regs.begin() + (long)j);
                }
                break;
            }
        }
        released.notify_all();
    }
    // Registers (or shares) the pages under the pageable views and fills in their device
    // addresses; `held` receives the registrations referenced.  Caller holds `lock`.
    int acquire(std::vector<View*>& pageable, std::vector<uintptr_t>& held,
                std::unique_lock<std::mutex>& lock) {
        std::vector<host::Range> bytes;
        for (View* v : pageable) {
            const uintptr_t p = reinterpret_cast<uintptr_t>(v->host);
            bytes.push_back({p, p + v->bytes});
        }
        std::vector<host::Range> need;
        if (!host::page_ranges(bytes, (uintptr_t)sysconf(_SC_PAGESIZE), need)) return kInvalid;
        std::vector<long> plan = host::plan(need, ranges());
        while (host::any_conflict(plan)) {
            released.wait(lock);
            plan = host::plan(need, ranges());
        }
        for (size_t i = 0; i < need.size(); ++i) {
            long j = plan[i];
            if (j == host::kNew) {
                // portable: a registration may be shared with a call on another device
                char* base = reinterpret_cast<char*>(need[i].lo);
                const hipError_t e = hipHostRegister(base, need[i].hi - need[i].lo,
                                                     hipHostRegisterMapped | hipHostRegisterPortable);
                if (e != hipSuccess) {
                    release(held);
                    held.clear();
                    return (int)e;
                }
                regs.push_back({need[i], 1});
                j = (long)regs.size() - 1;
                HistoryEntry& h = history[registered % kHistory];
                h = HistoryEntry{need[i].lo, need[i].hi, ++registered, kLive, 0};
            } else {
                ++regs[(size_t)j].refs;
            }
            held.push_back(regs[(size_t)j].r.lo);
            // the address the CURRENT device uses for this registration (asked per call: the
            // registration may have been made while another device was current)
            void* d = nullptr;
            const hipError_t e =
                hipHostGetDevicePointer(&d, reinterpret_cast<void*>(regs[(size_t)j].r.lo), 0);
            if (e != hipSuccess) {
                release(held);
                held.clear();
                return (int)e;
            }
            for (View* v : pageable) {
                const uintptr_t p = reinterpret_cast<uintptr_t>(v->host);
                if (p >= need[i].lo && p < need[i].hi)
                    v->dev = static_cast<char*>(d) + (p - regs[(size_t)j].r.lo);
            }
        }
        return 0;
    }
};

Registry& registry() {
    static Registry r;
    return r;
}

// Small batches: the pageable buffers are copied through library-owned pinned memory instead
// of being registered.  Registering and releasing three page ranges costs ≈ 6 µs a call
// (INTEGRATION.md §1), more than copying up to kStageBytes, and leaves the caller's pages alone:
// KFD keeps registered pages mapped for the GPU after their release.  Stages
// come from a process-wide pool and are never freed, so no HIP call runs at thread or process
// exit.
constexpr size_t kStageBytes = 128 << 10;
constexpr size_t kStageAlign = 256;

struct Stage {
    char* host = nullptr;  // pinned, mapped
    char* dev = nullptr;   // its device address
};

struct StagePool {
    std::mutex mu;
    std::vector<Stage*> idle;

    int take(Stage*& out) {
        {
            std::lock_guard<std::mutex> lock(mu);
            if (!idle.empty()) {
                out = idle.back();
                idle.pop_back();
                return 0;
            }
        }
        auto* st = new Stage();
        // coherent (fine-grained): the GPU never holds a stale line of a stage another call refilled
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&st->host), kStageBytes,
                                     hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&st->dev), st->host, 0);
        if (e != hipSuccess) {  // nothing half-made is kept
            if (st->host) (void)hipHostFree(st->host);
            delete st;
            return (int)e;
        }
        out = st;
        return 0;
    }
    void give_back(Stage* st) {
        std::lock_guard<std::mutex> lock(mu);
        idle.push_back(st);
    }
};

StagePool& stage_pool() {
    static StagePool* p = new StagePool();  // never destroyed
    return *p;
}

size_t stage_round(size_t b) { return (b + kStageAlign - 1) / kStageAlign * kStageAlign; }

// Bytes a batch's pageable views take in a stage (each at a kStageAlign boundary).
size_t staged_bytes(const std::vector<View*>& pageable) {
    size_t b = 0;
    for (const View* x : pageable) b += stage_round(x->bytes);
    return b;
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
    Registry& reg = registry();
    std::unique_lock<std::mutex> lock(reg.mu);
    std::vector<View*> pageable;
    for (View& x : v) {
        if (reg.owns_any(x.host, x.bytes)) {  // pages another call registered: pageable
            pageable.push_back(&x);
            continue;
        }
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
    Stage* st = nullptr;
    if (!pageable.empty() && staged_bytes(pageable) <= kStageBytes) {
        // a stage that cannot be made (pinned memory exhausted) leaves the call to the
        // registration below, with the allocation's own error cleared
        if (stage_pool().take(st) != 0) {
            st = nullptr;
            (void)hipGetLastError();
        }
    }
    if (st) {
        lock.unlock();  // no registration: the registry is not involved
        int rc = 0;
        size_t off = 0, h_off = 0;
        bool h_staged = false;
        for (View* x : pageable) {
            if (x == &v[2]) {  // H: written by the kernel into the stage, copied out after
                h_staged = true;
                h_off = off;
            } else {
                std::memcpy(st->host + off, x->host, x->bytes);
            }
            x->dev = st->dev + off;
            off += stage_round(x->bytes);
        }
        rc = run();
        if (rc == 0 && h_staged) std::memcpy(H, st->host + h_off, v[2].bytes);
        stage_pool().give_back(st);
        return rc;
    }
    std::vector<uintptr_t> held;
    if (!pageable.empty()) {
        const int rc = reg.acquire(pageable, held, lock);
        if (rc) return rc;
    }
    lock.unlock();  // the solve itself runs unlocked: other calls may share the registrations
    const int rc = run();
    if (!held.empty()) {
        lock.lock();
        reg.release(held);
    }
    return rc;
}

}  // namespace

extern "C" {

// Library-internal diagnostics (not in the public header): {live registrations, registrations
// made, unregistration failures, last failure code}.
int hg_internal_host_registry_stats(int64_t* out) {
    if (!out) return kInvalid;
    Registry& reg = registry();
    std::lock_guard<std::mutex> lock(reg.mu);
    out[0] = (int64_t)reg.regs.size();
    out[1] = (int64_t)reg.registered;
    out[2] = (int64_t)reg.unregister_failures;
    out[3] = reg.last_failure;
    return 0;
}

// The newest recorded registration whose page range holds `va`: its range, sequence number
// and state (1 live, 2 released, 3 release failed; 0 = none of the last 4096 holds it).
int hg_internal_host_registry_find(uint64_t va, uint64_t* lo, uint64_t* hi, uint64_t* seq) {
    Registry& reg = registry();
    std::lock_guard<std::mutex> lock(reg.mu);
    for (uint64_t k = 0; k < kHistory && k < reg.registered; ++k) {
        const HistoryEntry& h = reg.history[(reg.registered - 1 - k) % kHistory];
        if (va >= h.lo && va < h.hi) {
            if (lo) *lo = h.lo;
            if (hi) *hi = h.hi;
            if (seq) *seq = h.seq;
            return h.state;
        }
    }
    return 0;
}

int hg_solve_host_f32(int algo, const float* src, const float* tar, float* H, int64_t n,
                      int layout, int flags, void* stream) {
    return solve_host<float>(algo, src, tar, H, n, layout, flags, stream);
}

int hg_solve_host_f64(int algo, const double* src, const double* tar, double* H, int64_t n,
                      int layout, int flags, void* stream) {
    return solve_host<double>(algo, src, tar, H, n, layout, flags, stream);
}

}  // extern "C"
