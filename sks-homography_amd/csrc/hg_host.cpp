// hg_host.cpp -- host-resident batches (hg_solve_host_f32/_f64).  Pinned (device-mapped)
// buffers are read and written by the kernel in place over PCIe (zero-copy: both link
// directions carry traffic at once, no device buffer; at 10 M f32 AoS 12.0 ms against
// 17.7 ms for H2D + solve + D2H, profiles/r01/host_probe.json).  Pageable buffers go through a
// ring of library-owned pinned stages, filled and emptied by host threads while the kernel
// reads the stage before (solve_staged below): the caller's pages are never registered, so
// the call leaves no GPU mapping of them behind.  Registering them instead (zero-copy on the
// caller's pages) is opt-in, HG_FLAG_HOST_REGISTER: KFD keeps registered pages mapped for the
// GPU after hipHostUnregister, which is how heap pages reach a later HIP copy
// in the state the round-4/5 faults came from.
#include <hip/hip_runtime_api.h>
#include <emmintrin.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <unistd.h>
#include <vector>

#include "hg_host_ranges.hpp"
#include "hg_host_stage.hpp"
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

// Library-owned registrations of pageable host memory (HG_FLAG_HOST_REGISTER calls), shared
// between concurrent calls.  A staged call also consults the registry: pages a registering
// call holds read as pinned memory, and are still the caller's pageable memory to it.
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

// ---------------------------------------------------------------------------------------------
// Pageable buffers (the default): a ring of library-owned pinned stages (hg_host_stage.hpp).
// The caller's pages are only ever read and written by host threads, so the call leaves them
// exactly as it found them -- no registration, no GPU mapping.  Chunk k is
// copied into stage k % D while the kernels of the chunks before it read their stages over
// PCIe; a stage is refilled once its chunk's kernel has finished (an event per stage) and that
// chunk's H has been copied out.  Batches whose staged bytes fit kSmallStageBytes take one
// small stage and no helper thread (about 6 us cheaper a call than registering three page
// ranges).  Stages come from a process-wide pool and are never freed, so no
// HIP call runs at thread or process exit; they are portable (mapped for every device) and
// their device address is looked up per device.
constexpr size_t kSmallStageBytes = 128 << 10;
constexpr int kDevSlots = 64;

// Ring shape: 8 MiB stages, 6 deep (48 MiB of pinned memory and 48 MiB of device buffers while a
// large call runs), 8 copy threads, the copy engines moving each stage in and the kernel writing
// H straight into the stage.  At 10 M f32 AoS from pageable memory (tools/ring_probe.py,
// profiles/r06/ring_*.json): 8 MiB x 4 / x 6 13.1 ms, 12 x 6 13.3, 16 x 6 13.6, 32 x 4 13.0 (the GPU
// side alone 11.6-12.5: the host copies are what is left); with H brought back by the copy
// engines too (mode 1) 14.2-14.5 -- one engine's queue serialises the two directions; with the
// kernel reading the stage itself (mode 0) 16.1 at 32 x 6 (the pinned zero-copy call: 12.0).
struct StageConfig {
    std::atomic<int64_t> ring_bytes{8 << 20};  // one ring stage
    std::atomic<int> depth{6};                  // ring stages (and streams) a call cycles through
    std::atomic<int> coherent{1};              // stage memory fine-grained (1) or not (0)
    std::atomic<int> probe{0};  // tools only, wrong results: 1 no host copies, 2 no kernels
    std::atomic<int> dma{2};    // ring chunks: in by the copy engines, H by the kernel into the
                                // stage (2); both ways by the copy engines (1); read and written
                                // in the stage by the kernel over PCIe (0)
};

StageConfig& stage_config() {
    static StageConfig* c = new StageConfig();  // never destroyed
    return *c;
}

host::CopyPool& copy_pool() {
    static host::CopyPool* p = [] {
        auto* q = new host::CopyPool();  // never destroyed: its helpers never exit
        cpu_set_t set;
        int cpus = 8;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
        q->set_threads(std::max(1, std::min(cpus, 8)));
        return q;
    }();
    return *p;
}

struct Stage {
    char* host = nullptr;  // pinned, mapped, portable; coherent or not (StageConfig)
    size_t bytes = 0;
    int coherent = 1;
    char* dev[kDevSlots] = {};  // its address on device d (filled on first use there)
};

struct StageStats {
    std::atomic<int64_t> made{0}, calls{0}, chunks{0}, leaked{0}, ring_calls{0};
    std::atomic<int64_t> copy_ns{0}, wait_ns{0}, copy_bytes{0};  // host copies; event waits
};

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

StageStats& stage_stats() {
    static StageStats* s = new StageStats();
    return *s;
}

struct StagePool {
    std::mutex mu;
    std::vector<Stage*> idle;

    // An idle stage of exactly `bytes` and kind, or a new one.
    int take(size_t bytes, int coherent, Stage*& out) {
        {
            std::lock_guard<std::mutex> lock(mu);
            for (size_t i = idle.size(); i-- > 0;) {
                if (idle[i]->bytes != bytes || idle[i]->coherent != coherent) continue;
                out = idle[i];
                idle.erase(idle.begin() + (long)i);
                return 0;
            }
        }
        auto* st = new Stage();
        // coherent (fine-grained): the GPU never holds a stale line of a stage another call
        // refilled; portable: a stage serves calls on any device of the process
        const hipError_t e = hipHostMalloc(
            reinterpret_cast<void**>(&st->host), bytes,
            hipHostMallocMapped | hipHostMallocPortable |
                (coherent ? hipHostMallocCoherent : hipHostMallocNonCoherent));
        if (e != hipSuccess) {  // nothing half-made is kept
            delete st;
            return (int)e;
        }
        st->bytes = bytes;
        st->coherent = coherent;
        ++stage_stats().made;
        out = st;
        return 0;
    }
    // Idle stages are kept up to kIdleCap bytes (so a burst of concurrent large calls does not
    // pin its peak for the process's life); a stage past the cap is freed here, in the call.
    static constexpr size_t kIdleCap = (size_t)1 << 30;
    void give_back(Stage* st) {
        {
            std::lock_guard<std::mutex> lock(mu);
            size_t held = 0;
            for (const Stage* x : idle) held += x->bytes;
            if (held + st->bytes <= kIdleCap) {
                idle.push_back(st);
                return;
            }
        }
        (void)hipHostFree(st->host);
        delete st;
    }
};

StagePool& stage_pool() {
    static StagePool* p = new StagePool();  // never destroyed
    return *p;
}

// The stage's address on the current device.
int stage_dev(Stage* st, char*& out) {
    int d = 0;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess) return (int)e;
    if (d >= 0 && d < kDevSlots && st->dev[d]) {
        out = st->dev[d];
        return 0;
    }
    void* p = nullptr;
    e = hipHostGetDevicePointer(&p, st->host, 0);
    if (e != hipSuccess) return (int)e;
    out = static_cast<char*>(p);
    if (d >= 0 && d < kDevSlots) st->dev[d] = out;
    return 0;
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

// Streams of the ring, per device: created on first need, never destroyed (no HIP call at
// exit), handed to one call at a time.  Consecutive chunks run on different streams, so their
// kernels overlap: one chunk's kernel alone cannot keep both PCIe directions busy through its
// ramp-up and drain (profiles/r06: 145 us per 8 MiB chunk on one stream, the link's rate only
// with several in flight).
struct StreamPool {
    std::mutex mu;
    std::vector<std::pair<int, hipStream_t>> idle;

    int take(int dev, hipStream_t& out) {
        {
            std::lock_guard<std::mutex> lock(mu);
            for (size_t i = idle.size(); i-- > 0;) {
                if (idle[i].first != dev) continue;
                out = idle[i].second;
                idle.erase(idle.begin() + (long)i);
                return 0;
            }
        }
        return (int)hipStreamCreateWithFlags(&out, hipStreamNonBlocking);
    }
    void give_back(int dev, hipStream_t x) {
        std::lock_guard<std::mutex> lock(mu);
        idle.push_back({dev, x});
    }
};

StreamPool& stream_pool() {
    static StreamPool* p = new StreamPool();  // never destroyed
    return *p;
}

// Device buffers of the ring's DMA form, per device and size: made on first need, never freed
// (device memory, HBM: a few stages' worth per concurrent call), handed to one call at a time.
struct DevPool {
    struct Buf {
        int dev;
        size_t bytes;
        char* p;
    };
    std::mutex mu;
    std::vector<Buf> idle;

    int take(int dev, size_t bytes, char*& out) {
        {
            std::lock_guard<std::mutex> lock(mu);
            for (size_t i = idle.size(); i-- > 0;) {
                if (idle[i].dev != dev || idle[i].bytes != bytes) continue;
                out = idle[i].p;
                idle.erase(idle.begin() + (long)i);
                return 0;
            }
        }
        void* p = nullptr;
        const hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) return (int)e;
        out = static_cast<char*>(p);
        return 0;
    }
    void give_back(int dev, size_t bytes, char* p) {
        std::lock_guard<std::mutex> lock(mu);
        idle.push_back({dev, bytes, p});
    }
};

DevPool& dev_pool() {
    static DevPool* p = new DevPool();  // never destroyed
    return *p;
}

// Waits for `ev` by polling: hipEventSynchronize may put the thread to sleep, and each wake-up
// cost the ring ~0.5 ms a chunk at 1 M problems (8.7 ms a call against 1.6 ms polled;
// tools/crossover.py, profiles/r06).  After 50 ms of polling the wait blocks in HIP instead, so
// a long kernel does not keep a core busy.  (Stream drains keep hipStreamSynchronize: polling
// hipStreamQuery made the one-chunk calls 4-5 us slower.)
int wait_poll(hipEvent_t ev) {
    const int64_t t0 = now_ns();
    for (;;) {
        const hipError_t q = hipEventQuery(ev);
        if (q != hipErrorNotReady) return (int)q;
        if (now_ns() - t0 > 50000000) break;
        _mm_pause();
    }
    return (int)hipEventSynchronize(ev);
}

// The staged solve of a batch with at least one pageable buffer (v[i].dev == nullptr).  `s` is
// the caller's stream: device-memory buffers are ordered after the work queued on it.
template <typename T>
int solve_staged(int algo, View (&v)[3], int64_t n, int layout, int flags, hipStream_t s) {
    host::StagePlan p;
    p.n = n;
    p.elem = sizeof(T);
    p.soa = layout == HG_LAYOUT_SOA;
    for (int i = 0; i < 3; ++i) p.mode[i] = v[i].dev ? host::kDirect : host::kCpu;
    size_t per = 0;
    for (int i = 0; i < 3; ++i)
        if (p.staged(i)) per += host::align_up((size_t)n * p.per_problem(i));
    const bool small = per <= kSmallStageBytes;
    const size_t cap = small ? kSmallStageBytes : (size_t)stage_config().ring_bytes.load();
    if (!host::plan_chunks(p, cap)) return kInvalid;
    if (p.soa && p.chunks > 1) {
        // an SoA chunk is C-wide rows: a buffer used in place would have n-wide rows, so every
        // buffer goes through the stage -- host memory by the copy threads, device memory by
        // the DMA engines
        for (int i = 0; i < 3; ++i)
            if (p.mode[i] == host::kDirect) p.mode[i] = v[i].in_host ? host::kCpu : host::kDma;
        if (!host::plan_chunks(p, cap)) return kInvalid;
    }
    const bool device_data = !v[0].in_host || !v[1].in_host || !v[2].in_host;
    const int64_t K = p.chunks;
    const int D = (int)std::min<int64_t>(K, std::max(1, stage_config().depth.load()));
    // one chunk: the caller's stream; several: a ring stream per stage
    const bool ring = K > 1;
    // Past the small stage the copy engines move each stage's src / tar to a device buffer and
    // the kernel reads them from HBM, writing H straight into the stage over PCIe (posted
    // writes): the link's two directions are driven by different agents.  A chunk kernel that
    // also reads the stage over PCIe runs one round of waves whose reads barely overlap (15 ms
    // of kernels alone at 10 M against 12 ms for one zero-copy kernel over pinned memory), and
    // H brought back by the copy engines too shares their queue with the inputs (13.6 ms of GPU
    // side alone); this form's GPU side takes 11.6-12.5 ms (tools/ring_probe.py `parts`,
    // profiles/r06).
    bool dma = !small && stage_config().dma.load() != 0;
    const bool h_by_kernel = stage_config().dma.load() == 2;
    std::vector<Stage*> st((size_t)D, nullptr);
    std::vector<char*> sd((size_t)D, nullptr);
    std::vector<char*> db((size_t)D, nullptr);  // device buffers (dma)
    std::vector<hipStream_t> ss((size_t)D, s);
    std::vector<bool> own((size_t)D, false);
    std::vector<hipEvent_t> ev;
    int rc = 0, dev = 0;
    const int coherent = stage_config().coherent.load();
    rc = (int)hipGetDevice(&dev);
    for (int j = 0; j < D && !rc; ++j) {
        rc = stage_pool().take(cap, coherent, st[(size_t)j]);
        if (!rc) rc = stage_dev(st[(size_t)j], sd[(size_t)j]);
        if (!rc && dma && dev_pool().take(dev, cap, db[(size_t)j]) != 0) {
            // device memory short (another allocation holds the card): this call's kernels read
            // the stages over PCIe instead -- slower, same bits
            (void)hipGetLastError();
            for (int i = 0; i < j; ++i) dev_pool().give_back(dev, cap, db[(size_t)i]);
            std::fill(db.begin(), db.end(), nullptr);
            dma = false;
        }
    }
    if (!rc && ring) {
        for (int j = 0; j < D && !rc; ++j) {
            rc = stream_pool().take(dev, ss[(size_t)j]);
            own[(size_t)j] = rc == 0;
        }
        ev.assign((size_t)D + 1, nullptr);
        for (int j = 0; j <= D && !rc; ++j)
            rc = (int)hipEventCreateWithFlags(&ev[(size_t)j], hipEventDisableTiming);
        if (!rc && device_data) {  // the ring streams start after the caller's queued work
            rc = (int)hipEventRecord(ev[(size_t)D], s);
            for (int j = 0; j < D && !rc; ++j) rc = (int)hipStreamWaitEvent(ss[(size_t)j], ev[(size_t)D], 0);
        }
    }
    ++stage_stats().calls;
    if (!small) ++stage_stats().ring_calls;
    host::CopyPool& pool = copy_pool();
    std::vector<host::Piece> pieces;
    const char* in_user[3] = {static_cast<const char*>(v[0].host),
                              static_cast<const char*>(v[1].host), nullptr};
    char* H_user = static_cast<char*>(const_cast<void*>(v[2].host));
    auto copy_out = [&](int64_t k, int j) {
        if (p.mode[2] == host::kCpu)
            host::chunk_pieces(p, 2, k, nullptr, H_user, st[(size_t)j]->host, false, pieces);
    };
    auto copy_in = [&](int64_t k, int j) {
        for (int i = 0; i < 2; ++i)
            if (p.mode[i] == host::kCpu)
                host::chunk_pieces(p, i, k, in_user[i], nullptr, st[(size_t)j]->host, true, pieces);
    };
    const size_t E = sizeof(T);
    StageStats& stats = stage_stats();
    const int probe = stage_config().probe.load();
    auto run_pieces = [&]() {
        if (probe & 1) return;
        const int64_t t0 = now_ns();
        pool.run(pieces);
        stats.copy_ns += now_ns() - t0;
        int64_t b = 0;
        for (const host::Piece& x : pieces) b += (int64_t)x.bytes;
        stats.copy_bytes += b;
    };
    // chunks launched whose H has not been copied out yet, oldest first (chunk k is in stage
    // k % D); H leaves as soon as a chunk is done, so only the last chunk's copy is exposed
    int64_t out_next = 0;
    auto take_done = [&](int64_t upto, bool wait_first) -> int {  // copy out chunks < upto that are done
        while (out_next < upto) {
            const int j = (int)(out_next % D);
            if (ring) {
                if (wait_first) {
                    const int64_t t0 = now_ns();
                    const int e = wait_poll(ev[(size_t)j]);
                    stats.wait_ns += now_ns() - t0;
                    if (e) return e;
                    wait_first = false;
                } else {
                    const hipError_t q = hipEventQuery(ev[(size_t)j]);
                    if (q == hipErrorNotReady) break;
                    if (q != hipSuccess) return (int)q;
                }
            }
            copy_out(out_next, j);
            ++out_next;
        }
        return 0;
    };
    for (int64_t k = 0; k < K && !rc; ++k) {
        const int j = (int)(k % D);
        hipStream_t q = ss[(size_t)j];
        pieces.clear();
        // stage j still holds chunk k - D: it (and any chunk before it) must be out first;
        // chunks after it that are already done leave too
        rc = take_done(k - D + 1, k >= D && out_next <= k - D);
        if (!rc) rc = take_done(k, false);
        if (rc) break;
        copy_in(k, j);
        run_pieces();
        const int64_t lo = p.lo(k), c = p.count(k);
        char* ptr[3];
        bool host_ptr = !dma;  // a kernel pointer into host memory: the host cache policy
        char* const buf = dma ? db[(size_t)j] : sd[(size_t)j];  // where the staged regions live
        for (int i = 0; i < 3; ++i) {
            if (p.mode[i] == host::kDirect) {  // AoS (or a one-chunk SoA batch): in place
                ptr[i] = static_cast<char*>(v[i].dev) + (size_t)lo * p.per_problem(i);
                host_ptr = host_ptr || v[i].in_host;
            } else {
                ptr[i] = buf + p.off[i];
            }
        }
        const bool h_direct = dma && h_by_kernel && p.mode[2] == host::kCpu;
        if (h_direct) {  // H into the stage by the kernel itself
            ptr[2] = sd[(size_t)j] + p.off[2];
            host_ptr = true;
        }
        for (int i = 0; i < 2 && !rc; ++i) {
            const size_t bytes = (size_t)c * p.per_problem(i);  // the region, rows c wide in SoA
            if (p.mode[i] == host::kCpu && dma)  // the stage's region to the device buffer
                rc = (int)hipMemcpyAsync(buf + p.off[i], st[(size_t)j]->host + p.off[i], bytes,
                                         hipMemcpyHostToDevice, q);
            else if (p.mode[i] == host::kDma)  // device-memory SoA rows, cut to the chunk
                rc = (int)hipMemcpy2DAsync(dma ? buf + p.off[i] : st[(size_t)j]->host + p.off[i],
                                           (size_t)c * E,
                                           static_cast<const char*>(v[i].dev) + (size_t)lo * E,
                                           (size_t)n * E, (size_t)c * E, (size_t)p.rows[i],
                                           dma ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, q);
        }
        if (!rc && !(probe & 2))
            rc = launch<T>(algo, reinterpret_cast<const T*>(ptr[0]),
                           reinterpret_cast<const T*>(ptr[1]), reinterpret_cast<T*>(ptr[2]), c,
                           layout, flags, q, host_ptr);
        if (!rc && p.mode[2] == host::kCpu && dma && !h_direct)  // H to the stage
            rc = (int)hipMemcpyAsync(st[(size_t)j]->host + p.off[2], buf + p.off[2],
                                     (size_t)c * p.per_problem(2), hipMemcpyDeviceToHost, q);
        if (!rc && p.mode[2] == host::kDma)
            rc = (int)hipMemcpy2DAsync(static_cast<char*>(v[2].dev) + (size_t)lo * E,
                                       (size_t)n * E, dma ? buf + p.off[2] : st[(size_t)j]->host + p.off[2],
                                       (size_t)c * E, (size_t)c * E, (size_t)p.rows[2],
                                       dma ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, q);
        if (!rc && ring) rc = (int)hipEventRecord(ev[(size_t)j], q);
        ++stats.chunks;
    }
    // the chunks still out, in order, each copied as soon as it is done
    if (ring) {
        while (!rc && out_next < K) {
            pieces.clear();
            rc = take_done(out_next + 1, true);
            if (!rc) rc = take_done(K, false);
            if (!rc) run_pieces();
        }
    }
    // every stream drained (also after an error: no stage is reused under a running kernel)
    const int64_t t_drain = now_ns();
    hipError_t e = hipSuccess;
    for (int j = 0; j < (ring ? D : 1); ++j) {
        const hipError_t x = hipStreamSynchronize(ss[(size_t)j]);
        if (e == hipSuccess) e = x;
    }
    stats.wait_ns += now_ns() - t_drain;
    if (!ring && !rc && e == hipSuccess) {  // one chunk: H out now
        pieces.clear();
        copy_out(0, 0);
        run_pieces();
    }
    for (hipEvent_t x : ev)
        if (x) (void)hipEventDestroy(x);
    // a stream that did not drain may still have a kernel reading or writing a stage: neither
    // is handed to another call
    for (int j = 0; j < D; ++j) {
        if (own[(size_t)j] && e == hipSuccess) stream_pool().give_back(dev, ss[(size_t)j]);
        if (db[(size_t)j] && e == hipSuccess) dev_pool().give_back(dev, cap, db[(size_t)j]);
    }
    for (Stage* x : st) {
        if (!x) continue;
        if (e == hipSuccess) stage_pool().give_back(x);
        else ++stage_stats().leaked;
    }
    return rc ? rc : (int)e;
}

template <typename T>
int solve_host(int algo, const T* src, const T* tar, T* H, int64_t n, int layout, int flags,
               void* stream) {
    const int max_algo = sizeof(T) == 8 ? HG_ALGO_GPT : HG_ALGO_GE;
    if (algo < HG_ALGO_ACA || algo > max_algo || n < 0) return kInvalid;
    if (layout != HG_LAYOUT_AOS && layout != HG_LAYOUT_SOA) return kInvalid;
    if (flags & ~(HG_FLAG_NORMALIZE | HG_FLAG_HOST_REGISTER)) return kInvalid;
    const bool register_pages = flags & HG_FLAG_HOST_REGISTER;
    flags &= HG_FLAG_NORMALIZE;
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
    if (!pageable.empty() && !register_pages) {
        lock.unlock();  // no registration: the registry is not involved
        for (View* x : pageable) {
            x->dev = nullptr;  // a page another call registered is still the caller's pageable memory
            x->in_host = true;
        }
        return solve_staged<T>(algo, v, n, layout, flags, s);
    }
    std::vector<uintptr_t> held;
    if (!pageable.empty()) {  // HG_FLAG_HOST_REGISTER: the caller's pages, mapped for the call
        const int rc = reg.acquire(pageable, held, lock);
        if (rc) return rc;
    }
    lock.unlock();  // the solve itself runs unlocked: other calls may share the registrations
    int rc = launch<T>(algo, static_cast<const T*>(v[0].dev), static_cast<const T*>(v[1].dev),
                       static_cast<T*>(v[2].dev), n, layout, flags, s, !all_device);
    const hipError_t e = hipStreamSynchronize(s);  // H is complete when the call returns
    if (!rc) rc = (int)e;
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

// Library-internal (tests and tools/host_probe.py): the staged ring's shape -- bytes of a ring
// stage (>= 64 KiB), stages a call cycles through (1 ... 16), copy threads including the
// caller (1 ... 64); a value <= 0 leaves that setting as it is.  The previous settings go to
// prev[3] when given.
int hg_internal_host_stage_config(int64_t ring_bytes, int depth, int threads, int64_t* prev) {
    StageConfig& c = stage_config();
    if (prev) {
        prev[0] = c.ring_bytes.load();
        prev[1] = c.depth.load();
        prev[2] = copy_pool().threads();
    }
    if ((ring_bytes > 0 && ring_bytes < (64 << 10)) || depth > 16 || threads > 64) return kInvalid;
    if (ring_bytes > 0) c.ring_bytes = ring_bytes / (int64_t)hg::host::kStageAlign *
                                       (int64_t)hg::host::kStageAlign;
    if (depth > 0) c.depth = depth;
    if (threads > 0) copy_pool().set_threads(threads);
    return 0;
}

// Library-internal (tools/ring_probe.py): stage memory fine-grained (1, coherent) or coarse-
// grained (0, non-coherent) from now on; -1 only queries.  Returns the previous setting.
int hg_internal_host_stage_coherent(int coherent) {
    StageConfig& c = stage_config();
    const int prev = c.coherent.load();
    if (coherent == 0 || coherent == 1) c.coherent = coherent;
    return prev;
}

// Library-internal (tools/ring_probe.py, timing only -- results are WRONG while set): 1 skips
// the ring's host copies, 2 its kernels, 0 restores.  Returns the previous setting.
int hg_internal_host_stage_probe(int probe) {
    StageConfig& c = stage_config();
    const int prev = c.probe.load();
    if (probe >= 0 && probe <= 3) c.probe = probe;
    return prev;
}

// Library-internal (tools/ring_probe.py): the ring's chunks in by the copy engines and H written
// into the stage by the kernel (2, the default), both ways by the copy engines (1), or read and
// written in the stage by the kernel (0); -1 queries.
int hg_internal_host_stage_dma(int dma) {
    StageConfig& c = stage_config();
    const int prev = c.dma.load();
    if (dma >= 0 && dma <= 2) c.dma = dma;
    return prev;
}

// {stages allocated, staged calls, chunks solved, stages withheld after a failed stream,
// calls that took ring stages (not the small stage), ns in host copies, ns waiting for the
// GPU, bytes copied by the host} -- out[8].
int hg_internal_host_stage_stats(int64_t* out) {
    if (!out) return kInvalid;
    StageStats& s = stage_stats();
    out[0] = s.made.load();
    out[1] = s.calls.load();
    out[2] = s.chunks.load();
    out[3] = s.leaked.load();
    out[4] = s.ring_calls.load();
    out[5] = s.copy_ns.load();
    out[6] = s.wait_ns.load();
    out[7] = s.copy_bytes.load();
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
