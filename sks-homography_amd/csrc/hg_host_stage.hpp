// hg_host_stage.hpp -- the staged ring behind hg_solve_host_* for pageable buffers
// (hg_host.cpp), kept free of HIP so it builds and runs on the CPU under
// -fsanitize=address,undefined and -fsanitize=thread (tests/host_ranges_check.cpp,
// tests/test_sanitizers.py).
//
// A pageable batch is solved in chunks of C problems.  Each chunk's slice of every staged
// buffer is copied into a library-owned pinned stage (one region per buffer, 256-B aligned;
// SoA slices as C-wide rows, so the kernel sees an SoA batch of C problems), the kernel reads
// the stage and writes H into it, and H's slice is copied back out.  StagePlan fixes C and the
// regions; in_pieces / out_pieces list the byte copies of one chunk; CopyPool runs a list of
// copies on the calling thread plus helper threads.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <deque>
#include <emmintrin.h>
#include <mutex>
#include <thread>
#include <vector>

namespace hg {
namespace host {

constexpr size_t kStageAlign = 256;
constexpr int64_t kChunkQuantum = 64;  // C is a multiple of this: SoA rows stay 256-B aligned

inline size_t align_up(size_t b) { return (b + kStageAlign - 1) / kStageAlign * kStageAlign; }

// How a buffer (src, tar, H) reaches the kernel for a chunk.
enum StageMode : int {
    kDirect = 0,  // device-visible already (pinned host, device, managed): used in place
    kCpu = 1,     // copied into / out of the stage by host threads (pageable, or pinned host
                  // memory whose SoA rows must be cut into chunk rows)
    kDma = 2,     // device memory whose SoA rows must be cut: hipMemcpy2DAsync (hg_host.cpp)
};

struct StagePlan {
    int64_t n = 0;     // problems in the batch
    int64_t chunk = 0; // C: problems per chunk (the last chunk may be shorter)
    int64_t chunks = 0;
    size_t elem = 0;   // sizeof(T)
    bool soa = false;
    int rows[3] = {8, 8, 9};  // values per problem of src, tar, H
    int mode[3] = {kDirect, kDirect, kDirect};
    size_t off[3] = {0, 0, 0};  // region of each staged buffer in a stage
    size_t stage_bytes = 0;     // bytes of a stage the plan uses

    size_t per_problem(int i) const { return (size_t)rows[i] * elem; }
    bool staged(int i) const { return mode[i] != kDirect; }
    int64_t lo(int64_t k) const { return k * chunk; }
    int64_t count(int64_t k) const { return std::min(chunk, n - k * chunk); }
};

// Fills chunk, chunks, off and stage_bytes for a stage of `capacity` bytes; false when not even
// one chunk quantum fits or nothing is staged.  The batch fits in one chunk when n does (then
// the chunk is exactly n, whatever the quantum).
inline bool plan_chunks(StagePlan& p, size_t capacity) {
    size_t per = 0;
    int staged = 0;
    for (int i = 0; i < 3; ++i)
        if (p.staged(i)) {
            per += p.per_problem(i);
            ++staged;
        }
    if (!staged || p.n <= 0) return false;
    size_t whole = 0;  // the batch in one chunk, each region aligned
    for (int i = 0; i < 3; ++i)
        if (p.staged(i)) whole += align_up((size_t)p.n * p.per_problem(i));
    int64_t c = p.n;
    if (whole > capacity) {
        if (capacity <= (size_t)staged * kStageAlign) return false;
        c = (int64_t)((capacity - (size_t)staged * kStageAlign) / per);  // alignment slack
        c = c / kChunkQuantum * kChunkQuantum;
        if (c == 0) return false;
    }
    p.chunk = c;
    p.chunks = (p.n + c - 1) / c;
    size_t o = 0;
    for (int i = 0; i < 3; ++i) {
        p.off[i] = o;
        if (p.staged(i)) o += align_up((size_t)c * p.per_problem(i));
    }
    p.stage_bytes = o;
    return o <= capacity;
}

struct Piece {
    char* dst;
    const char* src;
    size_t bytes;
};

constexpr size_t kPieceBytes = 512 << 10;  // helpers take copies in pieces of at most this

inline void add_piece(std::vector<Piece>& out, char* dst, const char* src, size_t bytes) {
    while (bytes > 0) {
        const size_t b = std::min(bytes, kPieceBytes);
        out.push_back({dst, src, b});
        dst += b;
        src += b;
        bytes -= b;
    }
}

// The copies of chunk k's slice of buffer i between the caller's memory `user` (the whole
// batch) and `stage` (the stage's host address): into the stage when `in`, out of it else.
inline void chunk_pieces(const StagePlan& p, int i, int64_t k, const char* user_in, char* user_out,
                         char* stage, bool in, std::vector<Piece>& out) {
    const int64_t lo = p.lo(k), c = p.count(k);
    if (c <= 0) return;
    char* st = stage + p.off[i];
    if (!p.soa) {
        const size_t pp = p.per_problem(i), at = (size_t)lo * pp;
        if (in) add_piece(out, st, user_in + at, (size_t)c * pp);
        else add_piece(out, user_out + at, st, (size_t)c * pp);
        return;
    }
    const size_t row = (size_t)c * p.elem;  // one SoA row of the chunk
    for (int r = 0; r < p.rows[i]; ++r) {
        const size_t at = ((size_t)r * (size_t)p.n + (size_t)lo) * p.elem;
        if (in) add_piece(out, st + (size_t)r * row, user_in + at, row);
        else add_piece(out, user_out + at, st + (size_t)r * row, row);
    }
}

// One piece's copy with streaming (non-temporal) stores: the destination -- a stage the GPU
// reads next over PCIe, or the caller's H, read by nobody before the call returns -- is not
// read first (no read-for-ownership) and does not evict the copy threads' caches.  Measured on
// the MI355X box's EPYC host (tools/ring_probe.py, profiles/r06): the copies share the host's
// memory with the GPU's PCIe reads of the stages, and the read-for-ownership traffic of
// ordinary stores was what the ring ran short of.  Short or unaligned ends go through memcpy.
inline void copy_streaming(char* dst, const char* src, size_t bytes) {
    const size_t head = (64 - (reinterpret_cast<uintptr_t>(dst) & 63)) & 63;
    if (bytes < head + 256) {
        std::memcpy(dst, src, bytes);
        return;
    }
    std::memcpy(dst, src, head);
    dst += head;
    src += head;
    bytes -= head;
    const size_t body = bytes & ~(size_t)63;
    for (size_t i = 0; i < body; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
    std::memcpy(dst + body, src + body, bytes - body);
    _mm_sfence();  // the streamed lines are globally visible before the caller goes on
}

// Runs lists of copies on the calling thread and up to threads-1 helper threads.  Helpers
// are started on first need and never exit (no thread, and no library state, is torn down at
// process exit: the pool itself is never destroyed -- hg_host.cpp).  Each caller works on its
// own list as well, so a call always progresses, whatever other calls hold the helpers.
class CopyPool {
   public:
    static constexpr size_t kParallelMin = 1 << 20;  // smaller lists: the caller alone

    void set_threads(int t) {
        std::lock_guard<std::mutex> lock(mu_);
        want_ = std::max(1, std::min(t, 64));
    }
    int threads() {
        std::lock_guard<std::mutex> lock(mu_);
        return want_;
    }

    void run(const std::vector<Piece>& pieces) {
        size_t total = 0;
        for (const Piece& x : pieces) total += x.bytes;
        Job job;
        job.p = pieces.data();
        job.n = pieces.size();
        bool shared = false;
        if (total >= kParallelMin && pieces.size() > 1) {
            std::lock_guard<std::mutex> lock(mu_);
            const int helpers = std::min<int>(want_ - 1, (int)pieces.size() - 1);
            while (started_ < helpers) {
                std::thread([this] { helper(); }).detach();
                ++started_;
            }
            if (helpers > 0) {
                jobs_.push_back(&job);
                shared = true;
            }
        }
        if (shared) work_.notify_all();
        work_on(job);
        if (!shared) return;
        std::unique_lock<std::mutex> lock(mu_);
        auto it = std::find(jobs_.begin(), jobs_.end(), &job);
        if (it != jobs_.end()) jobs_.erase(it);  // no helper picks it up from now on
        idle_.wait(lock, [&] { return job.helpers == 0; });
    }

   private:
    struct Job {
        const Piece* p = nullptr;
        size_t n = 0;
        std::atomic<size_t> next{0};
        int helpers = 0;  // helpers working on it (under mu_)
    };

    static void work_on(Job& job) {
        for (size_t i = job.next.fetch_add(1); i < job.n; i = job.next.fetch_add(1))
            copy_streaming(job.p[i].dst, job.p[i].src, job.p[i].bytes);
    }

    void helper() {
        std::unique_lock<std::mutex> lock(mu_);
        for (;;) {
            work_.wait(lock, [&] { return !jobs_.empty(); });
            Job* job = jobs_.front();
            if (job->next.load() >= job->n) {  // every piece taken: retire it from the queue
                jobs_.pop_front();
                continue;
            }
            ++job->helpers;
            lock.unlock();
            work_on(*job);
            lock.lock();
            if (--job->helpers == 0) idle_.notify_all();
        }
    }

    std::mutex mu_;
    std::condition_variable work_, idle_;
    std::deque<Job*> jobs_;
    int started_ = 0;
    int want_ = 8;
};

}  // namespace host
}  // namespace hg
