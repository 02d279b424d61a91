// host_ranges_check.cpp -- CPU unit checks of hg_host_ranges.hpp (the page-range merge and
// the registration plan behind hg_solve_host_* with HG_FLAG_HOST_REGISTER) and of
// hg_host_stage.hpp (the staged ring behind the default pageable path: chunk plan, chunk
// copies, the copy thread pool), built by tests/test_sanitizers.py with
// -fsanitize=address,undefined and again with -fsanitize=thread.  Prints "host ranges ok" and
// exits 0 when every check holds.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>

#include "hg_host_ranges.hpp"
#include "hg_host_stage.hpp"

using hg::host::Range;

static std::atomic<int> failures{0};
#define CHECK(c)                                                       \
    do {                                                               \
        if (!(c)) {                                                    \
            std::fprintf(stderr, "%s:%d: CHECK(%s)\n", __FILE__, __LINE__, #c); \
            ++failures;                                                \
        }                                                              \
    } while (0)

// The staged ring of hg_host.cpp solve_staged, with a CPU "kernel" in place of the GPU one:
// each problem's H row is a function of its own src and tar values, read from wherever the
// plan puts them (the stage, or the caller's buffer in place), written to the stage or in
// place.  The H the ring leaves in the caller's buffer must equal the function applied to the
// whole batch directly, for AoS and SoA, f32- and f64-sized elements, one chunk and many, and
// every mix of staged and in-place buffers; the caller's inputs stay untouched.
template <typename T>
static void kernel_cpu(const T* s, const T* t, T* h, int64_t n, bool soa) {
    for (int64_t p = 0; p < n; ++p) {
        T a[8], b[8];
        for (int k = 0; k < 8; ++k) {
            a[k] = soa ? s[k * n + p] : s[p * 8 + k];
            b[k] = soa ? t[k * n + p] : t[p * 8 + k];
        }
        for (int k = 0; k < 9; ++k) {
            const T v = a[k % 8] * (T)(k + 1) - b[(k * 3) % 8] + (T)k;
            if (soa) h[k * n + p] = v;
            else h[p * 9 + k] = v;
        }
    }
}

template <typename T>
static void ring_case(std::mt19937_64& rng, hg::host::CopyPool& pool, int64_t n, bool soa,
                      const int (&mode)[3], size_t capacity, int depth) {
    using namespace hg::host;
    std::vector<T> s((size_t)n * 8), t((size_t)n * 8), h((size_t)n * 9, (T)-1), want((size_t)n * 9);
    for (auto& x : s) x = (T)(rng() % 1000);
    for (auto& x : t) x = (T)(rng() % 1000);
    const std::vector<T> s0 = s, t0 = t;
    kernel_cpu<T>(s.data(), t.data(), want.data(), n, soa);
    StagePlan p;
    p.n = n;
    p.elem = sizeof(T);
    p.soa = soa;
    for (int i = 0; i < 3; ++i) p.mode[i] = mode[i];
    if (!plan_chunks(p, capacity)) {
        CHECK(false);
        return;
    }
    if (soa && p.chunks > 1) {  // as solve_staged: every buffer through the stage
        for (int i = 0; i < 3; ++i)
            if (p.mode[i] == kDirect) p.mode[i] = kCpu;
        CHECK(plan_chunks(p, capacity));
    }
    CHECK(p.stage_bytes <= capacity);
    CHECK(p.chunk >= 1 && p.chunks == (n + p.chunk - 1) / p.chunk);
    if (p.chunks > 1) CHECK(p.chunk % kChunkQuantum == 0);
    for (int i = 0; i < 3; ++i) CHECK(p.off[i] % kStageAlign == 0);
    const int D = (int)std::min<int64_t>(p.chunks, depth);
    std::vector<std::vector<char>> stage((size_t)D, std::vector<char>(capacity + kStageAlign));
    std::vector<char*> base((size_t)D);
    for (int j = 0; j < D; ++j) {  // 256-B aligned, as hipHostMalloc's are
        char* b = stage[(size_t)j].data();
        base[(size_t)j] = b + (kStageAlign - reinterpret_cast<uintptr_t>(b) % kStageAlign) % kStageAlign;
    }
    const char* user_in[2] = {reinterpret_cast<const char*>(s.data()),
                              reinterpret_cast<const char*>(t.data())};
    char* user_h = reinterpret_cast<char*>(h.data());
    std::vector<Piece> pieces;
    std::vector<int64_t> pending((size_t)D, -1);  // the chunk each stage holds
    auto out_of = [&](int64_t k, int j) {
        if (p.mode[2] == kCpu) chunk_pieces(p, 2, k, nullptr, user_h, base[(size_t)j], false, pieces);
    };
    for (int64_t k = 0; k < p.chunks; ++k) {
        const int j = (int)(k % D);
        pieces.clear();
        if (pending[(size_t)j] >= 0) out_of(pending[(size_t)j], j);
        for (int i = 0; i < 2; ++i)
            if (p.mode[i] == kCpu) chunk_pieces(p, i, k, user_in[i], nullptr, base[(size_t)j], true, pieces);
        pool.run(pieces);
        const int64_t lo = p.lo(k), c = p.count(k);
        char* ptr[3];
        char* whole[3] = {reinterpret_cast<char*>(s.data()), reinterpret_cast<char*>(t.data()), user_h};
        for (int i = 0; i < 3; ++i)
            ptr[i] = p.mode[i] == kDirect ? whole[i] + (size_t)lo * p.per_problem(i)
                                          : base[(size_t)j] + p.off[i];
        kernel_cpu<T>(reinterpret_cast<const T*>(ptr[0]), reinterpret_cast<const T*>(ptr[1]),
                      reinterpret_cast<T*>(ptr[2]), c, soa);
        pending[(size_t)j] = k;
    }
    pieces.clear();
    for (int j = 0; j < D; ++j)
        if (pending[(size_t)j] >= 0) out_of(pending[(size_t)j], j);
    pool.run(pieces);
    CHECK(std::memcmp(h.data(), want.data(), h.size() * sizeof(T)) == 0);
    CHECK(s == s0 && t == t0);
}

static void stage_checks(int iters) {
    using namespace hg::host;
    // the plan: one chunk when the batch fits, exactly; else a quantum multiple
    StagePlan p;
    p.n = 1000;
    p.elem = 4;
    p.mode[0] = p.mode[1] = p.mode[2] = kCpu;
    CHECK(plan_chunks(p, 128 << 10));
    CHECK(p.chunks == 1 && p.chunk == 1000);
    CHECK(p.off[0] == 0 && p.off[1] == align_up(32000) && p.off[2] == 2 * align_up(32000));
    p.n = 10000000;
    CHECK(plan_chunks(p, 8 << 20));
    CHECK(p.chunk % kChunkQuantum == 0 && p.stage_bytes <= (8u << 20));
    CHECK(p.chunk * 100 > (8 << 20) - 100 * kChunkQuantum - 3 * kStageAlign);
    StagePlan q;  // nothing staged, or a stage too small for one quantum: refused
    q.n = 10;
    q.elem = 8;
    CHECK(!plan_chunks(q, 1 << 20));
    q.mode[2] = kCpu;
    q.n = 1 << 20;
    CHECK(!plan_chunks(q, 1024));

    // the ring against the direct computation, single- and multi-threaded pools
    std::mt19937_64 rng(11);
    // never destroyed, as the library's: helper threads never exit
    static hg::host::CopyPool* solo_p = new hg::host::CopyPool();
    static hg::host::CopyPool* team_p = new hg::host::CopyPool();
    hg::host::CopyPool &solo = *solo_p, &team = *team_p;
    solo.set_threads(1);
    team.set_threads(6);
    const int modes[][3] = {{kCpu, kCpu, kCpu}, {kDirect, kCpu, kCpu}, {kCpu, kDirect, kDirect},
                            {kDirect, kDirect, kCpu}, {kCpu, kCpu, kDirect}};
    for (int it = 0; it < iters && !failures; ++it) {
        const int64_t n = 1 + (int64_t)(rng() % 50000);
        const bool soa = rng() % 2;
        const auto& m = modes[rng() % 5];
        const size_t cap = (size_t)(16 << 10) << (rng() % 7);  // 16 KiB ... 1 MiB
        const int depth = 1 + (int)(rng() % 5);
        hg::host::CopyPool& pool = it % 3 ? team : solo;
        if (rng() % 2) ring_case<float>(rng, pool, n, soa, m, cap, depth);
        else ring_case<double>(rng, pool, n, soa, m, cap, depth);
    }
    // several callers sharing one pool at once (the helpers serve every caller's list)
    std::vector<std::thread> th;
    std::vector<int> bad(4, 0);
    for (int c = 0; c < 4; ++c)
        th.emplace_back([&, c] {
            std::mt19937_64 r(100 + c);
            const int before = failures;
            for (int it = 0; it < 10; ++it) {
                const int mm[3] = {kCpu, kCpu, kCpu};
                ring_case<float>(r, team, 200000 + c * 1001, it % 2, mm, 1 << 20, 3);
            }
            bad[(size_t)c] = failures != before;
        });
    for (auto& x : th) x.join();
    for (int b : bad) CHECK(!b);
}

int main(int argc, char** argv) {
    stage_checks(argc > 1 ? std::atoi(argv[1]) : 120);  // ring cases (fewer under -fsanitize=thread)
    const uintptr_t pg = 4096;
    std::vector<Range> out;

    // page rounding, merging of overlapping and adjacent ranges, sorting
    CHECK(hg::host::page_ranges({{5000, 5001}}, pg, out));
    CHECK(out.size() == 1 && out[0].lo == 4096 && out[0].hi == 8192);
    CHECK(hg::host::page_ranges({{9000, 12000}, {100, 200}, {4096, 8192}}, pg, out));
    CHECK(out.size() == 1 && out[0].lo == 0 && out[0].hi == 12288);  // 0-4K, 4K-8K, 8K-12K adjacent
    CHECK(hg::host::page_ranges({{0, 10}, {3 * pg, 3 * pg + 1}}, pg, out));
    CHECK(out.size() == 2 && out[0].hi == pg && out[1].lo == 3 * pg && out[1].hi == 4 * pg);
    // empty and wrapping ranges are rejected, the rest still planned
    CHECK(!hg::host::page_ranges({{10, 10}, {pg, pg + 1}}, pg, out));
    CHECK(out.size() == 1 && out[0].lo == pg);
    CHECK(!hg::host::page_ranges({{UINTPTR_MAX - 10, UINTPTR_MAX}}, pg, out));
    CHECK(out.empty());
    CHECK(!hg::host::page_ranges({{0, 1}}, 3000, out));  // not a power of two

    // the plan: share a containing registration, register new, wait on partial overlap
    const std::vector<Range> have = {{0, 4 * pg}, {8 * pg, 9 * pg}};
    auto p = hg::host::plan({{pg, 2 * pg}, {5 * pg, 6 * pg}, {8 * pg, 10 * pg}}, have);
    CHECK(p.size() == 3 && p[0] == 0 && p[1] == hg::host::kNew && p[2] == hg::host::kConflict);
    CHECK(hg::host::any_conflict(p));
    p = hg::host::plan({{4 * pg, 8 * pg}}, have);  // adjacent on both sides, overlapping none
    CHECK(p.size() == 1 && p[0] == hg::host::kNew);
    p = hg::host::plan({{3 * pg, 9 * pg}}, have);  // spans both
    CHECK(p[0] == hg::host::kConflict);
    CHECK(hg::host::touches({4 * pg - 1, 4 * pg}, have));
    CHECK(!hg::host::touches({4 * pg, 8 * pg}, have));

    // randomized: merged ranges are sorted, disjoint, non-adjacent, page-aligned, and cover
    // every input byte; the plan agrees with a brute-force page check
    std::mt19937_64 rng(7);
    for (int it = 0; it < 20000; ++it) {
        std::vector<Range> bytes;
        const int k = 1 + (int)(rng() % 6);
        for (int i = 0; i < k; ++i) {
            const uintptr_t lo = rng() % (64 * pg);
            bytes.push_back({lo, lo + 1 + rng() % (8 * pg)});
        }
        CHECK(hg::host::page_ranges(bytes, pg, out));
        for (size_t i = 0; i < out.size(); ++i) {
            CHECK(out[i].lo % pg == 0 && out[i].hi % pg == 0 && out[i].lo < out[i].hi);
            if (i) CHECK(out[i - 1].hi < out[i].lo);
        }
        for (const Range& b : bytes) {
            bool covered = false;
            for (const Range& m : out) covered |= m.lo <= b.lo && b.hi <= m.hi;
            CHECK(covered);
        }
        std::vector<Range> regs;
        for (uintptr_t a = 0; a < 80 * pg;) {  // disjoint registrations
            const uintptr_t len = (1 + rng() % 6) * pg;
            if (rng() % 2) regs.push_back({a, a + len});
            a += len + (rng() % 2) * pg;
        }
        const auto plan = hg::host::plan(out, regs);
        for (size_t i = 0; i < out.size(); ++i) {
            int touching = 0;
            long inside = -1;
            for (size_t j = 0; j < regs.size(); ++j) {
                if (hg::host::overlaps(out[i], regs[j])) {
                    ++touching;
                    if (hg::host::contains(regs[j], out[i])) inside = (long)j;
                }
            }
            const long want = touching == 0 ? hg::host::kNew
                              : (touching == 1 && inside >= 0) ? inside
                                                               : hg::host::kConflict;
            CHECK(plan[i] == want);
        }
        if (failures) break;
    }
    if (failures) {
        std::fprintf(stderr, "%d failures\n", failures.load());
        return 1;
    }
    std::printf("host ranges ok\n");
    return 0;
}
