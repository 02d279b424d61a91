// host_ranges_check.cpp -- CPU unit checks of hg_host_ranges.hpp (the page-range merge and
// the registration plan behind hg_solve_host_*), built by tests/test_sanitizers.py with
// -fsanitize=address,undefined.  Prints "host ranges ok" and exits 0 when every check holds.
#include <cstdio>
#include <cstdlib>
#include <random>

#include "hg_host_ranges.hpp"

using hg::host::Range;

static int failures = 0;
#define CHECK(c)                                                       \
    do {                                                               \
        if (!(c)) {                                                    \
            std::fprintf(stderr, "%s:%d: CHECK(%s)\n", __FILE__, __LINE__, #c); \
            ++failures;                                                \
        }                                                              \
    } while (0)

int main() {
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
        std::fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    std::printf("host ranges ok\n");
    return 0;
}
