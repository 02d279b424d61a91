// hg_host_ranges.hpp -- page-range bookkeeping for hg_solve_host_* (hg_host.cpp), kept free
// of HIP so it builds and runs on the CPU under -fsanitize=address,undefined
// (tests/host_ranges_check.cpp, tests/test_sanitizers.py).
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

namespace hg {
namespace host {

struct Range {
    uintptr_t lo, hi;  // [lo, hi)
};

inline bool overlaps(const Range& a, const Range& b) { return a.lo < b.hi && b.lo < a.hi; }
inline bool contains(const Range& outer, const Range& inner) {
    return outer.lo <= inner.lo && inner.hi <= outer.hi;
}

// The whole pages under each byte range [p, p + bytes), sorted, with overlapping or adjacent
// ranges merged (buffers cut from one allocation share a registration).  Empty ranges and
// ranges that would wrap the address space are dropped from the result and reported by a
// false return.
inline bool page_ranges(const std::vector<Range>& bytes, uintptr_t page, std::vector<Range>& out) {
    out.clear();
    if (page == 0 || (page & (page - 1)) != 0) return false;
    bool ok = true;
    std::vector<Range> r;
    r.reserve(bytes.size());
    for (const Range& b : bytes) {
        if (b.hi <= b.lo || b.hi > UINTPTR_MAX - (page - 1)) {
            ok = false;
            continue;
        }
        r.push_back({b.lo & ~(page - 1), (b.hi + page - 1) & ~(page - 1)});
    }
    std::sort(r.begin(), r.end(), [](const Range& a, const Range& b) { return a.lo < b.lo; });
    for (const Range& x : r) {
        if (!out.empty() && x.lo <= out.back().hi)
            out.back().hi = std::max(out.back().hi, x.hi);
        else
            out.push_back(x);
    }
    return ok;
}

// How each needed page range relates to the registrations the library already holds:
// the index of the registration that contains it (share it), kNew (it touches none:
// register it), or kConflict (it overlaps one or more without being inside one: it can
// be registered only once those are released).
constexpr long kNew = -1;
constexpr long kConflict = -2;

inline std::vector<long> plan(const std::vector<Range>& need, const std::vector<Range>& have) {
    std::vector<long> out(need.size(), kNew);
    for (size_t i = 0; i < need.size(); ++i) {
        for (size_t j = 0; j < have.size(); ++j) {
            if (!overlaps(need[i], have[j])) continue;
            if (out[i] == kNew && contains(have[j], need[i]))
                out[i] = (long)j;
            else
                out[i] = kConflict;
        }
    }
    return out;
}

inline bool any_conflict(const std::vector<long>& p) {
    return std::any_of(p.begin(), p.end(), [](long x) { return x == kConflict; });
}

// True if byte range [lo, hi) touches any of `have`.
inline bool touches(const Range& r, const std::vector<Range>& have) {
    return std::any_of(have.begin(), have.end(), [&](const Range& h) { return overlaps(r, h); });
}

}  // namespace host
}  // namespace hg
