// Seeded-sampler code-generation probe (tools/gpu_round.sh sample_flags): the shipped
// launch_sample_seeded compiled on its own, so tools/sample_flags_probe.sh can build it
// under different compiler flags (e.g. with and without the SLP vectoriser, which packs the
// ACA arithmetic into v_pk_* ops plus register moves).  Prints the mean us per launch at
// 16 M hypotheses over a 2540-point pool and a checksum of the H bits (equal checksums:
// identical results).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "hg_ransac.hpp"

int main(int argc, char** argv) {
    // argv[1]: a point file in the reference's format (count, then "x y u v" lines; e.g.
    // tests/golden/orig_pts_wall_restated.txt), or "synthetic" for 2540 random pairs
    const int64_t n = argc > 2 ? std::atoll(argv[2]) : (1 << 24);
    std::vector<float2> ps, pt;
    if (argc > 1 && std::string(argv[1]) != "synthetic") {
        FILE* f = std::fopen(argv[1], "r");
        if (!f) return 4;
        unsigned cnt = 0;
        if (std::fscanf(f, "%u", &cnt) != 1) return 5;
        for (unsigned i = 0; i < cnt; ++i) {
            float a, b, c, d;
            if (std::fscanf(f, "%f %f %f %f", &a, &b, &c, &d) != 4) return 6;
            ps.push_back(make_float2(a, b));
            pt.push_back(make_float2(c, d));
        }
        std::fclose(f);
    } else {
        uint64_t z = 12345;
        for (uint32_t i = 0; i < 2540; ++i) {
            z = z * 6364136223846793005ull + 1442695040888963407ull;
            ps.push_back(make_float2((float)(z >> 40) * 1e-3f, (float)((z >> 16) & 0xffffff) * 1e-3f));
            pt.push_back(make_float2(ps.back().x * 1.01f + 3.f, ps.back().y * 0.99f - 2.f));
        }
    }
    const uint32_t npool = (uint32_t)ps.size();
    float2 *dps, *dpt;
    float* dH;
    if (hipMalloc(&dps, npool * 8) || hipMalloc(&dpt, npool * 8) || hipMalloc(&dH, n * 36)) return 2;
    (void)hipMemcpy(dps, ps.data(), npool * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dpt, pt.data(), npool * 8, hipMemcpyHostToDevice);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    auto run = [&](int) { return hg::launch_sample_seeded(dps, dpt, npool, 11, 0, dH, n, 0, true, s); };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int variant = 0; variant < 3; ++variant) {  // three repeats
        for (int i = 0; i < 20; ++i)
            if (run(variant)) return 3;
        const int reps = 100;
        (void)hipEventRecord(e0, s);
        for (int i = 0; i < reps; ++i) (void)run(variant);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::vector<uint32_t> h(n * 9);
        (void)hipMemcpy(h.data(), dH, n * 36, hipMemcpyDeviceToHost);
        uint64_t sum = 0;
        for (size_t i = 0; i < h.size(); ++i) sum = sum * 1099511628211ull + h[i];
        std::printf("{\"n\": %lld, \"npool\": %u, \"us\": %.2f, \"checksum\": \"%016llx\"}\n",
                    (long long)n, npool, ms * 1e3 / reps, (unsigned long long)sum);
    }
    return 0;
}
