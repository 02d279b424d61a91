// runtime_test.cpp -- the reference GPU harness's flow ("C++ Codes/Runtime Test/GPU_Runtime
// Test/GPU_Runtime Test.cu": read_points, MRG32K3A draws, get_rand_list, cal_ACA / cal_SKS /
// cal_GPT / cal_GE timing loops) as a native C++ caller of the MI355X C ABI.  For each batch
// size N it draws 4*N MRG32K3A words with seed 11 and gathers N random 4-subsets of the
// file's correspondences on the device into the harness's SoA binary64 layout ((8,N) src /
// tar, (9,N) H) exactly as .cu:1443-1451 does (hg_rand_mrg32k3a_u32, hg_get_rand_list_f64),
// then times back-to-back launches the way cal_ACA does (one calibration launch, loops sized
// from it, event-timed mean), checks ACA against the GE baseline, and checks that the fused
// gather + solve (hg_gather_solve_f64) returns the same bits as gather-then-cal_Homo_ACA.
//
//   runtime_test <points.txt> [max_N] [seconds_per_case]
//
// Build (tests/test_gpu_cpp_api.py does):
//   g++ -std=c++17 -O2 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
//       examples/runtime_test.cpp -Lsks-homography_amd/lib -lsks_homography_amd
//       -L/opt/rocm/lib -lamdhip64 -o runtime_test
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <cstring>
#include <string>
#include <vector>

#include "sks_homography.h"

namespace {

#define CHECK(call)                                                                  \
    do {                                                                             \
        const int rc_ = (int)(call);                                                 \
        if (rc_ != 0) {                                                              \
            std::fprintf(stderr, "%s:%d: %s -> error %d\n", __FILE__, __LINE__, #call, \
                         rc_);                                                       \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

// The reference's point-file format (CPU_Runtime Test/utils.cpp:6-21): a count line,
// then "x1 y1 x2 y2" per correspondence.
bool read_points(const std::string& path, std::vector<double>& p1, std::vector<double>& p2) {
    std::ifstream in(path);
    long count = 0;
    if (!(in >> count) || count <= 0) return false;
    p1.resize(2 * count);
    p2.resize(2 * count);
    for (long i = 0; i < count; ++i) {
        float x1, y1, x2, y2;  // the reference parses with %f (binary32)
        if (!(in >> x1 >> y1 >> x2 >> y2)) return false;
        p1[2 * i] = x1; p1[2 * i + 1] = y1;
        p2[2 * i] = x2; p2[2 * i + 1] = y2;
    }
    return true;
}

using SolveF64 = int (*)(const double*, const double*, double*, int64_t, int, int, void*);

// cal_ACA's statistic: one launch to calibrate, loops = budget / that time, mean per launch.
double time_launches(SolveF64 fn, const double* s, const double* t, double* h, int64_t n,
                     double budget_ms) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float ms = 0.f;
    CHECK(hipEventRecord(e0, nullptr));
    CHECK(fn(s, t, h, n, HG_LAYOUT_SOA, 0, nullptr));
    CHECK(hipEventRecord(e1, nullptr));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    int loops = (int)(budget_ms / (ms > 1e-3f ? ms : 1e-3f));
    loops = loops < 10 ? 10 : (loops > 200000 ? 200000 : loops);
    for (int i = 0; i < loops; ++i) CHECK(fn(s, t, h, n, HG_LAYOUT_SOA, 0, nullptr));  // warm
    CHECK(hipEventRecord(e0, nullptr));
    for (int i = 0; i < loops; ++i) CHECK(fn(s, t, h, n, HG_LAYOUT_SOA, 0, nullptr));
    CHECK(hipEventRecord(e1, nullptr));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return (double)ms * 1e3 / loops;  // microseconds
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <points.txt> [max_N] [seconds_per_case]\n", argv[0]);
        return 2;
    }
    const int64_t max_n = argc > 2 ? std::atoll(argv[2]) : 1000000;
    const double budget_ms = (argc > 3 ? std::atof(argv[3]) : 0.2) * 1e3;
    std::vector<double> p1, p2;
    if (!read_points(argv[1], p1, p2)) {
        std::fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    const int64_t npool = (int64_t)p1.size() / 2;
    std::printf("%lld correspondences from %s (%s)\n", (long long)npool, argv[1], hg_version());

    // the correspondence pools on the device as Point2d (.cu:1414-1440)
    double *d_src_in, *d_tar_in;
    CHECK(hipMalloc(&d_src_in, p1.size() * sizeof(double)));
    CHECK(hipMalloc(&d_tar_in, p2.size() * sizeof(double)));
    CHECK(hipMemcpy(d_src_in, p1.data(), p1.size() * sizeof(double), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_tar_in, p2.data(), p2.size() * sizeof(double), hipMemcpyHostToDevice));
    int failures = 0;
    for (int64_t n = 1; n <= max_n; n *= 10) {
        // 4*N MRG32K3A words, seed 11, then get_rand_list (.cu:1443-1451)
        uint32_t* p_d;
        double *ds, *dt, *dh, *dg;
        CHECK(hipMalloc(&p_d, 4 * n * sizeof(uint32_t)));
        CHECK(hipMalloc(&ds, 8 * n * sizeof(double)));
        CHECK(hipMalloc(&dt, 8 * n * sizeof(double)));
        CHECK(hipMalloc(&dh, 9 * n * sizeof(double)));
        CHECK(hipMalloc(&dg, 9 * n * sizeof(double)));
        CHECK(hg_rand_mrg32k3a_u32(p_d, 4 * n, 11ULL, nullptr));
        CHECK(hg_get_rand_list_f64(p_d, (uint32_t)npool, d_src_in, d_tar_in, ds, dt, n, nullptr));
        const struct { const char* name; SolveF64 fn; double* out; } cases[] = {
            {"cal_Homo_ACA", hg_aca_f64, dh}, {"cal_Homo_SKS", hg_sks_f64, dg},
            {"cal_Homo_GPT", hg_gpt_f64, dg}, {"cal_Homo_GE ", hg_ge_f64, dg}};
        for (const auto& c : cases) {
            const double us = time_launches(c.fn, ds, dt, c.out, n, budget_ms);
            std::printf("%s N=%-8lld %10.3f us per launch  %8.2f G H/s\n", c.name, (long long)n,
                        us, n / us * 1e-3);
        }
        // ACA (unnormalised) against GE (H[8] = 1) after normalising: same homography.  The
        // C ABI is asynchronous (hg_rand_mrg32k3a_u32 included, since round 3): wait for the
        // stream before any host-side read
        CHECK(hipStreamSynchronize(nullptr));
        std::vector<double> ha(9 * n), hg(9 * n);
        CHECK(hipMemcpy(ha.data(), dh, 9 * n * sizeof(double), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hg.data(), dg, 9 * n * sizeof(double), hipMemcpyDeviceToHost));
        // the fused gather + cal_Homo_ACA: the same bits as gather-then-solve
        CHECK(hg_gather_solve_f64(HG_ALGO_ACA, d_src_in, d_tar_in, (uint32_t)npool, p_d, dg, n, 0,
                                  nullptr));
        std::vector<double> hf(9 * n);
        CHECK(hipMemcpy(hf.data(), dg, 9 * n * sizeof(double), hipMemcpyDeviceToHost));
        int64_t differ = 0;
        for (int64_t i = 0; i < 9 * n; ++i)
            differ += std::memcmp(&hf[i], &ha[i], sizeof(double)) != 0 &&
                      !(std::isnan(hf[i]) && std::isnan(ha[i]));
        std::printf("  fused gather + cal_Homo_ACA: %lld of %lld words differ from gather-then-solve\n",
                    (long long)differ, (long long)(9 * n));
        if (differ) ++failures;
        // draws + gather + cal_Homo_ACA in one launch (the words never reach memory): the
        // same bits again
        CHECK(hg_rand_gather_solve_f64(HG_ALGO_ACA, d_src_in, d_tar_in, (uint32_t)npool, 11ULL, dg,
                                       n, 0, nullptr));
        CHECK(hipMemcpy(hf.data(), dg, 9 * n * sizeof(double), hipMemcpyDeviceToHost));
        differ = 0;
        for (int64_t i = 0; i < 9 * n; ++i)
            differ += std::memcmp(&hf[i], &ha[i], sizeof(double)) != 0 &&
                      !(std::isnan(hf[i]) && std::isnan(ha[i]));
        std::printf("  draws + gather + cal_Homo_ACA in one launch: %lld of %lld words differ\n",
                    (long long)differ, (long long)(9 * n));
        if (differ) ++failures;
        int64_t agree = 0, finite = 0;
        for (int64_t i = 0; i < n; ++i) {
            const double w = ha[8 * n + i];
            bool ok = std::isfinite(w) && w != 0.0, fin = ok;
            double num = 0.0, den = 0.0;
            for (int k = 0; k < 9 && ok; ++k) {
                const double a = ha[k * n + i] / w, g = hg[k * n + i];
                if (!std::isfinite(a) || !std::isfinite(g)) { ok = false; fin = false; break; }
                num += (a - g) * (a - g);
                den += g * g;
            }
            finite += fin;
            agree += ok && num <= 1e-12 * den;
        }
        std::printf("  ACA vs GE: %lld of %lld finite solutions agree to 1e-6 relative\n",
                    (long long)agree, (long long)finite);
        if (finite > 0 && agree < finite * 99 / 100) ++failures;
        CHECK(hipFree(p_d)); CHECK(hipFree(ds)); CHECK(hipFree(dt)); CHECK(hipFree(dh));
        CHECK(hipFree(dg));
        std::printf("----------------------------------------------------------\n");
    }
    CHECK(hipFree(d_src_in));
    CHECK(hipFree(d_tar_in));
    return failures ? 1 : 0;
}
