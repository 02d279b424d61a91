// dropin_main.cpp -- a native C++ caller of the reference's solver interface, served by
// the MI355X library.  It makes the calls the reference's CPU harness makes
// ("C++ Codes/Runtime Test/CPU_Runtime Test/main.cpp:87-114": sks::runKernel_ACA /
// _ACA_double / _SKS / _SKS_double on 8-float point lists) and then the batch form a
// throughput caller should use (device buffers, one launch per batch; or host vectors,
// read and written by the kernel over PCIe).
//
// Build (see tests/test_gpu_cpp_api.py):
//   g++ -std=c++17 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ examples/dropin_main.cpp
//       -Lsks-homography_amd/lib -lsks_homography_amd -L/opt/rocm/lib -lamdhip64 -o dropin
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "sks_aca_sks.hpp"

static int check(int rc, const char* what) {
    if (rc != 0) std::fprintf(stderr, "%s failed: %d\n", what, rc);
    return rc;
}

int main() {
    // one 4-point set, the shape main.cpp:45-58 builds (M, N, P, Q)
    float src[8] = {0, 0, 200, 0, 50, 139, 181, 93};
    float tar[8] = {482.0f, 378.5714f, 650.2f, 512.7f, 544.9f, 596.4f, 711.3f, 549.8f};
    double srcd[8], tard[8];
    for (int k = 0; k < 8; ++k) { srcd[k] = src[k]; tard[k] = tar[k]; }
    float h_aca[9], h_sks[9];
    double hd_aca[9], hd_sks[9];
    if (check(sks::runKernel_ACA(src, tar, h_aca), "runKernel_ACA") ||
        check(sks::runKernel_SKS(src, tar, h_sks), "runKernel_SKS") ||
        check(sks::runKernel_ACA_double(srcd, tard, hd_aca), "runKernel_ACA_double") ||
        check(sks::runKernel_SKS_double(srcd, tard, hd_sks), "runKernel_SKS_double"))
        return 1;
    std::printf("ACA  H = [%.7g %.7g %.7g; %.7g %.7g %.7g; %.7g %.7g %.7g]\n", h_aca[0], h_aca[1],
                h_aca[2], h_aca[3], h_aca[4], h_aca[5], h_aca[6], h_aca[7], h_aca[8]);
    std::printf("SKS  H = [%.7g %.7g %.7g; %.7g %.7g %.7g; %.7g %.7g %.7g]\n", h_sks[0], h_sks[1],
                h_sks[2], h_sks[3], h_sks[4], h_sks[5], h_sks[6], h_sks[7], h_sks[8]);
    if (h_aca[8] != 1.0f || hd_aca[8] != 1.0) return 2;
    double diff = 0;
    for (int k = 0; k < 9; ++k) diff = std::fmax(diff, std::fabs((double)h_aca[k] - hd_aca[k]) /
                                                           (std::fabs(hd_aca[k]) + 1e-12));
    if (diff > 1e-3) { std::fprintf(stderr, "f32 vs f64 ACA differ: %g\n", diff); return 3; }

    // batch: the same set replicated n times on the device, one launch
    const int64_t n = 1 << 20;
    std::vector<float> hs(n * 8), ht(n * 8), hH(n * 9);
    for (int64_t i = 0; i < n; ++i) {
        std::memcpy(&hs[i * 8], src, sizeof src);
        std::memcpy(&ht[i * 8], tar, sizeof tar);
    }
    float *ds, *dt, *dH;
    if (hipMalloc(&ds, n * 32) || hipMalloc(&dt, n * 32) || hipMalloc(&dH, n * 36)) return 4;
    (void)hipMemcpy(ds, hs.data(), n * 32, hipMemcpyHostToDevice);
    (void)hipMemcpy(dt, ht.data(), n * 32, hipMemcpyHostToDevice);
    if (check(sks::runKernel_ACA_batch(ds, dt, dH, n), "runKernel_ACA_batch")) return 5;
    (void)hipMemcpy(hH.data(), dH, n * 36, hipMemcpyDeviceToHost);
    for (int64_t i = 0; i < n; ++i)
        if (std::memcmp(&hH[i * 9], h_aca, sizeof h_aca) != 0) {
            std::fprintf(stderr, "batch row %lld differs from the single call\n", (long long)i);
            return 6;
        }
    // the same batch straight from std::vector (pageable host memory, the reference's own
    // data placement): the kernel reads and writes it over PCIe (hg_solve_host_f32)
    std::vector<float> hH2(n * 9, -1.0f);
    if (check(sks::runKernel_ACA_batch(hs.data(), ht.data(), hH2.data(), n),
              "runKernel_ACA_batch(host vectors)"))
        return 11;
    if (std::memcmp(hH2.data(), hH.data(), n * 36) != 0) {
        std::fprintf(stderr, "host-vector batch differs from the device batch\n");
        return 12;
    }
    // many small batches in one grouped call (the C ABI): 40 slices of the device batch,
    // each of its own size, every row equal to the single call's
    {
        const int kGroups = 40;
        const float* gs[kGroups];
        const float* gt[kGroups];
        float* gh[kGroups];
        int64_t gn[kGroups];
        int64_t at = 0;
        for (int i = 0; i < kGroups; ++i) {
            gn[i] = 1 + 37 * i;
            gs[i] = ds + at * 8;
            gt[i] = dt + at * 8;
            gh[i] = dH + at * 9;
            at += gn[i];
        }
        (void)hipMemset(dH, 0, at * 36);
        if (check(hg_solve_grouped_f32(HG_ALGO_ACA, gs, gt, gh, gn, kGroups, HG_LAYOUT_AOS,
                                       HG_FLAG_NORMALIZE, nullptr),
                  "hg_solve_grouped_f32"))
            return 13;
        std::vector<float> gH(at * 9);
        (void)hipMemcpy(gH.data(), dH, at * 36, hipMemcpyDeviceToHost);
        for (int64_t i = 0; i < at; ++i)
            if (std::memcmp(&gH[i * 9], h_aca, sizeof h_aca) != 0) {
                std::fprintf(stderr, "grouped row %lld differs from the single call\n", (long long)i);
                return 14;
            }
    }
    // device pointers through the single-problem signature too
    if (check(sks::runKernel_SKS(ds, dt, dH), "runKernel_SKS(device ptrs)")) return 7;
    float row[9];
    (void)hipMemcpy(row, dH, 36, hipMemcpyDeviceToHost);
    if (std::memcmp(row, h_sks, sizeof row) != 0) return 8;
    // the reference's functions are pure and re-entrant: 8 host threads
    // calling the single-problem API at once must each get their own problem's bits
    const int kThreads = 8, kCalls = 200;
    std::vector<float> ts(kThreads * 8), tt(kThreads * 8), want(kThreads * 9);
    for (int t = 0; t < kThreads; ++t)
        for (int k = 0; k < 8; ++k) {
            ts[t * 8 + k] = src[k] + 3.25f * t * (k % 3);
            tt[t * 8 + k] = tar[k] - 1.5f * t * (k % 2);
        }
    (void)hipMemcpy(ds, ts.data(), kThreads * 32, hipMemcpyHostToDevice);
    (void)hipMemcpy(dt, tt.data(), kThreads * 32, hipMemcpyHostToDevice);
    if (check(sks::runKernel_SKS_batch(ds, dt, dH, kThreads), "runKernel_SKS_batch")) return 9;
    (void)hipMemcpy(want.data(), dH, kThreads * 36, hipMemcpyDeviceToHost);
    std::atomic<int> mismatches{0};
    std::vector<std::thread> pool;
    for (int t = 0; t < kThreads; ++t)
        pool.emplace_back([&, t] {
            float h[9];
            for (int c = 0; c < kCalls; ++c) {
                if (sks::runKernel_SKS(&ts[t * 8], &tt[t * 8], h) != 0 ||
                    std::memcmp(h, &want[t * 9], sizeof h) != 0)
                    mismatches.fetch_add(1);
            }
        });
    for (auto& th : pool) th.join();
    if (mismatches.load() != 0) {
        std::fprintf(stderr, "%d threaded calls differ from the batch result\n", mismatches.load());
        return 10;
    }
    std::printf("%d threads x %d calls: every result bit-identical to the batch\n", kThreads, kCalls);
    (void)hipFree(ds); (void)hipFree(dt); (void)hipFree(dH);
    std::printf("dropin ok: %lld batch rows bit-identical to the single call\n", (long long)n);
    return 0;
}
