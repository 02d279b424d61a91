// dropin_main.cpp -- a native C++ caller of the reference's solver interface, served by
// the MI355X library.  It makes the calls the reference's CPU harness makes
// ("C++ Codes/Runtime Test/CPU_Runtime Test/main.cpp:87-114": sks::runKernel_ACA /
// _ACA_double / _SKS / _SKS_double on 8-float point lists) and then the batch form a
// throughput caller should use (device buffers, one launch per batch; or host vectors,
// read and written by the kernel over PCIe).
//
// With a golden file (argv[1], written by tests/test_gpu_cpp_api.py from the reference's own
// outputs in tests/golden/cpp_uniform.npz and cpp_edge.npz), every problem in it goes
// through all four single-problem functions on host pointers and through the four batch
// overloads (std::vector and device buffers), and each H must equal the reference's bits
// (any NaN equal to any NaN: x86 and CDNA payloads differ).
//
// Build (see tests/test_gpu_cpp_api.py):
//   g++ -std=c++17 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ examples/dropin_main.cpp
//       -Lsks-homography_amd/lib -lsks_homography_amd -L/opt/rocm/lib -lamdhip64 -o dropin
//   ./dropin [golden.bin]
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

// Bit equality with every NaN equal to every NaN.
template <typename T>
static bool same_bits(const T* a, const T* b, int64_t count) {
    for (int64_t i = 0; i < count; ++i) {
        if (std::isnan(a[i]) && std::isnan(b[i])) continue;
        if (std::memcmp(&a[i], &b[i], sizeof(T)) != 0) return false;
    }
    return true;
}

// Golden file: int64 n, then src/tar/H_aca/H_sks in f32 ((n,8),(n,8),(n,9),(n,9)), then the
// same four in f64.  Returns 0 when every call reproduces the reference's bits.
template <typename T>
struct Golden {
    std::vector<T> src, tar, aca, sks;
    bool read(std::FILE* f, int64_t n) {
        src.resize(n * 8); tar.resize(n * 8); aca.resize(n * 9); sks.resize(n * 9);
        return std::fread(src.data(), sizeof(T), n * 8, f) == (size_t)(n * 8) &&
               std::fread(tar.data(), sizeof(T), n * 8, f) == (size_t)(n * 8) &&
               std::fread(aca.data(), sizeof(T), n * 9, f) == (size_t)(n * 9) &&
               std::fread(sks.data(), sizeof(T), n * 9, f) == (size_t)(n * 9);
    }
};

template <typename T>
static int check_golden(const Golden<T>& g, int64_t n, int (*aca)(T*, T*, T*),
                        int (*sks_)(T*, T*, T*),
                        int (*aca_b)(const T*, const T*, T*, int64_t, void*),
                        int (*sks_b)(const T*, const T*, T*, int64_t, void*), const char* tag) {
    std::vector<T> s = g.src, t = g.tar;  // the reference's pointers are non-const
    for (int algo = 0; algo < 2; ++algo) {
        const std::vector<T>& want = algo ? g.sks : g.aca;
        const char* name = algo ? "SKS" : "ACA";
        // single problems, host pointers (the reference's own call pattern)
        for (int64_t i = 0; i < n; ++i) {
            T h[9];
            const int rc = (algo ? sks_ : aca)(&s[i * 8], &t[i * 8], h);
            if (rc) return check(rc, "single call");
            if (!same_bits(h, &want[i * 9], 9)) {
                std::fprintf(stderr, "%s %s problem %lld differs from the reference\n", name, tag,
                             (long long)i);
                return 20;
            }
        }
        // batch from std::vector (pageable host memory)
        std::vector<T> hb(n * 9, T(-1));
        if (int rc = (algo ? sks_b : aca_b)(g.src.data(), g.tar.data(), hb.data(), n, nullptr))
            return check(rc, "batch (host vectors)");
        if (!same_bits(hb.data(), want.data(), n * 9)) {
            std::fprintf(stderr, "%s %s host-vector batch differs from the reference\n", name, tag);
            return 21;
        }
        // batch from device buffers
        T *ds, *dt, *dH;
        if (hipMalloc(&ds, n * 8 * sizeof(T)) || hipMalloc(&dt, n * 8 * sizeof(T)) ||
            hipMalloc(&dH, n * 9 * sizeof(T)))
            return 22;
        (void)hipMemcpy(ds, g.src.data(), n * 8 * sizeof(T), hipMemcpyHostToDevice);
        (void)hipMemcpy(dt, g.tar.data(), n * 8 * sizeof(T), hipMemcpyHostToDevice);
        if (int rc = (algo ? sks_b : aca_b)(ds, dt, dH, n, nullptr)) return check(rc, "batch (device)");
        std::vector<T> db(n * 9);
        (void)hipMemcpy(db.data(), dH, n * 9 * sizeof(T), hipMemcpyDeviceToHost);
        (void)hipFree(ds); (void)hipFree(dt); (void)hipFree(dH);
        if (!same_bits(db.data(), want.data(), n * 9)) {
            std::fprintf(stderr, "%s %s device batch differs from the reference\n", name, tag);
            return 23;
        }
    }
    return 0;
}

static int golden(const char* path) {
    std::FILE* f = std::fopen(path, "rb");
    if (!f) { std::fprintf(stderr, "cannot open %s\n", path); return 30; }
    int64_t n = 0;
    Golden<float> g32;
    Golden<double> g64;
    const bool ok = std::fread(&n, sizeof n, 1, f) == 1 && n > 0 && n < (1 << 20) &&
                    g32.read(f, n) && g64.read(f, n);
    std::fclose(f);
    if (!ok) { std::fprintf(stderr, "short golden file %s\n", path); return 31; }
    if (int rc = check_golden<float>(g32, n, sks::runKernel_ACA, sks::runKernel_SKS,
                                     sks::runKernel_ACA_batch, sks::runKernel_SKS_batch, "f32"))
        return rc;
    if (int rc = check_golden<double>(g64, n, sks::runKernel_ACA_double, sks::runKernel_SKS_double,
                                      sks::runKernel_ACA_double_batch,
                                      sks::runKernel_SKS_double_batch, "f64"))
        return rc;
    std::printf("golden ok: %lld problems x 4 functions, single calls and batches (host and "
                "device), bit-identical to the reference\n", (long long)n);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1) {
        if (int rc = golden(argv[1])) return rc;
    }
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
    if (h_aca[8] != 1.0f || hd_aca[8] != 1.0 || h_sks[8] != 1.0f || hd_sks[8] != 1.0) return 2;

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
