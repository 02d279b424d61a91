// multi_gpu.cpp -- one native process driving every visible GPU through the multi-GPU C ABI
// (include/sks_homography_multi.h; SURVEY.md 8(e), BASELINE configs[4]): the batch splits into
// contiguous rank-major blocks (hg_shard_range, shard.shard_range's split), each device
// generates and solves its own block on its own stream with no data-path collective
// (hg_solve_multi), and the H blocks are gathered on device 0 (hg_gather_multi: RCCL
// ncclSend / ncclRecv pairs over xGMI) only to check them.
//
//   multi_gpu [problems_per_device=10000000] [iters=50] [shards_per_device=1]
//
// Prints, for k = 1, 2, 4, ... up to the device count, the compute-resident throughput of k
// devices each solving its block (weak scaling, ACA AoS f32 normalised -- the bench
// headline's kernel), then the gather's time, then how many 32-bit words of the gathered H
// differ from one whole-batch solve on device 0 (0 expected: problems are independent).
// shards_per_device > 1 splits each device's block further over streams of that device;
// those blocks are then gathered by device-to-device copies (RCCL takes one rank per device).
//
// Build (tests/test_gpu_cpp_api.py does):
//   g++ -std=c++17 -O2 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
//       examples/multi_gpu.cpp -Lsks-homography_amd/lib -lsks_homography_multi
//       -lsks_homography_amd -L/opt/rocm/lib -lamdhip64 -o multi_gpu
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "sks_homography.h"
#include "sks_homography_multi.h"

namespace {

constexpr uint64_t kSeed = 11;  // bench.py's input stream

void check(int rc, const char* what) {
    if (rc == 0) return;
    if (HG_IS_RCCL_ERR(rc))
        std::fprintf(stderr, "%s failed: RCCL result %d\n", what, HG_RCCL_RESULT(rc));
    else
        std::fprintf(stderr, "%s failed: %d (%s)\n", what, rc,
                     hipGetErrorString(static_cast<hipError_t>(rc)));
    std::exit(1);
}

struct Shard {
    int device = 0;
    int64_t lo = 0, n = 0;
    float *src = nullptr, *tar = nullptr, *H = nullptr;
    hipStream_t stream = nullptr;
};

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

}  // namespace

int main(int argc, char** argv) {
    const int64_t per_dev = argc > 1 ? std::atoll(argv[1]) : 10'000'000;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 50;
    const int spd = argc > 3 ? std::atoi(argv[3]) : 1;
    int ndev = 0;
    check(static_cast<int>(hipGetDeviceCount(&ndev)), "hipGetDeviceCount");
    if (ndev < 1 || per_dev < 1 || iters < 1 || spd < 1) {
        std::fprintf(stderr, "usage: multi_gpu [problems_per_device] [iters] [shards_per_device]\n");
        return 2;
    }
    const int nshard = ndev * spd;
    const int64_t N = per_dev * ndev;
    std::printf("devices=%d shards=%d problems=%lld (%lld per device)\n", ndev, nshard,
                static_cast<long long>(N), static_cast<long long>(per_dev));

    // each device generates its own block of the one global batch: src = stream values
    // [0, 8N), tar = [8N, 16N); shard r holds rows [lo, lo + n) (bench.rank_block_inputs)
    std::vector<Shard> sh(nshard);
    for (int r = 0; r < nshard; ++r) {
        Shard& s = sh[r];
        int64_t hi = 0;
        check(hg_shard_range(N, nshard, r, &s.lo, &hi), "hg_shard_range");
        s.n = hi - s.lo;
        s.device = r / spd;
        check(static_cast<int>(hipSetDevice(s.device)), "hipSetDevice");
        check(static_cast<int>(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)),
              "hipStreamCreate");
        check(static_cast<int>(hipMalloc(&s.src, s.n * 32 + 16)), "hipMalloc src");
        check(static_cast<int>(hipMalloc(&s.tar, s.n * 32 + 16)), "hipMalloc tar");
        check(static_cast<int>(hipMalloc(&s.H, s.n * 36 + 16)), "hipMalloc H");
        check(hg_fill_uniform_f32(s.src, s.n * 8, kSeed, s.lo * 8, 0.f, 1024.f, s.stream),
              "fill src");
        check(hg_fill_uniform_f32(s.tar, s.n * 8, kSeed, (N + s.lo) * 8, 0.f, 1024.f, s.stream),
              "fill tar");
    }
    std::vector<hg_device_batch> b(nshard);
    for (int r = 0; r < nshard; ++r)
        b[r] = {sh[r].device, sh[r].src, sh[r].tar, sh[r].H, sh[r].n, sh[r].stream};
    check(hg_sync_multi(b.data(), nshard), "hg_sync_multi");

    // compute-resident weak scaling: the first k devices' shards, iters batches each
    std::vector<int> counts;
    for (int k = 1; k < ndev; k *= 2) counts.push_back(k);
    counts.push_back(ndev);
    for (const int k : counts) {
        const int ks = k * spd;
        for (int w = 0; w < 3; ++w)
            check(hg_solve_multi(HG_ALGO_ACA, HG_DTYPE_F32, b.data(), ks, HG_LAYOUT_AOS,
                                 HG_FLAG_NORMALIZE), "hg_solve_multi");
        check(hg_sync_multi(b.data(), ks), "hg_sync_multi");
        const double t0 = now_s();
        for (int i = 0; i < iters; ++i)
            check(hg_solve_multi(HG_ALGO_ACA, HG_DTYPE_F32, b.data(), ks, HG_LAYOUT_AOS,
                                 HG_FLAG_NORMALIZE), "hg_solve_multi");
        check(hg_sync_multi(b.data(), ks), "hg_sync_multi");
        const double dt = now_s() - t0;
        const double problems = static_cast<double>(per_dev) * k * iters;
        std::printf("solve_multi devices=%d: %.2f us per batch, %.1f M homographies/s "
                    "(%.2f TB/s at 100 B each)\n", k, dt / iters * 1e6, problems / dt / 1e6,
                    problems * 100.0 / dt / 1e12);
    }

    // the check: every block gathered on device 0 against one whole-batch solve there
    check(static_cast<int>(hipSetDevice(0)), "hipSetDevice");
    float *ws = nullptr, *wt = nullptr, *wH = nullptr, *all = nullptr;
    check(static_cast<int>(hipMalloc(&ws, N * 32)), "hipMalloc");
    check(static_cast<int>(hipMalloc(&wt, N * 32)), "hipMalloc");
    check(static_cast<int>(hipMalloc(&wH, N * 36)), "hipMalloc");
    check(static_cast<int>(hipMalloc(&all, N * 36)), "hipMalloc");
    check(static_cast<int>(hipMemset(all, 0xff, N * 36)), "hipMemset");  // NaN everywhere
    check(hg_fill_uniform_f32(ws, N * 8, kSeed, 0, 0.f, 1024.f, nullptr), "fill");
    check(hg_fill_uniform_f32(wt, N * 8, kSeed, N * 8, 0.f, 1024.f, nullptr), "fill");
    check(hg_aca_f32(ws, wt, wH, N, HG_LAYOUT_AOS, HG_FLAG_NORMALIZE, nullptr), "hg_aca_f32");
    check(static_cast<int>(hipDeviceSynchronize()), "hipDeviceSynchronize");
    check(hg_solve_multi(HG_ALGO_ACA, HG_DTYPE_F32, b.data(), nshard, HG_LAYOUT_AOS,
                         HG_FLAG_NORMALIZE), "hg_solve_multi");
    check(hg_sync_multi(b.data(), nshard), "hg_sync_multi");
    const double g0 = now_s();
    if (spd == 1) {
        std::vector<int> devs(ndev);
        for (int d = 0; d < ndev; ++d) devs[d] = d;
        std::vector<void*> comms(ndev, nullptr);
        check(hg_comm_init_all(ndev, devs.data(), comms.data()), "hg_comm_init_all");
        const double c0 = now_s();
        check(hg_gather_multi(b.data(), ndev, 0, HG_DTYPE_F32, all, comms.data()),
              "hg_gather_multi");
        check(hg_sync_multi(b.data(), nshard), "hg_sync_multi");
        const double c1 = now_s();
        std::printf("gather on device 0 (RCCL, %d ranks): %.3f ms, %.1f GB/s into device 0\n",
                    ndev, (c1 - c0) * 1e3,
                    static_cast<double>(N - sh[0].n) * 36 / (c1 - c0) / 1e9);
        check(hg_comm_destroy(ndev, comms.data()), "hg_comm_destroy");
    } else {
        for (const Shard& s : sh)
            check(static_cast<int>(hipMemcpyPeer(all + s.lo * 9, 0, s.H, s.device, s.n * 36)),
                  "hipMemcpyPeer");
        std::printf("gather on device 0 (copies): %.3f ms\n", (now_s() - g0) * 1e3);
    }
    std::vector<uint32_t> a(N * 9), w(N * 9);
    check(static_cast<int>(hipMemcpy(a.data(), all, N * 36, hipMemcpyDeviceToHost)), "copy");
    check(static_cast<int>(hipMemcpy(w.data(), wH, N * 36, hipMemcpyDeviceToHost)), "copy");
    int64_t differ = 0;
    for (int64_t i = 0; i < N * 9; ++i) differ += a[i] != w[i];
    std::printf("bits: %lld of %lld words differ from one whole-batch solve\n",
                static_cast<long long>(differ), static_cast<long long>(N * 9));
    for (Shard& s : sh) {
        (void)hipSetDevice(s.device);
        (void)hipFree(s.src);
        (void)hipFree(s.tar);
        (void)hipFree(s.H);
        (void)hipStreamDestroy(s.stream);
    }
    (void)hipSetDevice(0);
    (void)hipFree(ws);
    (void)hipFree(wt);
    (void)hipFree(wH);
    (void)hipFree(all);
    return differ == 0 ? 0 : 1;
}
