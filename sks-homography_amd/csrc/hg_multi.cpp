// hg_multi.cpp -- the multi-GPU C ABI (include/sks_homography_multi.h): one host thread
// driving every GPU of a node, each solving its contiguous block of the batch with no
// data-path collective, and the optional gather of the H blocks on one GPU
// through RCCL point-to-point (ncclGroupStart, ncclSend / ncclRecv, rccl.h:700-745) -- the
// native caller's form of shard.py's gather_blocks.  Host C++ over the product library.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <vector>

#include "sks_homography.h"
#include "sks_homography_multi.h"

namespace {

constexpr int kErrInvalid = (int)hipErrorInvalidValue;

// an RCCL failure, apart from the hipError_t codes (sks_homography_multi.h)
int rccl_err(ncclResult_t r) { return r == ncclSuccess ? 0 : HG_ERR_RCCL_BASE + (int)r; }

// Sets `device` current for the scope; the caller's device comes back on exit.
class DeviceScope {
   public:
    explicit DeviceScope(int device) {
        ok_ = hipGetDevice(&prev_) == hipSuccess;
        rc_ = (int)hipSetDevice(device);
    }
    ~DeviceScope() {
        if (ok_) (void)hipSetDevice(prev_);
    }
    int rc() const { return rc_; }

   private:
    int prev_ = 0;
    bool ok_ = false;
    int rc_ = 0;
};

using SolveF32 = int (*)(const float*, const float*, float*, int64_t, int, int, void*);
using SolveF64 = int (*)(const double*, const double*, double*, int64_t, int, int, void*);
constexpr SolveF32 kF32[4] = {hg_aca_f32, hg_sks_f32, hg_ge_f32, nullptr};
constexpr SolveF64 kF64[4] = {hg_aca_f64, hg_sks_f64, hg_ge_f64, hg_gpt_f64};

bool shards_ok(const hg_device_batch* shards, int ndev) {
    if (!shards || ndev < 1) return false;
    for (int i = 0; i < ndev; ++i)
        if (shards[i].n < 0) return false;
    return true;
}

}  // namespace

extern "C" {

int hg_shard_range(int64_t total, int world, int rank, int64_t* lo, int64_t* hi) {
    if (total < 0 || world < 1 || rank < 0 || rank >= world || !lo || !hi) return kErrInvalid;
    const int64_t base = total / world, extra = total % world;
    *lo = rank * base + (rank < extra ? rank : extra);
    *hi = *lo + base + (rank < extra ? 1 : 0);
    return 0;
}

int hg_solve_multi(int algo, int dtype, const hg_device_batch* shards, int ndev, int layout,
                   int flags) {
    if (!shards_ok(shards, ndev) || algo < 0 || algo > 3 || (dtype != HG_DTYPE_F32 &&
                                                            dtype != HG_DTYPE_F64))
        return kErrInvalid;
    if (dtype == HG_DTYPE_F32 && !kF32[algo]) return kErrInvalid;  // GPT-LU is binary64 only
    for (int i = 0; i < ndev; ++i) {
        const hg_device_batch& b = shards[i];
        if (b.n == 0) continue;
        DeviceScope on(b.device);
        if (on.rc()) return on.rc();
        const int rc = dtype == HG_DTYPE_F32
                           ? kF32[algo](static_cast<const float*>(b.src),
                                        static_cast<const float*>(b.tar), static_cast<float*>(b.H),
                                        b.n, layout, flags, b.stream)
                           : kF64[algo](static_cast<const double*>(b.src),
                                        static_cast<const double*>(b.tar),
                                        static_cast<double*>(b.H), b.n, layout, flags, b.stream);
        if (rc) return rc;
    }
    return 0;
}

int hg_sync_multi(const hg_device_batch* shards, int ndev) {
    if (!shards_ok(shards, ndev)) return kErrInvalid;
    for (int i = 0; i < ndev; ++i) {
        DeviceScope on(shards[i].device);
        if (on.rc()) return on.rc();
        const int rc = (int)hipStreamSynchronize(static_cast<hipStream_t>(shards[i].stream));
        if (rc) return rc;
    }
    return 0;
}

int hg_comm_init_all(int ndev, const int* devices, void** comms) {
    if (ndev < 1 || !devices || !comms) return kErrInvalid;
    std::vector<ncclComm_t> c(ndev);
    const ncclResult_t r = ncclCommInitAll(c.data(), ndev, devices);
    if (r != ncclSuccess) return rccl_err(r);
    for (int i = 0; i < ndev; ++i) comms[i] = c[i];
    return 0;
}

int hg_comm_destroy(int ndev, void** comms) {
    if (ndev < 1 || !comms) return kErrInvalid;
    int first = 0;
    for (int i = 0; i < ndev; ++i) {
        if (!comms[i]) continue;
        const ncclResult_t r = ncclCommDestroy(static_cast<ncclComm_t>(comms[i]));
        if (r != ncclSuccess && !first) first = rccl_err(r);
        comms[i] = nullptr;
    }
    return first;
}

int hg_gather_multi(const hg_device_batch* shards, int ndev, int root, int dtype, void* H_all,
                    void* const* comms) {
    if (!shards_ok(shards, ndev) || root < 0 || root >= ndev || !H_all || !comms ||
        (dtype != HG_DTYPE_F32 && dtype != HG_DTYPE_F64))
        return kErrInvalid;
    const size_t row = 9 * (dtype == HG_DTYPE_F32 ? sizeof(float) : sizeof(double));
    std::vector<int64_t> lo(ndev, 0);
    for (int i = 1; i < ndev; ++i) lo[i] = lo[i - 1] + shards[i - 1].n;
    for (int i = 0; i < ndev; ++i)
        if (!comms[i] || (shards[i].n > 0 && !shards[i].H)) return kErrInvalid;
    char* dst = static_cast<char*>(H_all);
    const hg_device_batch& rb = shards[root];
    // the root's own rows: a copy on its stream (nothing when the block already sits there)
    if (rb.n > 0 && dst + lo[root] * row != rb.H) {
        DeviceScope on(rb.device);
        if (on.rc()) return on.rc();
        const int rc = (int)hipMemcpyAsync(dst + lo[root] * row, rb.H, rb.n * row,
                                           hipMemcpyDeviceToDevice,
                                           static_cast<hipStream_t>(rb.stream));
        if (rc) return rc;
    }
    if (ndev == 1) return 0;
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return rccl_err(r);
    int first = 0;
    for (int i = 0; i < ndev && !first; ++i) {
        if (i == root || shards[i].n == 0) continue;
        const size_t bytes = shards[i].n * row;
        r = ncclSend(shards[i].H, bytes, ncclUint8, root, static_cast<ncclComm_t>(comms[i]),
                     static_cast<hipStream_t>(shards[i].stream));
        if (r == ncclSuccess)
            r = ncclRecv(dst + lo[i] * row, bytes, ncclUint8, i, static_cast<ncclComm_t>(comms[root]),
                         static_cast<hipStream_t>(rb.stream));
        if (r != ncclSuccess) first = rccl_err(r);
    }
    r = ncclGroupEnd();  // always closed, so a failed enqueue leaves no open group behind
    return first ? first : rccl_err(r);
}

}  // extern "C"
