/* sks_homography_multi.h -- the multi-GPU C ABI: one process driving the GPUs of one node.
 *
 * problems are independent, so a batch splits into contiguous rank-major
 * blocks, one per GPU, with no data-path collective; the only exchange is the optional
 * gather of every block's H on one GPU (RCCL point-to-point over xGMI: ncclGroupStart +
 * ncclSend / ncclRecv pairs, rccl.h:700-745), reported apart from the solve.  This is the
 * C/C++ caller's form of what sks-homography_amd/shard.py does for one-process-per-GPU
 * Python callers (torch.distributed); the split arithmetic is the same (shard_range).
 *
 * Library: sks-homography_amd/lib/libsks_homography_multi.so (links the product library and
 * librccl; the product library itself has no RCCL dependency).  Every call is asynchronous on
 * the shards' streams unless it says otherwise, and returns 0, a hipError_t code
 * (hipErrorInvalidValue = 1 for a bad argument), or HG_ERR_RCCL_BASE + an ncclResult_t when
 * RCCL itself failed (the two code spaces overlap, so RCCL's are moved apart: HG_IS_RCCL_ERR /
 * HG_RCCL_RESULT recover it).  N > 1 GPUs: correct by construction and unmeasured on hardware
 * (the build box has one GPU).
 */
#ifndef SKS_HOMOGRAPHY_MULTI_H_
#define SKS_HOMOGRAPHY_MULTI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HG_DTYPE_F32 0
#define HG_DTYPE_F64 1

#define HG_ERR_RCCL_BASE 0x10000
#define HG_IS_RCCL_ERR(rc) ((rc) >= HG_ERR_RCCL_BASE)
#define HG_RCCL_RESULT(rc) ((rc) - HG_ERR_RCCL_BASE)

/* One GPU's block of a batch: device memory on `device` (src, tar, H in `layout`, n problems,
 * the same contracts as hg_<algo>_<dtype>) and a stream on that device (NULL = its null
 * stream). */
typedef struct hg_device_batch {
    int device;
    const void* src;
    const void* tar;
    void* H;
    int64_t n;
    void* stream;
} hg_device_batch;

/* [*lo, *hi): rank's contiguous block of `total` problems split over `world` ranks, sizes
 * differing by at most one (rank r gets total/world, plus one for r < total % world) --
 * shard.shard_range's split. */
int hg_shard_range(int64_t total, int world, int rank, int64_t* lo, int64_t* hi);

/* Solves every shard's block on its own device and stream: hg_<algo>_<dtype>(src, tar, H, n,
 * layout, flags, stream) per shard (algo HG_ALGO_*, dtype HG_DTYPE_*), the calling thread's
 * current device restored afterwards.  Empty shards are skipped.  Bits equal one
 * hg_<algo>_<dtype> call on the whole batch (problems are independent). */
int hg_solve_multi(int algo, int dtype, const hg_device_batch* shards, int ndev, int layout,
                   int flags);

/* Waits for every shard's stream (synchronous). */
int hg_sync_multi(const hg_device_batch* shards, int ndev);

/* RCCL communicators for a process that owns `ndev` devices (ncclCommInitAll, rccl.h:236):
 * comms[i] is rank i on devices[i].  comms is an array of ndev opaque handles (ncclComm_t);
 * synchronous.  hg_comm_destroy releases them. */
int hg_comm_init_all(int ndev, const int* devices, void** comms);
int hg_comm_destroy(int ndev, void** comms);

/* Gathers every shard's H (AoS rows of 9 values of `dtype`, n_i rows contiguous) into H_all
 * on shards[root].device, block i at row lo_i = n_0 + ... + n_{i-1}: one ncclGroupStart /
 * ncclGroupEnd holding an ncclSend on each shard's comm and stream and the matching ncclRecv
 * on the root's, and a device-to-device copy of the root's own block (skipped when it is
 * already in place).  comms[i] must be rank i of an ndev-rank communicator on
 * shards[i].device (hg_comm_init_all).  Asynchronous on the streams. */
int hg_gather_multi(const hg_device_batch* shards, int ndev, int root, int dtype, void* H_all,
                    void* const* comms);

#ifdef __cplusplus
}
#endif

#endif /* SKS_HOMOGRAPHY_MULTI_H_ */
