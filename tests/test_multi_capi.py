"""The multi-GPU C ABI (include/sks_homography_multi.h, lib/libsks_homography_multi.so) on the
CPU: it loads, exports what its header declares (and the product library does not), its split
is shard.shard_range's exactly, and every argument check answers before any HIP call."""
import ctypes

import pytest

from test_capi import _c_decls


@pytest.fixture(scope="module")
def multi(pkg):
    return pkg._lib.multi()


def test_exports_its_header(pkg, multi):
    decls = _c_decls("sks_homography_multi.h")
    assert set(decls) == set(pkg._lib.MULTI_SIGNATURES)
    for name in decls:
        assert hasattr(multi, name), name
        assert not hasattr(pkg.lib(), name), f"{name} leaked into the product library"


def test_shard_range_equals_python_split(pkg, multi):
    lo, hi = ctypes.c_int64(), ctypes.c_int64()
    for total in (0, 1, 7, 8, 9, 1000, 10_000_000, 80_000_000, (1 << 40) + 3):
        for world in (1, 2, 3, 7, 8, 16):
            prev = 0
            for rank in range(world):
                assert multi.hg_shard_range(total, world, rank, ctypes.byref(lo), ctypes.byref(hi)) == 0
                assert (lo.value, hi.value) == pkg.shard_range(total, world, rank)
                assert lo.value == prev
                prev = hi.value
            assert prev == total
    for bad in ((-1, 2, 0), (5, 0, 0), (5, 2, 2), (5, 2, -1)):
        assert multi.hg_shard_range(*bad, ctypes.byref(lo), ctypes.byref(hi)) == 1
    assert multi.hg_shard_range(5, 2, 0, None, ctypes.byref(hi)) == 1


def _shards(pkg, *ns):
    arr = (pkg._lib.DeviceBatch * len(ns))()
    for i, n in enumerate(ns):
        arr[i].device, arr[i].n = 0, n
    return arr


def test_argument_checks_before_any_hip_call(pkg, multi):
    s = _shards(pkg, 0, 0)
    assert multi.hg_solve_multi(0, 0, None, 1, 0, 0) == 1          # no shards
    assert multi.hg_solve_multi(0, 0, s, 0, 0, 0) == 1             # ndev 0
    assert multi.hg_solve_multi(4, 0, s, 2, 0, 0) == 1             # algo
    assert multi.hg_solve_multi(0, 2, s, 2, 0, 0) == 1             # dtype
    assert multi.hg_solve_multi(3, 0, s, 2, 0, 0) == 1             # GPT-LU binary32
    assert multi.hg_solve_multi(0, 0, s, 2, 0, 0) == 0             # empty shards: nothing to do
    neg = _shards(pkg, 4, -1)
    assert multi.hg_solve_multi(0, 0, neg, 2, 0, 0) == 1           # n < 0
    assert multi.hg_sync_multi(None, 1) == 1
    comms = (ctypes.c_void_p * 2)()
    assert multi.hg_gather_multi(s, 2, 2, 0, 16, comms) == 1       # root out of range
    assert multi.hg_gather_multi(s, 2, 0, 0, None, comms) == 1     # no destination
    assert multi.hg_gather_multi(s, 2, 0, 3, 16, comms) == 1       # dtype
    assert multi.hg_gather_multi(s, 2, 0, 0, 16, comms) == 1       # NULL communicators
    assert multi.hg_comm_init_all(0, None, comms) == 1
    assert multi.hg_comm_destroy(0, comms) == 1
    assert multi.hg_comm_destroy(2, comms) == 0                    # NULL handles: nothing to free


def test_rccl_failures_have_their_own_codes(multi):
    """RCCL's ncclResult_t codes overlap hipError_t's (1 is both hipErrorInvalidValue and
    ncclUnhandledCudaError), so the multi ABI returns them as HG_ERR_RCCL_BASE + result.  With
    no GPU in this container, communicator set-up fails inside RCCL and says so."""
    import torch
    if torch.cuda.device_count() > 0:  # counts devices without initialising the runtime
        pytest.skip("a GPU is present: communicator set-up would succeed")
    devs = (ctypes.c_int * 1)(0)
    comms = (ctypes.c_void_p * 1)()
    rc = multi.hg_comm_init_all(1, devs, comms)
    assert rc >= 0x10000 and rc - 0x10000 > 0, hex(rc)  # HG_IS_RCCL_ERR, an ncclResult_t != 0
    assert comms[0] is None
