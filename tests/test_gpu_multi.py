"""The multi-GPU C ABI on the GPU box's one device (include/sks_homography_multi.h).

  * hg_solve_multi over one shard, and over the shard_range blocks of one batch given as
    several shards of device 0 on their own streams, equals one whole-batch solve bit for bit
    (AoS f32 normalised, SoA f64 unnormalised);
  * hg_comm_init_all / hg_gather_multi / hg_comm_destroy with one rank: RCCL initialises over
    the device and the gather lands the root's block in the gathered buffer.
N > 1 devices (the ncclSend / ncclRecv pairs) cannot run on a one-GPU box: correct by
construction, unmeasured on hardware.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(pkg, dev, n, dtype, layout):
    src = pkg.fill_uniform(n * 8, 11, 0, device=dev)
    tar = pkg.fill_uniform(n * 8, 11, n * 8, device=dev)
    if dtype == torch.float64:
        src, tar = src.double(), tar.double()
    shape = (8, n) if layout == "soa" else (n, 8)
    return src.view(shape), tar.view(shape)


@pytest.mark.parametrize("dtype,layout,norm", [(torch.float32, "aos", True),
                                               (torch.float64, "soa", False)])
@pytest.mark.parametrize("parts", [1, 3, 8])
def test_solve_multi_equals_whole_batch(pkg, dev, dtype, layout, norm, parts):
    """parts = 8: the shard loop the 8-GPU node runs (BASELINE configs[4]), every shard here
    on device 0 with its own stream; the calling thread's current device is left as it was."""
    multi = pkg._lib.multi()
    n = 1_000_003
    src, tar = _batch(pkg, dev, n, dtype, layout)
    want = pkg.solve("aca", src, tar, normalize=norm, layout=layout)
    dt = 0 if dtype == torch.float32 else 1
    streams = [torch.cuda.Stream(dev) for _ in range(parts)]
    keep, shards = [], (pkg._lib.DeviceBatch * parts)()
    for r in range(parts):
        lo, hi = pkg.shard_range(n, parts, r)
        if layout == "aos":
            s, t = src[lo:hi].contiguous(), tar[lo:hi].contiguous()
            H = torch.empty((hi - lo, 9), dtype=dtype, device=dev)
        else:
            s, t = src[:, lo:hi].contiguous(), tar[:, lo:hi].contiguous()
            H = torch.empty((9, hi - lo), dtype=dtype, device=dev)
        keep.append((s, t, H))
        shards[r].device, shards[r].n = dev.index or 0, hi - lo
        shards[r].src, shards[r].tar, shards[r].H = s.data_ptr(), t.data_ptr(), H.data_ptr()
        shards[r].stream = streams[r].cuda_stream
    torch.cuda.synchronize(dev)
    hip = ctypes.CDLL("libamdhip64.so.7")
    before, after = ctypes.c_int(-1), ctypes.c_int(-1)
    assert hip.hipGetDevice(ctypes.byref(before)) == 0
    assert multi.hg_solve_multi(0, dt, shards, parts, 1 if layout == "soa" else 0, 1 if norm else 0) == 0
    assert hip.hipGetDevice(ctypes.byref(after)) == 0 and after.value == before.value
    assert multi.hg_sync_multi(shards, parts) == 0
    got = torch.cat([H for *_, H in keep], dim=0 if layout == "aos" else 1)
    assert torch.equal(got.view(torch.uint8), want.view(torch.uint8))


def test_one_rank_rccl_gather(pkg, dev):
    multi = pkg._lib.multi()
    n = 4099
    src, tar = _batch(pkg, dev, n, torch.float32, "aos")
    H = pkg.solve("aca", src, tar, normalize=True)
    comms = (ctypes.c_void_p * 1)()
    devs = (ctypes.c_int * 1)(dev.index or 0)
    assert multi.hg_comm_init_all(1, devs, comms) == 0 and comms[0]
    try:
        shards = (pkg._lib.DeviceBatch * 1)()
        shards[0].device, shards[0].H, shards[0].n = dev.index or 0, H.data_ptr(), n
        shards[0].stream = torch.cuda.current_stream(dev).cuda_stream
        full = torch.full((n, 9), float("nan"), device=dev)
        assert multi.hg_gather_multi(shards, 1, 0, 0, full.data_ptr(), comms) == 0
        torch.cuda.synchronize(dev)
        assert torch.equal(full.view(torch.int32), H.view(torch.int32))
        # in place: nothing to move
        assert multi.hg_gather_multi(shards, 1, 0, 0, H.data_ptr(), comms) == 0
    finally:
        assert multi.hg_comm_destroy(1, comms) == 0
