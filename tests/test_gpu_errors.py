"""C-ABI error attribution: a call's return code is its own
launch's status, never an error an unrelated earlier HIP call left pending on the thread,
and the library leaves such a pending error in place for its owner.

The pending error is provoked with hipSetDevice(9999) (hipErrorInvalidDevice, non-fatal)
through the same HIP runtime the library uses (one libamdhip64.so.7 per process)."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

HIP_ERROR_INVALID_DEVICE = 101


@pytest.fixture()
def hip(pkg, dev):
    pkg.lib()
    h = ctypes.CDLL("libamdhip64.so.7")
    h.hipSetDevice.argtypes = [ctypes.c_int]
    torch.cuda.synchronize(dev)
    h.hipGetLastError()  # start clean
    yield h
    h.hipGetLastError()  # leave clean for the next test


def _pend(hip):
    assert hip.hipSetDevice(9999) == HIP_ERROR_INVALID_DEVICE
    assert hip.hipPeekAtLastError() == HIP_ERROR_INVALID_DEVICE


def _bits_equal(orc, a, b):
    return orc.same_bits(np.asarray(a), np.asarray(b)).all()


def test_solver_launch_ignores_pending_error(hip, pkg, dev, orc):
    g = load_golden("cpp_uniform.npz")
    s = torch.from_numpy(g["src_f32"]).to(dev)
    t = torch.from_numpy(g["tar_f32"]).to(dev)
    n = s.shape[0]
    stream = torch.cuda.current_stream(dev).cuda_stream
    lib = pkg.lib()
    for fn, key in ((lib.hg_aca_f32, "aca_f32"), (lib.hg_sks_f32, "sks_f32")):
        H = torch.full((n, 9), -1.0, device=dev)
        _pend(hip)
        assert fn(s.data_ptr(), t.data_ptr(), H.data_ptr(), n, 0, 1, stream) == 0
        # the caller's error is still there, unread, for its owner
        assert hip.hipPeekAtLastError() == HIP_ERROR_INVALID_DEVICE
        hip.hipGetLastError()
        torch.cuda.synchronize(dev)
        assert _bits_equal(orc, H.cpu().numpy(), g[key])


def test_rect_launch_ignores_pending_error(hip, pkg, dev, orc, oracle):
    g = load_golden("torch_tensor_aca.npz")
    sh = torch.from_numpy(g["f_src_h"]).to(dev)
    th = torch.from_numpy(g["f_tar_h"]).to(dev)
    B = th.shape[0]
    sc = torch.tensor([128.0], device=dev)
    dv = torch.tensor([1.0], device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    lib = pkg.lib()
    H = torch.full((B, 3, 3), -1.0, device=dev)
    H2 = torch.full((B, 3, 3), -1.0, device=dev)
    torch.cuda.synchronize(dev)
    # (torch's own launches check hipGetLastError, so no torch op may run while it pends)
    _pend(hip)
    assert lib.hg_tensor_aca_rect_f32(sh.data_ptr(), th.data_ptr(), H.data_ptr(), B, sc.data_ptr(),
                                      dv.data_ptr(), stream) == 0
    assert hip.hipPeekAtLastError() == HIP_ERROR_INVALID_DEVICE
    assert lib.hg_tensor_aca_rect_f32_hostscalar(sh.data_ptr(), th.data_ptr(), H2.data_ptr(), B,
                                                 128.0, 1.0, stream) == 0
    assert hip.hipPeekAtLastError() == HIP_ERROR_INVALID_DEVICE
    hip.hipGetLastError()
    torch.cuda.synchronize(dev)
    assert _bits_equal(orc, H.cpu().numpy(), g["f_rect"])
    assert _bits_equal(orc, H2.cpu().numpy(), g["f_rect"])


def test_other_launchers_ignore_pending_error(hip, pkg, dev, oracle):
    stream = torch.cuda.current_stream(dev).cuda_stream
    lib = pkg.lib()
    out = torch.empty(1000, device=dev)
    bits = torch.empty(4000, dtype=torch.int32, device=dev)
    w = load_golden("cpp_wall.npz")
    ps = torch.from_numpy(w["pool_src"]).to(dev)
    pt = torch.from_numpy(w["pool_tar"]).to(dev)
    H = torch.empty((1000, 9), device=dev)
    torch.cuda.synchronize(dev)
    _pend(hip)
    assert lib.hg_fill_uniform_f32(out.data_ptr(), 1000, 11, 0, 0.0, 1024.0, stream) == 0
    assert lib.hg_fill_bits_u32(bits.data_ptr(), 4000, 11, 0, stream) == 0
    assert lib.hg_sample_solve_f32(ps.data_ptr(), pt.data_ptr(), ps.shape[0], bits.data_ptr(),
                                   H.data_ptr(), 1000, 0, 1, stream) == 0
    assert hip.hipPeekAtLastError() == HIP_ERROR_INVALID_DEVICE
    hip.hipGetLastError()
    torch.cuda.synchronize(dev)
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.fill_uniform(1000, 11, 0))


def test_table8_launchers_ignore_pending_error(hip, pkg, dev, orc):
    """the Table-8 entry points too (the MRG32K3A draws, get_rand_list, the fused
    gather + solve and the fused draws + gather + solve)."""
    stream = torch.cuda.current_stream(dev).cuda_stream
    lib = pkg.lib()
    w = load_golden("cpp_wall.npz")
    ps = torch.from_numpy(w["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(w["pool_tar"].astype(np.float64)).to(dev)
    n = 1000
    rl = torch.empty((4, n), dtype=torch.int32, device=dev)
    d_src = torch.empty((8, n), dtype=torch.float64, device=dev)
    d_tar = torch.empty((8, n), dtype=torch.float64, device=dev)
    H1 = torch.empty((9, n), dtype=torch.float64, device=dev)
    H2 = torch.empty((9, n), dtype=torch.float64, device=dev)
    torch.cuda.synchronize(dev)
    _pend(hip)
    assert lib.hg_rand_mrg32k3a_u32(rl.data_ptr(), 4 * n, 11, stream) == 0
    assert lib.hg_get_rand_list_f64(rl.data_ptr(), ps.shape[0], ps.data_ptr(), pt.data_ptr(),
                                    d_src.data_ptr(), d_tar.data_ptr(), n, stream) == 0
    assert lib.hg_gather_solve_f64(0, ps.data_ptr(), pt.data_ptr(), ps.shape[0], rl.data_ptr(),
                                   H1.data_ptr(), n, 0, stream) == 0
    assert lib.hg_rand_gather_solve_f64(0, ps.data_ptr(), pt.data_ptr(), ps.shape[0], 11,
                                        H2.data_ptr(), n, 0, stream) == 0
    assert hip.hipPeekAtLastError() == HIP_ERROR_INVALID_DEVICE
    hip.hipGetLastError()
    torch.cuda.synchronize(dev)
    assert _bits_equal(orc, H1.cpu().numpy(), H2.cpu().numpy())
    assert _bits_equal(orc, H1.cpu().numpy(),
                       pkg.solve("aca", d_src, d_tar, normalize=False, layout="soa").cpu().numpy())


def test_host_pointer_calls_ignore_pending_error(hip, pkg, dev, orc):
    """sks::runKernel_ACA on host pointers and hg_solve_host_f32 on pageable memory probe
    their pointers first (hipPointerGetAttributes succeeds on unregistered memory on this
    runtime, tools/probe_lasterror.cpp) -- neither reports nor consumes the pending error."""
    g = load_golden("cpp_uniform.npz")
    lib = pkg.lib()
    one = lib._ZN3sks13runKernel_ACAEPfS0_S0_
    one.restype = ctypes.c_int
    s = np.ascontiguousarray(g["src_f32"])
    t = np.ascontiguousarray(g["tar_f32"])
    h9 = np.empty(9, np.float32)
    fp = ctypes.POINTER(ctypes.c_float)
    _pend(hip)
    assert one(s[3].ctypes.data_as(fp), t[3].ctypes.data_as(fp), h9.ctypes.data_as(fp)) == 0
    assert hip.hipPeekAtLastError() == HIP_ERROR_INVALID_DEVICE
    assert _bits_equal(orc, h9, g["aca_f32"][3])
    H = np.full((s.shape[0], 9), -1, np.float32)
    assert lib.hg_solve_host_f32(0, s.ctypes.data, t.ctypes.data, H.ctypes.data, s.shape[0], 0, 1,
                                 None) == 0
    assert hip.hipPeekAtLastError() == HIP_ERROR_INVALID_DEVICE
    hip.hipGetLastError()
    assert _bits_equal(orc, H, g["aca_f32"])


def test_refused_arguments_raise_no_hip_error(hip, pkg, dev):
    """Arguments a launcher refuses return non-zero without raising a HIP error (nothing
    was launched, so nothing is left pending on the thread)."""
    lib = pkg.lib()
    x = torch.zeros(8, device=dev)
    out = torch.zeros(1, device=dev)
    assert lib.hg_sum_rows_f32(x.data_ptr(), 70000, 0, out.data_ptr(), None) != 0  # rows > 65535
    assert lib.hg_aca_f32(x.data_ptr(), x.data_ptr(), out.data_ptr(), 1, 7, 1, None) != 0  # layout
    assert hip.hipPeekAtLastError() == 0
