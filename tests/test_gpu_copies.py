"""The test process's own host copies leave no GPU mapping of its heap.

HIP copies a pageable buffer of 2 MB or more by mapping the user's pages for the GPU in place,
and KFD keeps that mapping after the copy; every GPU fault this project's suites ever had was
such a copy writing a reused heap page.  tests/conftest.py keeps this process's copies on HIP's
staged path (GPU_PINNED_MIN_XFER_SIZE, read when the runtime starts).  These tests check that
the setting took: after .cpu() / .to() copies of 2-64 MB, KFD reports the copied pages as not
accessible to the GPU (tests/fault_probe.c asks hsa_amd_svm_attributes_get, a host-side
query).  The library's own host entry maps none of the caller's pages (it stages pageable
memory through its own pinned buffers; tests/test_gpu_host_nomap.py checks that without the
knob) except with HG_FLAG_HOST_REGISTER, whose pages KFD keeps mapped after the call, so this
file runs before any library host call (tests/conftest.py orders it with the first tier)."""
import ctypes
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NO_ACCESS = 0x202  # HSA_AMD_SVM_ATTRIB_AGENT_NO_ACCESS


@pytest.fixture(scope="module")
def svm_access():
    path = os.path.join(ROOT, "tests", "_build", "libfault_probe.so")
    if not os.path.exists(path):
        pytest.skip("tests/_build/libfault_probe.so not built (__graft_entry__.build())")
    fp = ctypes.CDLL(path)
    u64 = ctypes.c_uint64
    fp.hg_fault_probe_svm.argtypes = [u64, u64] + [ctypes.POINTER(u64)] * 3
    assert fp.hg_fault_probe_install() == 0

    def query(p):
        acc, ro, gf = u64(), u64(), u64()
        rc = fp.hg_fault_probe_svm(p // 4096 * 4096, 4096, ctypes.byref(acc), ctypes.byref(ro),
                                   ctypes.byref(gf))
        assert rc == 0, f"hsa_amd_svm_attributes_get failed ({rc})"
        return acc.value
    return query


def test_conftest_sets_the_staged_copy_knob():
    assert int(os.environ["GPU_PINNED_MIN_XFER_SIZE"]) >= 65536


@pytest.mark.parametrize("mb", [2, 6, 64])
def test_pageable_copies_leave_no_gpu_mapping(dev, svm_access, mb):
    n = mb * 2**20 // 4
    a = torch.arange(n, dtype=torch.float32)
    d = a.to(dev)                       # host -> device: the host pages are the source
    b = torch.empty(n, dtype=torch.float32)
    b.copy_(d)                          # device -> host: the host pages are the destination
    torch.cuda.synchronize(dev)
    assert torch.equal(a, b)
    for t in (a, b):
        # interior pages only: an edge page may be shared with a neighbouring allocation
        for p in (t.data_ptr() + 8192, t.data_ptr() + t.numel() * 2, t.data_ptr() + t.numel() * 4 - 8192):
            assert svm_access(p) == NO_ACCESS, f"{mb} MB copy left page {p:#x} GPU-mapped"
