"""hg_tensor_aca_rect_backward_sum_f32 (csrc/hg_rect_sum.hpp): the TensorACA_rect all-gradient
backward with ATen-CPU's batch sum of the scale / div terms, the sum's first level folded into
the backward kernel.  Its contract is the two-launch form's bits -- the terms kernel
(hg_tensor_aca_rect_backward_terms_f32) then hg_sum_aten_f32 -- which
tests/test_gpu_aten_sum.py and tests/test_gpu_rect_grad.py pin to oracle/aten_sum.py, ATen
autograd and the reference's fixtures.  Checked here bit for bit against that form and against
the oracle's sum of the terms: batch sizes from 1 to 16 M (every cascade shape: no level-0
block, partial super-blocks, one and several chunks, the last chunk shorter), ATen thread
counts 1 ... 64, lanes 4 / 8 / 16, with and without dL/dsrc, misaligned tensors (the two-launch
fallback), and the op (sks_amd::tensor_aca_rect_backward) that now takes this path."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
from aten_sum import aten_sum  # noqa: E402

pytestmark = pytest.mark.gpu


def _batch(pkg, dev, B, seed=0):
    torch.manual_seed(seed)
    _, _, src, tar, scale, div = pkg.adjust(dev, B)
    gH = torch.randn(B, 3, 3, device=dev)
    return src.contiguous(), tar.contiguous(), gH, scale, div


def _two_launch(pkg, dev, src, tar, gH, scale, div, want_src, lanes, threads):
    B = tar.shape[0]
    gs = torch.full((B, 3, 4), float("nan"), device=dev) if want_src else None
    gt = torch.full((B, 3, 4), float("nan"), device=dev)
    terms = torch.empty((2, 3 * B), device=dev)
    out = torch.full((2,), float("nan"), device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    pkg._lib.call("hg_tensor_aca_rect_backward_terms_f32", src.data_ptr(), tar.data_ptr(), gH.data_ptr(),
                  B, scale.data_ptr(), div.data_ptr(), gs.data_ptr() if want_src else None,
                  gt.data_ptr(), terms.data_ptr(), st)
    terms_copy = terms.clone()
    pkg._lib.call("hg_sum_aten_f32", terms.data_ptr(), 2, 3 * B, 3 * B, 1, lanes, threads,
                  out.data_ptr(), st)
    return gs, gt, out, terms_copy


def _fused(pkg, dev, src, tar, gH, scale, div, want_src, lanes, threads):
    B = tar.shape[0]
    gs = torch.full((B, 3, 4), float("nan"), device=dev) if want_src else None
    gt = torch.full((B, 3, 4), float("nan"), device=dev)
    ws = torch.full((6 * B,), float("nan"), device=dev)
    out = torch.full((2,), float("nan"), device=dev)
    pkg._lib.call("hg_tensor_aca_rect_backward_sum_f32", src.data_ptr(), tar.data_ptr(), gH.data_ptr(),
                  B, scale.data_ptr(), div.data_ptr(), gs.data_ptr() if want_src else None,
                  gt.data_ptr(), ws.data_ptr(), lanes, threads, out.data_ptr(),
                  torch.cuda.current_stream(dev).cuda_stream)
    return gs, gt, out


def _bits(x):
    return x.view(torch.int32)


CASES = [  # (B, threads, lanes)
    (1, 1, 8), (2, 16, 8), (5, 1, 8), (11, 4, 8), (170, 1, 8), (171, 1, 8), (1000, 16, 8),
    (10923, 1, 8), (10924, 2, 8), (43691, 16, 8), (65536, 1, 8), (65536, 16, 8), (65536, 64, 8),
    (65536, 16, 4), (65536, 16, 16), (100003, 3, 8), (349525, 1, 8), (1 << 20, 16, 8),
    (1 << 20, 7, 8), ((1 << 20) + 7, 64, 8), (3_000_001, 16, 8),
]


@pytest.mark.parametrize("B,T,W", CASES)
def test_fused_equals_two_launch_form(pkg, dev, B, T, W):
    src, tar, gH, scale, div = _batch(pkg, dev, B, seed=B % 97)
    for want_src in (True, False):
        gs0, gt0, out0, terms = _two_launch(pkg, dev, src, tar, gH, scale, div, want_src, W, T)
        gs1, gt1, out1 = _fused(pkg, dev, src, tar, gH, scale, div, want_src, W, T)
        assert torch.equal(_bits(gt1), _bits(gt0)), (B, T, W)
        if want_src:
            assert torch.equal(_bits(gs1), _bits(gs0)), (B, T, W)
        assert _bits(out1).tolist() == _bits(out0).tolist(), (B, T, W, out1.tolist(), out0.tolist())
    if B <= 1_100_000:  # and the oracle's ATen-order sum of the same terms
        t = terms.cpu().numpy()
        want = np.array([aten_sum(t[0], W, T), aten_sum(t[1], W, T)], np.float32)
        assert out1.cpu().numpy().tobytes() == want.tobytes(), (B, T, W)


def test_fused_at_bench_size(pkg, dev):
    """B = 16 M (the bench's large backward), T = 16 and 1 (one chunk: level step 32)."""
    B = 16 * 1024 * 1024
    src, tar, gH, scale, div = _batch(pkg, dev, B, seed=3)
    for T in (16, 1):
        gs0, gt0, out0, _ = _two_launch(pkg, dev, src, tar, gH, scale, div, True, 8, T)
        gs1, gt1, out1 = _fused(pkg, dev, src, tar, gH, scale, div, True, 8, T)
        assert torch.equal(_bits(gt1), _bits(gt0)) and torch.equal(_bits(gs1), _bits(gs0))
        assert _bits(out1).tolist() == _bits(out0).tolist(), T
        del gs0, gt0, gs1, gt1
        torch.cuda.empty_cache()


def test_misaligned_views_take_the_two_launch_form(pkg, dev):
    B = 40000
    src, tar, gH, scale, div = _batch(pkg, dev, B, seed=9)
    buf = torch.empty(B * 12 + 1, device=dev)
    tar_u = buf[1:].view(B, 3, 4)  # 4 B past a 16-B boundary
    tar_u.copy_(tar)
    gs0, gt0, out0, _ = _two_launch(pkg, dev, src, tar, gH, scale, div, True, 8, 16)
    gs1, gt1, out1 = _fused(pkg, dev, src, tar_u, gH, scale, div, True, 8, 16)
    assert torch.equal(_bits(gt1), _bits(gt0)) and torch.equal(_bits(gs1), _bits(gs0))
    assert _bits(out1).tolist() == _bits(out0).tolist()


def test_argument_checks(pkg, dev):
    lib = pkg.lib()
    f = lib.hg_tensor_aca_rect_backward_sum_f32
    x = torch.zeros(16, device=dev)
    p = x.data_ptr()
    assert f(p, p, p, -1, p, p, None, p, p, 8, 1, p, None) == 1    # B < 0
    assert f(p, p, p, 4, p, p, None, p, p, 0, 1, p, None) == 1     # lanes
    assert f(p, p, p, 4, p, p, None, p, p, 2, 4, p, None) == 1     # lanes < 4 with threads
    assert f(p, p, p, 4, p, p, None, p, None, 8, 1, p, None) == 1  # no workspace
    assert f(p, p, p, 4, p, p, None, p, p, 8, 1, None, None) == 1  # no output
    out = torch.full((2,), 5.0, device=dev)
    assert f(None, None, None, 0, None, None, None, None, None, 8, 1, out.data_ptr(), None) == 0
    torch.cuda.synchronize(dev)
    assert out.tolist() == [0.0, 0.0]


def test_op_takes_the_fused_path(pkg, dev):
    """sks_amd::tensor_aca_rect_backward (aten order, one-value scale / div): equal to the
    two-launch form for T = the op's aten_threads."""
    B = 1 << 20
    src, tar, gH, scale, div = _batch(pkg, dev, B, seed=5)
    for T in (1, 16):
        gs_op, gt_op, gsc, gdv = pkg.tensor_aca_rect_backward(src, tar, gH, scale, div, True, True,
                                                              aten_threads=T)
        gs0, gt0, out0, _ = _two_launch(pkg, dev, src, tar, gH, scale, div, True, 8, T)
        assert torch.equal(_bits(gt_op), _bits(gt0)) and torch.equal(_bits(gs_op), _bits(gs0))
        assert _bits(gsc.reshape(1)).tolist() + _bits(gdv.reshape(1)).tolist() == _bits(out0).tolist()
