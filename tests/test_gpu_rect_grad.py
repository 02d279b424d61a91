"""TensorACA_rect's backward on the GPU against ATen autograd through the reference's own
statements (Modules_Runtime_Test.py:294-302), bit for bit.

The reference gets its gradients from ATen autograd over its seven statements.  Those write
H in place, and column 2 reads columns 0 and 1 back, so autograd differentiates them with
respect to tar, scale and div only (with src requiring grad its backward raises; recorded in
the fixture).  The product's backward (hg_solvers.hpp tensor_aca_rect_grad_rows) restates the
autograd graph op for op: the zero-filled slice gradients (+0), the order dL/dh_temp arrives
in, ATen's FMA-contracted cross product as the cross's backward.

Pins:
  * tests/golden/torch_rect_grad.npz (tools/make_golden.py --torch-grad, the reference's
    statements under autograd on CPU torch here): dL/dtar in every case, dL/dscale and dL/ddiv
    where ATen reduces them per problem or not at all -- through the op's backward and
    torch.autograd;
  * ATen autograd through the same statements on THIS box's CPU, 200 003 problems each of
    random bit patterns, a special-value mixture and quads over 20 decades (AVX-512 hosts:
    ATen's cross takes its FMA path there; skipped, not weakened, elsewhere).
A batch-uniform (1,) scale / div gradient is ATen's batch-wide sum of the (B,3,1) terms; the
op sums the same terms in ATen-CPU's order (hg_sum_aten_f32, restated in oracle/aten_sum.py),
so it is bit for bit too -- with the thread count of the process that made the fixture (the
order depends on it from 32768 terms up; tests/test_gpu_aten_sum.py covers B = 64 K and 1 M).
"""
import zlib

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gold():
    return load_golden("torch_rect_grad.npz")


def _same(orc, got, want, what):
    got = got.detach().cpu().numpy() if torch.is_tensor(got) else np.asarray(got)
    ok = orc.same_bits(np.ascontiguousarray(got, np.float32), np.ascontiguousarray(want, np.float32))
    assert ok.all(), f"{what}: {int((~ok).sum())}/{ok.size} differ; first at {np.argwhere(~ok)[:3].tolist()}"


def test_backward_equals_reference_autograd_fixture(orc, oracle, pkg, dev, gold):
    assert bool(gold["src_grad_refused"])
    for tag in (str(t) for t in gold["cases"]):
        src, tar, gH = (torch.from_numpy(gold[f"{tag}_{k}"]).to(dev) for k in ("src", "tar", "gH"))
        sc_np, dv_np = gold[f"{tag}_scale"], gold[f"{tag}_div"]
        sc, dv = torch.from_numpy(sc_np).to(dev), torch.from_numpy(dv_np).to(dev)
        B = tar.shape[0]
        _, g_tar, g_sc, g_dv = pkg.tensor_aca_rect_backward(src, tar, gH, sc, dv, False, True)
        _same(orc, g_tar, gold[f"{tag}_gtar"], f"grad tar {tag}")
        # through torch.autograd, src constant as in the reference
        t = tar.clone().requires_grad_()
        s_, d_ = sc.clone().requires_grad_(), dv.clone().requires_grad_()
        pkg.TensorACA_rect(B, src, t, s_, d_).backward(gH)
        _same(orc, t.grad, gold[f"{tag}_gtar"], f"autograd tar {tag}")
        for got, via, key in ((g_sc, s_.grad, "gscale"), (g_dv, d_.grad, "gdiv")):
            want = gold[f"{tag}_{key}"]
            _same(orc, via, got.cpu().numpy(), f"autograd {key} {tag}")
            _same(orc, got, want, f"{key} {tag}")  # (1,) ones too: ATen's order, bit for bit


B = 200_003
SPECIALS = np.array([0.0, -0.0, 1.0, -1.0, 2.0, 0.5, 3.0, 1024.0, np.inf, -np.inf, np.nan,
                     1e-45, -1.2e-40, 3e38, -3e38], np.float32)
WEIGHTS = np.array([8, 6, 8, 6, 6, 4, 4, 4, 1, 1, 1, 1, 1, 1, 1], np.float64)


def _inputs(kind, rng, shape):
    if kind == "random_bits":
        return rng.integers(0, 2**32 - 1, size=shape, dtype=np.uint32, endpoint=True).view(np.float32)
    if kind == "special_mixture":
        return rng.choice(SPECIALS, size=shape, p=WEIGHTS / WEIGHTS.sum()).astype(np.float32)
    return (rng.uniform(-1, 1, shape) * 10.0 ** rng.integers(-10, 11, (shape[0], 1, 1))).astype(np.float32)


@pytest.mark.parametrize("kind", ["random_bits", "special_mixture", "scaled"])
@pytest.mark.parametrize("per_problem", [False, True])
def test_backward_equals_aten_autograd_on_box_cpu(orc, pkg, dev, kind, per_problem):
    """bench.torch_tensor_aca_rect (the reference's statements) under autograd on this box's
    CPU, with its own thread count: dL/dtar, dL/dscale and dL/ddiv bit for bit, for
    batch-uniform (1,) and per-problem (B,1,1) scale / div -- through the op with its default
    (this process's ATen threads) and through torch.autograd."""
    if not orc.cpu_has_avx512():
        pytest.skip("ATen's CPU cross takes its AVX-512 FMA path only on an AVX-512 host")
    import bench
    rng = np.random.default_rng(zlib.crc32(repr((kind, per_problem)).encode()))
    src, tar = _inputs(kind, rng, (B, 3, 4)), _inputs(kind, rng, (B, 3, 4))
    gH = _inputs(kind, rng, (B, 3, 3))
    if per_problem:
        sc = (rng.random((B, 1, 1)) * 64 + 64).astype(np.float32)
        dv = (rng.random((B, 1, 1)) + 0.5).astype(np.float32)
    else:
        sc, dv = np.array([50.0], np.float32), np.array([1.25], np.float32)
    t = torch.from_numpy(tar).requires_grad_()
    s_, d_ = torch.from_numpy(sc).requires_grad_(), torch.from_numpy(dv).requires_grad_()
    bench.torch_tensor_aca_rect(torch.from_numpy(src), t, s_, d_).backward(torch.from_numpy(gH))
    _, g_tar, g_sc, g_dv = pkg.tensor_aca_rect_backward(
        torch.from_numpy(src).to(dev), torch.from_numpy(tar).to(dev), torch.from_numpy(gH).to(dev),
        torch.from_numpy(sc).to(dev), torch.from_numpy(dv).to(dev), False, True)
    _same(orc, g_tar, t.grad.numpy(), f"grad tar {kind}")
    _same(orc, g_sc, s_.grad.numpy(), f"grad scale {kind}")
    _same(orc, g_dv, d_.grad.numpy(), f"grad div {kind}")
    # the same through torch.autograd on the GPU leaves
    tg = torch.from_numpy(tar).to(dev).requires_grad_()
    sg = torch.from_numpy(sc).to(dev).requires_grad_()
    dg = torch.from_numpy(dv).to(dev).requires_grad_()
    pkg.TensorACA_rect(B, torch.from_numpy(src).to(dev), tg, sg, dg).backward(torch.from_numpy(gH).to(dev))
    _same(orc, sg.grad, s_.grad.numpy(), f"autograd scale {kind}")
    _same(orc, dg.grad, d_.grad.numpy(), f"autograd div {kind}")


def test_offsets_gradient_equals_aten_autograd_through_the_reference_construction(orc, pkg, dev):
    """The compact deep-homography form against what a reference user writes: the source
    rectangle built as getInput builds it, tar = src + offsets as getTar does (.py:9-21), the
    homogeneous tensors as adjust makes them (.py:24-37), then TensorACA_rect's statements
    under autograd on this box's CPU -- the offsets' gradient equals the op's bit for bit."""
    if not orc.cpu_has_avx512():
        pytest.skip("ATen's CPU cross takes its AVX-512 FMA path only on an AVX-512 host")
    import bench
    n = 100_003
    rng = np.random.default_rng(2718)
    corner = rng.integers(10, 30, (n, 2)).astype(np.float32)
    offs = (rng.random((n, 4, 2)) * 32).astype(np.float32)
    gH = rng.standard_normal((n, 3, 3)).astype(np.float32)
    rect = torch.tensor([[0.0, 0.0], [128.0, 0.0], [0.0, 128.0], [128.0, 128.0]])
    src = torch.from_numpy(corner)[:, None, :] + rect[None]
    off_t = torch.from_numpy(offs).requires_grad_()
    tar = src + off_t
    ones = torch.ones((n, 1, 4))
    src_h = torch.cat((src.transpose(1, 2), ones), dim=1)
    tar_h = torch.cat((tar.transpose(1, 2), ones), dim=1)
    H = bench.torch_tensor_aca_rect(src_h, tar_h, torch.tensor([128.0]), torch.tensor([1.0]))
    H.backward(torch.from_numpy(gH))
    g_off, _ = pkg.tensor_aca_offsets_backward(torch.from_numpy(corner).to(dev),
                                               torch.from_numpy(offs).to(dev),
                                               torch.from_numpy(gH).to(dev), 128.0, 128.0, False)
    _same(orc, H.detach().numpy(), pkg.tensor_aca_offsets(torch.from_numpy(corner).to(dev),
                                                           torch.from_numpy(offs).to(dev),
                                                           128.0, 128.0).cpu().numpy(), "forward")
    _same(orc, g_off, off_t.grad.numpy(), "grad offsets")
