"""TensorACA_rect with order="rocm" against the reference's statements run by torch-ROCm on
this GPU -- the reference's own default run (Modules_Runtime_Test.py:393, device='cuda') --
bit for bit.

The checker here is the reference itself on its default device: bench.torch_tensor_aca_rect
(the statements of Modules_Runtime_Test.py:294-302) on cuda tensors, forward and under
torch.autograd.  torch-ROCm sums every three-term reduction as ((0 + t0) + t2) + t1 (the
forward's torch.sum over the cross terms, the backward's sum_to_size over three rows;
profiles/r04/rocm_grad_probe_r04j.json); order="rocm" evaluates the same statements that way
(hg_solvers.hpp sum3<kAtenRocm>).  Pinned:
  * H for (1,), (B,1,1), (3,1) and (B,3,1) scale / div, on fractional, special-value and
    random-bit batches;
  * dL/dtar and dL/dscale, dL/ddiv for every shape: per problem ((B,1,1): three rows), none
    ((B,3,1)), and the batch-wide sums of a (1,) or (3,1) parameter, which follow ATen-ROCm's
    reduction tree (hg_sum_rocm_f32, restated in oracle/aten_rocm_sum.py).
The default order="cpu" stays the fixtures' (tests/test_gpu_rect_grad.py); the last test shows
the two orders differ on fractional inputs and agree on the reference's integer batches.
"""
import zlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B = 100_003
SPECIALS = np.array([0.0, -0.0, 1.0, -1.0, 2.0, 0.5, 3.0, 1024.0, np.inf, -np.inf, np.nan,
                     1e-45, -1.2e-40, 3e38, -3e38], np.float32)


def _same(orc, got, want, what):
    got = np.ascontiguousarray(got.detach().cpu().numpy(), np.float32)
    want = np.ascontiguousarray(want.detach().cpu().numpy(), np.float32)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    ok = orc.same_bits(got, want)
    assert ok.all(), f"{what}: {int((~ok).sum())}/{ok.size} differ; first at {np.argwhere(~ok)[:3].tolist()}"


def _batch(kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "fractional":
        s = rng.uniform(0, 160, (B, 3, 4)).astype(np.float32)
        t = rng.uniform(0, 160, (B, 3, 4)).astype(np.float32)
    elif kind == "special":
        s = rng.choice(SPECIALS, (B, 3, 4)).astype(np.float32)
        t = rng.choice(SPECIALS, (B, 3, 4)).astype(np.float32)
    else:  # random bit patterns
        s = rng.integers(0, 2**32 - 1, (B, 3, 4), dtype=np.uint32, endpoint=True).view(np.float32)
        t = rng.integers(0, 2**32 - 1, (B, 3, 4), dtype=np.uint32, endpoint=True).view(np.float32)
    if kind != "random_bits":
        s[:, 2, :] = 1.0
        t[:, 2, :] = 1.0
    g = rng.standard_normal((B, 3, 3)).astype(np.float32)
    return s, t, g, rng


def _params(shape, rng):
    if shape == "one":
        return np.array([50.0], np.float32), np.array([1.25], np.float32)
    dims = {"per_problem": (B, 1, 1), "per_row": (3, 1), "per_problem_row": (B, 3, 1)}[shape]
    return (rng.uniform(20, 160, dims).astype(np.float32),
            rng.uniform(0.5, 2.0, dims).astype(np.float32))


SHAPES = ["one", "per_problem", "per_row", "per_problem_row"]


@pytest.mark.parametrize("kind", ["fractional", "special", "random_bits"])
@pytest.mark.parametrize("shape", SHAPES)
def test_forward_equals_torch_rocm(orc, pkg, dev, kind, shape):
    import bench
    s_np, t_np, _, rng = _batch(kind, zlib.crc32(repr(("fwd", kind, shape)).encode()))
    sc_np, dv_np = _params(shape, rng)
    s, t = torch.from_numpy(s_np).to(dev), torch.from_numpy(t_np).to(dev)
    sc, dv = torch.from_numpy(sc_np).to(dev), torch.from_numpy(dv_np).to(dev)
    want = bench.torch_tensor_aca_rect(s, t, sc, dv)
    _same(orc, pkg.tensor_aca_rect(s, t, sc, dv, order="rocm"), want, f"H {kind} {shape}")
    out = torch.empty(B, 3, 3, device=dev)
    pkg.tensor_aca_rect(s, t, sc, dv, out=out, order="rocm")
    _same(orc, out, want, f"H out= {kind} {shape}")
    if shape == "one":  # Python numbers take the same path in this order
        _same(orc, pkg.tensor_aca_rect(s, t, 50.0, 1.25, order="rocm"), want, f"H numbers {kind}")
    # strided (unaligned) views take the generic kernel
    s2, t2 = (torch.cat([x.reshape(-1), x.new_zeros(1)])[1:].view(B, 3, 4) for x in (s, t))
    s2.copy_(s)
    t2.copy_(t)
    _same(orc, pkg.tensor_aca_rect(s2, t2, sc, dv, order="rocm"), want, f"H unaligned {kind} {shape}")


@pytest.mark.parametrize("kind", ["fractional", "special"])
@pytest.mark.parametrize("shape", SHAPES)
def test_backward_equals_torch_rocm_autograd(orc, pkg, dev, kind, shape):
    """dL/dtar, dL/dscale and dL/ddiv equal torch-ROCm's autograd through the statements,
    through the op's backward and through torch.autograd (B = 100 003: the one-value path's div
    terms start at an unaligned address)."""
    import bench
    s_np, t_np, g_np, rng = _batch(kind, zlib.crc32(repr(("bwd", kind, shape)).encode()))
    sc_np, dv_np = _params(shape, rng)
    s, t, gH = (torch.from_numpy(x).to(dev) for x in (s_np, t_np, g_np))
    sc, dv = torch.from_numpy(sc_np).to(dev), torch.from_numpy(dv_np).to(dev)
    tg, sg, dg = (x.clone().requires_grad_() for x in (t, sc, dv))
    bench.torch_tensor_aca_rect(s, tg, sg, dg).backward(gH)

    _, g_tar, g_sc, g_dv = pkg.tensor_aca_rect_backward(s, t, gH, sc, dv, False, True,
                                                         order="rocm")
    _same(orc, g_tar, tg.grad, f"dtar {kind} {shape}")
    # unaligned views take the generic kernels (the aligned one-value case is the staged form)
    su, tu = (torch.cat([x.reshape(-1), x.new_zeros(1)])[1:].view(B, 3, 4) for x in (s, t))
    su.copy_(s)
    tu.copy_(t)
    _, g_tar_u, g_sc_u, g_dv_u = pkg.tensor_aca_rect_backward(su, tu, gH, sc, dv, True, True,
                                                              order="rocm")
    _same(orc, g_tar_u, tg.grad, f"dtar unaligned {kind} {shape}")
    _same(orc, g_sc_u, g_sc, f"dscale unaligned {kind} {shape}")
    _same(orc, g_dv_u, g_dv, f"ddiv unaligned {kind} {shape}")
    t2, s2_, d2_ = (x.clone().requires_grad_() for x in (t, sc, dv))
    pkg.tensor_aca_rect_autograd(s, t2, s2_, d2_, order="rocm").backward(gH)
    _same(orc, t2.grad, tg.grad, f"autograd dtar {kind} {shape}")
    # the reference-signature mirror with the keyword
    t3, s3_, d3_ = (x.clone().requires_grad_() for x in (t, sc, dv))
    pkg.TensorACA_rect(B, s, t3, s3_, d3_, order="rocm").backward(gH)
    for got, want, name in ((t3.grad, tg.grad, "tar"), (s3_.grad, sg.grad, "scale"),
                            (d3_.grad, dg.grad, "div")):
        _same(orc, got, want, f"TensorACA_rect {name} {kind} {shape}")
    for got, via, want, name in ((g_sc, s2_.grad, sg.grad, "dscale"), (g_dv, d2_.grad, dg.grad, "ddiv")):
        _same(orc, via, got, f"autograd {name} {kind} {shape}")
        # every shape, the batch-wide sums of (1,) and (3,1) included (hg_sum_rocm_f32)
        _same(orc, got, want, f"{name} {kind} {shape}")


def test_orders_differ_on_fractions_and_agree_on_integers(orc, pkg, dev):
    import bench
    s_np, t_np, g_np, _ = _batch("fractional", 5)
    s, t = torch.from_numpy(s_np).to(dev), torch.from_numpy(t_np).to(dev)
    sc, dv = torch.tensor([50.0], device=dev), torch.tensor([1.25], device=dev)
    cpu_o = pkg.tensor_aca_rect(s, t, sc, dv)
    rocm_o = pkg.tensor_aca_rect(s, t, sc, dv, order="rocm")
    frac = float((cpu_o != rocm_o).float().mean())
    assert 0.05 < frac < 0.6, frac  # ~24 % on the probe's batch
    # a few float32 roundings of the cross-term sum apart, measured against each problem's
    # largest entry (single elements cancel, so an element-wise relative bound would be
    # meaningless): 1.05e-5 at most on this batch
    scale = cpu_o.abs().amax(dim=(1, 2), keepdim=True)
    assert float(((rocm_o - cpu_o).abs() / scale).max()) < 1e-4
    # the reference's own batches (integer corners and jitter): every order gives the same bits
    torch.manual_seed(3)
    _, _, src_h, tar_h, scale, div = pkg.adjust(dev, 4096)
    a = pkg.tensor_aca_rect(src_h, tar_h, scale, div)
    b = pkg.tensor_aca_rect(src_h, tar_h, scale, div, order="rocm")
    _same(orc, a, b, "integer batch, orders")
    _same(orc, b, bench.torch_tensor_aca_rect(src_h, tar_h, scale, div), "integer batch vs torch")


def test_order_argument_validated(pkg, dev):
    s = torch.zeros(4, 3, 4, device=dev)
    with pytest.raises(ValueError, match="order"):
        pkg.tensor_aca_rect(s, s, 1.0, 1.0, order="gpu")
    with pytest.raises(RuntimeError, match="order must be 0"):
        torch.ops.sks_amd.tensor_aca_rect(s, s, torch.ones(1, device=dev), torch.ones(1, device=dev), 2)
