"""Compact TensorACA (corner + 4 offsets): forward bit-exact against
the oracle's TensorACA_rect on the equivalently-built (B,3,4) tensors; backward
bit-exact against the oracle gradient mapped to offsets; autograd close to float64."""
import numpy as np
import pytest
import torch

from test_gpu_parity import _bits

pytestmark = pytest.mark.gpu


def _build_h(corner, offsets, w, h):
    """(B,3,4) src/tar exactly as getInput/getTar/adjust build them (float32 adds)."""
    c = corner.astype(np.float32)
    o = offsets.reshape(-1, 4, 2).astype(np.float32)
    w, h = np.float32(w), np.float32(h)
    sx = np.stack([c[:, 0], c[:, 0] + w, c[:, 0], c[:, 0] + w], 1)
    sy = np.stack([c[:, 1], c[:, 1], c[:, 1] + h, c[:, 1] + h], 1)
    ones = np.ones_like(sx)
    src = np.stack([sx, sy, ones], 1)
    tar = np.stack([sx + o[:, :, 0], sy + o[:, :, 1], ones], 1)
    return src.astype(np.float32), tar.astype(np.float32)


@pytest.mark.parametrize("B", [1, 127, 128, 129, 4096, 100_001])
@pytest.mark.parametrize("wh", [(128.0, 128.0), (50.0, 40.0)])
def test_offsets_forward_backward_vs_oracle(orc, oracle, pkg, dev, B, wh):
    w, h = wh
    g = torch.Generator(device=dev).manual_seed(B)
    corner = (torch.rand(B, 2, device=dev, generator=g) * 20 + 10).floor() + 0.25
    offsets = torch.rand(B, 4, 2, device=dev, generator=g) * 32
    H = pkg.tensor_aca_offsets(corner, offsets, w, h)
    src, tar = _build_h(corner.cpu().numpy(), offsets.cpu().numpy(), w, h)
    div = float(np.float32(w) / np.float32(h))
    want = oracle.tensor_aca_rect(src, tar, w, div)
    ok = orc.same_bits(H.cpu().numpy(), want)
    assert ok.all(), f"{(~ok).sum()} differ"
    gH = torch.randn(B, 3, 3, device=dev, generator=g)
    g_off, g_cor = pkg.tensor_aca_offsets_backward(corner, offsets, gH, w, h, True)
    ws, wt, _ = oracle.tensor_aca_rect_backward(src, tar, gH.cpu().numpy(), w, div)
    want_off = np.stack([wt[:, 0, :], wt[:, 1, :]], 2)  # (B,4,2)
    assert orc.same_bits(g_off.cpu().numpy(), want_off).all()
    want_cx = ws[:, 0, 0] + (((wt[:, 0, 0] + wt[:, 0, 1]) + wt[:, 0, 2]) + wt[:, 0, 3])
    want_cy = ws[:, 1, 0] + (((wt[:, 1, 0] + wt[:, 1, 1]) + wt[:, 1, 2]) + wt[:, 1, 3])
    assert orc.same_bits(g_cor.cpu().numpy(), np.stack([want_cx, want_cy], 1)).all()


def test_offsets_unaligned_views(orc, oracle, pkg, dev):
    B = 3001
    corner = torch.rand(B, 2, device=dev) * 20
    offsets = torch.rand(B, 4, 2, device=dev) * 32
    cbig = torch.zeros(B * 2 + 1, device=dev)
    cbig[1:] = corner.reshape(-1)
    obig = torch.zeros(B * 8 + 1, device=dev)
    obig[1:] = offsets.reshape(-1)
    H = pkg.tensor_aca_offsets(cbig[1:].view(B, 2), obig[1:].view(B, 4, 2), 128.0, 128.0)
    assert torch.equal(H, pkg.tensor_aca_offsets(corner, offsets, 128.0, 128.0))


def test_offsets_autograd_vs_float64(pkg, dev):
    B = 2048
    corner = (torch.rand(B, 2, device=dev) * 20 + 10).requires_grad_()
    offsets = (torch.rand(B, 4, 2, device=dev) * 32).requires_grad_()
    H = torch.ops.sks_amd.tensor_aca_offsets(corner, offsets, 50.0, 40.0)
    gH = torch.randn(B, 3, 3, device=dev)
    H.backward(gH)
    c64 = corner.detach().double().requires_grad_()
    o64 = offsets.detach().double().requires_grad_()
    w, h = 50.0, 40.0
    sx = torch.stack([c64[:, 0], c64[:, 0] + w, c64[:, 0], c64[:, 0] + w], 1)
    sy = torch.stack([c64[:, 1], c64[:, 1], c64[:, 1] + h, c64[:, 1] + h], 1)
    ones = torch.ones_like(sx)
    src = torch.stack([sx, sy, ones], 1)
    tar = torch.stack([sx + o64[:, :, 0], sy + o64[:, :, 1], ones], 1)
    from test_oracle_golden import _functional_rect
    _functional_rect(src, tar, w, w / h).backward(gH.double())

    def rel(a, b):
        return ((a.double() - b).abs().max() / b.abs().max()).item()

    assert rel(offsets.grad, o64.grad) < 1e-5
    assert rel(corner.grad, c64.grad) < 1e-4


@pytest.mark.parametrize("wh", [(128.0, 128.0), (64.0, 64.0), (0.0, 0.0), (np.inf, np.inf),
                                (96.0, 64.0)])
def test_square_specialisation_same_bits(orc, oracle, pkg, dev, wh):
    """ACA_rect.m:28's square case (ratio 1, no multiply by div) is dispatched on the host
    when width == height (compact form) or div == 1.0 (host-scalar rect form); it must give
    the general form's bits, and 0/0 or inf/inf ratios (NaN) must stay on the general path."""
    w, h = wh
    B = 4096 + 37
    g = torch.Generator(device=dev).manual_seed(5)
    corner = (torch.rand(B, 2, device=dev, generator=g) * 20 + 10).floor()
    offsets = (torch.rand(B, 4, 2, device=dev, generator=g) * 32).floor()
    H = pkg.tensor_aca_offsets(corner, offsets, w, h)
    src, tar = _build_h(corner.cpu().numpy(), offsets.cpu().numpy(), w, h)
    with np.errstate(invalid="ignore"):
        div = float(np.float32(w) / np.float32(h))
    want = oracle.tensor_aca_rect(src, tar, w, div)
    assert orc.same_bits(H.cpu().numpy(), want).all()
    # rect form: host scalars (square path when div == 1) vs device scalars (general path)
    s_d, t_d = torch.from_numpy(src).to(dev), torch.from_numpy(tar).to(dev)
    Hh = pkg.tensor_aca_rect(s_d, t_d, w, div)
    Hd = pkg.tensor_aca_rect(s_d, t_d, torch.tensor([w], device=dev),
                             torch.tensor([div], device=dev))
    assert orc.same_bits(Hh.cpu().numpy(), Hd.cpu().numpy()).all()
    assert orc.same_bits(Hh.cpu().numpy(), want).all()


def test_native_ops_pass_torch_opcheck(pkg, dev):
    """torch.library.opcheck over the native operators (csrc/hg_torch_ops.cpp): schema,
    Meta/fake-tensor kernels, autograd registration and AOT dispatch agree with the real
    GPU kernels."""
    B = 1000
    torch.manual_seed(0)
    _, _, src, tar, scale, div = pkg.adjust(dev, B)
    corner = src[:, 0:2, 0].contiguous()
    offs = (tar[:, 0:2, :] - src[:, 0:2, :]).transpose(1, 2).contiguous()
    ops = torch.ops.sks_amd
    tests = ("test_schema", "test_autograd_registration", "test_faketensor",
             "test_aot_dispatch_dynamic")
    offs_g = offs.clone().requires_grad_(True)
    tar_g = tar.clone().requires_grad_(True)
    torch.library.opcheck(ops.tensor_aca_offsets.default, (corner, offs_g, 128.0, 128.0),
                          test_utils=tests)
    torch.library.opcheck(ops.tensor_aca_rect.default, (src, tar_g, scale, div), test_utils=tests)
    # the torch-ROCm evaluation order (int order=1), and its backward op with a per-problem scale
    torch.library.opcheck(ops.tensor_aca_rect.default, (src, tar_g, scale, div, 1), test_utils=tests)
    torch.library.opcheck(ops.tensor_aca_rect_backward.default,
                          (src, tar, torch.randn(B, 3, 3, device=dev), torch.full((B, 1, 1), 128.0,
                           device=dev), div, True, True, 0, 1),
                          test_utils=("test_schema", "test_faketensor"))
    q = torch.rand(B, 4, 2, device=dev) * 100
    torch.library.opcheck(ops.aca.default, (q, q + 1.5, True),
                          test_utils=("test_schema", "test_faketensor"))
    # ACA_vanilla's differentiable form (normalize=False), float32 and float64
    for dt in (torch.float32, torch.float64):
        qg = q.to(dt).clone().requires_grad_(True)
        torch.library.opcheck(ops.aca.default, (qg, (q + 1.5).to(dt), False), test_utils=tests)
        torch.library.opcheck(ops.aca_backward.default,
                              (q.to(dt), (q + 1.5).to(dt), torch.randn(B, 3, 3, device=dev, dtype=dt),
                               True, True), test_utils=("test_schema", "test_faketensor"))
    torch.library.opcheck(ops.sks.default, (q, q + 1.5, False),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))
    # the host-scalar overload: differentiable in src and tar (scale / div are constants)
    tar_s = tar.clone().requires_grad_(True)
    torch.library.opcheck(ops.tensor_aca_rect.scalar, (src, tar_s, 128.0, 1.0), test_utils=tests)


def test_autograd_refusals_and_constants(orc, pkg, dev):
    """Every native op answers inputs that require grad explicitly, with one policy: the
    forms the reference never differentiates -- sks_amd::sks, aca with normalize=True and
    solve (the C++ API's forms) -- raise naming the missing backward while grad mode is on,
    and run as inference under torch.no_grad() or on detached inputs; the scalar TensorACA
    overload gives src / tar the tensor overload's gradients bit for bit."""
    ops = torch.ops.sks_amd
    q = (torch.rand(64, 4, 2, device=dev) * 100).requires_grad_(True)
    t = q.detach() + 1.5
    with pytest.raises(RuntimeError, match="sks_amd::sks has no backward"):
        ops.sks.default(q, t, False)
    with pytest.raises(RuntimeError, match="normalize=True .* has no backward"):
        ops.aca.default(q, t, True)
    with pytest.raises(RuntimeError, match="sks_amd::solve has no backward"):
        ops.solve.default(q.view(64, 8), t.view(64, 8), 1, True, 0)
    with torch.no_grad():
        assert ops.sks.default(q, t, False).shape == (64, 3, 3)
        H = ops.aca.default(q, t, True)
        Hs = ops.solve.default(q.view(64, 8), t.view(64, 8), 1, True, 0)
    assert ops.sks.default(q.detach(), t, True).grad_fn is None
    assert H.grad_fn is None and not H.requires_grad
    assert Hs.grad_fn is None and not Hs.requires_grad
    _bits(orc, H, ops.aca.default(q.detach(), t, True).cpu().numpy(), "aca normalize=True, no_grad")
    B = 777
    torch.manual_seed(1)
    _, _, sh, th, sc, dv = pkg.adjust(dev, B)
    th = th + torch.rand_like(th)
    gH = torch.randn(B, 3, 3, device=dev)
    t1, t2 = th.clone().requires_grad_(True), th.clone().requires_grad_(True)
    s1, s2 = sh.clone().requires_grad_(True), sh.clone().requires_grad_(True)
    ops.tensor_aca_rect.scalar(s1, t1, 128.0, 1.0).backward(gH)
    ops.tensor_aca_rect.default(s2, t2, torch.tensor([128.0], device=dev),
                                torch.tensor([1.0], device=dev)).backward(gH)
    _bits(orc, t1.grad, t2.grad.cpu().numpy(), "scalar overload dL/dtar")
    _bits(orc, s1.grad, s2.grad.cpu().numpy(), "scalar overload dL/dsrc")


def test_fit_offsets_example(pkg, dev):
    """examples/fit_offsets.py: gradient descent through the compact TensorACA op and its
    HIP backward recovers known corner offsets (the deep-homography training signal)."""
    import importlib.util
    import os
    from conftest import ROOT
    spec = importlib.util.spec_from_file_location("fit_offsets",
                                                  os.path.join(ROOT, "examples", "fit_offsets.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.fit(batch=2048, steps=300) < 0.5


def test_rect_and_offsets_edge_values_vs_oracle(orc, oracle, pkg, dev):
    """Degenerate and extreme TensorACA inputs (coincident corners, zero-area targets,
    +-Inf, NaN, 1e30, subnormals) propagate exactly as the restatement of the reference
    statements does (no guards), forward and backward."""
    rng = np.random.default_rng(3)
    B = 4096 + 13
    corner = np.floor(rng.uniform(10, 30, (B, 2))).astype(np.float32)
    offs = rng.uniform(-16, 16, (B, 4, 2)).astype(np.float32)
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e30, -1e30, 1e-40, -128.0],
                        np.float32)
    for i in range(0, B, 7):  # sprinkle special values into offsets and corners
        offs[i, rng.integers(0, 4), rng.integers(0, 2)] = specials[i % len(specials)]
        if i % 5 == 0:
            corner[i, rng.integers(0, 2)] = specials[(i // 5) % len(specials)]
    offs[1] = -np.array([[0, 0], [128, 0], [0, 128], [128, 128]], np.float32)  # all corners -> M
    dc, do = torch.from_numpy(corner).to(dev), torch.from_numpy(offs).to(dev)
    for w, h in ((128.0, 128.0), (64.0, 48.0)):
        src, tar = _build_h(corner, offs, w, h)
        div = float(np.float32(w) / np.float32(h))
        want = oracle.tensor_aca_rect(src, tar, w, div)
        assert orc.same_bits(pkg.tensor_aca_offsets(dc, do, w, h).cpu().numpy(), want).all()
        Hr = pkg.tensor_aca_rect(torch.from_numpy(src).to(dev), torch.from_numpy(tar).to(dev), w, div)
        assert orc.same_bits(Hr.cpu().numpy(), want).all()
        gH = torch.from_numpy(rng.standard_normal((B, 3, 3)).astype(np.float32)).to(dev)
        g_off, _ = pkg.tensor_aca_offsets_backward(dc, do, gH, w, h, True)
        _, wt, _ = oracle.tensor_aca_rect_backward(src, tar, gH.cpu().numpy(), w, div)
        assert orc.same_bits(g_off.cpu().numpy(), np.stack([wt[:, 0, :], wt[:, 1, :]], 2)).all()
