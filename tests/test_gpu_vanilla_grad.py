"""ACA_vanilla's backward on the GPU against ATen autograd through the reference's own
statements (Modules_Runtime_Test.py:322-382), bit for bit.

The reference's ACA_vanilla is differentiable w.r.t. src and tar (ATen autograd over its
statements); `ACA_vanilla` / `aca_vanilla` / torch.ops.sks_amd.aca(normalize=False) are too,
through one HIP kernel (hg_aca_backward_f32/_f64: hg_solvers.hpp aca_vanilla_grad, the
autograd engine's order restated).

Pins:
  * tests/golden/torch_vanilla_grad.npz (tools/make_golden.py --torch-vanilla-grad: the
    reference's statements under autograd on CPU torch here), binary32 and binary64 --
    through the C ABI, the op's backward and torch.autograd, for src and tar together and
    alone, in the (B,4,2) and (B,8) layouts, aligned (LDS-staged kernel) and misaligned views
    (per-lane kernel);
  * ATen autograd through the same statements (bench.torch_aca_vanilla, pinned to the
    fixture in the CPU suite) on THIS box's CPU, 200 003 problems each of random bit patterns,
    a special-value mixture and quads over 20 decades.
Elementwise ops only (no cross product), so no CPU-capability condition applies.
"""
import zlib

import numpy as np
import pytest
import torch

from bench import torch_aca_vanilla
from conftest import default_dtype, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gold():
    return load_golden("torch_vanilla_grad.npz")


def _same(orc, got, want, what):
    got = got.detach().cpu().numpy() if torch.is_tensor(got) else np.asarray(got)
    want = np.asarray(want)
    ok = orc.same_bits(np.ascontiguousarray(got.reshape(want.shape)), np.ascontiguousarray(want))
    assert ok.all(), f"{what}: {int((~ok).sum())}/{ok.size} differ; first at {np.argwhere(~ok)[:3].tolist()}"


def test_backward_equals_reference_autograd_fixture(orc, pkg, dev, gold):
    for tag in (str(t) for t in gold["cases"]):
        src, tar, gH = (torch.from_numpy(gold[f"{tag}_{k}"]).to(dev) for k in ("src", "tar", "gH"))
        B = src.shape[0]
        ws, wt = gold[f"{tag}_gsrc"], gold[f"{tag}_gtar"]
        g_src, g_tar = pkg.aca_backward(src, tar, gH)
        _same(orc, g_src, ws, f"op grad src {tag}")
        _same(orc, g_tar, wt, f"op grad tar {tag}")
        assert g_src.shape == src.shape and g_tar.shape == tar.shape
        # one side only
        only_s, none_t = pkg.aca_backward(src, tar, gH, True, False)
        none_s, only_t = pkg.aca_backward(src, tar, gH, False, True)
        assert none_t.numel() == 0 and none_s.numel() == 0
        _same(orc, only_s, ws, f"op grad src alone {tag}")
        _same(orc, only_t, wt, f"op grad tar alone {tag}")
        # torch.autograd through the reference-API mirror (with the fixture's default dtype),
        # and the (B,8) layout
        S, T = src.clone().requires_grad_(), tar.clone().requires_grad_()
        with default_dtype(src.dtype):
            H = pkg.ACA_vanilla(B, S, T)
        _same(orc, H, gold[f"{tag}_H"], f"forward {tag}")
        H.backward(gH)
        _same(orc, S.grad, ws, f"autograd src {tag}")
        _same(orc, T.grad, wt, f"autograd tar {tag}")
        S8, T8 = src.reshape(B, 8).clone().requires_grad_(), tar.reshape(B, 8).clone().requires_grad_()
        torch.ops.sks_amd.aca(S8, T8, False).backward(gH)
        assert S8.grad.shape == (B, 8)
        _same(orc, S8.grad, ws.reshape(B, 8), f"autograd (B,8) src {tag}")
        _same(orc, T8.grad, wt.reshape(B, 8), f"autograd (B,8) tar {tag}")
        # tar alone requiring grad (the deep-homography case: a fixed source quad)
        T1 = tar.clone().requires_grad_()
        with default_dtype(src.dtype):
            H1 = pkg.ACA_vanilla(B, src, T1)
        H1.backward(gH)
        _same(orc, T1.grad, wt, f"autograd tar alone {tag}")


def test_backward_c_abi_misaligned_and_ragged(orc, oracle, pkg, dev):
    """The per-lane kernel (views one element off 16-B alignment) and ragged last waves of
    the staged kernel equal the oracle; a NULL pair and n < 0 are refused."""
    rng = np.random.default_rng(77)
    for n in (1, 63, 64, 65, 255, 257, 100_003):
        s = rng.uniform(0, 1024, (n, 8)).astype(np.float32)
        t = rng.uniform(0, 1024, (n, 8)).astype(np.float32)
        g = rng.standard_normal((n, 9)).astype(np.float32)
        ws, wt = oracle.aca_vanilla_backward(s, t, g)
        for shift in (0, 1):
            buf = torch.zeros(3, n * 9 + 8, device=dev)
            S = buf[0, shift:shift + n * 8]
            T = buf[1, shift:shift + n * 8]
            G = buf[2, shift:shift + n * 9]
            S.copy_(torch.from_numpy(s.ravel()))
            T.copy_(torch.from_numpy(t.ravel()))
            G.copy_(torch.from_numpy(g.ravel()))
            out = torch.zeros(2, n * 8 + 4, device=dev)
            gs, gt = out[0, shift:shift + n * 8], out[1, shift:shift + n * 8]
            stream = torch.cuda.current_stream(dev).cuda_stream
            pkg._lib.call("hg_aca_backward_f32", S.data_ptr(), T.data_ptr(), G.data_ptr(), n,
                          gs.data_ptr(), gt.data_ptr(), stream)
            _same(orc, gs, ws.ravel(), f"C ABI grad src n={n} shift={shift}")
            _same(orc, gt, wt.ravel(), f"C ABI grad tar n={n} shift={shift}")
    x = torch.zeros(64, device=dev)
    with pytest.raises(pkg.HipError):
        pkg._lib.call("hg_aca_backward_f32", x.data_ptr(), x.data_ptr(), x.data_ptr(), 1, None,
                      None, None)
    with pytest.raises(pkg.HipError):
        pkg._lib.call("hg_aca_backward_f32", x.data_ptr(), x.data_ptr(), x.data_ptr(), -1,
                      x.data_ptr(), None, None)


def test_normalised_form_refuses_grad_inputs(pkg, dev):
    """normalize=True (the C++ API's H / H[8], ACA_SKS.cpp:94-98) has no gradient in the
    reference: with inputs that require grad (grad mode on) the op raises, naming the
    differentiable form, rather than returning H with its graph silently cut; under
    torch.no_grad() or on detached inputs it returns H, the same bits either way."""
    src = torch.rand(8, 4, 2, device=dev, requires_grad=True)
    tar = torch.rand(8, 4, 2, device=dev)
    with pytest.raises(RuntimeError, match="normalize=False"):
        torch.ops.sks_amd.aca(src, tar, True)
    with torch.no_grad():
        H = torch.ops.sks_amd.aca(src, tar, True)
    assert H.shape == (8, 3, 3) and H.grad_fn is None and not H.requires_grad
    assert torch.equal(torch.ops.sks_amd.aca(src.detach(), tar, True), H)


B = 200_003
SPECIALS = np.array([0.0, -0.0, 1.0, -1.0, 2.0, 0.5, 3.0, 1024.0, np.inf, -np.inf, np.nan,
                     1e-45, -1.2e-40, 3e38, -3e38], np.float32)
WEIGHTS = np.array([8, 6, 8, 6, 6, 4, 4, 4, 1, 1, 1, 1, 1, 1, 1], np.float64)


def _inputs(kind, rng, shape):
    if kind == "random_bits":
        return rng.integers(0, 2**32 - 1, size=shape, dtype=np.uint32, endpoint=True).view(np.float32)
    if kind == "special_mixture":
        return rng.choice(SPECIALS, size=shape, p=WEIGHTS / WEIGHTS.sum()).astype(np.float32)
    return (rng.uniform(-1, 1, shape) * 10.0 ** rng.integers(-10, 11, (shape[0],) + (1,) * (len(shape) - 1))
            ).astype(np.float32)


@pytest.mark.parametrize("kind", ["random_bits", "special_mixture", "scaled"])
def test_backward_equals_aten_autograd_on_box_cpu(orc, pkg, dev, kind):
    rng = np.random.default_rng(zlib.crc32(kind.encode()))
    src, tar, gH = _inputs(kind, rng, (B, 4, 2)), _inputs(kind, rng, (B, 4, 2)), _inputs(kind, rng, (B, 3, 3))
    S = torch.from_numpy(src).requires_grad_()
    T = torch.from_numpy(tar).requires_grad_()
    H = torch_aca_vanilla(S, T)
    H.backward(torch.from_numpy(gH))
    ds, dt = torch.from_numpy(src).to(dev), torch.from_numpy(tar).to(dev)
    _same(orc, pkg.ACA_vanilla(B, ds, dt), H.detach().numpy(), f"forward {kind}")
    g_src, g_tar = pkg.aca_backward(ds, dt, torch.from_numpy(gH).to(dev))
    _same(orc, g_src, S.grad.numpy(), f"grad src {kind}")
    _same(orc, g_tar, T.grad.numpy(), f"grad tar {kind}")


@pytest.mark.parametrize("kind", ["scaled", "random_bits", "special_mixture"])
def test_backward_f64_equals_aten_autograd_on_box_cpu(orc, pkg, dev, kind):
    rng = np.random.default_rng(zlib.crc32(("f64" + kind).encode()))
    n = 100_003

    def draw(shape):
        if kind == "random_bits":
            return rng.integers(0, 2**64 - 1, size=shape, dtype=np.uint64, endpoint=True).view(np.float64)
        if kind == "special_mixture":
            return rng.choice(SPECIALS.astype(np.float64), size=shape, p=WEIGHTS / WEIGHTS.sum())
        return rng.uniform(-512, 512, shape) * 10.0 ** rng.integers(-6, 7, (shape[0],) + (1,) * (len(shape) - 1))

    src, tar, gH = draw((n, 4, 2)), draw((n, 4, 2)), draw((n, 3, 3))
    S, T = torch.from_numpy(src).requires_grad_(), torch.from_numpy(tar).requires_grad_()
    with default_dtype(torch.float64):
        H = torch_aca_vanilla(S, T)
    H.backward(torch.from_numpy(gH))
    g_src, g_tar = pkg.aca_backward(torch.from_numpy(src).to(dev), torch.from_numpy(tar).to(dev),
                                    torch.from_numpy(gH).to(dev))
    _same(orc, g_src, S.grad.numpy(), f"f64 grad src {kind}")
    _same(orc, g_tar, T.grad.numpy(), f"f64 grad tar {kind}")


def test_binary64_inputs_under_the_float32_default(orc, pkg, dev, gold):
    """The reference's statements write into torch.ones((bs, 9)) -- torch's default dtype
    (.py:372) -- so binary64 inputs under the float32 default give a float32 H (each binary64
    value rounded once) and binary64 gradients of a float32 upstream gradient.  ACA_vanilla does
    the same, and its gradients equal ATen autograd's through the statements on the CPU."""
    tag = "f64_uniform"
    src, tar = (torch.from_numpy(gold[f"{tag}_{k}"]) for k in ("src", "tar"))
    B = src.shape[0]
    g32 = torch.from_numpy(gold[f"{tag}_gH"].astype(np.float32))
    S, T = src.clone().requires_grad_(), tar.clone().requires_grad_()
    H = torch_aca_vanilla(S, T)  # the float32 default
    assert H.dtype is torch.float32
    H.backward(g32)
    Sd, Td = src.to(dev).requires_grad_(), tar.to(dev).requires_grad_()
    Hd = pkg.ACA_vanilla(B, Sd, Td)
    assert Hd.dtype is torch.float32
    _same(orc, Hd, H.detach().numpy(), "forward, f32 default")
    Hd.backward(g32.to(dev))
    _same(orc, Sd.grad, S.grad.numpy(), "grad src, f32 default")
    _same(orc, Td.grad, T.grad.numpy(), "grad tar, f32 default")


@pytest.mark.parametrize("kind", ["random_bits", "special_mixture", "scaled"])
def test_equals_the_reference_statements_run_on_this_gpu(orc, pkg, dev, kind):
    """The reference runs its statements with device='cuda' (.py:393): ACA_vanilla's are
    element-wise products and differences only, so ROCm's ATen evaluates them exactly as the
    CPU does, and autograd sums the same terms in the same order -- forward and both gradients
    equal the op's bit for bit on the GPU itself (unlike TensorACA_rect, whose torch.sum order
    differs on ROCm: tests/test_gpu_parity.py)."""
    rng = np.random.default_rng(zlib.crc32(("gpu" + kind).encode()))
    src, tar, gH = (torch.from_numpy(_inputs(kind, rng, sh)).to(dev) for sh in ((B, 4, 2), (B, 4, 2), (B, 3, 3)))
    S, T = src.clone().requires_grad_(), tar.clone().requires_grad_()
    H = torch_aca_vanilla(S, T)
    H.backward(gH)
    S2, T2 = src.clone().requires_grad_(), tar.clone().requires_grad_()
    H2 = pkg.ACA_vanilla(B, S2, T2)
    H2.backward(gH)
    _same(orc, H2, H.detach().cpu().numpy(), f"forward {kind}")
    _same(orc, S2.grad, S.grad.cpu().numpy(), f"grad src {kind}")
    _same(orc, T2.grad, T.grad.cpu().numpy(), f"grad tar {kind}")
