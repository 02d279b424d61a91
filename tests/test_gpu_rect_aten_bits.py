"""TensorACA_rect on the GPU against the reference's own ATen composition run on the CPU of the
same box, bit for bit, on inputs well beyond the fixtures: random binary32 bit patterns, a
special-value mixture (signed zeros, +-Inf, NaN, subnormals, near-overflow) and quads over 20
decades of scale, with ordinary, fractional and infinite rectangle scalars.

The composition is `bench.torch_tensor_aca_rect`, the seven statements of
Modules_Runtime_Test.py:294-302 (torch.zeros, the d / cross / sum / three slice writes).  On
an AVX-512 host ATen's CPU cross contracts to FMA, which is what the kernel reproduces
(DESIGN.md section 2); on a host without AVX-512 ATen takes another path and the test is
skipped rather than weakened.  Bar: every bit, every NaN equal to every NaN.
"""
import zlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B = 200_003
SPECIALS = np.array([0.0, -0.0, 1.0, -1.0, 2.0, 0.5, 3.0, 1024.0, np.inf, -np.inf, np.nan,
                     1e-45, -1.2e-40, 3e38, -3e38], np.float32)
WEIGHTS = np.array([8, 6, 8, 6, 6, 4, 4, 4, 1, 1, 1, 1, 1, 1, 1], np.float64)


def _inputs(kind, rng):
    if kind == "random_bits":
        return tuple(rng.integers(0, 2**32 - 1, size=(B, 3, 4), dtype=np.uint32, endpoint=True)
                     .view(np.float32) for _ in range(2))
    if kind == "special_mixture":
        p = WEIGHTS / WEIGHTS.sum()
        return tuple(rng.choice(SPECIALS, size=(B, 3, 4), p=p).astype(np.float32) for _ in range(2))
    return tuple((rng.uniform(-1, 1, (B, 3, 4)) * 10.0 ** rng.integers(-10, 11, (B, 1, 1)))
                 .astype(np.float32) for _ in range(2))


@pytest.mark.parametrize("kind", ["random_bits", "special_mixture", "scaled"])
@pytest.mark.parametrize("scale,div", [(128.0, 1.0), (50.0, 1.25), (float("inf"), 0.5)])
def test_rect_equals_aten_cpu_composition(orc, pkg, dev, kind, scale, div):
    if not orc.cpu_has_avx512():
        pytest.skip("ATen's CPU cross takes its AVX-512 FMA path only on an AVX-512 host")
    import bench
    rng = np.random.default_rng(zlib.crc32(repr((kind, scale, div)).encode()))
    src, tar = (np.ascontiguousarray(a) for a in _inputs(kind, rng))
    sc, dv = torch.tensor([scale], dtype=torch.float32), torch.tensor([div], dtype=torch.float32)
    want = bench.torch_tensor_aca_rect(torch.from_numpy(src), torch.from_numpy(tar), sc, dv).numpy()
    ds, dt = torch.from_numpy(src).to(dev), torch.from_numpy(tar).to(dev)
    for what, got in (
            ("device scalars", pkg.TensorACA_rect(B, ds, dt, sc.to(dev), dv.to(dev))),
            ("host scalars", pkg.TensorACA_rect(B, ds, dt, scale, div))):
        got = got.cpu().numpy()
        ok = orc.same_bits(got, want)
        bad = np.flatnonzero(~ok)
        if not ok.all():
            i = bad[0] // 9
            raise AssertionError(
                f"{kind} scale={scale} div={div} {what}: {bad.size}/{ok.size} differ; first at "
                f"problem {i}, element {bad[0] % 9}: got {got[i].ravel().tolist()} want "
                f"{want[i].ravel().tolist()} src {src[i].ravel().view(np.uint32).tolist()} "
                f"tar {tar[i].ravel().view(np.uint32).tolist()}")


@pytest.mark.parametrize("tag,scale,div", [("128_1", 128.0, 1.0), ("50_125", 50.0, 1.25),
                                           ("inf_05", float("inf"), 0.5)])
def test_rect_and_vanilla_equal_reference_special_fixture(orc, pkg, dev, tag, scale, div):
    """tests/golden/torch_special.npz -- the reference's own TensorACA_rect and ACA_vanilla
    statements executed on CPU torch here (tools/make_golden.py --torch-special) over special
    values, problem 0 an all-(-0) cross product -- through both scalar forms and ACA_vanilla."""
    from conftest import load_golden
    g = load_golden("torch_special.npz")
    B = g["rect_src"].shape[0]
    ds, dt = torch.from_numpy(g["rect_src"]).to(dev), torch.from_numpy(g["rect_tar"]).to(dev)
    sc = torch.tensor([scale], dtype=torch.float32, device=dev)
    dv = torch.tensor([div], dtype=torch.float32, device=dev)
    for what, got in (("device scalars", pkg.TensorACA_rect(B, ds, dt, sc, dv)),
                      ("host scalars", pkg.TensorACA_rect(B, ds, dt, scale, div))):
        ok = orc.same_bits(got.cpu().numpy(), g[f"rect_{tag}"])
        assert ok.all(), f"{tag} {what}: {int((~ok).sum())} differ"
    H = pkg.ACA_vanilla(B, torch.from_numpy(g["van_src"]).to(dev), torch.from_numpy(g["van_tar"]).to(dev))
    ok = orc.same_bits(H.cpu().numpy(), g["vanilla"])
    assert ok.all(), f"ACA_vanilla: {int((~ok).sum())} differ"


def test_scale_and_div_shapes_the_reference_refuses(pkg, dev):
    """A (2,) scale or div does not broadcast to the (B,3,1) column it scales, so the
    reference's own composition refuses it (.py:301-302); so do the op and its backward (the
    accepted broadcast shapes are tests/test_gpu_rect_bcast.py's)."""
    torch.manual_seed(0)
    _, _, sh, th, sc, dv = pkg.adjust(dev, 16)
    assert pkg.TensorACA_rect(16, sh, th, sc, dv).shape == (16, 3, 3)
    two = torch.tensor([128.0, 64.0], device=dev)
    for bad_scale, bad_div in ((two, dv), (sc, two), (torch.tensor([128.0, 64.0]), 1.0)):
        with pytest.raises((RuntimeError, ValueError)):
            pkg.TensorACA_rect(16, sh, th, bad_scale, bad_div)
    with pytest.raises((RuntimeError, ValueError)):
        pkg.tensor_aca_rect_backward(sh, th, torch.ones((16, 3, 3), device=dev), two, dv)
