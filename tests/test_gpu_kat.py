"""The Matlab camera-model KAT (Matlab Codes/veri_4Pts.m) on the GPU.

Quad case (veri_4Pts.m:9-53) through every general solver, and the rectangle case
(veri_4Pts.m:82-95: w = 50, h = 40, M = (36, 81)) through the TensorACA forms:
hg_tensor_aca_rect_f32 with device scalars, with host scalars, and the compact
hg_tensor_aca_offsets_f32.  Each result equals the oracle bit for bit and, normalised,
lies within 1e-5 (normwise) of H_real_norm."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _normwise(H, Hn):
    H = np.asarray(H, np.float64).reshape(3, 3)
    H = (H / H[2, 2]).reshape(9)
    return np.linalg.norm(H - Hn) / np.linalg.norm(Hn)


def test_kat_quad_gpu(orc, oracle, pkg, dev):
    g = load_golden("kat_veri4pts.npz")
    Hn = g["H_real_norm"].reshape(9)
    s32 = torch.from_numpy(g["src_f32"]).to(dev)
    t32 = torch.from_numpy(g["tar_f32"]).to(dev)
    s64 = torch.from_numpy(g["src"]).to(dev)
    t64 = torch.from_numpy(g["tar"]).to(dev)
    for algo in ("aca", "sks"):
        h32 = pkg.solve(algo, s32, t32).cpu().numpy()
        assert orc.same_bits(h32, g[f"{algo}_f32"]).all()
        assert _normwise(h32, Hn) < 1e-6
        h64 = pkg.solve(algo, s64, t64).cpu().numpy()
        assert orc.same_bits(h64, oracle.solve(algo, g["src"], g["tar"])).all()
        np.testing.assert_allclose(h64[0], Hn, rtol=1e-9, atol=1e-12)


def _rect_case():
    g = load_golden("kat_veri4pts.npz")
    w, h, mx, my = (float(x) for x in g["rect_whm"])
    src = np.vstack([g["rect_src"].T, np.ones(4)])[None].astype(np.float32)  # (1,3,4)
    tar = np.vstack([g["rect_tar"].T, np.ones(4)])[None].astype(np.float32)
    return g, w, h, mx, my, src, tar


def test_kat_rect_gpu(orc, oracle, pkg, dev):
    g, w, h, mx, my, src, tar = _rect_case()
    Hn = g["H_real_norm"].reshape(9)
    div = float(np.float32(w) / np.float32(h))
    want = oracle.tensor_aca_rect(src, tar, w, div)
    assert _normwise(want[0], Hn) < 1e-5
    lib = pkg.lib()
    stream = torch.cuda.current_stream(dev).cuda_stream
    ds = torch.from_numpy(src).to(dev)
    dt = torch.from_numpy(tar).to(dev)
    sc = torch.tensor([w], dtype=torch.float32, device=dev)
    dv = torch.tensor([div], dtype=torch.float32, device=dev)
    H1 = torch.full((1, 3, 3), -1.0, device=dev)
    H2 = torch.full((1, 3, 3), -1.0, device=dev)
    assert lib.hg_tensor_aca_rect_f32(ds.data_ptr(), dt.data_ptr(), H1.data_ptr(), 1, sc.data_ptr(),
                                      dv.data_ptr(), stream) == 0
    assert lib.hg_tensor_aca_rect_f32_hostscalar(ds.data_ptr(), dt.data_ptr(), H2.data_ptr(), 1, w,
                                                 div, stream) == 0
    torch.cuda.synchronize(dev)
    for H in (H1, H2):
        got = H.cpu().numpy()
        assert orc.same_bits(got, want).all(), (got, want)
        assert _normwise(got[0], Hn) < 1e-5
    # the torch op and the reference-named wrapper reach the same kernel
    H3 = pkg.TensorACA_rect(1, ds, dt, sc, dv)
    assert orc.same_bits(H3.cpu().numpy(), want).all()


def test_kat_rect_compact_offsets_gpu(orc, oracle, pkg, dev):
    """The rectangle KAT in the deep-homography 4-offset form: corner M and the four
    predicted corner offsets (tar - src, float32); the kernel rebuilds the target with
    float adds, so the oracle is run on the same assembled tensors."""
    g, w, h, mx, my, src, tar = _rect_case()
    Hn = g["H_real_norm"].reshape(9)
    np.testing.assert_array_equal(src[0, 0], [mx, mx + w, mx, mx + w])
    np.testing.assert_array_equal(src[0, 1], [my, my, my + h, my + h])
    offs = np.ascontiguousarray((tar[0, :2, :] - src[0, :2, :]).T, np.float32)[None]  # (1,4,2)
    corner = np.array([[mx, my]], np.float32)
    tar_rebuilt = src.copy()
    tar_rebuilt[0, :2, :] = src[0, :2, :] + offs[0].T
    div = float(np.float32(w) / np.float32(h))
    want = oracle.tensor_aca_rect(src, tar_rebuilt, w, div)
    H = pkg.tensor_aca_offsets(torch.from_numpy(corner).to(dev), torch.from_numpy(offs).to(dev), w, h)
    got = H.cpu().numpy()
    assert orc.same_bits(got, want).all(), (got, want)
    assert _normwise(got[0], Hn) < 1e-5
    # raw C ABI as well
    lib = pkg.lib()
    Hc = torch.full((1, 3, 3), -1.0, device=dev)
    dc = torch.from_numpy(corner).to(dev)
    do = torch.from_numpy(offs).to(dev)
    assert lib.hg_tensor_aca_offsets_f32(dc.data_ptr(), do.data_ptr(), Hc.data_ptr(), 1, w, h,
                                         torch.cuda.current_stream(dev).cuda_stream) == 0
    torch.cuda.synchronize(dev)
    assert orc.same_bits(Hc.cpu().numpy(), want).all()


@pytest.mark.parametrize("B", [1, 65, 4099])
def test_kat_rect_replicated(orc, oracle, pkg, dev, B):
    """The KAT rectangle replicated B times (full tiles and ragged tails of the vector
    kernel): every row equals the single problem's bits."""
    g, w, h, mx, my, src, tar = _rect_case()
    div = float(np.float32(w) / np.float32(h))
    want = oracle.tensor_aca_rect(src, tar, w, div)
    ds = torch.from_numpy(np.repeat(src, B, 0)).to(dev)
    dt = torch.from_numpy(np.repeat(tar, B, 0)).to(dev)
    H = pkg.ops.tensor_aca_rect(ds, dt, w, div)
    got = H.cpu().numpy()
    assert orc.same_bits(got, np.repeat(want, B, 0)).all()
