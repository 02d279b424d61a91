"""Pins the oracle (oracle/hg_oracle.c) against fixtures produced by the reference
itself (tools/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from conftest import load_golden


def _assert_bits(orc, got, want, what):
    ok = orc.same_bits(got, want)
    assert ok.all(), f"{what}: {int((~ok).sum())}/{ok.size} elements differ; first at " \
                     f"{np.argwhere(~ok)[:3].tolist()}"


@pytest.mark.parametrize("algo", ["aca", "sks"])
def test_oracle_vs_reference_cpp_uniform(orc, oracle, algo):
    g = load_golden("cpp_uniform.npz")
    _assert_bits(orc, oracle.solve(algo, g["src_f32"], g["tar_f32"]), g[f"{algo}_f32"],
                 f"{algo} f32")
    _assert_bits(orc, oracle.solve(algo, g["src_f64"], g["tar_f64"]), g[f"{algo}_f64"],
                 f"{algo} f64")


@pytest.mark.parametrize("algo", ["aca", "sks"])
def test_oracle_vs_reference_cpp_wall(orc, oracle, algo):
    g = load_golden("cpp_wall.npz")
    _assert_bits(orc, oracle.solve(algo, g["src"], g["tar"]), g[algo], f"{algo} wall")


@pytest.mark.parametrize("algo", ["aca", "sks"])
def test_oracle_vs_reference_cpp_edge(orc, oracle, algo):
    g = load_golden("cpp_edge.npz")
    _assert_bits(orc, oracle.solve(algo, g["src"], g["tar"]), g[algo], f"{algo} edge f32")
    _assert_bits(orc, oracle.solve(algo, g["src_f64"], g["tar_f64"]), g[f"{algo}_f64"],
                 f"{algo} edge f64")


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_oracle_vs_compiled_reference_random(orc, oracle, dtype):
    """Where the reference was compiled (oracle/_ref, built from /root/reference),
    the restatement must equal it on fresh random quads too."""
    if not orc.RefOracle.available():
        pytest.skip("oracle/_ref not built here")
    ref = orc.RefOracle()
    rng = np.random.default_rng(123)
    n = 200_000
    s = rng.uniform(-3000, 3000, (n, 8)).astype(dtype)
    t = rng.uniform(-3000, 3000, (n, 8)).astype(dtype)
    for algo in ("aca", "sks"):
        _assert_bits(orc, oracle.solve(algo, s, t), ref.solve(algo, s, t), f"{algo} {dtype}")


def test_oracle_soa_equals_aos(orc, oracle):
    g = load_golden("cpp_uniform.npz")
    for algo in ("aca", "sks"):
        aos = oracle.solve(algo, g["src_f32"], g["tar_f32"], normalize=False)
        soa = oracle.solve(algo, g["src_f32"].T.copy(), g["tar_f32"].T.copy(), normalize=False,
                           layout="soa")
        _assert_bits(orc, soa.T, aos, f"{algo} soa")


def test_oracle_unnormalised_vs_reference_aca_vanilla(orc, oracle):
    """ACA_vanilla (Modules_Runtime_Test.py:312-388) is the unnormalised ACA."""
    g = load_golden("torch_tensor_aca.npz")
    for tag in ("int", "f"):
        src = g[f"{tag}_src"].reshape(-1, 8)
        tar = g[f"{tag}_tar"].reshape(-1, 8)
        got = oracle.solve("aca", src, tar, normalize=False)
        _assert_bits(orc, got, g[f"{tag}_vanilla"].reshape(-1, 9), f"ACA_vanilla {tag}")


@pytest.mark.parametrize("tag", ["uniform", "wall", "edge"])
def test_oracle_unnormalised_f64_vs_reference_aca_vanilla_f64(orc, oracle, tag):
    """Unnormalised binary64 ACA -- cal_Homo_ACA's contract (GPU_Runtime Test.cu:81-151) --
    pinned by reference output: ACA_vanilla's own statements executed on float64 CPU tensors
    (tests/golden/torch_aca_f64.npz).  The same fixture normalised the C++ way
    (ACA_SKS.cpp:94-98) equals the compiled reference's runKernel_ACA_double, so two
    reference artifacts agree on these bits."""
    g = load_golden("torch_aca_f64.npz")
    src, tar = g[f"{tag}_src"].reshape(-1, 8), g[f"{tag}_tar"].reshape(-1, 8)
    want = g[f"{tag}_H"].reshape(-1, 9)
    _assert_bits(orc, oracle.solve("aca", src, tar, normalize=False), want, f"f64 {tag}")
    _assert_bits(orc, oracle.solve("aca", np.ascontiguousarray(src.T), np.ascontiguousarray(tar.T),
                                   normalize=False, layout="soa").T, want, f"f64 {tag} soa")
    if orc.RefOracle.available():
        norm = want.copy()
        with np.errstate(divide="ignore", invalid="ignore"):
            r = 1.0 / norm[:, 8]
            norm[:, :8] *= r[:, None]
        norm[:, 8] = 1.0
        _assert_bits(orc, norm, orc.RefOracle().solve("aca", src, tar), f"f64 {tag} vs C++")


@pytest.mark.parametrize("key,scale,div", [("int_rect", None, None), ("f_rect", 128.0, 1.0),
                                           ("f_rect_div125", 50.0, 1.25)])
def test_oracle_vs_reference_tensor_aca_rect(orc, oracle, key, scale, div):
    g = load_golden("torch_tensor_aca.npz")
    tag = key.split("_")[0]
    if scale is None:
        scale, div = float(g["int_scale"][0]), float(g["int_div"][0])
    got = oracle.tensor_aca_rect(g[f"{tag}_src_h"], g[f"{tag}_tar_h"], scale, div)
    _assert_bits(orc, got, g[key], key)


def test_rect_equals_normalised_aca(oracle):
    """TensorACA_rect is ACA up to scale."""
    g = load_golden("torch_tensor_aca.npz")
    Hr = oracle.tensor_aca_rect(g["int_src_h"], g["int_tar_h"], float(g["int_scale"][0]),
                                float(g["int_div"][0])).reshape(-1, 9).astype(np.float64)
    Ha = oracle.solve("aca", g["int_src"].reshape(-1, 8).astype(np.float64),
                      g["int_tar"].reshape(-1, 8).astype(np.float64))
    # both are f32 pipelines of different length: compare normwise per problem
    err = np.linalg.norm(Hr / Hr[:, 8:9] - Ha, axis=1) / np.linalg.norm(Ha, axis=1)
    assert err.max() < 1e-5, err.max()


def test_kat_veri4pts(oracle):
    """veri_4Pts.m: H_real ./ H must be constant (checked on the normalised H)."""
    g = load_golden("kat_veri4pts.npz")
    Hn = g["H_real_norm"].reshape(9)
    for algo, tol in (("aca", 1e-6), ("sks", 1e-6)):
        h64 = oracle.solve(algo, g["src"], g["tar"])[0]
        np.testing.assert_allclose(h64, Hn, rtol=1e-9, atol=1e-12)
        h32 = oracle.solve(algo, g["src_f32"], g["tar_f32"])[0]
        assert np.linalg.norm(h32 - Hn) / np.linalg.norm(Hn) < tol
        np.testing.assert_array_equal(h32, g[f"{algo}_f32"][0])
    # rectangle (veri_4Pts.m:82-95) through TensorACA_rect's (B,3,4) form
    w, h, mx, my = g["rect_whm"]
    src = np.vstack([g["rect_src"].T, np.ones(4)])[None].astype(np.float32)
    tar = np.vstack([g["rect_tar"].T, np.ones(4)])[None].astype(np.float32)
    Hr = oracle.tensor_aca_rect(src, tar, w, w / h)[0].astype(np.float64)
    Hr = (Hr / Hr[2, 2]).reshape(9)
    assert np.linalg.norm(Hr - Hn) / np.linalg.norm(Hn) < 1e-5


def test_reference_generator_restated(pkg):
    """sks-homography_amd.adjust reproduces the reference's draws (seed 0)."""
    g = load_golden("torch_generator.npz")
    torch.manual_seed(0)
    out = pkg.adjust("cpu", 8)
    for k, v in zip(["src", "tar", "src_h", "tar_h", "scale", "div"], out):
        np.testing.assert_array_equal(v.numpy(), g[k], err_msg=k)


def test_uniform_stream_known_values(oracle):
    a = oracle.fill_uniform(16, 11, 0)
    b = oracle.fill_uniform(8, 11, 8)
    np.testing.assert_array_equal(a[8:], b)
    assert a.dtype == np.float32 and (a >= 0).all() and (a < 1024).all()


@pytest.mark.parametrize("seed", [11, 3])
@pytest.mark.parametrize("offset", [0, 2**33 + 7])
def test_uniform_stream_vs_independent_restatement(oracle, seed, offset):
    """The input stream of every bench and parity batch (oracle_fill_uniform_f32, the GPU's
    hg_fill_uniform_f32) against tests/restate_streams.py, which shares no code with it:
    the first 10**5 values bit for bit (numpy uint64 restatement), the first 2000 also
    through the literal Python-integer statement; then lo/hi other than the default."""
    import restate_streams as rs
    got = oracle.fill_uniform(100_000, seed, offset)
    np.testing.assert_array_equal(got.view(np.uint32), rs.uniform_f32(100_000, seed, offset).view(np.uint32))
    np.testing.assert_array_equal(got[:2000].view(np.uint32),
                                  rs.uniform_f32_pyint(2000, seed, offset).view(np.uint32))
    got = oracle.fill_uniform(4099, seed, offset, -3000.0, 3000.0)
    np.testing.assert_array_equal(got.view(np.uint32),
                                  rs.uniform_f32(4099, seed, offset, -3000.0, 3000.0).view(np.uint32))


def test_uniform_stream_counter_wraps(oracle):
    """Counters wrap mod 2**64 (offsets near the top of the range)."""
    import restate_streams as rs
    off = (1 << 64) - 5 - (11 * rs.K_UNIFORM) % (1 << 64)
    got = oracle.fill_uniform(64, 11, off % (1 << 64))
    np.testing.assert_array_equal(got.view(np.uint32), rs.uniform_f32(64, 11, off % (1 << 64)).view(np.uint32))


def _functional_rect(src, tar, scale, div):
    """Out-of-place statement of the reference composition (.py:296-302); the
    reference writes H by slices in place, which autograd can differentiate w.r.t.
    tar/scale/div but not w.r.t. src."""
    d = tar[:, :, 1:] - tar[:, :, 0:1]
    q = torch.cross(d[:, 1:2, :], d[:, 0:1, :], dim=2)
    b = q.sum(2, keepdim=True) * tar[:, :, 0:1]
    h0 = tar[:, :, 1:2] * q[:, :, 0:1] - b
    h1 = div * (tar[:, :, 2:3] * q[:, :, 1:2] - b)
    h2 = scale * b - src[:, 0:1, 0:1] * h0 - src[:, 1:2, 0:1] * h1
    return torch.cat([h0, h1, h2], 2)


@pytest.mark.parametrize("scale,div", [(128.0, 1.0), (50.0, 1.25)])
def test_oracle_rect_backward_vs_autograd_f64(oracle, scale, div):
    """The hand-derived TensorACA gradient against float64 autograd of
    the reference composition."""
    g = load_golden("torch_tensor_aca.npz")
    sh, th = torch.from_numpy(g["f_src_h"]), torch.from_numpy(g["f_tar_h"])
    gH = torch.randn(th.shape[0], 3, 3, generator=torch.Generator().manual_seed(1))
    gs, gt, gsd = oracle.tensor_aca_rect_backward(sh.numpy(), th.numpy(), gH.numpy(), scale, div)
    s64 = sh.double().requires_grad_()
    t64 = th.double().requires_grad_()
    sc = torch.tensor([scale], dtype=torch.float64, requires_grad=True)
    dv = torch.tensor([div], dtype=torch.float64, requires_grad=True)
    _functional_rect(s64, t64, sc, dv).backward(gH.double())

    def rel(a, b):
        return float(np.abs(a - b).max() / np.abs(b).max())

    assert rel(gt, t64.grad.numpy()) < 1e-6
    assert rel(gs, s64.grad.numpy()) < 1e-6
    assert abs(gsd[:, 0].astype(np.float64).sum() / sc.grad.item() - 1) < 1e-5
    assert abs(gsd[:, 1].astype(np.float64).sum() / dv.grad.item() - 1) < 1e-5


def test_oracle_ge_vs_reference(orc, oracle):
    """RHO-GE baseline (cv::runKernel_GE, GE.cpp:41-188) against the compiled reference."""
    for fx, sk, tk, hk in (("cpp_uniform.npz", "src_f32", "tar_f32", "ge_f32"),
                           ("cpp_wall.npz", "src", "tar", "ge"),
                           ("cpp_edge.npz", "src", "tar", "ge")):
        g = load_golden(fx)
        _assert_bits(orc, oracle.solve("ge", g[sk], g[tk]), g[hk], f"ge {fx}")


def test_oracle_gpt_lu_vs_lapack(oracle):
    """GPT-LU baseline (cal_Homo_GPT, GPU_Runtime Test.cu:301-357): the reference needs
    nvcc, so the restatement is pinned against LAPACK's solve of the same 8x8 system."""
    rng = np.random.default_rng(8)
    n = 2000
    s = rng.uniform(0, 1024, (n, 8))
    t = rng.uniform(0, 1024, (n, 8))
    H = oracle.solve("gpt", s, t)
    for i in range(0, n, 7):
        A = np.zeros((8, 8))
        b = np.zeros(8)
        for k in range(4):
            x, y, u, v = s[i, 2 * k], s[i, 2 * k + 1], t[i, 2 * k], t[i, 2 * k + 1]
            A[k] = [x, y, 1, 0, 0, 0, -x * u, -y * u]
            A[k + 4] = [0, 0, 0, x, y, 1, -x * v, -y * v]
            b[k], b[k + 4] = u, v
        want = np.linalg.solve(A, b)
        np.testing.assert_allclose(H[i, :8], want, rtol=1e-7, atol=1e-9 * np.abs(want).max())
        assert H[i, 8] == 1.0


def test_oracle_ge_f64_tracks_reference_f32(orc, oracle):
    """The binary64 GE restatement (cal_Homo_GE) agrees with the reference's binary32
    GE.cpp to f32 accuracy on the uniform fixture (same statements, wider type)."""
    g = load_golden("cpp_uniform.npz")
    h64 = oracle.solve("ge", g["src_f32"].astype(np.float64), g["tar_f32"].astype(np.float64))
    h32 = g["ge_f32"].astype(np.float64)
    rel = np.abs(h64 - h32) / np.maximum(np.abs(h64), 1e-12)
    assert np.median(rel) < 1e-5


def test_tensor_aca_restatement_equals_aten_on_special_values(orc, oracle):
    """The TensorACA restatement against the reference's ATen composition on CPU torch
    (bench.torch_tensor_aca_rect, Modules_Runtime_Test.py:294-302) beyond the fixtures:
    special values, signed zeros (three -0 cross terms: torch.sum starts from +0) and random
    bit patterns, bit for bit.  AVX-512 hosts only (ATen's cross contracts to FMA there)."""
    import pytest
    import torch

    import bench
    if not orc.cpu_has_avx512():
        pytest.skip("ATen's CPU cross takes its FMA path only on an AVX-512 host")
    rng = np.random.default_rng(48259)
    vals = np.array([0.0, -0.0, 1.0, -1.0, 2.0, 0.5, 1024.0, np.inf, -np.inf, np.nan, 1e-45,
                     -1.2e-40, 3e38], np.float32)
    B = 50_000
    cases = [tuple(rng.choice(vals, size=(B, 3, 4)).astype(np.float32) for _ in range(2)),
             tuple(rng.integers(0, 2**32 - 1, size=(B, 3, 4), dtype=np.uint32, endpoint=True)
                   .view(np.float32) for _ in range(2))]
    # the case that showed it: every cross term -0 (underflowing products of tiny differences)
    one = np.array([[[1.4e-45, -0.0, 0.0, 0.0], [-1.2e-40, 0.0, -0.0, 0.0], [-0.0, 1024.0, -0.0, 0.0]]],
                   np.float32)
    cases.append((np.full((1, 3, 4), 2.0, np.float32), one))
    for src, tar in cases:
        for scale, div in ((128.0, 1.0), (50.0, 1.25), (float("inf"), 0.5)):
            want = bench.torch_tensor_aca_rect(torch.from_numpy(src), torch.from_numpy(tar),
                                               torch.tensor([scale]), torch.tensor([div])).numpy()
            got = oracle.tensor_aca_rect(src, tar, scale, div)
            assert orc.same_bits(got, want).all(), (scale, div, int((~orc.same_bits(got, want)).sum()))


@pytest.mark.parametrize("tag,scale,div", [("128_1", 128.0, 1.0), ("50_125", 50.0, 1.25),
                                           ("inf_05", float("inf"), 0.5)])
def test_tensor_aca_restatement_equals_reference_special_fixture(orc, oracle, tag, scale, div):
    """torch_special.npz: the reference's own TensorACA_rect statements on special values
    (tools/make_golden.py --torch-special), problem 0 an all-(-0) cross product."""
    g = load_golden("torch_special.npz")
    got = oracle.tensor_aca_rect(g["rect_src"], g["rect_tar"], scale, div)
    ok = orc.same_bits(got, g[f"rect_{tag}"])
    assert ok.all(), int((~ok).sum())


def test_aca_vanilla_restatement_equals_reference_special_fixture(orc, oracle):
    g = load_golden("torch_special.npz")
    B = g["van_src"].shape[0]
    got = oracle.solve("aca", g["van_src"].reshape(B, 8), g["van_tar"].reshape(B, 8),
                       normalize=False).reshape(B, 3, 3)
    ok = orc.same_bits(got, g["vanilla"])
    assert ok.all(), int((~ok).sum())


def _bcast_cases():
    g = load_golden("torch_rect_bcast.npz")
    return g, [(k, str(n), bool(a)) for k, (n, a) in enumerate(zip(g["cases"], g["accepted"]))]


def test_oracle_rect_broadcast_scale_div_vs_reference(orc, oracle):
    """TensorACA with per-problem / per-row scale and div (the reference composition's own
    broadcasting, .py:301-302): the oracle's row form equals the reference statements' H bit
    for bit on every shape the composition accepts (tests/golden/torch_rect_bcast.npz), and
    so does its gradient of tar, against ATen autograd's through those statements."""
    g, cases = _bcast_cases()
    assert sum(a for _, _, a in cases) >= 9 and sum(not a for _, _, a in cases) >= 8
    for k, name, acc in cases:
        if not acc:
            continue
        sc, dv = g[f"c{k}_scale"], g[f"c{k}_div"]
        _assert_bits(orc, oracle.tensor_aca_rect_rows(g["src_h"], g["tar_h"], sc, dv),
                     g[f"c{k}_H"], f"rect {name}")
        _, gt, *_ = oracle.tensor_aca_rect_rows_backward(g["src_h"], g["tar_h"], g["gH"], sc, dv)
        _assert_bits(orc, gt, g[f"c{k}_gtar"], f"grad tar {name}")


def test_rect_op_accepts_the_reference_shapes_on_meta(pkg):
    """torch.ops.sks_amd.tensor_aca_rect accepts exactly the scale / div shapes the reference
    composition accepts and refuses the others (checked on meta tensors: the shape rule is
    the op's own, no GPU needed)."""
    import torch
    g, cases = _bcast_cases()
    B = 64
    m = lambda *s: torch.empty(*s, device="meta")  # noqa: E731
    op = torch.ops.sks_amd.tensor_aca_rect.default
    for k, name, acc in cases:
        sc, dv = g[f"c{k}_scale"], g[f"c{k}_div"]
        if acc:
            assert op(m(B, 3, 4), m(B, 3, 4), m(sc.shape), m(dv.shape)).shape == (B, 3, 3), name
        else:
            with pytest.raises(RuntimeError):
                op(m(B, 3, 4), m(B, 3, 4), m(sc.shape), m(dv.shape))


def _rect_grad_reduced(gss, gds, gsr, gdr, sc, dv):
    """The oracle's per-problem / per-row partials in the parameter's shape, where ATen's
    reduction to that shape is a three-row sum (B,1,1) or none (B,3,1)."""
    if sc.ndim == 3 and sc.shape[1] == 1:
        return gss.reshape(sc.shape), gds.reshape(dv.shape)
    return gsr.reshape(sc.shape), gdr.reshape(dv.shape)


def test_oracle_rect_backward_equals_reference_autograd(orc, oracle):
    """tests/golden/torch_rect_grad.npz: ATen autograd through the reference's own
    TensorACA_rect statements (tools/make_golden.py --torch-grad) -- the adjust() batches with
    signed-zero gradients and identity problems, fractional quads, special values, random bit
    patterns.  dL/dtar bit for bit in every case; dL/dscale, dL/ddiv bit for bit where ATen
    reduces them per problem ((B,1,1): three rows) or not at all ((B,3,1)); a batch-uniform
    (1,) parameter's gradient is a sum over the whole batch, in ATen's own vectorised order,
    so there the per-problem partials sum to it within binary32 accumulation error."""
    g = load_golden("torch_rect_grad.npz")
    assert bool(g["src_grad_refused"])  # the statements cannot differentiate src (in-place H)
    for tag in (str(t) for t in g["cases"]):
        sc, dv = g[f"{tag}_scale"], g[f"{tag}_div"]
        _, gt, gsr, gdr, gss, gds = oracle.tensor_aca_rect_rows_backward(
            g[f"{tag}_src"], g[f"{tag}_tar"], g[f"{tag}_gH"], sc, dv)
        _assert_bits(orc, gt, g[f"{tag}_gtar"], f"grad tar {tag}")
        if sc.size == 1:
            for part, key in ((gss, "gscale"), (gds, "gdiv")):
                want = float(g[f"{tag}_{key}"][0])
                got = float(np.asarray(part, np.float64).sum())
                if np.isfinite(want):
                    assert abs(got - want) <= 1e-5 * np.abs(part).astype(np.float64).sum(), (tag, key)
                else:
                    assert not np.isfinite(got), (tag, key)
        else:
            ws, wd = _rect_grad_reduced(gss, gds, gsr, gdr, sc, dv)
            _assert_bits(orc, ws, g[f"{tag}_gscale"], f"grad scale {tag}")
            _assert_bits(orc, wd, g[f"{tag}_gdiv"], f"grad div {tag}")


def test_oracle_aca_vanilla_backward_equals_reference_autograd(orc, oracle):
    """tests/golden/torch_vanilla_grad.npz: ATen autograd through the reference's own
    ACA_vanilla statements (tools/make_golden.py --torch-vanilla-grad) in binary32 and
    binary64 -- uniform quads, adjust() batches with signed-zero gradients, point-file subsets,
    the edge set, special values, random bit patterns.  The oracle's dL/dsrc and dL/dtar
    equal it bit for bit, and so does its forward (unnormalised ACA)."""
    g = load_golden("torch_vanilla_grad.npz")
    for tag in (str(t) for t in g["cases"]):
        src, tar = g[f"{tag}_src"], g[f"{tag}_tar"]
        n = src.shape[0]
        gs, gt = oracle.aca_vanilla_backward(src, tar, g[f"{tag}_gH"])
        _assert_bits(orc, gs, g[f"{tag}_gsrc"].reshape(n, 8), f"grad src {tag}")
        _assert_bits(orc, gt, g[f"{tag}_gtar"].reshape(n, 8), f"grad tar {tag}")
        H = oracle.solve("aca", src.reshape(n, 8), tar.reshape(n, 8), normalize=False)
        _assert_bits(orc, H, g[f"{tag}_H"].reshape(n, 9), f"H {tag}")


def test_vanilla_restatement_builds_the_reference_graph(orc):
    """bench.torch_aca_vanilla (the composition the GPU tests run under autograd on the box's
    CPU, and bench times on the GPU) gives the fixture's H and gradients bit for bit: the
    same graph as the reference's statements."""
    import torch
    from bench import torch_aca_vanilla
    from conftest import default_dtype
    g = load_golden("torch_vanilla_grad.npz")
    for tag in (str(t) for t in g["cases"]):
        S = torch.from_numpy(g[f"{tag}_src"].copy()).requires_grad_()
        T = torch.from_numpy(g[f"{tag}_tar"].copy()).requires_grad_()
        with default_dtype(S.dtype):  # as the fixture was made
            H = torch_aca_vanilla(S, T)
        H.backward(torch.from_numpy(g[f"{tag}_gH"]))
        _assert_bits(orc, H.detach().numpy(), g[f"{tag}_H"], f"H {tag}")
        _assert_bits(orc, S.grad.numpy(), g[f"{tag}_gsrc"], f"grad src {tag}")
        _assert_bits(orc, T.grad.numpy(), g[f"{tag}_gtar"], f"grad tar {tag}")
