"""The binary64 SoA kernels against a STAND-IN build of the reference's GPU kernel
statements, bit for bit -- a restatement check, not a parity pin.

oracle/_ref/libsks_ref_cu.so holds the statements of cal_Homo_ACA / cal_Homo_SKS /
cal_Homo_GE / cal_Homo_GPT ("GPU_Runtime Test.cu:81-507") compiled by hipcc behind a
prepended HIP header (nvcc and the CUDA headers are not in the image), -ffp-contract=off
(every operation rounded on its own, in the statement order), launched as the reference's
host drivers launch them (<<<ceil(N/32), 32>>>, SoA (8,N) -> (9,N), unnormalised).  It
checks that our kernels evaluate those statements in order with IEEE rounding; it does
not show what the reference's own nvcc build produces.  What pins the rows:
unnormalised binary64 ACA by the reference's ACA_vanilla statements run in float64
(test_gpu_parity.py::test_golden_aca_f64_unnormalised); unnormalised binary64 SKS, GE f64
(cal_Homo_GE) and GPT-LU (cal_Homo_GPT) by restatement only -- parity unpinned.
Also the CPU oracle's restatement of the same four, on uniform, wall-pool and edge inputs.
"""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st
from hypothesis.extra.numpy import arrays

from conftest import load_golden

pytestmark = pytest.mark.gpu

ALGOS = ["aca", "sks", "ge", "gpt"]


@pytest.fixture(scope="module")
def refcu(orc):
    if not orc.RefCuOracle.available():
        pytest.fail(f"{orc.REF_CU_SO} missing: oracle/build.sh builds it where /root/reference is")
    return orc.RefCuOracle()


def _inputs():
    """(8, n) binary64 SoA sets: uniform U[0,1024) (the bench stream), random 4-subsets of
    the reference's own wall correspondences, and the 64 edge cases (duplicates, collinear,
    +-Inf, NaN, subnormals, 1e18)."""
    import restate_streams as rs
    n = 100_003
    u_s = rs.uniform_f32(n * 8, 11, 0).astype(np.float64).reshape(n, 8)
    u_t = rs.uniform_f32(n * 8, 11, n * 8).astype(np.float64).reshape(n, 8)
    w = load_golden("cpp_wall.npz")
    e = load_golden("cpp_edge.npz")
    sets = {
        "uniform": (u_s, u_t),
        "wall": (w["src"].astype(np.float64), w["tar"].astype(np.float64)),
        "edge": (e["src_f64"], e["tar_f64"]),
    }
    return {k: (np.ascontiguousarray(s.T), np.ascontiguousarray(t.T)) for k, (s, t) in sets.items()}


@pytest.mark.parametrize("algo", ALGOS)
def test_hip_f64_soa_equals_reference_kernels(orc, pkg, dev, refcu, algo):
    for name, (s, t) in _inputs().items():
        want = refcu.solve(algo, s, t)
        got = pkg.solve(algo, torch.from_numpy(s).to(dev), torch.from_numpy(t).to(dev),
                        normalize=False, layout="soa").cpu().numpy()
        ok = orc.same_bits(got, want)
        assert ok.all(), f"{algo} {name}: {int((~ok).sum())}/{ok.size} differ"


@pytest.mark.parametrize("algo", ALGOS)
def test_oracle_restatement_equals_reference_kernels(orc, oracle, refcu, algo):
    for name, (s, t) in _inputs().items():
        want = refcu.solve(algo, s, t)
        got = oracle.solve(algo, s, t, normalize=False, layout="soa")
        ok = orc.same_bits(got, want)
        assert ok.all(), f"{algo} {name}: {int((~ok).sum())}/{ok.size} differ"


def test_reference_kernels_normalised_equal_reference_cpp(orc, refcu):
    """Closing the loop: cal_Homo_ACA/SKS normalised as the C++ does (r = 1/H[8], eight
    multiplies, H[8] = 1) equal runKernel_ACA_double / _SKS_double on the uniform fixture."""
    g = load_golden("cpp_uniform.npz")
    s, t = np.ascontiguousarray(g["src_f64"].T), np.ascontiguousarray(g["tar_f64"].T)
    for algo in ("aca", "sks"):
        H = refcu.solve(algo, s, t).T.copy()
        r = 1.0 / H[:, 8:9]
        H[:, :8] *= r
        H[:, 8] = 1.0
        assert orc.same_bits(H, g[f"{algo}_f64"]).all(), algo


def test_reference_kernels_large_batch(orc, pkg, dev, refcu):
    """A 2 M-problem batch (SoA f64: the MALL-resident/streaming policy switch of the SoA
    dispatcher lies at 1 M): every element of hg_aca_f64 / hg_gpt_f64 equals the reference
    kernel's."""
    import restate_streams as rs
    n = 2_000_001
    s = np.ascontiguousarray(rs.uniform_f32(n * 8, 3, 0).astype(np.float64).reshape(8, n))
    t = np.ascontiguousarray(rs.uniform_f32(n * 8, 3, n * 8).astype(np.float64).reshape(8, n))
    ds, dt = torch.from_numpy(s).to(dev), torch.from_numpy(t).to(dev)
    for algo in ("aca", "gpt"):
        want = refcu.solve(algo, s, t)
        got = pkg.solve(algo, ds, dt, normalize=False, layout="soa").cpu().numpy()
        assert orc.same_bits(got, want).all(), algo


def _special_mixtures(n, seed):
    """(8, n) SoA sets whose every coordinate is drawn from a small set of special values:
    signed zeros, ties of equal magnitude (+-1, +-2), +-Inf, NaN, subnormals and near-overflow
    magnitudes.  Pivot searches meet exact ties and all-zero / NaN columns on almost every
    problem, which is where a register-resident partial pivoting (the first row of strictly
    larger magnitude wins) and any structural shortcut in it would show."""
    vals = np.array([0.0, -0.0, 1.0, -1.0, 2.0, -2.0, 0.5, 3.0, 1024.0,
                     np.inf, -np.inf, np.nan, 5e-324, -2.5e-310, 1e308, -1e308])
    w = np.array([8, 6, 8, 6, 6, 4, 4, 4, 4, 1, 1, 1, 1, 1, 1, 1], dtype=np.float64)
    rng = np.random.default_rng(seed)
    s = rng.choice(vals, size=(8, n), p=w / w.sum())
    t = rng.choice(vals, size=(8, n), p=w / w.sum())
    # a third of the problems keep ordinary source points, so the target side alone is special
    k = n // 3
    s[:, :k] = rng.integers(-4, 5, size=(8, k)).astype(np.float64)
    return np.ascontiguousarray(s), np.ascontiguousarray(t)


@pytest.mark.parametrize("n", [65_536, 65_537])
def test_special_value_mixtures_equal_reference_kernels(orc, oracle, pkg, dev, refcu, n):
    """Every solver, both SoA kernel forms (even n from 32 K: two problems per lane in 16-B
    registers; odd n: one per lane), the AoS form, and the CPU restatement, against the
    reference kernels on special-value mixtures -- NaN for NaN, signed zeros included."""
    s, t = _special_mixtures(n, 7 + n)
    ds, dt = torch.from_numpy(s).to(dev), torch.from_numpy(t).to(dev)
    for algo in ALGOS:
        want = refcu.solve(algo, s, t)
        got = pkg.solve(algo, ds, dt, normalize=False, layout="soa").cpu().numpy()
        ok = orc.same_bits(got, want)
        assert ok.all(), f"{algo} GPU: {int((~ok).sum())}/{ok.size} differ"
        aos = pkg.solve(algo, ds.T.contiguous(), dt.T.contiguous(), normalize=False,
                        layout="aos").cpu().numpy()
        ok = orc.same_bits(aos, want.T)
        assert ok.all(), f"{algo} GPU AoS: {int((~ok).sum())}/{ok.size} differ"
        ok = orc.same_bits(oracle.solve(algo, s, t, normalize=False, layout="soa"), want)
        assert ok.all(), f"{algo} oracle: {int((~ok).sum())}/{ok.size} differ"


@settings(max_examples=20, deadline=None, suppress_health_check=list(HealthCheck))
@given(arrays(np.float64, (16, 257), elements=st.floats(width=64, allow_nan=True,
                                                        allow_infinity=True, allow_subnormal=True)))
def test_arbitrary_doubles_equal_reference_kernels(orc, pkg, dev, refcu, batch):
    """Arbitrary binary64 bit patterns (NaN, +-Inf, subnormals, huge and tiny values drawn by
    hypothesis), 257 problems a draw: every solver's SoA output equals the reference
    kernel's, NaN for NaN."""
    s = np.ascontiguousarray(batch[:8])
    t = np.ascontiguousarray(batch[8:])
    ds, dt = torch.from_numpy(s).to(dev), torch.from_numpy(t).to(dev)
    for algo in ALGOS:
        want = refcu.solve(algo, s, t)
        got = pkg.solve(algo, ds, dt, normalize=False, layout="soa").cpu().numpy()
        ok = orc.same_bits(got, want)
        assert ok.all(), f"{algo}: {int((~ok).sum())} differ"
