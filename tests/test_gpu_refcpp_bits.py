"""The headline f32 path (and its f64 twin) against the reference's OWN C++ on arbitrary
bit patterns.

`oracle/_ref/libsks_ref.so` is `C++ Codes/modules/ACA_SKS.cpp` + `GE.cpp` compiled where
they lie (oracle/build.sh): `sks::runKernel_ACA/_SKS` (ACA_SKS.cpp:24-102, :189-303), their
`_double` forms (:104-179, :305-418) and RHO-GE (GE.cpp:43).  The golden fixtures pin
those on uniform, wall-pool and hand-picked edge inputs; here every binary32 / binary64 bit
pattern is fair game -- NaNs of any payload, +-Inf, subnormals, signed zeros, huge and
tiny magnitudes -- so any operation whose rounding, exception or special-value handling
on gfx950 differs from x86 SSE (division, reciprocal, FMA contraction, denormal flushing)
would show.  Bar: bit-exact, every NaN equal to every NaN (payloads are not part of the
contract: x86 propagates an operand's, the GPU may return the canonical one).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ref(orc):
    if not orc.RefOracle.available():
        pytest.fail(f"{orc.REF_SO} missing: oracle/build.sh builds it where /root/reference is")
    return orc.RefOracle()


def _check(orc, got, want, what):
    got = got.cpu().numpy() if isinstance(got, torch.Tensor) else got
    ok = orc.same_bits(got, want)
    bad = np.flatnonzero(~ok)
    assert ok.all(), (f"{what}: {bad.size}/{ok.size} differ; first at {bad[:3].tolist()} "
                      f"got {got.ravel()[bad[:3]]} want {np.asarray(want).ravel()[bad[:3]]}")


def _random_bits(n, dtype, seed):
    """(n,8) src/tar whose words are uniform random bit patterns of `dtype` (every exponent,
    NaN and Inf included: 1/256 of binary32 words have the all-ones exponent)."""
    rng = np.random.default_rng(seed)
    u = np.uint32 if dtype == np.float32 else np.uint64
    s = rng.integers(0, np.iinfo(u).max, size=(n, 8), dtype=u, endpoint=True).view(dtype)
    t = rng.integers(0, np.iinfo(u).max, size=(n, 8), dtype=u, endpoint=True).view(dtype)
    return np.ascontiguousarray(s), np.ascontiguousarray(t)


F32_SPECIALS = np.array([0.0, -0.0, 1.0, -1.0, 2.0, -2.0, 0.5, 3.0, 1024.0, np.inf, -np.inf,
                         np.nan, 1e-45, -1.2e-40, 1.1754942e-38, 3.0e38, -3.0e38], np.float32)


def _special_mixture(n, seed):
    """(n,8) src/tar drawn from binary32 special values and ties; the first third keeps small
    integer source points so the target side alone is special there."""
    rng = np.random.default_rng(seed)
    w = np.array([8, 6, 8, 6, 6, 4, 4, 4, 4, 1, 1, 1, 1, 1, 1, 1, 1], np.float64)
    s = rng.choice(F32_SPECIALS, size=(n, 8), p=w / w.sum()).astype(np.float32)
    t = rng.choice(F32_SPECIALS, size=(n, 8), p=w / w.sum()).astype(np.float32)
    k = n // 3
    s[:k] = rng.integers(-4, 5, size=(k, 8)).astype(np.float32)
    return np.ascontiguousarray(s), np.ascontiguousarray(t)


def _random_mantissas(n, seed):
    """Every sign and mantissa bit random, binary exponents in [-16, 16]: finite inputs whose
    outputs are mostly finite too, so each operation's rounding is exercised bit by bit."""
    rng = np.random.default_rng(seed)

    def words():
        sign = rng.integers(0, 2, size=(n, 8), dtype=np.uint32) << np.uint32(31)
        expo = (rng.integers(-16, 17, size=(n, 8)) + 127).astype(np.uint32) << np.uint32(23)
        mant = rng.integers(0, 1 << 23, size=(n, 8), dtype=np.uint32)
        return np.ascontiguousarray((sign | expo | mant).view(np.float32))

    return words(), words()


def _scaled_uniform(n, seed):
    """Ordinary quads over 16 decades of scale: the products and the normalisation's
    reciprocal reach overflow and the subnormal range without any special input."""
    rng = np.random.default_rng(seed)
    scale = np.float32(10.0) ** rng.integers(-8, 9, size=(n, 1)).astype(np.float32)
    s = (rng.uniform(-1, 1, (n, 8)).astype(np.float32) * scale).astype(np.float32)
    t = (rng.uniform(-1, 1, (n, 8)).astype(np.float32) * scale).astype(np.float32)
    return np.ascontiguousarray(s), np.ascontiguousarray(t)


INPUTS_F32 = {
    "random_bits": lambda n: _random_bits(n, np.float32, 101),
    "special_mixture": lambda n: _special_mixture(n, 102),
    "random_mantissas": lambda n: _random_mantissas(n, 106),
    "scaled_uniform": lambda n: _scaled_uniform(n, 103),
}


@pytest.mark.parametrize("kind", list(INPUTS_F32))
@pytest.mark.parametrize("n", [4099, 1_000_003])
def test_f32_every_solver_equals_reference_cpp(orc, ref, pkg, dev, kind, n):
    """sks::runKernel_ACA / _SKS and RHO-GE (normalised, as the C++ returns them) through
    the AoS headline kernels, the SoA kernels and the unaligned generic path."""
    s, t = INPUTS_F32[kind](n)
    ds, dt = torch.from_numpy(s).to(dev), torch.from_numpy(t).to(dev)
    for algo in ("aca", "sks", "ge"):
        want = ref.solve(algo, s, t)
        _check(orc, pkg.solve(algo, ds, dt, normalize=True), want, f"{kind} {algo} aos")
        Hs = pkg.solve(algo, ds.T.contiguous(), dt.T.contiguous(), normalize=True, layout="soa")
        _check(orc, Hs.T, want, f"{kind} {algo} soa")
    # 4-B-aligned views (not 16-B): the generic one-problem-per-lane kernel
    flat_s = torch.empty(n * 8 + 1, dtype=torch.float32, device=dev)
    flat_t = torch.empty(n * 8 + 1, dtype=torch.float32, device=dev)
    flat_s[1:] = ds.view(-1)
    flat_t[1:] = dt.view(-1)
    us, ut = flat_s[1:].view(n, 8), flat_t[1:].view(n, 8)
    for algo in ("aca", "sks"):
        _check(orc, pkg.solve(algo, us, ut, normalize=True), ref.solve(algo, s, t),
               f"{kind} {algo} unaligned")


@pytest.mark.parametrize("n", [4099, 1_000_003])
def test_f64_equals_reference_cpp_double(orc, ref, pkg, dev, n):
    """sks::runKernel_ACA_double / _SKS_double on arbitrary binary64 bit patterns and on a
    binary64 special-value mixture, AoS and SoA."""
    s, t = _random_bits(n, np.float64, 104)
    ms, mt = _special_mixture(n, 105)
    for name, (a, b) in {"random_bits": (s, t),
                         "special_mixture": (ms.astype(np.float64), mt.astype(np.float64))}.items():
        da, db = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
        for algo in ("aca", "sks"):
            want = ref.solve(algo, a, b)
            _check(orc, pkg.solve(algo, da, db, normalize=True), want, f"f64 {name} {algo} aos")
            Hs = pkg.solve(algo, da.T.contiguous(), db.T.contiguous(), normalize=True, layout="soa")
            _check(orc, Hs.T, want, f"f64 {name} {algo} soa")


@pytest.mark.parametrize("npool", [2540, 9000])
def test_sampler_pairs_equal_reference_cpp(orc, oracle, ref, pkg, dev, npool):
    """The RANSAC samplers solve two hypotheses per lane as packed f32x2 pairs (their own
    arithmetic path, not the headline kernel's).  On a pool of arbitrary binary32 points,
    the indexed and seeded samplers (LDS pool at 2540 pairs, global gather at 9000) equal
    the reference C++ run on the gathered problems."""
    rng = np.random.default_rng(npool)
    pool = rng.integers(0, 2**32 - 1, size=(npool, 4), dtype=np.uint32, endpoint=True).view(np.float32)
    # a quarter of the pool ordinary points, so most hypotheses mix both kinds
    pool[: npool // 4] = rng.uniform(0, 1024, (npool // 4, 4)).astype(np.float32)
    ps_np, pt_np = np.ascontiguousarray(pool[:, :2]), np.ascontiguousarray(pool[:, 2:])
    ps, pt = torch.from_numpy(ps_np).to(dev), torch.from_numpy(pt_np).to(dev)
    n = 65_539
    idx = pkg.fill_bits(4 * n, 21, 5, dev).view(n, 4)
    s, t = oracle.sample_problems(ps_np, pt_np, idx.cpu().numpy())
    for algo in ("aca", "sks"):
        want = ref.solve(algo, s, t)
        _check(orc, pkg.sample_solve(ps, pt, idx, algo=algo), want, f"indexed {algo} npool={npool}")
        seeded = pkg.sample_solve_seeded(ps, pt, n, 21, 5, algo=algo)
        _check(orc, seeded, want, f"seeded {algo} npool={npool}")


def test_single_call_and_host_batch_equal_reference_cpp(orc, ref, pkg, dev):
    """The two other kernel forms behind the reference's own signatures: the single-problem
    sks::runKernel_* calls on host pointers (points in the launch arguments, hg_solve_one_*)
    and host-resident batches (hg_solve_host_*, the kernel reading the caller's pageable
    memory over PCIe), on random binary32 / binary64 bit patterns and special mixtures."""
    import ctypes

    from test_gpu_parity import _sks_api
    fns = _sks_api(pkg)
    s32, t32 = _random_bits(256, np.float32, 107)
    m32, n32 = _special_mixture(256, 108)
    s64, t64 = _random_bits(256, np.float64, 109)
    for key, algo, (s, t) in (("aca", "aca", (s32, t32)), ("sks", "sks", (s32, t32)),
                              ("aca", "aca", (m32, n32)), ("sks", "sks", (m32, n32)),
                              ("aca64", "aca", (s64, t64)), ("sks64", "sks", (s64, t64))):
        f, ct = fns[key]
        P = ctypes.POINTER(ct)
        want = ref.solve(algo, s, t)
        got = np.zeros_like(want)
        for i in range(s.shape[0]):
            si, ti, hi = (np.ascontiguousarray(a[i]) for a in (s, t, got))
            assert f(si.ctypes.data_as(P), ti.ctypes.data_as(P), hi.ctypes.data_as(P)) == 0
            got[i] = hi
        _check(orc, got, want, f"sks::{key} single calls")
    for s, t in ((_random_bits(100_003, np.float32, 110)), (_random_bits(100_003, np.float64, 111))):
        for algo in ("aca", "sks"):
            H = pkg.solve_host(algo, torch.from_numpy(s), torch.from_numpy(t), normalize=True)
            _check(orc, H, ref.solve(algo, s, t), f"solve_host {algo} {s.dtype}")
