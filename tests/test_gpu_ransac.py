"""RANSAC extension on the GPU: draws, fused sampler and inlier scorer
are bit-exact against the oracle; the pipeline finds the dominant homography of the
reference's own correspondence file (orig_pts_wall.txt, via tests/golden)."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _pool(dev):
    g = load_golden("cpp_wall.npz")
    return (g["pool_src"], g["pool_tar"], torch.from_numpy(g["pool_src"]).to(dev),
            torch.from_numpy(g["pool_tar"]).to(dev))


def test_fill_bits_matches_host(oracle, pkg, dev):
    for off in (0, 2, 977, (1 << 34) + 3):
        for count in (1, 2, 3, 50_001, 50_002):
            got = pkg.fill_bits(count, 7, off, dev).cpu().numpy().view(np.uint32)
            np.testing.assert_array_equal(got, oracle.fill_bits(count, 7, off), err_msg=f"{off} {count}")


def test_fill_bits_unaligned_output(oracle, pkg, dev):
    """An output 4-B but not 8-B aligned takes the per-word store path (the paired uint2
    store needs 8 B): same words, nothing written outside [0, count)."""
    buf = torch.full((1 + 4099 + 1,), -1, dtype=torch.int32, device=dev)
    for off in (0, 1):
        buf.fill_(-1)
        pkg._lib.call("hg_fill_bits_u32", buf.data_ptr() + 4, 4099, 9, off,
                      torch.cuda.current_stream(dev).cuda_stream)
        got = buf.cpu().numpy().view(np.uint32)
        assert got[0] == 0xFFFFFFFF and got[-1] == 0xFFFFFFFF
        np.testing.assert_array_equal(got[1:-1], oracle.fill_bits(4099, 9, off))


@pytest.mark.parametrize("n", [1, 127, 128, 129, 1000, 65_537])
@pytest.mark.parametrize("algo", ["aca", "sks"])
def test_sample_solve_ragged_vs_oracle(orc, oracle, pkg, dev, n, algo):
    ps, pt, dps, dpt = _pool(dev)
    idx = pkg.fill_bits(n * 4, 11, 0, dev).view(n, 4)
    H = pkg.sample_solve(dps, dpt, idx, algo=algo)
    s, t = oracle.sample_problems(ps, pt, idx.cpu().numpy().view(np.uint32))
    ok = orc.same_bits(H.cpu().numpy(), oracle.solve(algo, s, t))
    assert ok.all(), f"{(~ok).sum()} differ"


@pytest.mark.parametrize("npool", [1, 3, 4, 2047, 2048, 2049, 2540])
def test_score_vs_oracle(oracle, pkg, dev, npool):
    ps, pt, dps, dpt = _pool(dev)
    ps, pt, dps, dpt = ps[:npool], pt[:npool], dps[:npool], dpt[:npool]
    n = 3001
    idx = pkg.fill_bits(n * 4, 5, 0, dev).view(n, 4)
    H = pkg.sample_solve(dps, dpt, idx)
    for thresh in (0.5, 3.0):
        got = pkg.ransac_score(H, dps, dpt, thresh).cpu().numpy().view(np.uint32)
        want = oracle.ransac_score(H.cpu().numpy(), ps, pt, thresh)
        np.testing.assert_array_equal(got, want)


def test_ransac_end_to_end(oracle, pkg, dev):
    ps, pt, dps, dpt = _pool(dev)
    res = pkg.ransac(dps, dpt, hypotheses=20_000, thresh=3.0, seed=11)
    counts = res.counts.cpu().numpy()
    assert res.inliers == counts.max() and counts[res.index] == res.inliers
    assert res.index == int(np.flatnonzero(counts == counts.max())[0])
    # the oracle agrees on the winner's count
    want = oracle.ransac_score(res.H.cpu().numpy()[None], ps, pt, 3.0)[0]
    assert want == res.inliers
    # a wall seen from two views: the best of 20 K hypotheses explains most pairs
    assert res.inliers > 0.5 * ps.shape[0], res.inliers


def _tune_sample(pkg):
    import ctypes
    f = pkg._lib.tune().hg_tune_sample
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    f.restype = ctypes.c_int
    return f


def _div_special_operands():
    """Division operands where the expansion's scaling and fix-up steps matter: signed zeros,
    subnormals (smallest, largest, in between), the normal range's ends, powers of two,
    mantissas of all ones, +-Inf and NaNs -- every pairing of them, both orders."""
    f = np.float32
    tiny, big = np.finfo(f).tiny, np.finfo(f).max
    vals = [0.0, -0.0, 1.0, -1.0, 3.0, 0.1, tiny, -tiny, big, -big, big / 2, tiny * 2,
            np.nextafter(f(1), f(2)), np.nextafter(f(1), f(0)), np.nextafter(f(2), f(0)),
            float(2.0 ** 64), float(2.0 ** -64), float(2.0 ** 126), float(2.0 ** -126),
            np.inf, -np.inf, np.nan]
    bits = [0x00000001, 0x80000001, 0x007FFFFF, 0x00400000, 0x00000100, 0x7FC00001, 0xFFC00000,
            0x7F7FFFFF, 0x3FFFFFFF, 0x4B7FFFFF, 0x1FFFFFFF, 0x5F7FFFFF]
    v = np.concatenate([np.array(vals, f), np.array(bits, np.uint32).view(f)])
    a, b = np.meshgrid(v, v)
    return a.ravel(), b.ravel()


def test_packed_division_is_ieee(pkg, dev):
    """div_rn's packed expansion (the samplers' divisions, hg_solvers.hpp) is binary32 IEEE
    division: on 4 M random bit patterns plus every pairing of the special operands it equals
    numpy's float32 a / b (correctly rounded) bit for bit -- NaN for NaN -- and equals the
    compiler's own scalar divisions to the last bit, NaN payloads and signs included."""
    import ctypes
    f = pkg._lib.tune().hg_tune_div_pairs
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                  ctypes.c_void_p]
    f.restype = ctypes.c_int
    rng = np.random.default_rng(20261016)
    sa, sb = _div_special_operands()
    n_rand = 1 << 22
    a = np.concatenate([rng.integers(0, 2 ** 32, n_rand, dtype=np.uint64).astype(np.uint32).view(np.float32), sa])
    b = np.concatenate([rng.integers(0, 2 ** 32, n_rand, dtype=np.uint64).astype(np.uint32).view(np.float32), sb])
    # quotients in every binade: b within a few binades of a, so few over/underflow to Inf/0
    near = rng.integers(0, 2 ** 32, 1 << 20, dtype=np.uint64).astype(np.uint32)
    shift = rng.integers(-(24 << 23), 24 << 23, 1 << 20).astype(np.int64)
    b_near = np.clip(near.astype(np.int64) % (1 << 31) + shift, 0, 0x7F7FFFFF).astype(np.uint32)
    b_near |= near & 0x80000000
    a = np.concatenate([a, near.view(np.float32)])
    b = np.concatenate([b, b_near.view(np.float32)])
    if a.size % 2:
        a, b = a[:-1], b[:-1]
    da, db = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    out = {}
    for packed in (1, 0):
        q = torch.empty_like(da)
        assert f(packed, da.data_ptr(), db.data_ptr(), q.data_ptr(), a.size,
                 torch.cuda.current_stream(dev).cuda_stream) == 0
        out[packed] = q.cpu().numpy()
    np.testing.assert_array_equal(out[1].view(np.uint32), out[0].view(np.uint32))
    with np.errstate(all="ignore"):
        want = a / b
    nan = np.isnan(want)
    assert (np.isnan(out[1]) == nan).all()
    bad = np.flatnonzero(out[1][~nan].view(np.uint32) != want[~nan].view(np.uint32))
    assert bad.size == 0, [(a[~nan][i], b[~nan][i]) for i in bad[:5]]


@pytest.mark.parametrize("npool", [1, 2, 3, 4, 7, 8, 1024, 1025, 2540, 3900, 20_000])
@pytest.mark.parametrize("variant", [0, 1, 2])
def test_sample_solve_variants_vs_oracle(orc, oracle, pkg, dev, npool, variant):
    """Every sampler form (global gather; pool staged in LDS, P = 1/2) against the oracle:
    pools from 1 point (the remainder clamp) and powers of two to beyond the LDS limit (the LDS
    forms fall back), ragged batches over the persistent grid, indices spanning all of
    uint32 (modulo reduction as get_rand_list, .cu:56-59)."""
    g = np.random.default_rng(npool)
    ps = (g.random((npool, 2)) * 1000).astype(np.float32)
    pt = (g.random((npool, 2)) * 1000).astype(np.float32)
    dps, dpt = torch.from_numpy(ps).to(dev), torch.from_numpy(pt).to(dev)
    f = _tune_sample(pkg)
    for n in (1, 255, 70_001):
        idx = pkg.fill_bits(n * 4, npool + n, 0, dev).view(n, 4)
        idx[0, 0] = -1  # 0xFFFFFFFF
        for algo in (0, 1):
            H = torch.empty((n, 9), device=dev)
            rc = f(variant, dps.data_ptr(), dpt.data_ptr(), npool, idx.data_ptr(), H.data_ptr(), n,
                   algo, 1, torch.cuda.current_stream(dev).cuda_stream)
            assert rc == 0
            s, t = oracle.sample_problems(ps, pt, idx.cpu().numpy().view(np.uint32))
            ok = orc.same_bits(H.cpu().numpy(), oracle.solve("aca" if algo == 0 else "sks", s, t))
            assert ok.all(), f"variant {variant} npool {npool} n {n}: {(~ok).sum()} differ"


def test_score_special_values_vs_oracle(oracle, pkg, dev):
    """Hypotheses and pool points with NaN / +-Inf / 0 / huge entries: the division-free
    inlier test gives the restatement's counts exactly (w' = 0 never counts)."""
    rng = np.random.default_rng(8)
    npool, n = 777, 5003
    ps = rng.uniform(0, 1000, (npool, 2)).astype(np.float32)
    pt = rng.uniform(0, 1000, (npool, 2)).astype(np.float32)
    H = rng.standard_normal((n, 9)).astype(np.float32)
    H[:, 8] = 1.0
    specials = np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 1e30, 1e-40], np.float32)
    H[::11, 6:9] = 0.0                                   # w' == 0 for every point
    for i in range(0, n, 5):
        H[i, rng.integers(0, 9)] = specials[i % len(specials)]
    for i in range(0, npool, 9):
        ps[i, rng.integers(0, 2)] = specials[i % len(specials)]
    H[7] = [1, 0, 0, 0, 1, 0, 0, 0, 1]                   # identity: inliers where src == tar
    pt[::3] = ps[::3]
    for thresh in (0.0, 2.0):
        got = pkg.ransac_score(torch.from_numpy(H).to(dev), torch.from_numpy(ps).to(dev),
                               torch.from_numpy(pt).to(dev), thresh).cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(got, oracle.ransac_score(H, ps, pt, thresh))


@pytest.mark.parametrize("npool", [1, 3, 2540, 5000, 20_000])
def test_sample_solve_seeded_vs_oracle(orc, oracle, pkg, dev, npool):
    """The seeded fused sampler (draws made in the kernel) equals fill_bits + the indexed
    sampler bit for bit, and both equal the oracle: LDS-pool and global-gather forms
    (npool 20 000 exceeds the LDS pool; at 5000 the seeded launch keeps the pool in LDS,
    past its 64 KiB opt-in, while the indexed one gathers from global memory), ragged
    batches, offsets past 2^32, both solvers, normalised or not."""
    g = np.random.default_rng(npool + 1)
    ps = (g.random((npool, 2)) * 1000).astype(np.float32)
    pt = (g.random((npool, 2)) * 1000).astype(np.float32)
    dps, dpt = torch.from_numpy(ps).to(dev), torch.from_numpy(pt).to(dev)
    for n, seed, off in ((1, 3, 0), (129, 11, 977), (70_001, 12345, (1 << 33) + 5)):
        bits = pkg.fill_bits(n * 4, seed, off, dev).view(n, 4)
        s, t = oracle.sample_problems(ps, pt, oracle.fill_bits(n * 4, seed, off).reshape(n, 4))
        for algo in ("aca", "sks"):
            for norm in (True, False):
                H = pkg.sample_solve_seeded(dps, dpt, n, seed, off, algo=algo, normalize=norm)
                ref = pkg.sample_solve(dps, dpt, bits, algo=algo, normalize=norm)
                assert torch.equal(H.view(torch.int32), ref.view(torch.int32)), (n, algo, norm)
                ok = orc.same_bits(H.cpu().numpy(), oracle.solve(algo, s, t, normalize=norm))
                assert ok.all(), f"npool {npool} n {n} {algo} norm={norm}: {(~ok).sum()} differ"


def test_sample_solve_seeded_packed_shapes_vs_indexed(orc, oracle, pkg, dev):
    """Past kSeededPairMinN (4 M) the seeded ACA launch switches to the 4-wave packed-pair
    shape (SKS uses packed pairs at every size): still fill_bits + the indexed sampler bit
    for bit, NaN bits included, and the oracle NaN for NaN, on the reference's wall pool,
    a ragged batch and an odd stream offset."""
    g = load_golden("cpp_wall.npz")
    ps, pt = g["pool_src"], g["pool_tar"]
    dps, dpt = torch.from_numpy(ps).to(dev), torch.from_numpy(pt).to(dev)
    n, seed, off = (1 << 22) + 129, 11, 3
    bits = pkg.fill_bits(n * 4, seed, off, dev).view(n, 4)
    s, t = oracle.sample_problems(ps, pt, bits.cpu().numpy())
    for algo in ("aca", "sks"):
        H = pkg.sample_solve_seeded(dps, dpt, n, seed, off, algo=algo)
        ref = pkg.sample_solve(dps, dpt, bits, algo=algo)
        assert torch.equal(H.view(torch.int32), ref.view(torch.int32)), algo
        ok = orc.same_bits(H.cpu().numpy(), oracle.solve(algo, s, t, normalize=True))
        assert ok.all(), f"{algo}: {(~ok).sum()} differ"


def test_sample_solve_seeded_zero_and_errors(pkg, dev):
    ps = torch.rand(10, 2, device=dev)
    assert pkg.sample_solve_seeded(ps, ps, 0, 1).shape == (0, 9)
    with pytest.raises(ValueError):
        pkg.sample_solve_seeded(ps, ps, 5, 1, algo="ge")
    with pytest.raises(ValueError):
        pkg.sample_solve_seeded(ps, ps, -1, 1)


def test_generators_validate_out(pkg, dev):
    """fill_uniform's `out` must hold `count` contiguous float32 elements on the GPU."""
    with pytest.raises(ValueError, match="out must be"):
        pkg.fill_uniform(100, 1, out=torch.empty(99, device=dev))
    with pytest.raises(ValueError, match="out must be"):
        pkg.fill_uniform(10, 1, out=torch.empty(10, dtype=torch.float64, device=dev))
    with pytest.raises(ValueError, match="out must be"):
        pkg.fill_uniform(10, 1, out=torch.empty(20, device=dev)[::2])
    o = torch.empty(12, device=dev)
    assert pkg.fill_uniform(10, 1, out=o) is o
    with pytest.raises(ValueError, match="stream_copy"):
        pkg.stream_copy(torch.zeros(8, device=dev), torch.zeros(4, device=dev))


from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402
from hypothesis.extra.numpy import arrays  # noqa: E402


@settings(max_examples=25, deadline=None, suppress_health_check=list(HealthCheck))
@given(pool=arrays(np.float32, st.tuples(st.integers(1, 48), st.just(4)),
                   elements=st.floats(width=32, allow_nan=True, allow_infinity=True,
                                      allow_subnormal=True)),
       n=st.integers(1, 300), seed=st.integers(0, 2**32), off=st.integers(0, 2**34))
def test_samplers_on_arbitrary_pools(orc, oracle, pkg, dev, pool, n, seed, off):
    """Pools of arbitrary binary32 bit patterns (subnormals, +-Inf, NaN, huge and tiny values
    drawn by hypothesis): the packed-pair samplers -- seeded and indexed -- agree with each
    other bit for bit and with the scalar oracle NaN for NaN, both solvers, normalised or not
    (the packed f32 instructions keep subnormals exactly as the scalar ones do)."""
    ps = np.ascontiguousarray(pool[:, :2])
    pt = np.ascontiguousarray(pool[:, 2:])
    dps, dpt = torch.from_numpy(ps).to(dev), torch.from_numpy(pt).to(dev)
    bits = pkg.fill_bits(n * 4, seed, off, dev).view(n, 4)
    s, t = oracle.sample_problems(ps, pt, bits.cpu().numpy())
    for algo in ("aca", "sks"):
        for norm in (True, False):
            H = pkg.sample_solve_seeded(dps, dpt, n, seed, off, algo=algo, normalize=norm)
            ref = pkg.sample_solve(dps, dpt, bits, algo=algo, normalize=norm)
            assert torch.equal(H.view(torch.int32), ref.view(torch.int32)), (algo, norm)
            ok = orc.same_bits(H.cpu().numpy(), oracle.solve(algo, s, t, normalize=norm))
            assert ok.all(), f"{algo} norm={norm}: {(~ok).sum()} differ"
