"""The hand-written MRG32K3A generator (csrc/hg_mrg32k3a.hpp, hg_gather.hpp) and the fused
draws + gather + solve of the reference's Table-8 flow (GPU_Runtime Test.cu:1443-1451).

Pins:
  * hg_rand_mrg32k3a_u32 equals rocrand_generate (ROCRAND_RNG_PSEUDO_MRG32K3A, default
    ordering; built into the tune library as the checker) word for word: seeds 11 (the
    reference's), 3, 0, 2^64 - 1 and a 64-bit pattern; counts 1, 37, 2^17 - 1, 2^17,
    2^17 + 1, 300001, 2^22 + 3 and 40 M (the 4 x 10 M words of a 10 M-hypothesis call);
  * and equals the independent numpy restatement (tests/restate_mrg32k3a.py);
  * hg_rand_gather_solve_f64 equals hg_rand_mrg32k3a_u32(4 n) + hg_gather_solve_f64 bit for
    bit: every algorithm, both normalisations, LDS and global pools, ragged n across the
    2^17 residue classes, and the reference's wall file;
  * both are asynchronous and graph-capturable.
"""
import ctypes

import numpy as np
import pytest
import torch

import restate_mrg32k3a as R
from conftest import load_golden

pytestmark = pytest.mark.gpu

SEEDS = [11, 3, 0, (1 << 64) - 1, 0x0123456789ABCDEF]
COUNTS = [1, 37, (1 << 17) - 1, 1 << 17, (1 << 17) + 1, 300_001, (1 << 22) + 3]


@pytest.fixture(scope="module")
def tune(pkg):
    t = pkg._lib.tune()
    vp, i64, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64
    t.hg_tune_rocrand_mrg32k3a_u32.argtypes = [vp, i64, u64, vp]
    t.hg_tune_mrg_words.argtypes = [vp, i64, u64, i64, vp]
    t.hg_tune_rand_gather_solve_f64.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_uint32,
                                                u64, vp, i64, vp]
    return t


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def rocrand_words(tune, dev, count, seed):
    out = torch.empty(count, dtype=torch.int32, device=dev)
    assert tune.hg_tune_rocrand_mrg32k3a_u32(out.data_ptr(), count, seed, _stream(dev)) == 0
    return out


@pytest.mark.parametrize("seed", SEEDS)
def test_words_equal_rocrand(pkg, dev, tune, seed):
    for count in COUNTS:
        ours = pkg.rand_mrg32k3a(count, seed, dev)
        ref = rocrand_words(tune, dev, count, seed)
        assert torch.equal(ours, ref), f"seed {seed} count {count}: " \
            f"{int((ours != ref).sum())} words differ"


def test_words_equal_rocrand_40m(pkg, dev, tune):
    """The 4 x 10 M words of a 10 M-hypothesis Table-8 call (positions up to 305 per
    subsequence: 16 chunks per subsequence in the shipped split)."""
    count = 40_000_003
    ours = pkg.rand_mrg32k3a(count, 11, dev)
    ref = rocrand_words(tune, dev, count, 11)
    assert torch.equal(ours, ref)
    # every split of the subsequences over threads gives the same words
    for chunk in (1, 3, 64, 1000):
        o = torch.empty(count, dtype=torch.int32, device=dev)
        assert tune.hg_tune_mrg_words(o.data_ptr(), count, 11, chunk, _stream(dev)) == 0
        assert torch.equal(o, ref), chunk


@pytest.mark.parametrize("seed", [11, 3])
def test_words_equal_restatement(pkg, dev, seed):
    count = 300_001
    ours = pkg.rand_mrg32k3a(count, seed, dev).cpu().numpy().view(np.uint32)
    assert np.array_equal(ours, R.generate(seed, count))


def test_words_equal_committed_rocrand_fixture(pkg, dev):
    g = load_golden("mrg32k3a_rocrand.npz")
    for seed in [int(s) for s in g["seeds"]]:
        w = pkg.rand_mrg32k3a(300_001, seed, dev).cpu().numpy().view(np.uint32)
        assert np.array_equal(w[g[f"s{seed}_n300001_idx"]], g[f"s{seed}_n300001_val"]), seed
        assert np.array_equal(w[:37], g[f"s{seed}_n37"])


def test_words_graph_capture(pkg, dev):
    count = (1 << 20) + 5
    want = pkg.rand_mrg32k3a(count, 11, dev)
    out = torch.empty(count, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        pkg._lib.call("hg_rand_mrg32k3a_u32", out.data_ptr(), count, 11, s.cuda_stream)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, want)


def _wall(dev):
    g = load_golden("cpp_wall.npz")
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(dev)
    return ps, pt


def _random_pool(dev, npool, seed):
    rng = np.random.default_rng(seed)
    pool = rng.integers(0, 2**64 - 1, size=(npool, 4), dtype=np.uint64, endpoint=True).view(np.float64)
    pool[: (npool + 1) // 2] = rng.uniform(0, 1024, ((npool + 1) // 2, 4))
    return (torch.from_numpy(np.ascontiguousarray(pool[:, :2])).to(dev),
            torch.from_numpy(np.ascontiguousarray(pool[:, 2:])).to(dev))


def _same(orc, a, b, what):
    ok = orc.same_bits(a.cpu().numpy(), b.cpu().numpy())
    assert ok.all(), f"{what}: {int((~ok).sum())}/{ok.size} differ"


# 70000 / 200000: groups whose first class already wrapped (g C + b_k >= 2^17) for some row
@pytest.mark.parametrize("n", [1, 37, 4096, 70_000, (1 << 17) - 3, 1 << 17, (1 << 17) + 1,
                               200_000, 1_000_003])
def test_fused_equals_words_then_gather_wall(orc, pkg, dev, n):
    ps, pt = _wall(dev)
    rl = pkg.rand_mrg32k3a(4 * n, 11, dev).view(4, n)
    for algo in ("aca", "sks", "ge", "gpt"):
        for norm in (False, True):
            _same(orc, pkg.rand_gather_solve(ps, pt, n, 11, algo, norm),
                  pkg.gather_solve(ps, pt, rl, algo, norm), f"{algo} norm={norm} n={n}")


@pytest.mark.parametrize("npool", [1, 2, 97, 4048, 4049, 20_000])
def test_fused_arbitrary_pools(orc, pkg, dev, npool):
    """4048 pairs is the largest ACA / SKS pool kept in LDS beside the draws buffers (1024-lane
    blocks), 4049 the first gathered from global memory."""
    ps, pt = _random_pool(dev, npool, npool)
    n = 300_007
    rl = pkg.rand_mrg32k3a(4 * n, 3, dev).view(4, n)
    for algo in ("aca", "sks", "ge", "gpt"):
        _same(orc, pkg.rand_gather_solve(ps, pt, n, 3, algo),
              pkg.gather_solve(ps, pt, rl, algo), f"{algo} npool={npool}")


def test_fused_large_and_global_variant(orc, pkg, dev, tune):
    """10 M hypotheses (the bench size): shipped form and the global-pool variant against
    the unfused pair; seed 2^64 - 1 exercises the seeding's wrap-around."""
    ps, pt = _wall(dev)
    n = 10_000_019
    seed = (1 << 64) - 1
    rl = pkg.rand_mrg32k3a(4 * n, seed, dev).view(4, n)
    for algo, aid in (("aca", 0), ("sks", 1)):
        want = pkg.gather_solve(ps, pt, rl, algo)
        _same(orc, pkg.rand_gather_solve(ps, pt, n, seed, algo), want, algo)
        H = torch.empty_like(want)
        assert tune.hg_tune_rand_gather_solve_f64(0, aid, ps.data_ptr(), pt.data_ptr(), ps.shape[0],
                                                  seed, H.data_ptr(), n, _stream(dev)) == 0
        _same(orc, H, want, f"{algo} global pool")
        del want, H


def test_fused_graph_capture_and_empty(orc, pkg, dev):
    ps, pt = _wall(dev)
    n = 65_537
    want = pkg.rand_gather_solve(ps, pt, n, 11, "sks")
    H = torch.empty_like(want)
    s = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        pkg._lib.call("hg_rand_gather_solve_f64", 1, ps.data_ptr(), pt.data_ptr(), ps.shape[0], 11,
                      H.data_ptr(), n, 0, s.cuda_stream)
    H.zero_()
    g.replay()
    torch.cuda.synchronize()
    _same(orc, H, want, "graph")
    assert pkg.rand_gather_solve(ps, pt, 0, 11).shape == (9, 0)
