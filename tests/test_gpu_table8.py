"""The reference's Table-8 sampling pipeline in its own formats (GPU_Runtime Test.cu:1443-1451):
MRG32K3A words, get_rand_list (:52-78) and cal_Homo_* (:81-507), through
hg_rand_mrg32k3a_u32 / hg_get_rand_list_f64 / hg_gather_solve_f64.

Pins:
  * get_rand_list: the (8,n) rows equal a numpy restatement of its statements (an exact
    gather: every bit);
  * the fused gather + solve equals the cal_Homo_{ACA,SKS,GE,GPT} statements (the hipcc
    stand-in build oracle/_ref/libsks_ref_cu.so, a cross-check -- DESIGN.md §3) run on those rows, bit for
    bit, NaN for NaN -- on the reference's own point file and on pools of arbitrary binary64
    bit patterns, through the LDS-pool form (small pools, and the 2540-pair wall file with
    the LDS opt-in) and the global-gather form (pools over 160 KiB);
  * MRG32K3A: the hand-written generator's words equal rocrand_generate's and the
    restatement's (tests/test_gpu_mrg32k3a.py); here: determinism across calls and streams,
    seed sensitivity, range and moments.  Equality with cuRAND's own stream is parity
    unpinned (no cuRAND in this image).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

ALGOS = ["aca", "sks", "ge", "gpt"]


@pytest.fixture(scope="module")
def refcu(orc):
    if not orc.RefCuOracle.available():
        pytest.fail(f"{orc.REF_CU_SO} missing: oracle/build.sh builds it where /root/reference is")
    return orc.RefCuOracle()


def _wall(dev):
    g = load_golden("cpp_wall.npz")
    ps = g["pool_src"].astype(np.float64)  # Point2f -> Point2d, as .cu:1414-1416 copies them
    pt = g["pool_tar"].astype(np.float64)
    return ps, pt


def _restated_rand_list(rl, ps, pt):
    """get_rand_list (.cu:52-78) in numpy: word k of hypothesis id at rl[k, id], each taken
    modulo the pool size; rows 2k / 2k+1 are x / y of the selected point."""
    r = rl.astype(np.uint32) % np.uint32(ps.shape[0])
    d_src = np.empty((8, rl.shape[1]), np.float64)
    d_tar = np.empty((8, rl.shape[1]), np.float64)
    for k in range(4):
        d_src[2 * k], d_src[2 * k + 1] = ps[r[k], 0], ps[r[k], 1]
        d_tar[2 * k], d_tar[2 * k + 1] = pt[r[k], 0], pt[r[k], 1]
    return d_src, d_tar


def _check(orc, got, want, what):
    got = got.cpu().numpy() if isinstance(got, torch.Tensor) else got
    ok = orc.same_bits(got, want)
    assert ok.all(), f"{what}: {int((~ok).sum())}/{ok.size} differ"


@pytest.mark.parametrize("n", [1, 4096, 100_003])
def test_wall_pipeline_equals_reference_kernels(orc, pkg, dev, refcu, n):
    """The harness's own flow (numsOfH = 1 << 12 by default, .cu:1419) on orig_pts_wall.txt:
    draws -> get_rand_list -> cal_Homo_*, unfused and fused, against the reference kernels."""
    ps, pt = _wall(dev)
    dps, dpt = torch.from_numpy(ps).to(dev), torch.from_numpy(pt).to(dev)
    rl = pkg.rand_mrg32k3a(4 * n, 11, dev).view(4, n)
    d_src, d_tar = pkg.get_rand_list(rl, dps, dpt)
    ws, wt = _restated_rand_list(rl.cpu().numpy().view(np.uint32), ps, pt)
    _check(orc, d_src, ws, "get_rand_list src")
    _check(orc, d_tar, wt, "get_rand_list tar")
    for algo in ALGOS:
        want = refcu.solve(algo, ws, wt)
        _check(orc, pkg.gather_solve(dps, dpt, rl, algo), want, f"fused {algo}")
        _check(orc, pkg.solve(algo, d_src, d_tar, normalize=False, layout="soa"), want,
               f"unfused {algo}")
        # normalised: the same bits as the SoA solver's normalised output
        _check(orc, pkg.gather_solve(dps, dpt, rl, algo, normalize=True),
               pkg.solve(algo, d_src, d_tar, normalize=True, layout="soa").cpu().numpy(),
               f"fused normalised {algo}")


@pytest.mark.parametrize("npool", [1, 2, 97, 2048, 5120, 5121, 20_000])
def test_arbitrary_pools_and_words(orc, pkg, dev, refcu, npool):
    """Pools of arbitrary binary64 bit patterns (NaN, +-Inf, subnormals) mixed with ordinary
    points, and words over the whole uint32 range (0, 0xFFFFFFFF, multiples of the pool
    size): 5120 pairs is the largest LDS pool (160 KiB), 5121 the first global-gather one."""
    rng = np.random.default_rng(npool)
    pool = rng.integers(0, 2**64 - 1, size=(npool, 4), dtype=np.uint64, endpoint=True).view(np.float64)
    pool[: (npool + 1) // 2] = rng.uniform(0, 1024, ((npool + 1) // 2, 4))
    ps, pt = np.ascontiguousarray(pool[:, :2]), np.ascontiguousarray(pool[:, 2:])
    n = 65_541
    words = rng.integers(0, 2**32 - 1, size=(4, n), dtype=np.uint32, endpoint=True)
    words[:, :6] = [[0, 0xFFFFFFFF, npool, npool - 1, 2 * npool, 0xFFFFFFFE]] * 4
    dps, dpt = torch.from_numpy(ps).to(dev), torch.from_numpy(pt).to(dev)
    rl = torch.from_numpy(words.view(np.int32)).to(dev)
    ws, wt = _restated_rand_list(words, ps, pt)
    d_src, d_tar = pkg.get_rand_list(rl, dps, dpt)
    _check(orc, d_src, ws, f"get_rand_list src npool={npool}")
    _check(orc, d_tar, wt, f"get_rand_list tar npool={npool}")
    for algo in ALGOS:
        _check(orc, pkg.gather_solve(dps, dpt, rl, algo), refcu.solve(algo, ws, wt),
               f"fused {algo} npool={npool}")


def test_large_batch_fused_equals_unfused(orc, pkg, dev):
    """4 M hypotheses (a grid of many persistent passes per block) on the wall pool: the
    fused kernel equals get_rand_list + the shipped SoA solver bit for bit."""
    ps, pt = _wall(dev)
    dps, dpt = torch.from_numpy(ps).to(dev), torch.from_numpy(pt).to(dev)
    n = 4_000_037
    rl = pkg.rand_mrg32k3a(4 * n, 7, dev).view(4, n)
    d_src, d_tar = pkg.get_rand_list(rl, dps, dpt)
    for algo in ("aca", "sks"):
        _check(orc, pkg.gather_solve(dps, dpt, rl, algo),
               pkg.solve(algo, d_src, d_tar, normalize=False, layout="soa").cpu().numpy(), algo)


def test_mrg32k3a_stream(pkg, dev):
    """MRG32K3A (the reference's CURAND_RNG_PSEUDO_MRG32K3A, seed 11): the same words on
    every call, other words for another seed, and the moments of a uniform draw."""
    a = pkg.rand_mrg32k3a(1 << 22, 11, dev)
    b = pkg.rand_mrg32k3a(1 << 22, 11, dev)
    c = pkg.rand_mrg32k3a(1 << 22, 12, dev)
    assert torch.equal(a, b)
    assert not torch.equal(a, c)
    # every call restarts its seed's stream: a request of another size and seed in between,
    # or on another stream, leaves the next call's words alone
    pkg.rand_mrg32k3a(12345, 99, dev)
    s2 = torch.cuda.Stream(dev)
    with torch.cuda.stream(s2):
        d = pkg.rand_mrg32k3a(1 << 22, 11, dev)
    s2.synchronize()
    assert torch.equal(a, d)
    u = a.cpu().numpy().view(np.uint32).astype(np.float64)
    assert u.max() <= 2.0**32 - 1
    x = u / 2.0**32
    assert abs(x.mean() - 0.5) < 2e-3 and abs(x.var() - 1 / 12) < 2e-3
    # the empty request is a no-op
    assert pkg.rand_mrg32k3a(0, 11, dev).numel() == 0


def test_argument_checks(pkg, dev):
    ps = torch.zeros((10, 2), dtype=torch.float64, device=dev)
    rl = torch.zeros((4, 8), dtype=torch.int32, device=dev)
    with pytest.raises(ValueError):
        pkg.gather_solve(ps.float(), ps.float(), rl)          # pools must be float64
    with pytest.raises(ValueError):
        pkg.gather_solve(ps, ps, rl.view(8, 4))               # rand_list must be (4,n)
    with pytest.raises(ValueError):
        pkg.gather_solve(ps, ps[:5], rl)                      # pool sizes differ
    with pytest.raises(ValueError):
        pkg.gather_solve(ps, ps, rl, algo="dlt")
    H = pkg.gather_solve(ps, ps, torch.zeros((4, 0), dtype=torch.int32, device=dev))
    assert H.shape == (9, 0)
