"""CPU: the MRG32K3A restatement (tests/restate_mrg32k3a.py) pinned three ways, and the
library's host-side engine setup (hg_mrg32k3a_state) checked against it.

1. The recurrence and its jumps against constants L'Ecuyer published independently of any
   GPU library: the 2^76 (substream) and 2^127 (stream) jump matrices of RngStreams
   (L'Ecuyer, Simard, Chen & Kelton, Operations Research 50(6), 2002, A1p76 / A2p76 /
   A1p127 / A2p127).
2. Pure-Python integers against the vectorised numpy form.
3. Both against rocrand_generate's own words, dumped on the MI355X box
   (tests/golden/mrg32k3a_rocrand.npz; tools/mrg_dump.py, tools/make_mrg_fixture.py):
   seeds 0, 1, 3, 11, 2^32 + 7, 2^64 - 1 and 0x0123456789abcdef, calls of 37 and 300001
   words (2^17 + 1 and 2^18 + 1 subsequence wraps) and of 2^22 + 3 words at seed 11.

cuRAND's seeding, uint conversion and host ordering stay unpinned (not in this image).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

import restate_mrg32k3a as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "mrg32k3a_rocrand.npz")

# RngStreams' published jump matrices (A^(2^76), A^(2^127) of each component)
A1P76 = ((82758667, 1871391091, 4127413238), (3672831523, 69195019, 1871391091),
         (3672091415, 3528743235, 69195019))
A2P76 = ((1511326704, 3759209742, 1610795712), (4292754251, 1511326704, 3889917532),
         (3859662829, 4292754251, 3708466080))
A1P127 = ((2427906178, 3580155704, 949770784), (226153695, 1230515664, 3580155704),
          (1988835001, 986791581, 1230515664))
A2P127 = ((1464411153, 277697599, 1610723613), (32183930, 1464411153, 1022607788),
          (2824425944, 32183930, 2093834863))


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLDEN)


def test_jump_matrices_equal_lecuyer_published():
    assert R.mat_pow(R.A1, 1 << 76, R.M1) == A1P76
    assert R.mat_pow(R.A2, 1 << 76, R.M2) == A2P76
    assert R.mat_pow(R.A1, 1 << 127, R.M1) == A1P127
    assert R.mat_pow(R.A2, 1 << 127, R.M2) == A2P127


def test_step_matrix_is_the_recurrence():
    g1, g2 = R.seed_state(11)
    ref = R.words_python(11, 0, 0, 5)
    # five steps by the matrices, output by hand
    x1, x2 = g1, g2
    out = []
    for _ in range(5):
        x1, x2 = R.mat_vec(R.A1, x1, R.M1), R.mat_vec(R.A2, x2, R.M2)
        z = (x1[2] - x2[2]) % R.M1 or R.M1
        out.append(R.to_uint(z))
    assert out == ref


def test_python_ints_equal_numpy():
    for seed in (11, 3, (1 << 64) - 1):
        w = R.generate(seed, 3 * R.ORDER_SUBSEQUENCES + 5)
        for s in (0, 1, 4095, R.ORDER_SUBSEQUENCES - 1):
            want = R.words_python(seed, s, 0, 3 if s < 5 else 3)
            got = [int(w[s + p * R.ORDER_SUBSEQUENCES]) for p in range(3)]
            assert got == want, (seed, s)
        assert R.words_python(seed, 2, 0, 4)[3] == int(w[2 + 3 * R.ORDER_SUBSEQUENCES])


def test_restatement_equals_rocrand_words(gold):
    seeds = [int(s) for s in gold["seeds"]]
    assert set(seeds) >= {0, 1, 3, 11, (1 << 64) - 1}
    for seed in seeds:
        assert np.array_equal(R.generate(seed, 37), gold[f"s{seed}_n37"]), seed
        w = R.generate(seed, 300001)
        idx = gold[f"s{seed}_n300001_idx"]
        assert np.array_equal(w[idx], gold[f"s{seed}_n300001_val"]), seed
        # a shorter call's words are a longer call's prefix
        assert np.array_equal(w[:37], gold[f"s{seed}_n37"])
    n = int(gold["s11_big_n"])
    w = R.generate(11, n)
    assert np.array_equal(w[gold["s11_big_idx"]], gold["s11_big_val"])


def test_word_order_is_subsequence_major(gold):
    """word i = position i >> 17 of subsequence i & (2^17 - 1): the pure-Python engine at
    (subsequence, offset) reproduces the dumped words at their indices"""
    idx = gold["s3_n300001_idx"]
    val = gold["s3_n300001_val"]
    pick = [0, 1, 2, len(idx) // 2, len(idx) - 1]
    for j in pick:
        i = int(idx[j])
        s, p = i % R.ORDER_SUBSEQUENCES, i // R.ORDER_SUBSEQUENCES
        assert R.words_python(3, s, p, 1)[0] == int(val[j])


CASES = [(11, 0, 0), (11, 5, 3), (3, 131071, 1000), (0, 7, 0), (1, 0, 1),
         ((1 << 64) - 1, (1 << 40) + 3, (1 << 50) + 11), (0x0123456789ABCDEF, 99, (1 << 63) + 5),
         ((1 << 32) + 7, (1 << 64) - 1, (1 << 64) - 1)]


@pytest.mark.parametrize("seed,sub,off", CASES)
def test_host_engine_state_equals_restatement(pkg, seed, sub, off):
    g1, g2 = R.state_at(seed, sub, off)
    assert pkg.mrg32k3a_state(seed, sub, off) == tuple(g1) + tuple(g2)


def test_host_engine_state_random_seeds(pkg):
    rng = np.random.default_rng(5)
    for _ in range(200):
        seed = int(rng.integers(0, 1 << 63)) * 2 + int(rng.integers(0, 2))
        sub, off = int(rng.integers(0, 1 << 17)), int(rng.integers(0, 1 << 40))
        g1, g2 = R.state_at(seed, sub, off)
        assert pkg.mrg32k3a_state(seed, sub, off) == tuple(g1) + tuple(g2)
