"""ATen-CPU's float32 sum order, restated in oracle/aten_sum.py, pinned on this CPU (no GPU).

The reference's batch-uniform scale / div gradients are ATen autograd's sum_to_size of the
(B,3,1) per-(problem, row) terms (Modules_Runtime_Test.py:301-302 under .backward()).  The
restatement must give torch.sum's bits:
  * over run lengths 0 .. 4.2 M: below and above the 32768-element grain, every cascade
    depth, ragged vector and scalar tails;
  * for several at::get_num_threads() values (the two-pass chunking);
  * for the strided column reduction of a (3,1) parameter;
and, through the oracle's per-row gradient terms, it must reproduce ATen autograd's own
gradients recorded in tests/golden/torch_rect_grad_large.npz for every thread count.
"""
import hashlib
import os
import sys

import numpy as np
import pytest
import torch

from conftest import load_golden

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
from aten_sum import aten_column_sums, aten_sum, ceil_log2  # noqa: E402

SIZES = [0, 1, 3, 7, 8, 9, 31, 32, 33, 255, 256, 257, 4095, 4097, 32767, 32768, 32769,
         65536, 100003, 196608, 262145, 1048577, 3 * 1048576 + 7]


@pytest.fixture
def threads():
    prev = torch.get_num_threads()
    yield
    torch.set_num_threads(prev)


def _data(m, seed):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal(m) * 10.0 ** rng.integers(-3, 4, m)).astype(np.float32)


@pytest.mark.parametrize("T", [1, 2, 3, 8, 16])
def test_full_reduction_bits_equal_torch_sum(threads, T):
    torch.set_num_threads(T)
    for m in SIZES:
        x = _data(m, m + T)
        want = torch.from_numpy(x).sum().numpy()
        got = aten_sum(x, lanes=8, threads=T)
        assert want.tobytes() == np.float32(got).tobytes(), (T, m, want, got)


def test_sum_kernel_is_8_lanes_on_this_host(threads):
    """ATen's sum runs its 8-lane build even where the capability is AVX-512: a 16-lane
    restatement differs from torch.sum where the 8-lane one does not."""
    torch.set_num_threads(1)
    x = _data(4097, 5)
    want = torch.from_numpy(x).sum().numpy().tobytes()
    assert np.float32(aten_sum(x, 8, 1)).tobytes() == want
    assert np.float32(aten_sum(x, 16, 1)).tobytes() != want


@pytest.mark.parametrize("T", [1, 8])
def test_column_sums_bits_equal_torch(threads, T):
    """(B,3,1) -> (3,1): each column in row_sum's one-lane order, independent of T."""
    torch.set_num_threads(T)
    for B in (1, 5, 63, 1024, 10923, 65536, 262147):
        x = _data(3 * B, B).reshape(B, 3)
        want = torch.from_numpy(x).view(B, 3, 1).sum(0).numpy().ravel()
        assert want.tobytes() == aten_column_sums(x).tobytes(), B


def test_special_values():
    """Signed zeros, infinities and NaN follow torch's float32 additions."""
    torch.set_num_threads(1)
    rng = np.random.default_rng(9)
    vals = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, 3e38, -3e38, 1e-45], np.float32)
    for m in (1, 7, 64, 70000):
        x = rng.choice(vals, m).astype(np.float32)
        want = torch.from_numpy(x).sum().numpy()
        got = np.float32(aten_sum(x, 8, 1))
        assert (np.isnan(want) and np.isnan(got)) or want.tobytes() == got.tobytes(), m
    assert np.float32(aten_sum(np.full(9, -0.0, np.float32), 8, 1)).tobytes() == \
        torch.full((9,), -0.0).sum().numpy().tobytes()


def test_ceil_log2():
    assert [ceil_log2(x) for x in (0, 1, 2, 3, 4, 5, 8, 9, 65536, 65537)] == [1, 1, 1, 2, 2, 3, 3, 4, 16, 17]


def test_fixture_gradients_are_oracle_terms_in_aten_order(oracle):
    """tests/golden/torch_rect_grad_large.npz (ATen autograd through the reference's
    statements at B = 64 K and 1 M, several thread counts): the oracle's (problem, row)
    gradient terms summed by aten_sum give every recorded dL/dscale, dL/ddiv bit for bit,
    and the thread count really changes the recorded bits (the test can fail)."""
    from oracle import rect_grad_batch
    g = load_golden("torch_rect_grad_large.npz")
    seed = int(g["seed"])
    differs = 0
    for B in (int(b) for b in g["B"]):
        sh, th, gH = rect_grad_batch(oracle, B, seed + B)
        for tag in ("uniform", "frac", "per_row"):
            key = f"B{B}_{tag}"
            sc, dv = g[f"{key}_scale"], g[f"{key}_div"]
            _, gt, gsr, gdr, _, _ = oracle.tensor_aca_rect_rows_backward(sh, th, gH, sc, dv)
            Ts = sorted(int(k.split("_T")[1].split("_")[0]) for k in g
                        if k.startswith(key + "_T") and k.endswith("_gscale"))
            seen = set()
            for T in Ts:
                want_s, want_d = g[f"{key}_T{T}_gscale"], g[f"{key}_T{T}_gdiv"]
                if tag == "per_row":
                    got_s, got_d = aten_column_sums(gsr), aten_column_sums(gdr)
                else:
                    got_s = np.array([aten_sum(gsr, 8, T)], np.float32)
                    got_d = np.array([aten_sum(gdr, 8, T)], np.float32)
                assert got_s.tobytes() == want_s.astype(np.float32).ravel().tobytes(), (key, T)
                assert got_d.tobytes() == want_d.astype(np.float32).ravel().tobytes(), (key, T)
                assert hashlib.sha256(gt.tobytes()).hexdigest() == str(g[f"{key}_T{T}_gtar_sha256"])
                seen.add((want_s.tobytes(), want_d.tobytes()))
            differs += len(seen) > 1
    assert differs >= 2, "the recorded gradients should depend on the thread count"
