"""hg_sum_aten_f32 (csrc/hg_reduce.hpp) against ATen-CPU's float32 sum order, and the
batch-uniform TensorACA scale / div gradients at the reference's batch size and beyond.

Pins:
  * the kernel equals oracle/aten_sum.py (pinned against torch.sum by
    tests/test_aten_sum_order.py) bit for bit over run lengths 0 .. 12.6 M, every cascade
    depth, thread counts 1 .. 64, one and several rows, strided rows, special values;
  * it equals torch.sum on THIS box's CPU with this process's thread count;
  * tests/golden/torch_rect_grad_large.npz: ATen autograd through the reference's
    TensorACA_rect statements at B = 64 K (BASELINE configs[3]) and 1 M, for every recorded
    at::get_num_threads(): the op's dL/dscale, dL/ddiv bit for bit (aten_threads = T), and
    dL/dtar's SHA-256.
"""
import hashlib
import os
import sys

import numpy as np
import pytest
import torch

from conftest import load_golden

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
from aten_sum import aten_column_sums, aten_sum  # noqa: E402

pytestmark = pytest.mark.gpu


def _data(m, seed):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal(m) * 10.0 ** rng.integers(-3, 4, m)).astype(np.float32)


def _sum_gpu(pkg, dev, x_np, rows, m, row_stride, es, lanes, threads):
    x = torch.from_numpy(x_np).to(dev)
    out = torch.full((rows,), 7.0, device=dev)
    pkg._lib.call("hg_sum_aten_f32", x.data_ptr(), rows, m, row_stride, es, lanes, threads,
                  out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    return out.cpu().numpy()


@pytest.mark.parametrize("T", [1, 2, 8, 16, 64])
def test_kernel_equals_restatement(orc, pkg, dev, T):
    for m in (0, 1, 7, 8, 33, 255, 4097, 32767, 32768, 65537, 196608, 1048579, 3 * 4194304 + 5):
        if m > 2_000_000 and T not in (1, 16):
            continue
        x = _data(m, m + 31 * T)
        got = _sum_gpu(pkg, dev, x, 1, m, 0, 1, 8, T)
        want = np.array([aten_sum(x, 8, T)], np.float32)
        assert got.tobytes() == want.tobytes(), (m, T, got, want)


@pytest.mark.parametrize("m,T", [(2**25 + 63, 2), (3 * 2**24 + 95, 3)])
def test_last_run_with_a_smaller_level_step(orc, pkg, dev, m, T):
    """Chunked runs whose LAST (shorter) chunk falls below a level-power boundary: run 0 has
    2^19 + 1 rows per stream (step 32, 512 super-blocks), the last 2^19 (step 16, 2048
    super-blocks).  The launch grids must cover the largest extent over every run, not run
    0's (grids sized from run 0 skipped the last run's super-blocks 513..2047)."""
    x = _data(m, 77 + T)
    got = _sum_gpu(pkg, dev, x, 1, m, 0, 1, 8, T)
    want = np.array([aten_sum(x, 8, T)], np.float32)
    assert got.tobytes() == want.tobytes(), (m, T, got, want)


def test_rows_strides_and_column_form(orc, pkg, dev):
    """Several rows at once; a (B,3) array's columns as strided rows (elem stride 3) and as
    (3,B) rows, both in the one-lane column order of a (3,1) parameter."""
    for B in (5, 1000, 65536, 262147):
        x = _data(3 * B, B).reshape(B, 3)
        want = aten_column_sums(x)
        got_strided = _sum_gpu(pkg, dev, np.ascontiguousarray(x), 3, B, 1, 3, 1, 1)
        got_rows = _sum_gpu(pkg, dev, np.ascontiguousarray(x.T), 3, B, B, 1, 1, 1)
        assert got_strided.tobytes() == want.tobytes(), B
        assert got_rows.tobytes() == want.tobytes(), B
    m = 200003
    xs = np.stack([_data(m, 1), _data(m, 2)])
    got = _sum_gpu(pkg, dev, xs, 2, m, m, 1, 8, 8)
    want = np.array([aten_sum(xs[0], 8, 8), aten_sum(xs[1], 8, 8)], np.float32)
    assert got.tobytes() == want.tobytes()


def test_special_values(orc, pkg, dev):
    rng = np.random.default_rng(4)
    vals = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, 3e38, -3e38, 1e-45], np.float32)
    for m in (1, 9, 64, 70001, 300000):
        for T in (1, 8):
            x = rng.choice(vals, m).astype(np.float32)
            got = _sum_gpu(pkg, dev, x, 1, m, 0, 1, 8, T)[0]
            want = np.float32(aten_sum(x, 8, T))
            assert (np.isnan(got) and np.isnan(want)) or got.tobytes() == want.tobytes(), (m, T)
    neg0 = np.full(100, -0.0, np.float32)
    assert _sum_gpu(pkg, dev, neg0, 1, 100, 0, 1, 8, 1).tobytes() == \
        torch.from_numpy(neg0).sum().numpy().reshape(1).tobytes()


def test_kernel_equals_torch_sum_on_this_box(pkg, dev):
    """torch.sum on the GPU box's own CPU, with this process's ATen thread count."""
    T = torch.get_num_threads()
    for m in (1000, 40000, 600009, 3 * 1048576):
        x = _data(m, m)
        want = torch.from_numpy(x).sum().numpy().reshape(1)
        got = _sum_gpu(pkg, dev, x, 1, m, 0, 1, 8, min(T, 1024))
        assert got.tobytes() == want.tobytes(), (m, T)


def test_argument_checks(pkg, dev):
    x = torch.zeros(10, device=dev)
    out = torch.zeros(1, device=dev)
    bad = [(1, 10, 0, 1, 0, 1), (1, 10, 0, 1, 17, 1), (1, 10, 0, 1, 8, 0), (1, 10, 0, 1, 8, 1025),
           (1, 10, 0, 1, 2, 4), (-1, 10, 0, 1, 8, 1), (1, -1, 0, 1, 8, 1)]
    for rows, m, rs, es, lanes, threads in bad:
        assert pkg._lib.lib().hg_sum_aten_f32(x.data_ptr(), rows, m, rs, es, lanes, threads,
                                              out.data_ptr(), None) != 0, (lanes, threads)


def test_large_batch_gradients_equal_reference_autograd(orc, oracle, pkg, dev):
    """B = 64 K and 1 M: the op's batch-uniform and per-row scale / div gradients equal ATen
    autograd's through the reference statements for every thread count the fixture holds."""
    g = load_golden("torch_rect_grad_large.npz")
    seed = int(g["seed"])
    for B in (int(b) for b in g["B"]):
        sh, th, gH = (torch.from_numpy(a).to(dev) for a in orc.rect_grad_batch(oracle, B, seed + B))
        for tag in ("uniform", "frac", "per_row"):
            key = f"B{B}_{tag}"
            sc = torch.from_numpy(g[f"{key}_scale"]).to(dev)
            dv = torch.from_numpy(g[f"{key}_div"]).to(dev)
            Ts = sorted(int(k.split("_T")[1].split("_")[0]) for k in g
                        if k.startswith(key + "_T") and k.endswith("_gscale"))
            for T in Ts:
                _, g_tar, g_sc, g_dv = pkg.tensor_aca_rect_backward(sh, th, gH, sc, dv, False, True,
                                                                    aten_threads=T)
                assert g_sc.cpu().numpy().tobytes() == g[f"{key}_T{T}_gscale"].tobytes(), (key, T)
                assert g_dv.cpu().numpy().tobytes() == g[f"{key}_T{T}_gdiv"].tobytes(), (key, T)
                digest = hashlib.sha256(g_tar.cpu().numpy().tobytes()).hexdigest()
                assert digest == str(g[f"{key}_T{T}_gtar_sha256"]), (key, T)
