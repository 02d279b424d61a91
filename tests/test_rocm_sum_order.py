"""ATen-ROCm's float32 GPU sum, restated (oracle/aten_rocm_sum.py), against its own output on
the MI355X (tests/golden/rocm_sum.npz, tools/make_rocm_sum_golden.py): the order torch-ROCm's
autograd sums TensorACA_rect's (B,3,1) scale / div gradient terms to a (1,) or (3,1)
parameter -- the last reduction of the reference's device='cuda' run (.py:301-302, :393) that
order="rocm" reproduces (hg_sum_rocm_f32; tests/test_gpu_rect_rocm_order.py on the GPU)."""
import os
import sys

import numpy as np
import pytest

from conftest import load_golden

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import aten_rocm_sum as ars  # noqa: E402


@pytest.fixture(scope="module")
def gold():
    return load_golden("rocm_sum.npz")


def test_restatement_reproduces_the_gpu_sums(gold):
    num_mp, max_tpm = int(gold["num_mp"]), int(gold["max_tpm"])
    assert int(gold["warp"]) == ars.WARP
    bad = []
    for kind, B, seed, flavour, bits in zip(gold["kind"], gold["B"], gold["seed"], gold["flavour"],
                                            gold["bits"]):
        t = ars.rocm_sum_case(str(kind), int(B), int(seed), str(flavour))
        got = ars.rocm_sum(t, str(kind), num_mp, max_tpm)
        want = bits[:got.size]
        if not (got.view(np.uint32) == want).all():
            bad.append((str(kind), int(B), str(flavour)))
    assert not bad, bad[:10]
    assert len(gold["B"]) == 198


def test_configs_cover_every_regime(gold):
    """The fixture's sizes reach every launch shape the two reductions take: unvectorised and
    vectorised full sums, one and many CTAs, and column sums with and without the y split."""
    num_mp, max_tpm = int(gold["num_mp"]), int(gold["max_tpm"])
    shapes = set()
    for kind, B in zip(gold["kind"], gold["B"]):
        if str(kind) == "cols" and int(B) < 2:
            continue
        c = ars.Config(str(kind), int(B), num_mp, max_tpm)
        shapes.add((str(kind), c.vectorize, c.ctas > 1, c.input_mult[1] != 0, c.bw, c.bh))
    assert ("full", False, False, False, 64, 1) in shapes or any(
        s[0] == "full" and not s[1] for s in shapes)
    assert any(s[0] == "full" and s[1] and s[2] for s in shapes)       # vectorised, global
    assert any(s[0] == "full" and s[1] and not s[2] for s in shapes)   # vectorised, one CTA
    assert any(s[0] == "cols" and s[3] for s in shapes)                # y split
    assert any(s[0] == "cols" and not s[3] for s in shapes)            # one thread per column


def test_signed_zero_sums_start_from_plus_zero():
    for kind in ("full", "cols"):
        t = -np.zeros((1000, 3), np.float32)
        r = ars.rocm_sum(t, kind, 256, 2048)
        assert (r.view(np.uint32) == 0).all()


def test_library_plans_the_restated_launch(pkg):
    """hg_sum_rocm_plan (the C++ host side of hg_sum_rocm_f32) picks ATen's launch shape --
    the restatement's Config -- for every B from 2 to 5000 and a spread beyond, on this GPU's
    (256 CUs, 2048 threads per CU) and on other CU counts."""
    import ctypes
    lib = pkg.lib()
    plan = (ctypes.c_int64 * 12)()
    sizes = list(range(2, 5001)) + [10922, 10923, 43690, 43691, 65536, 100003, 174762, 174763,
                                     262144, 1 << 20, 3_000_001, 1 << 24, 700_000_000]
    for num_mp, max_tpm in ((256, 2048), (304, 2048), (120, 2048), (80, 2048), (64, 1024)):
        for kind_i, kind in ((0, "full"), (1, "cols")):
            for B in sizes if num_mp == 256 else sizes[::37]:
                assert lib.hg_sum_rocm_plan(B, kind_i, num_mp, max_tpm, plan) == 0
                c = ars.Config(kind, B, num_mp, max_tpm)
                want = (c.bw, c.bh, c.ctas, *c.input_mult, *c.output_mult, c.step_input,
                        c.step_output, int(c.vectorize), c.grid_x)
                assert tuple(plan) == want, (kind, B, num_mp, tuple(plan), want)
    assert lib.hg_sum_rocm_plan(1, 0, 256, 2048, plan) == 1
    assert lib.hg_sum_rocm_plan(5, 2, 256, 2048, plan) == 1
    assert lib.hg_sum_rocm_f32(None, 0, 0, None, None, None) == 1       # NULL out
    assert lib.hg_sum_rocm_f32(None, 5, 3, 16, None, None) == 1         # kind
    assert lib.hg_sum_rocm_f32(None, -1, 0, 16, None, None) == 1        # B < 0
    assert lib.hg_sum_rocm_f32(None, 5, 0, 16, None, None) == 1         # NULL x
