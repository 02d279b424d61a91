"""hg_sum_rocm_f32 on the GPU against torch.sum on the same GPU -- ATen-ROCm's own float32
reduction, which torch-ROCm's autograd runs to sum TensorACA_rect's (B,3,1) scale / div
gradient terms to a (1,) or (3,1) parameter (at::sum_to) -- bit for bit, at the fixture's sizes
and beyond (up to 16 M problems, several CTAs per output), on aligned and unaligned buffers
(the kernel keeps the aligned tensor's order), and against tests/golden/rocm_sum.npz."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import load_golden

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import aten_rocm_sum as ars  # noqa: E402

pytestmark = pytest.mark.gpu


def _ours(pkg, x, B, kind):
    out = torch.empty(1 if kind == 0 else 3, device=x.device)
    ws = torch.empty(1024, device=x.device)
    pkg._lib.call("hg_sum_rocm_f32", x.data_ptr(), B, kind, out.data_ptr(), ws.data_ptr(),
                  torch.cuda.current_stream(x.device).cuda_stream)
    return out


def _torch(x, B, kind):
    v = x.view(B, 3, 1)
    return (v.sum_to_size(1) if kind == 0 else v.sum_to_size(3, 1)).reshape(-1)


def _same(orc, got, want, what):
    ok = orc.same_bits(got.cpu().numpy(), want.cpu().numpy())
    assert ok.all(), (what, got.cpu().numpy().tolist(), want.cpu().numpy().tolist())


SIZES = [0, 1, 2, 3, 5, 21, 42, 43, 100, 171, 341, 342, 1000, 1366, 2731, 10922, 10923,
         43690, 43691, 65536, 100003, 174763, 262144, 1 << 20, 3_000_001, 1 << 24]


@pytest.mark.parametrize("kind", [0, 1])
def test_equals_torch_sum_on_this_gpu(orc, pkg, dev, kind):
    props = torch.cuda.get_device_properties(dev)
    rng = np.random.default_rng(kind)
    for B in SIZES:
        t = (rng.standard_normal((B, 3)) * 10.0 ** rng.integers(-3, 4, (B, 1))).astype(np.float32)
        x = torch.from_numpy(t).to(dev).reshape(-1)
        want = _torch(x, B, kind) if B else torch.zeros(1 if kind == 0 else 3, device=dev)
        _same(orc, _ours(pkg, x, B, kind), want, (kind, B))
        if 2 <= B <= 262144:  # the restatement agrees on this device's properties too
            r = ars.rocm_sum(t, "full" if kind == 0 else "cols", props.multi_processor_count,
                             props.max_threads_per_multi_processor)
            _same(orc, torch.from_numpy(r), want, ("restated", kind, B))
        if B:  # the same values one float past an aligned address: the aligned order
            buf = torch.empty(3 * B + 1, device=dev)
            buf[1:] = x
            _same(orc, _ours(pkg, buf[1:], B, kind), want, ("unaligned", kind, B))


def test_fixture(orc, pkg, dev):
    g = load_golden("rocm_sum.npz")
    props = torch.cuda.get_device_properties(dev)
    if (props.multi_processor_count, props.max_threads_per_multi_processor) != (int(g["num_mp"]),
                                                                                int(g["max_tpm"])):
        pytest.skip("another device shape than the fixture's")
    for kind, B, seed, flavour, bits in zip(g["kind"], g["B"], g["seed"], g["flavour"], g["bits"]):
        t = ars.rocm_sum_case(str(kind), int(B), int(seed), str(flavour))
        x = torch.from_numpy(t).to(dev).reshape(-1)
        got = _ours(pkg, x, int(B), 0 if str(kind) == "full" else 1).cpu().numpy()
        assert (got.view(np.uint32) == bits[:got.size]).all(), (str(kind), int(B), str(flavour))


def test_special_values(orc, pkg, dev):
    """Signed zeros sum to +0 from ATen's +0 accumulators; Inf and NaN propagate as torch's."""
    for kind in (0, 1):
        for B in (7, 4096, 300_000):
            for fill in (-0.0, float("inf"), float("nan")):
                x = torch.full((3 * B,), fill, device=dev)
                x[::5] = -0.0
                _same(orc, _ours(pkg, x, B, kind), _torch(x, B, kind), (kind, B, fill))
