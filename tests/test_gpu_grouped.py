"""Many small batches in few launches (hg_solve_grouped_*, ops.solve_grouped): every batch's
H bit-identical to solving it alone (which tests/test_gpu_parity.py pins to the oracle),
ragged sizes including empty batches, more batches than one launch carries, both layouts,
both precisions, every solver; one group also checked against the oracle directly."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [1, 0, 63, 64, 65, 255, 256, 257, 1000, 4097, 2, 3] * 6  # 72 batches: 3 launches


def _bits(x):
    return x.view(torch.int32 if x.dtype is torch.float32 else torch.int64)


def _batches(pkg, dev, dtype, layout, sizes, seed=9):
    srcs, tars, off = [], [], 0
    for m in sizes:
        s = pkg.fill_uniform(max(m, 1) * 8, seed, off, device=dev)[:m * 8]
        t = pkg.fill_uniform(max(m, 1) * 8, seed, off + 10_000_000, device=dev)[:m * 8]
        off += 8 * max(m, 1)
        shape = (m, 8) if layout == "aos" else (8, m)
        srcs.append(s.view(shape).to(dtype).contiguous())
        tars.append(t.view(shape).to(dtype).contiguous())
    return srcs, tars


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("layout", ["aos", "soa"])
def test_grouped_matches_per_batch(pkg, dev, dtype, layout):
    srcs, tars = _batches(pkg, dev, dtype, layout, SIZES)
    algos = ["aca", "sks", "ge"] + (["gpt"] if dtype is torch.float64 else [])
    for algo in algos:
        for norm in (True, False):
            got = pkg.solve_grouped(algo, srcs, tars, normalize=norm, layout=layout)
            for i, (s, t, h) in enumerate(zip(srcs, tars, got)):
                want = pkg.solve(algo, s, t, normalize=norm, layout=layout) if s.numel() else h
                assert torch.equal(_bits(h), _bits(want)), (algo, norm, i, SIZES[i])


def test_grouped_vs_oracle(pkg, dev, oracle):
    srcs, tars = _batches(pkg, dev, torch.float32, "aos", [5, 300, 77], seed=4)
    for algo in ("aca", "sks"):
        got = pkg.solve_grouped(algo, srcs, tars)
        for s, t, h in zip(srcs, tars, got):
            want = oracle.solve(algo, s.cpu().numpy(), t.cpu().numpy(), normalize=True)
            assert np.array_equal(h.cpu().numpy().view(np.uint32), want.view(np.uint32))


def test_grouped_out_and_errors(pkg, dev):
    srcs, tars = _batches(pkg, dev, torch.float32, "aos", [10, 20])
    outs = [torch.full((10, 9), float("nan"), device=dev), torch.full((20, 9), float("nan"), device=dev)]
    got = pkg.solve_grouped("aca", srcs, tars, outs=outs)
    assert got[0].data_ptr() == outs[0].data_ptr()
    assert torch.equal(_bits(outs[1]), _bits(pkg.solve("aca", srcs[1], tars[1])))
    assert pkg.solve_grouped("aca", [], []) == []
    with pytest.raises(ValueError):
        pkg.solve_grouped("aca", srcs, tars[:1])
    with pytest.raises(TypeError):
        pkg.solve_grouped("gpt", srcs, tars)


def test_grouped_in_a_graph(pkg, dev):
    """The grouped launches are capturable like every other entry point."""
    srcs, tars = _batches(pkg, dev, torch.float64, "soa", [1000] * 40)
    outs = [torch.empty((9, 1000), dtype=torch.float64, device=dev) for _ in srcs]
    want = [pkg.solve("aca", s, t, normalize=False, layout="soa") for s, t in zip(srcs, tars)]
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        pkg.solve_grouped("aca", srcs, tars, normalize=False, layout="soa", outs=outs)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            pkg.solve_grouped("aca", srcs, tars, normalize=False, layout="soa", outs=outs)
    torch.cuda.current_stream(dev).wait_stream(s)
    for o in outs:
        o.zero_()
    g.replay()
    torch.cuda.synchronize(dev)
    for o, w in zip(outs, want):
        assert torch.equal(_bits(o), _bits(w))
