"""Where the time of one differentiable ACA_vanilla / TensorACA_rect step goes at the
config-4 batch (B = 64 K).  Host-bound steps: the per-call figure is
wall time over many back-to-back calls (the device idles between kernels), so each variant
below removes one layer:

  full          pkg.ACA_vanilla(...).backward(gH)         (bench's aca_vanilla_autograd)
  op            torch.ops.sks_amd.aca(S, T, False).backward(gH)   (no Python wrapper)
  op_grad       torch.autograd.grad(op, (S, T), gH)        (no AccumulateGrad into .grad)
  fwd_grad      the forward alone, inputs requiring grad   (graph node built, no backward)
  fwd_nograd    the forward alone under no_grad
  raw           hg_aca_f32 + hg_aca_backward_f32 through ctypes (the launches alone)
  engine_floor  a one-element mul + .backward()            (autograd's own per-step floor)
  graph         the full step captured once in a CUDA graph, replayed
and the same for TensorACA_rect with a grad-requiring tar.  Prints one JSON object.
Run on the GPU box: python tools/autograd_cost.py
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def per_call_us(fn, n=2000, warm=200):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def best_of(variants, rounds=3):
    """Each variant timed `rounds` times, interleaved (clock / allocator warm-up and
    neighbours on the box hit every variant alike); the minimum per variant."""
    best = {k: float("inf") for k in variants}
    for _ in range(rounds):
        for k, fn in variants.items():
            best[k] = min(best[k], per_call_us(fn))
    return {k: round(v, 2) for k, v in best.items()}


def graphed_us(step, per_graph=1, n=500):
    """us per step when `per_graph` steps are captured in one CUDA graph and replayed."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(5):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            step()
    us = per_call_us(g.replay, n, 20) / per_graph
    del g
    return round(us, 2)


def main():
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    B = 65536
    torch.manual_seed(0)
    src, tar, sh, th, sc, dv = pkg.adjust(dev, B)
    tar = (tar + torch.rand_like(tar)).contiguous()
    gH = torch.randn(B, 3, 3, device=dev)
    S, T = src.clone().requires_grad_(), tar.clone().requires_grad_()
    ops = torch.ops.sks_amd
    out = {"batch": B}

    def full():
        S.grad = None
        T.grad = None
        pkg.ACA_vanilla(B, S, T).backward(gH)

    def op():
        S.grad = None
        T.grad = None
        ops.aca.default(S, T, False).backward(gH)

    import bench
    Hb = torch.empty(B, 3, 3, device=dev)
    gs, gt = torch.empty_like(src), torch.empty_like(tar)
    lib = pkg._lib.lib()
    st = torch.cuda.current_stream(dev).cuda_stream
    sp, tp, hp, gp = src.data_ptr(), tar.data_ptr(), Hb.data_ptr(), gH.data_ptr()
    gsp, gtp = gs.data_ptr(), gt.data_ptr()

    def raw():
        lib.hg_aca_f32(sp, tp, hp, B, 0, 0, st)
        lib.hg_aca_backward_f32(sp, tp, gp, B, gsp, gtp, st)

    x = torch.ones(1, device=dev, requires_grad=True)
    g1 = torch.ones(1, device=dev)

    def floor():
        x.grad = None
        (x * 2.0).backward(g1)

    def torch_full():
        S.grad = None
        T.grad = None
        bench.torch_aca_vanilla(S, T).backward(gH)

    def nograd_wrapper():
        with torch.no_grad():
            pkg.ACA_vanilla(B, S, T)

    out["aca_vanilla"] = best_of({
        "full": full, "op": op,
        "op_grad": lambda: torch.autograd.grad(ops.aca.default(S, T, False), (S, T), gH),
        "fwd_grad": lambda: ops.aca.default(S, T, False),
        "fwd_nograd_wrapper": nograd_wrapper,
        "raw_two_launches": raw, "engine_floor_1elem_mul": floor,
        "torch_composed_full": torch_full,
    })

    def gstep():
        torch.autograd.grad(ops.aca.default(S, T, False), (S, T), gH)

    def gstep_torch():
        torch.autograd.grad(bench.torch_aca_vanilla(S, T), (S, T), gH)

    for name, fn in (("graph_1", (gstep, 1)), ("graph_100", (gstep, 100)),
                     ("torch_composed_graph_100", (gstep_torch, 100))):
        try:
            out["aca_vanilla"][name] = graphed_us(*fn)
        except Exception as e:  # noqa: BLE001
            out["aca_vanilla"][name] = f"{type(e).__name__}: {e}"

    Th = th.clone().requires_grad_()

    def rect_full():
        Th.grad = None
        pkg.TensorACA_rect(B, sh, Th, sc, dv).backward(gH)

    def rect_op():
        Th.grad = None
        ops.tensor_aca_rect.default(sh, Th, sc, dv).backward(gH)

    def rect_torch():
        Th.grad = None
        bench.torch_tensor_aca_rect(sh, Th, sc, dv).backward(gH)

    out["tensor_aca_rect"] = best_of({"full": rect_full, "op": rect_op, "torch_composed_full": rect_torch})
    for name, fn in (("graph_100", lambda: torch.autograd.grad(ops.tensor_aca_rect.default(sh, Th, sc, dv), (Th,), gH)),
                     ("torch_composed_graph_100",
                      lambda: torch.autograd.grad(bench.torch_tensor_aca_rect(sh, Th, sc, dv), (Th,), gH))):
        try:
            out["tensor_aca_rect"][name] = graphed_us(fn, 100)
        except Exception as e:  # noqa: BLE001
            out["tensor_aca_rect"][name] = f"{type(e).__name__}: {e}"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
