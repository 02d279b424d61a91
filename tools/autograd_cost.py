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
    return round((time.perf_counter() - t0) / n * 1e6, 2)


def graphed_us(step, n=2000):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(5):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    return per_call_us(g.replay, n), g


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

    out["aca_vanilla"] = {
        "full": per_call_us(full),
        "op": per_call_us(op),
        "op_grad": per_call_us(lambda: torch.autograd.grad(ops.aca.default(S, T, False), (S, T), gH)),
        "fwd_grad": per_call_us(lambda: ops.aca.default(S, T, False)),
    }
    with torch.no_grad():
        out["aca_vanilla"]["fwd_nograd"] = per_call_us(lambda: ops.aca.default(S, T, False))
    Hb = torch.empty(B, 3, 3, device=dev)
    gs, gt = torch.empty_like(src), torch.empty_like(tar)
    lib = pkg._lib.lib()
    st = torch.cuda.current_stream(dev).cuda_stream
    sp, tp, hp, gp = src.data_ptr(), tar.data_ptr(), Hb.data_ptr(), gH.data_ptr()
    gsp, gtp = gs.data_ptr(), gt.data_ptr()

    def raw():
        lib.hg_aca_f32(sp, tp, hp, B, 0, 0, st)
        lib.hg_aca_backward_f32(sp, tp, gp, B, gsp, gtp, st)

    out["aca_vanilla"]["raw"] = per_call_us(raw)
    x = torch.ones(1, device=dev, requires_grad=True)
    g1 = torch.ones(1, device=dev)

    def floor():
        x.grad = None
        (x * 2.0).backward(g1)

    out["engine_floor"] = per_call_us(floor)

    # graph-captured full step: .grad tensors accumulate in the graph's own memory
    def gstep():
        S.grad = None
        T.grad = None
        ops.aca.default(S, T, False).backward(gH)
    try:
        us, g = graphed_us(gstep)
        out["aca_vanilla"]["graph"] = us
        del g
    except Exception as e:  # noqa: BLE001
        out["aca_vanilla"]["graph"] = f"{type(e).__name__}: {e}"

    Th = th.clone().requires_grad_()

    def rect_full():
        Th.grad = None
        pkg.TensorACA_rect(B, sh, Th, sc, dv).backward(gH)

    def rect_op():
        Th.grad = None
        ops.tensor_aca_rect.default(sh, Th, sc, dv).backward(gH)

    out["tensor_aca_rect"] = {"full": per_call_us(rect_full), "op": per_call_us(rect_op)}
    try:
        us, g = graphed_us(rect_op)
        out["tensor_aca_rect"]["graph"] = us
        del g
    except Exception as e:  # noqa: BLE001
        out["tensor_aca_rect"]["graph"] = f"{type(e).__name__}: {e}"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
