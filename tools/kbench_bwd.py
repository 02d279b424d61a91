"""TensorACA backward kernels (rect and compact forms) at B = 64 K and 16 M: device time
per call from HIP-graph replays, algorithmic GB/s.  Bytes per problem: rect in tar 48 +
src 8 + dL/dH 36, out dL/dtar 48 (+ dL/dsrc 48 + scale/div partials 8); compact in
corner 8 + offsets 32 + dL/dH 36, out dL/doffsets 32 (+ dL/dcorner 8)."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def timed(fn, calls):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(calls):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / calls * 1e3)
    return statistics.median(ts)


def main():
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    out = {}
    for B in (65536, 16 << 20):
        torch.manual_seed(0)
        _, _, src, tar, sc, dv = pkg.adjust(dev, B)
        gH = torch.randn(B, 3, 3, device=dev)
        corner = src[:, 0:2, 0].contiguous()
        offs = (tar[:, 0:2, :] - src[:, 0:2, :]).transpose(1, 2).contiguous()
        calls = 100 if B <= 65536 else 10
        cases = {
            "rect bwd (tar only)": (lambda: pkg.tensor_aca_rect_backward(src, tar, gH, sc, dv, False, False), 92 + 48),
            "rect bwd (all)": (lambda: pkg.tensor_aca_rect_backward(src, tar, gH, sc, dv, True, True), 92 + 48 + 48 + 8),
            "offsets bwd (offsets only)": (lambda: pkg.tensor_aca_offsets_backward(corner, offs, gH, 128.0, 128.0, False), 76 + 32),
            "offsets bwd (+corner)": (lambda: pkg.tensor_aca_offsets_backward(corner, offs, gH, 128.0, 128.0, True), 76 + 40),
            "offsets fwd": (lambda: pkg.tensor_aca_offsets(corner, offs, 128.0, 128.0), 76),
        }
        if B % 64 == 0:  # the all-gradient kernel alone and its no-arithmetic twin (tune library)
            t = pkg._lib.tune()
            vp = ctypes.c_void_p
            t.hg_tune_rect_backward.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int64, vp, vp, vp,
                                                vp, vp, vp]
            gs_, gt_ = torch.empty_like(src), torch.empty_like(tar)
            terms = torch.empty((2, B, 3), device=dev)
            cur = lambda: torch.cuda.current_stream(dev).cuda_stream  # noqa: E731 -- the capture stream
            for v, name in ((0, "rect bwd kernel (all, raw)"), (1, "rect bwd kernel twin (no arithmetic)")):
                cases[name] = ((lambda v=v: t.hg_tune_rect_backward(
                    v, src.data_ptr(), tar.data_ptr(), gH.data_ptr(), B, sc.data_ptr(), dv.data_ptr(),
                    gs_.data_ptr(), gt_.data_ptr(), terms.data_ptr(), cur())), 92 + 48 + 48 + 24)
            # a copy of the same 252 B per problem (hg_stream_copy: half read, half written)
            cbuf = torch.empty(B * 126 // 4, dtype=torch.float32, device=dev)
            cdst = torch.empty_like(cbuf)
            cases["copy yardstick (252 B per problem)"] = (
                lambda: pkg._lib.call("hg_stream_copy", cbuf.data_ptr(), cdst.data_ptr(), B * 126, cur()),
                252)
        res = {}
        for name, (fn, bpp) in cases.items():
            us = timed(fn, calls)
            res[name] = {"us": round(us, 2), "algorithmic_gbps": round(B * bpp / us / 1e3, 1)}
            print(B, name, res[name], flush=True)
        out[str(B)] = res
        del src, tar, gH, corner, offs
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench_bwd.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
