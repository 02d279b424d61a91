"""TensorACA tile sweep (tools/kbench_rect.py): hg_tune_rect variants (rect and compact
forms, P = 1/2/4 problems per lane) at small and large B.  Device time per launch from
a HIP graph of back-to-back launches (the small-B case is launch-bound on the host, so
eager timing would only measure the host), interleaved rounds, median reported; every
variant's output is compared bit for bit with the shipped op's."""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

NAMES = ["rect P1 (shipped)", "rect P2", "rect P4", "offsets P1 (shipped)", "offsets P2",
         "offsets P4", "rect P1 cached", "offsets P1 cached"]


def main():
    pkg = ge.load_package()
    lib = pkg._lib.tune()
    f = lib.hg_tune_rect
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                  ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
    f.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    out = {}
    for B in (4096, 65536, 1 << 20, 16 << 20):
        torch.manual_seed(0)
        _, _, src, tar, _, _ = pkg.adjust(dev, B)
        corner = src[:, 0:2, 0].contiguous()
        offs = (tar[:, 0:2, :] - src[:, 0:2, :]).transpose(1, 2).contiguous()
        want_r = pkg.tensor_aca_rect(src, tar, 128.0, 1.0)
        want_o = pkg.tensor_aca_offsets(corner, offs, 128.0, 128.0)
        H = torch.empty((B, 3, 3), device=dev)
        calls = 100 if B <= 65536 else 10
        graphs, ok = {}, {}
        s = torch.cuda.Stream(dev)
        for v, name in enumerate(NAMES):
            is_rect = name.startswith("rect")
            a, b = (src, tar) if is_rect else (corner, offs)
            wb = (128.0, 1.0) if is_rect else (128.0, 128.0)

            def launch(v=v, a=a, b=b, wb=wb):
                rc = f(v, a.data_ptr(), b.data_ptr(), H.data_ptr(), B, wb[0], wb[1],
                       torch.cuda.current_stream(dev).cuda_stream)
                assert rc == 0, rc

            H.zero_()
            launch()
            torch.cuda.synchronize()
            ok[name] = bool(torch.equal(H.view(torch.int32),
                                        (want_r if is_rect else want_o).view(torch.int32)))
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(calls):
                        launch()
            torch.cuda.current_stream(dev).wait_stream(s)
            graphs[name] = g
        times = {n: [] for n in NAMES}
        for _ in range(9):
            for name, g in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / calls * 1e3)
        res = {}
        for name in NAMES:
            med = statistics.median(times[name])
            bpp = 92 if name.startswith("rect") else 76
            res[name] = {"us": round(med, 3), "algorithmic_gbps": round(B * bpp / med / 1e3, 1),
                         "bit_exact": ok[name]}
            print(B, name, res[name], flush=True)
        out[str(B)] = res
        del graphs
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench_rect.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
