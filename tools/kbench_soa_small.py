"""SoA solver across N (the Table 8 sizes): device time per launch from HIP graphs of
back-to-back launches, shipped non-temporal kernel vs plain (cached) loads/stores
(hg_tune_soa variants), f64 as the reference's cal_Homo_ACA/SKS.  Bit-exact check."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    lib = pkg._lib.tune()
    lib.hg_tune_soa_variant_name.restype = ctypes.c_char_p
    lib.hg_tune_soa_variant_name.argtypes = [ctypes.c_int]
    f = lib.hg_tune_soa
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    f.restype = ctypes.c_int
    names = {v: lib.hg_tune_soa_variant_name(v).decode() for v in (0, 7)}
    dev = torch.device("cuda:0")
    out = {}
    for n in (1000, 10_000, 100_000, 1_000_000, 10_000_000):
        src = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(8, n).double()
        tar = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(8, n).double()
        Hs = {v: torch.empty((9, n), dtype=torch.float64, device=dev) for v in names}
        calls = 100 if n <= 100_000 else 20
        graphs = {}
        s = torch.cuda.Stream(dev)
        for v in names:
            def launch(v=v):
                assert f(0, v, src.data_ptr(), tar.data_ptr(), Hs[v].data_ptr(), n, 8,
                         torch.cuda.current_stream(dev).cuda_stream) == 0
            launch()
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(calls):
                        launch()
            torch.cuda.current_stream(dev).wait_stream(s)
            graphs[v] = g
        torch.cuda.synchronize()
        exact = bool(torch.equal(Hs[0].view(torch.int64), Hs[7].view(torch.int64)))
        times = {v: [] for v in names}
        for _ in range(9):
            for v, g in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / calls * 1e3)
        out[str(n)] = {names[v]: round(statistics.median(times[v]), 3) for v in names}
        out[str(n)]["bit_exact"] = exact
        print(n, out[str(n)], flush=True)
        del graphs, src, tar, Hs
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench_soa_small.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
