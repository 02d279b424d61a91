"""SoA solver across N (the Table 8 sizes): device time per launch from HIP graphs of
back-to-back launches, f64 as the reference's cal_Homo_ACA/SKS: the 16-B register form
(non-temporal / plain loads and stores), the LDS-DMA tile and the narrow one-problem-per-lane
form (non-temporal / plain) -- hg_tune_soa variants by name.  Bit-exact against the first."""
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
    lib.hg_tune_num_soa_variants.restype = ctypes.c_int
    dt = os.environ.get("KB_DT", "f64")
    w = "W8" if dt == "f64" else "W4"
    want = (f"{dt} G1 one-shot (shipped)", f"{dt} G1 one-shot plain (cached) ld/st",
            f"{dt} LDS-DMA tile nt", f"{dt} narrow {w} (1 problem per lane)",
            f"{dt} narrow {w} plain (cached) ld/st")
    tdt = torch.float64 if dt == "f64" else torch.float32
    allv = {lib.hg_tune_soa_variant_name(v).decode(): v
            for v in range(lib.hg_tune_num_soa_variants())}
    names = {allv[w]: w for w in want}
    first = allv[want[0]]
    dev = torch.device("cuda:0")
    out = {}
    for n in (1000, 10_000, 100_000, 1_000_000, 10_000_000):
        src = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(8, n).to(tdt)
        tar = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(8, n).to(tdt)
        Hs = {v: torch.empty((9, n), dtype=tdt, device=dev) for v in names}
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
        exact = all(bool(torch.equal(Hs[first].view(torch.int64), Hs[v].view(torch.int64)))
                    for v in names)
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
    with open(os.path.join(ROOT, "gpurun_out", f"kbench_soa_small_{dt}.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
