"""binary64 AoS variant sweep at 10 M (hg_tune_aos_f64): interleaved rounds, median per
launch, algorithmic GB/s at 200 B per problem, bits compared with the shipped path."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

NAMES = {0: "P1 nt lds-dma (shipped)", 1: "P2 nt lds-dma", 2: "P1 nt register-staged",
         3: "P1 lds-dma default policy", 4: "P1 nt lds-dma, NO SOLVE (pattern ceiling)"}


def main():
    pkg = ge.load_package()
    f = pkg._lib.tune().hg_tune_aos_f64
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_int64, ctypes.c_void_p]
    f.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    n = 10_000_000
    src = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(n, 8).double()
    tar = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(n, 8).double()
    H = torch.empty((n, 9), dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for algo in (0, 1):
        want = pkg.solve("aca" if algo == 0 else "sks", src, tar)
        exact, times = {}, {v: [] for v in NAMES}
        for v in NAMES:
            H.zero_()
            assert f(algo, v, src.data_ptr(), tar.data_ptr(), H.data_ptr(), n, st) == 0
            torch.cuda.synchronize()
            exact[v] = bool(torch.equal(H.view(torch.int64), want.view(torch.int64)))
        for _ in range(7):
            for v in NAMES:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    f(algo, v, src.data_ptr(), tar.data_ptr(), H.data_ptr(), n, st)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / 20 * 1e3)
        for v, name in NAMES.items():
            us = statistics.median(times[v])
            key = f"{'aca' if algo == 0 else 'sks'} {name}"
            out[key] = {"us": round(us, 2), "gbps": round(n * 200 / us / 1e3, 1), "bit_exact": exact[v]}
            print(key, out[key], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench_f64.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
