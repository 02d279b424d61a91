"""The binary64 baseline solvers (GPT-LU, GE) in the SoA layout across the kernel shapes,
interleaved in one process (tools/gpu_round.sh kbench_gpt).  These two are VALU-bound, not
HBM-bound like ACA/SKS, so the shape the dispatcher picks for ACA (two problems per lane in
16-B registers when MALL-resident, one per lane beyond) is not necessarily theirs.  Every
variant's output is compared bit for bit with the shipped path; median of 5 rounds x 20."""
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

ALGOS = {"ge": 2, "gpt": 3}
VARIANTS = ("f64 G1 one-shot (shipped)", "f64 G1 one-shot plain (cached) ld/st", "f64 G2 one-shot",
            "f64 narrow W8 (1 problem per lane)", "f64 narrow W8 plain (cached) ld/st")


def main():
    rounds, iters = 5, 20
    pkg = ge.load_package()
    lib = pkg._lib.tune()
    lib.hg_tune_num_soa_variants.restype = ctypes.c_int
    lib.hg_tune_soa_variant_name.restype = ctypes.c_char_p
    lib.hg_tune_soa_variant_name.argtypes = [ctypes.c_int]
    lib.hg_tune_soa.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    lib.hg_tune_soa.restype = ctypes.c_int
    names = {lib.hg_tune_soa_variant_name(v).decode(): v for v in range(lib.hg_tune_num_soa_variants())}
    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream(dev).cuda_stream
    out = {}
    for n in (1_000_000, 10_000_000):
        s = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(8, n).double()
        t = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(8, n).double()
        H = torch.empty(9, n, dtype=torch.float64, device=dev)
        cases, bits = {}, {}
        for algo, a in ALGOS.items():
            want = pkg.solve(algo, s, t, normalize=False, layout="soa").clone()

            def shipped(algo=algo):
                pkg.solve(algo, s, t, normalize=False, layout="soa", out=H)
            cases[(algo, "shipped dispatch")] = shipped
            for name in VARIANTS:
                v = names[name]

                def run(a=a, v=v):
                    assert lib.hg_tune_soa(a, v, s.data_ptr(), t.data_ptr(), H.data_ptr(), n, 8, sp) == 0
                cases[(algo, name)] = run
            for key, f in cases.items():
                if key[0] != algo:
                    continue
                H.zero_()
                f()
                torch.cuda.synchronize()
                bits[key] = bool(torch.equal(H.view(torch.int64), want.view(torch.int64)))
            del want
        times = {k: [] for k in cases}
        for _ in range(rounds):
            for k, f in cases.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    f()
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / iters * 1e3)
        rec = {}
        for (algo, name), ts in times.items():
            us = statistics.median(ts)
            rec[f"{algo} | {name}"] = {"us": round(us, 2), "gbps": round(n * 200 / us / 1e3, 1),
                                       "bit_exact": bits[(algo, name)]}
            print(n, algo, name, rec[f"{algo} | {name}"], flush=True)
        out[f"n={n}"] = rec
        del s, t, H
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench_gpt.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
