"""Probe: bench's 10 M one-launch Table-8 timing (table8_pipeline_section's large part: warm-up
of one-launch / two-launch / write-only, then launch_stats of the one-launch kernel) run
standalone, ACA then SKS and SKS then ACA, three times -- to see whether the bench's SKS
figure (~150 us against 118-137 us in the kernel sweeps) is the kernel or its context.
    python tools/t8_order_probe.py   -> gpurun_out/t8_order_probe.json"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    d = bench.Dist("gloo")
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(d.dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(d.dev)
    stream = torch.cuda.current_stream(d.dev).cuda_stream
    big = 10_000_000
    tune = pkg._lib.tune()
    import ctypes
    tune.hg_tune_copy.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    wbuf = torch.empty(big * 18, dtype=torch.float32, device=d.dev)
    f_write = lambda: tune.hg_tune_copy(5, None, wbuf.data_ptr(), big * 72, stream)  # noqa: E731
    wb = torch.empty(4 * big, dtype=torch.int32, device=d.dev)
    out = []
    for rep in range(3):
        for order in (("aca", "sks"), ("sks", "aca")):
            rec = {"rep": rep, "order": "->".join(order)}
            for algo in order:
                aid = {"aca": 0, "sks": 1}[algo]
                Hb = torch.empty((9, big), dtype=torch.float64, device=d.dev)
                f_one = lambda: pkg._lib.call("hg_rand_gather_solve_f64", aid, ps.data_ptr(), pt.data_ptr(),  # noqa: E731
                                              ps.shape[0], 11, Hb.data_ptr(), big, 0, stream)

                def f_two():
                    pkg._lib.call("hg_rand_mrg32k3a_u32", wb.data_ptr(), 4 * big, 11, stream)
                    pkg._lib.call("hg_gather_solve_f64", aid, ps.data_ptr(), pt.data_ptr(), ps.shape[0],
                                  wb.data_ptr(), Hb.data_ptr(), big, 0, stream)

                for _ in range(5):
                    f_one()
                    f_two()
                    f_write()
                rec[algo] = bench.launch_stats(d, f_one, groups=10)["median_us"]
                rec[algo + "_alone"] = bench.launch_stats(d, f_one, groups=10)["median_us"]
                del Hb
            print(rec, flush=True)
            out.append(rec)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "t8_order_probe.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
