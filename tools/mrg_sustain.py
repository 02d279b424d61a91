"""Does the one-launch draws + gather + solve slow down under sustained back-to-back launches?
bench.py's table8_pipeline times 10 groups of 10 launches of one kernel; tools/kbench_mrg.py
interleaves groups of 5 with other kernels -- and the two disagreed at 10 M (SKS 160 vs
118-137 us on the same box).  This times the same launch in groups of 1, 5, 10, 50 and 200,
interleaved and back to back, ACA and SKS, 10 M hypotheses, with the write-only stream between.
    python tools/mrg_sustain.py   -> gpurun_out/mrg_sustain.json
"""
import ctypes
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def group_time(f, k, st):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(k):
        f()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k


def main():
    pkg = ge.load_package()
    lib = pkg.lib()
    t = pkg._lib.tune()
    t.hg_tune_policy.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                 ctypes.c_void_p]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    s = st.cuda_stream
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(dev)
    n = 10_000_000
    H = torch.empty((9, n), dtype=torch.float64, device=dev)
    w = torch.empty(n * 18, dtype=torch.float32, device=dev)
    out = {}
    fw = lambda: t.hg_tune_policy(0, w.data_ptr(), w.data_ptr(), n * 72, s)  # noqa: E731
    for algo, aid in (("aca", 0), ("sks", 1)):
        f = lambda: lib.hg_rand_gather_solve_f64(aid, ps.data_ptr(), pt.data_ptr(), ps.shape[0],  # noqa: E731
                                                 11, H.data_ptr(), n, 0, s)
        for _ in range(5):
            f()
        rec = {}
        for k in (1, 5, 10, 50, 200):
            samples = [group_time(f, k, st) for _ in range(max(3, 400 // k))]
            rec[f"back_to_back_{k}"] = round(statistics.median(samples), 2)
        inter = []
        for _ in range(20):
            fw()
            inter.append(group_time(f, 5, st))
        rec["after_write_5"] = round(statistics.median(inter), 2)
        rec["write_only_10"] = round(statistics.median([group_time(fw, 10, st) for _ in range(10)]), 2)
        out[algo] = rec
        print(algo, rec, flush=True)
    # placement: the same launch into other 720 MB buffers (bench.py allocates one per
    # algorithm after a 160 MB word buffer), and SKS before ACA
    del H
    wb = torch.empty(4 * n, dtype=torch.int32, device=dev)
    for order in (("sks", 1), ("aca", 0)), (("aca", 0), ("sks", 1)):
        for algo, aid in order:
            Hb = torch.empty((9, n), dtype=torch.float64, device=dev)
            f = lambda: lib.hg_rand_gather_solve_f64(aid, ps.data_ptr(), pt.data_ptr(),  # noqa: E731
                                                     ps.shape[0], 11, Hb.data_ptr(), n, 0, s)
            for _ in range(5):
                f()
            key = f"{algo}_fresh_buffer_{order[0][0]}_first"
            out[key] = {"us": round(statistics.median([group_time(f, 10, st) for _ in range(10)]), 2),
                        "ptr_mod_2M": Hb.data_ptr() % (2 << 20)}
            print(key, out[key], flush=True)
            del Hb
    del wb
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "mrg_sustain.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
