"""The fused Table-8 SKS launch (10 M) over time: 60 groups of 20 back-to-back launches on one
output buffer, the mean of each group, then the same after a 2 s idle gap -- how many launches
the card takes to settle under this VALU-heavy load (tools/t8_placement_probe.py found the
launch time falling over the first few hundred launches whatever the buffer), and whether an
idle gap undoes it.  Also ACA and the write-only stream of the same 720 MB for reference.
    python tools/t8_ramp_probe.py  -> gpurun_out/t8_ramp.json"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
N = 10_000_000


def main():
    import numpy as np
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    H = torch.empty((9, N), dtype=torch.float64, device=dev)
    t = pkg._lib.tune()
    t.hg_tune_policy.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    w = torch.empty(N * 18, dtype=torch.float32, device=dev)

    def series(fn, groups=60, per=20):
        out = []
        for _ in range(groups):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(per):
                fn()
            e1.record()
            e1.synchronize()
            out.append(round(e0.elapsed_time(e1) * 1e3 / per, 1))
        return out

    sks = lambda: pkg._lib.call("hg_rand_gather_solve_f64", 1, ps.data_ptr(), pt.data_ptr(),  # noqa: E731
                                ps.shape[0], 11, H.data_ptr(), N, 0, st)
    aca = lambda: pkg._lib.call("hg_rand_gather_solve_f64", 0, ps.data_ptr(), pt.data_ptr(),  # noqa: E731
                                ps.shape[0], 11, H.data_ptr(), N, 0, st)
    wr = lambda: t.hg_tune_policy(0, w.data_ptr(), w.data_ptr(), N * 72, st)  # noqa: E731
    res = {"write_only_72B": series(wr, 10), "sks": series(sks)}
    time.sleep(2.0)
    res["sks_after_2s_idle"] = series(sks, 20)
    res["aca"] = series(aca, 30)
    res["sks_after_aca"] = series(sks, 20)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "t8_ramp.json"), "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res.items():
        print(k, v, flush=True)


if __name__ == "__main__":
    main()
