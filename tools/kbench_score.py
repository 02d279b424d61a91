"""RANSAC scorer variant sweep (interleaved, one process); counts must match the
shipped scorer exactly."""
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


NV = 7  # hg_tune_score variants (csrc/hg_ransac.hip)


def main():
    pkg = ge.load_package()
    lib = pkg._lib.tune()
    lib.hg_tune_score.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_uint32, ctypes.c_float,
                                  ctypes.c_void_p, ctypes.c_void_p]
    lib.hg_tune_score.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"]).to(dev)
    pt = torch.from_numpy(g["pool_tar"]).to(dev)
    n = 1 << 20
    idx = pkg.fill_bits(n * 4, 11, 0, dev).view(n, 4)
    H = pkg.sample_solve(ps, pt, idx)
    want = pkg.ransac_score(H, ps, pt, 3.0)
    out = torch.empty_like(want)
    sp = torch.cuda.current_stream(dev).cuda_stream
    res = {}
    times = {v: [] for v in range(NV)}
    for v in range(NV):
        assert lib.hg_tune_score(v, H.data_ptr(), n, ps.data_ptr(), pt.data_ptr(), ps.shape[0],
                                 3.0, out.data_ptr(), sp) == 0
        torch.cuda.synchronize()
        res[v] = bool(torch.equal(out, want))
    for _ in range(5):
        for v in range(NV):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                lib.hg_tune_score(v, H.data_ptr(), n, ps.data_ptr(), pt.data_ptr(), ps.shape[0],
                                  3.0, out.data_ptr(), sp)
            e1.record()
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / 5)
    pairs = n * ps.shape[0]
    recs = []
    for v in range(NV):
        med = statistics.median(times[v])
        rec = {"variant": v, "ms": round(med, 4), "G_pairs_per_s": round(pairs / med / 1e6, 1),
               "exact": res[v]}
        recs.append(rec)
        print(json.dumps(rec))
    with open(os.path.join(ROOT, "gpurun_out", "kbench_score.json"), "w") as f:
        json.dump(recs, f, indent=1)


if __name__ == "__main__":
    main()
