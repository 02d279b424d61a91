"""Short fixed dispatch list of the MRG32K3A kernels for rocprofv3 (round 3): the standalone
generator at 1 M .. 40 M words and several split thresholds, and the fused draws + gather +
solve at 1 M and 10 M hypotheses; each 10 times.  Run under
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mrg -- python tools/mrg_probe.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    lib = pkg.lib()
    t = pkg._lib.tune()
    vp, i64, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64
    t.hg_tune_mrg_words.argtypes = [vp, i64, u64, i64, vp]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev).cuda_stream
    buf = torch.empty(40_000_000, dtype=torch.int32, device=dev)
    for count in (1 << 20, 1 << 21, 4_000_000, 1 << 23, 40_000_000):
        for chunk in (16, 64, 1 << 30):
            for _ in range(10):
                assert t.hg_tune_mrg_words(buf.data_ptr(), count, 11, chunk, st) == 0
            torch.cuda.synchronize()
            print("words", count, chunk, flush=True)
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(dev)
    H = torch.empty((9, 10_000_000), dtype=torch.float64, device=dev)
    for n in (1_000_000, 10_000_000):
        for algo in (0, 1):
            for _ in range(10):
                assert lib.hg_rand_gather_solve_f64(algo, ps.data_ptr(), pt.data_ptr(), ps.shape[0],
                                                    11, H.data_ptr(), n, 0, st) == 0
            torch.cuda.synchronize()
            print("fused", n, algo, flush=True)


if __name__ == "__main__":
    main()
