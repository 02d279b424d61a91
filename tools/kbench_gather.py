"""The fused get_rand_list + cal_Homo_* kernel (hg_gather.hpp, binary64, the reference's formats)
in its tune shapes (hg_tune_gather_solve_f64: 0 pool in LDS with 1024-lane persistent blocks =
shipped, 1 global gather, 2 / 3 pool in LDS with 512 / 256-lane blocks, 4-6 the LDS forms with two
hypotheses per lane) on the reference's
wall file, 1 M and 10 M hypotheses.  Device time per launch from event-bracketed back-to-back
launches, interleaved rounds, median; algorithmic GB/s at 16 B of words + 72 B of H per
hypothesis.  Outputs compared bit for bit with variant 0."""
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

NAMES = {0: "pool in LDS, 1024-lane persistent blocks (shipped)", 1: "global gather",
         2: "pool in LDS, 512-lane blocks", 3: "pool in LDS, 256-lane blocks",
         4: "pool in LDS, 1024-lane blocks, 2 per lane", 5: "pool in LDS, 512-lane blocks, 2 per lane",
         6: "pool in LDS, 256-lane blocks, 2 per lane",
         7: "pool in LDS, 1024-lane blocks, default-policy H stores"}
if os.environ.get("KB_GATHER_VARIANTS"):  # e.g. "0,7"
    NAMES = {int(v): NAMES[int(v)] for v in os.environ["KB_GATHER_VARIANTS"].split(",")}
ROUNDS = int(os.environ.get("KB_ROUNDS", "7"))


def main():
    pkg = ge.load_package()
    f = pkg._lib.tune().hg_tune_gather_solve_f64
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    f.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    out = {}
    for algo in (0, 1):
        for n in (1_000_000, 10_000_000):  # even: the two-per-lane forms need it
            rl = pkg.rand_mrg32k3a(4 * n, 11, dev).view(4, n)
            Hs = {v: torch.empty((9, n), dtype=torch.float64, device=dev) for v in NAMES}

            def run(v):
                rc = f(v, algo, ps.data_ptr(), pt.data_ptr(), ps.shape[0], rl.data_ptr(),
                       Hs[v].data_ptr(), n, st)
                assert rc == 0, (v, rc)

            for v in NAMES:
                for _ in range(5):
                    run(v)
            times = {v: [] for v in NAMES}
            loops = 50 if n == 1_000_000 else 20
            for _ in range(ROUNDS):
                for v in NAMES:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(loops):
                        run(v)
                    e1.record()
                    e1.synchronize()
                    times[v].append(e0.elapsed_time(e1) * 1e3 / loops)
            ref = Hs[0].view(torch.int64)
            for v, name in NAMES.items():
                us = statistics.median(times[v])
                rec = {"us": round(us, 2), "gbps": round(n * 88 / (us * 1e-6) / 1e9, 1),
                       "bit_exact": bool(torch.equal(Hs[v].view(torch.int64), ref))}
                out[f"{'aca' if algo == 0 else 'sks'} n={n} {name}"] = rec
                print(f"{'aca' if algo == 0 else 'sks'} {n} {name} {rec}", flush=True)
            del rl, Hs
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench_gather.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
