"""HBM ceilings on this box (tools/gpu_round.sh hbm_ceilings): read-only, write-only and
copy streams over 1 GB, each timed over 50 launches (median of 7 rounds), to place the
headline kernel's 64:36 read/write mix between them."""
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
    f = pkg._lib.tune().hg_tune_copy
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    f.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    nbytes = 1 << 30
    a = torch.ones(nbytes // 4, device=dev)
    b = torch.empty_like(a)
    st = torch.cuda.current_stream().cuda_stream
    names = {0: ("copy U4 nt", 2), 3: ("copy LDS-DMA", 2), 4: ("read-only U4 nt", 1),
             5: ("write-only U4 nt", 1)}
    times = {v: [] for v in names}
    for v in names:
        for _ in range(5):
            assert f(v, a.data_ptr(), b.data_ptr(), nbytes, st) == 0
    for _ in range(7):
        for v in names:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                f(v, a.data_ptr(), b.data_ptr(), nbytes, st)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 50)
    out = {}
    for v, (name, mult) in names.items():
        ms = statistics.median(times[v])
        out[name] = {"ms": round(ms, 4), "gbps": round(nbytes * mult / ms / 1e6, 1)}
        print(name, out[name], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "hbm_ceilings.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
