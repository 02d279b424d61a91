"""Store / load cache-policy bits on a 1 GB stream (tools/gpu_round.sh hbm_policy):
hg_tune_policy's buffer stores and loads with aux 0 / sc0 / nt / sc0|nt / sc1 / sc1|nt,
median of 7 interleaved rounds of 30 launches, beside the shipped write-only / read-only
(global_store / global_load nt) streams of hg_tune_copy."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

AUX = ["0", "sc0", "nt", "sc0|nt", "sc1", "sc1|nt"]


def main():
    pkg = ge.load_package()
    lib = pkg._lib.tune()
    fp, fc = lib.hg_tune_policy, lib.hg_tune_copy
    for f in (fp, fc):
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        f.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    nbytes = 1 << 30
    a = torch.ones(nbytes // 4, device=dev)
    b = torch.empty_like(a)
    st = torch.cuda.current_stream().cuda_stream
    cases = {f"store {x}": (fp, i) for i, x in enumerate(AUX)}
    cases.update({f"load {x}": (fp, 6 + i) for i, x in enumerate(AUX)})
    cases["write-only global nt (hg_tune_copy 5)"] = (fc, 5)
    cases["read-only global nt (hg_tune_copy 4)"] = (fc, 4)
    for name, (f, v) in cases.items():
        for _ in range(3):
            assert f(v, a.data_ptr(), b.data_ptr(), nbytes, st) == 0
    times = {k: [] for k in cases}
    for _ in range(7):
        for name, (f, v) in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(30):
                f(v, a.data_ptr(), b.data_ptr(), nbytes, st)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 30)
    out = {}
    for name in cases:
        ms = statistics.median(times[name])
        out[name] = {"ms": round(ms, 4), "gbps": round(nbytes / ms / 1e6, 1)}
        print(name, out[name], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "hbm_policy.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
