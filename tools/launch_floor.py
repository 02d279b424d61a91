"""Host-launch floor vs the solver's launch at tiny N (tools/gpu_round.sh launch_floor):
hg_tune_launch_loop runs `loops` back-to-back launches from C++, event-timed.  algo 2 is
an empty kernel (the raw launch floor)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
loop = pkg._lib.tune().hg_tune_launch_loop
loop.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                 ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
loop.restype = ctypes.c_double
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
s = torch.rand(8, 2048, dtype=torch.float64, device=dev)
H = torch.empty(9, 2048, dtype=torch.float64, device=dev)
for rep in range(2):
    row = {"empty": round(loop(2, 8, 0, 0, 0, 0, 1, 0, 20000, st), 2),
           "empty+getlasterror": round(loop(3, 8, 0, 0, 0, 0, 1, 0, 20000, st), 2)}
    a = torch.rand(8, 1000, dtype=torch.float64, device=dev)
    h = torch.empty(9, 1000, dtype=torch.float64, device=dev)
    row["aca1000_raw"] = round(loop(4, 8, a.data_ptr(), a.data_ptr(), h.data_ptr(), 1000, 1, 0,
                                    20000, st), 2)
    row["aca1000_raw_nt"] = round(loop(5, 8, a.data_ptr(), a.data_ptr(), h.data_ptr(), 1000, 1, 0,
                                       20000, st), 2)
    row["store_one"] = round(loop(6, 8, 0, 0, h.data_ptr(), 0, 1, 0, 20000, st), 2)
    for algo, name in ((8, "store_one_sc0sc1"), (9, "store_one_sc1"), (10, "store_one_sc0sc1nt"),
                       (11, "store_one_nt")):
        row[name] = round(loop(algo, 8, 0, 0, h.data_ptr(), 0, 1, 0, 20000, st), 2)
    row["load_one"] = round(loop(12, 8, a.data_ptr(), 0, h.data_ptr(), 0, 1, 0, 20000, st), 2)
    row["args_unused"] = round(loop(13, 8, a.data_ptr(), 0, h.data_ptr(), 0, 1, 0, 20000, st), 2)
    row["args_read"] = round(loop(14, 8, a.data_ptr(), 0, h.data_ptr(), 7, 1, 0, 20000, st), 2)
    row["aca1000_generic_raw"] = round(loop(7, 8, a.data_ptr(), a.data_ptr(), h.data_ptr(), 1000,
                                            1, 0, 20000, st), 2)
    for n in (1, 2, 3, 4, 10, 1000):
        for algo in (0, 1):
            # SoA views of n problems inside the (8, 2048) buffer need stride n: use fresh tensors
            a = torch.rand(8, n, dtype=torch.float64, device=dev)
            h = torch.empty(9, n, dtype=torch.float64, device=dev)
            row[f"{'aca' if algo == 0 else 'sks'}{n}"] = round(
                loop(algo, 8, a.data_ptr(), a.data_ptr(), h.data_ptr(), n, 1, 0, 20000, st), 2)
    for n in (1, 2, 3, 64, 65):  # AoS, f32 (n, 8) -> (n, 9)
        a = torch.rand(n, 8, device=dev)
        h = torch.empty(n, 9, device=dev)
        row[f"aos_f32_aca{n}"] = round(loop(0, 4, a.data_ptr(), a.data_ptr(), h.data_ptr(), n, 0, 1,
                                            20000, st), 2)
    row["HIP_FORCE_DEV_KERNARG"] = os.environ.get("HIP_FORCE_DEV_KERNARG")
    print(row, flush=True)
