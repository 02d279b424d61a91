"""Why the fused Table-8 launch (hg_rand_gather_solve_f64, 10 M, (9,n) binary64 H) runs at
different speeds on different output allocations of the same size (KERNEL_NOTES: 'placement'):
six H buffers allocated in turn, each timed over 20 back-to-back launches after 5 warm-up ones,
with the device address of each (its alignment), in three passes (buffer order, reversed, again):
a time tied to the buffer repeats, one tied to the run's clock does not.  Run under rocprofv3 --pmc with
PLACEMENT_PMC=1 (3 launches per buffer, in buffer order) to count address-translation misses
per launch (tools/pmc_tlb.py's counters).
    python tools/t8_placement_probe.py [--reduce counter_collection.csv]"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NBUF = 6
N = 10_000_000


def run():
    import numpy as np
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    Hs = [torch.empty((9, N), dtype=torch.float64, device=dev) for _ in range(NBUF)]
    pmc = os.environ.get("PLACEMENT_PMC") == "1"
    out = {"buffers": []}
    order = list(range(NBUF))
    passes = [order, order[::-1], order] if not pmc else [order]
    for algo, aid, idx, pas in [(a, i, o, k) for a, i in (("sks", 1), ("aca", 0))
                                for k, o in enumerate(passes)]:
        for i in idx:
            H = Hs[i]
            f = lambda: pkg._lib.call("hg_rand_gather_solve_f64", aid, ps.data_ptr(), pt.data_ptr(),  # noqa: E731
                                      ps.shape[0], 11, H.data_ptr(), N, 0, st)
            if pmc:
                for _ in range(3):
                    f()
                torch.cuda.synchronize()
                continue
            for _ in range(5):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            e1.synchronize()
            rec = {"algo": algo, "pass": pas, "buffer": i, "us": round(e0.elapsed_time(e1) * 1e3 / 20, 2),
                   "addr_mod_2MiB": H.data_ptr() % (2 << 20), "addr_hex": hex(H.data_ptr())}
            out["buffers"].append(rec)
            print(json.dumps(rec), flush=True)
    if not pmc:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", "t8_placement.json"), "w") as fh:
            json.dump(out, fh, indent=1)


def reduce(path):
    rows = list(csv.DictReader(open(path)))
    by = {}
    for r in rows:
        if "mrg_gather_solve" not in r.get("Kernel_Name", ""):
            continue
        key = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        by.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    disp = [by[k] for k in sorted(by)]
    res = []
    for j, c in enumerate(disp):
        res.append({"launch": j, "algo": "sks" if j < 3 * NBUF else "aca", "buffer": (j % (3 * NBUF)) // 3, **c})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--reduce":
        reduce(sys.argv[2])
    else:
        run()
