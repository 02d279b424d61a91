"""Workload for a counter pass over the seeded RANSAC sampler (tools/gpu_round.sh
pmc_sample): 16 M hypotheses over the 2540-pair wall pool, 3 ACA then 3 SKS launches.
`--reduce <counter_collection.csv> [out.json]` turns the pass into per-kernel figures:
VALU wave-instructions per 64 hypotheses (one per lane), VALU busy against the CU's busy
cycles (4 cycles per wave64 instruction), LDS instructions per 128 hypotheses."""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
N = 1 << 24
CUS = 256


def run():
    import numpy as np
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"]).to(dev)
    pt = torch.from_numpy(g["pool_tar"]).to(dev)
    for algo in ("aca", "sks"):
        for _ in range(3):
            pkg.sample_solve_seeded(ps, pt, N, 11, 0, algo=algo)
        torch.cuda.synchronize()
    # SAMPLE_VARIANTS="26,28,29": seeded tune shapes (hg_tune_sample_seeded), ACA, 3 launches each
    variants = [int(v) for v in os.environ.get("SAMPLE_VARIANTS", "").split(",") if v]
    if variants:
        import ctypes
        fs = pkg._lib.tune().hg_tune_sample_seeded
        fs.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64,
                       ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                       ctypes.c_void_p]
        H = torch.empty((N, 9), device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        for v in variants:
            for _ in range(3):
                assert fs(v, ps.data_ptr(), pt.data_ptr(), ps.shape[0], 11, 0, H.data_ptr(), N, 0, 1, st) == 0
            torch.cuda.synchronize()
    print("pmc_sample done")


def reduce(path):
    per = {}
    meta = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "sample_solve" not in name:
            continue
        per.setdefault(name, {}).setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
        meta[name] = {k: r.get(k) for k in ("Grid_Size", "Workgroup_Size", "VGPR_Count", "LDS_Block_Size")}
    out = {}
    for name, disp in per.items():
        keys = sorted(set().union(*disp.values()))
        med = {k: statistics.median(d[k] for d in disp.values() if k in d) for k in keys}
        busy = med["SQ_BUSY_CU_CYCLES"] / CUS
        quad = med["SQ_ACTIVE_INST_VALU"] / (CUS * 4)
        out[name] = {**meta[name], "dispatches": len(disp), "median_counters": med, "derived": {
            "valu_wave_instr_per_64_hypotheses": round(med["SQ_INSTS_VALU"] / (N / 64), 1),
            "lds_wave_instr_per_128_hypotheses": round(med["SQ_INSTS_LDS"] / (N / 128), 1),
            "valu_busy_quadcycles_per_simd": round(quad),
            "busy_cycles_per_cu": round(busy),
            "valu_busy_frac_if_4_cycles_per_wave64_instr": round(4 * quad / busy, 3),
            **({"waves_per_simd": round(4 * med["SQ_WAVE_CYCLES"] / (CUS * 4) / busy, 2)}
               if "SQ_WAVE_CYCLES" in med else {})}}
    print(json.dumps({k[:80]: v["derived"] for k, v in out.items()}, indent=1))
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--reduce":
        res = reduce(sys.argv[2])
        if len(sys.argv) > 3:
            json.dump(res, open(sys.argv[3], "w"), indent=1)
    else:
        run()
