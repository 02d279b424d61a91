"""Workload for a counter pass over the fused Table-8 pipeline (MRG32K3A draws + get_rand_list
gather + cal_Homo_*, binary64, hg_rand_gather_solve_f64; GPU_Runtime Test.cu:52-78, :81-240,
:1443-1451) at the bench size: 10 M hypotheses over the reference's wall pool, 3 ACA then 3
SKS launches (tools/gpu_round.sh pmc_table8); then 3 launches of the seeded f32 sampler
(hg_sample_solve_seeded_f32) at its bench size, 16 M.
`--reduce <counter_collection.csv> [out.json]` turns the pass into per-kernel figures: VALU
wave-instructions per hypothesis-wave (64 hypotheses), VALU busy against the CU's busy cycles
(a wave64 VALU instruction holds a SIMD 4 cycles at full rate), waves resident per SIMD
(wave-cycles / busy cycles), SALU and LDS instructions per hypothesis-wave, and the fraction
of wave-cycles spent waiting on anything (SQ_WAIT_INST_ANY)."""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
N = 10_000_000
SEEDED_N = 16 << 20
SEEDED = "sample_solve_lds_kernel<0, true, 2, 0, 4, 1"  # the seeded ACA instantiation
CUS = 256


def run():
    import numpy as np
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(dev)
    # T8_VARIANT >= 0: a tune-library variant instead (hg_tune_rand_gather_solve_f64: 2 no
    # solve, 4 no engine steps -- the VALU split of VERDICT r05 item 5; wrong bits, counts only)
    variant = int(os.environ.get("T8_VARIANT", "-1"))
    if variant >= 0:
        import ctypes
        t = pkg._lib.tune()
        vp = ctypes.c_void_p
        t.hg_tune_rand_gather_solve_f64.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_uint32,
                                                    ctypes.c_uint64, vp, ctypes.c_int64, vp]
        H = torch.empty((9, N), dtype=torch.float64, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
    for aid, algo in enumerate(("aca", "sks")):
        for _ in range(3):
            if variant < 0:
                pkg.rand_gather_solve(ps, pt, N, 11, algo, False)
            else:
                assert t.hg_tune_rand_gather_solve_f64(variant, aid, ps.data_ptr(), pt.data_ptr(),
                                                       ps.shape[0], 11, H.data_ptr(), N, st) == 0
        torch.cuda.synchronize()
    # the seeded f32 sampler at its bench size (16 M hypotheses, the draws made in the kernel,
    # hg_sample_solve_seeded_f32; VERDICT r04 item 3 asks for the same reading)
    ps32 = torch.from_numpy(g["pool_src"]).to(dev)
    pt32 = torch.from_numpy(g["pool_tar"]).to(dev)
    for _ in range(3):
        pkg.sample_solve_seeded(ps32, pt32, SEEDED_N, 7, 0)
    torch.cuda.synchronize()
    print("pmc_table8 done")


def reduce(path):
    per, meta = {}, {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "mrg_gather_solve" not in name and SEEDED not in name:
            continue
        per.setdefault(name, {}).setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
        meta[name] = {k: r.get(k) for k in ("Grid_Size", "Workgroup_Size", "VGPR_Count", "Accum_VGPR_Count",
                                            "SGPR_Count", "LDS_Block_Size", "Scratch_Size")}
    out = {}
    for name, disp in per.items():
        keys = sorted(set().union(*disp.values()))
        med = {k: statistics.median(d[k] for d in disp.values() if k in d) for k in keys}
        hw = (SEEDED_N if SEEDED in name else N) / 64  # hypothesis-waves
        busy = med.get("SQ_BUSY_CU_CYCLES", 0) / CUS
        derived = {"valu_wave_instr_per_hypothesis_wave": round(med["SQ_INSTS_VALU"] / hw, 1)}
        if "SQ_INSTS_SALU" in med:
            derived["salu_instr_per_hypothesis_wave"] = round(med["SQ_INSTS_SALU"] / hw, 1)
        if "SQ_INSTS_LDS" in med:
            derived["lds_instr_per_hypothesis_wave"] = round(med["SQ_INSTS_LDS"] / hw, 1)
        if busy and "SQ_ACTIVE_INST_VALU" in med:
            quad = med["SQ_ACTIVE_INST_VALU"] / (CUS * 4)  # quad-cycles per SIMD
            derived["valu_active_frac_of_busy"] = round(4 * quad / busy, 3)
            derived["valu_issue_floor_frac_of_busy"] = round(4 * med["SQ_INSTS_VALU"] / (CUS * 4) / busy, 3)
        if busy and "SQ_WAVE_CYCLES" in med:
            derived["waves_per_simd"] = round(4 * med["SQ_WAVE_CYCLES"] / (CUS * 4) / busy, 2)
        if "SQ_WAIT_INST_ANY" in med and "SQ_WAVE_CYCLES" in med:
            derived["wait_any_frac_of_wave_cycles"] = round(med["SQ_WAIT_INST_ANY"] / med["SQ_WAVE_CYCLES"], 3)
        if busy and "GRBM_GUI_ACTIVE" in med:
            derived["busy_frac_of_gui_active"] = round(busy / med["GRBM_GUI_ACTIVE"], 3)
        out[name] = {**meta[name], "dispatches": len(disp), "median_counters": med, "derived": derived}
    print(json.dumps({k[:80]: {**v["derived"], "vgpr": v["VGPR_Count"]} for k, v in out.items()}, indent=1))
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--reduce":
        res = reduce(sys.argv[2])
        if len(sys.argv) > 3:
            json.dump(res, open(sys.argv[3], "w"), indent=1)
    else:
        run()
