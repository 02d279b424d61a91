"""The fused Table-8 kernel (hg_rand_gather_solve_f64: MRG32K3A draws + get_rand_list gather +
cal_Homo_*, binary64; GPU_Runtime Test.cu:52-78, :81-240, :1443-1451) in its chunk shapes
(round 5): positions per chunk Q (a lane solves Q / 4 hypotheses per
chunk, one barrier per chunk) and lanes per block KB (the VGPR budget: 128 at 1024 lanes,
168 at 768, 256 at 512), ACA and SKS at 10 M on the reference's wall pool, against the write-
only stream of the same 720 MB.  Every variant's H is compared bit for bit with the shipped
launch.  Device time per launch from events around back-to-back launches, interleaved rounds,
median.
    python tools/kbench_t8q.py   -> gpurun_out/kbench_t8q.json
"""
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

ROUNDS = int(os.environ.get("KB_ROUNDS", "7"))
VARIANTS = {  # hg_tune_rand_gather_solve_f64 variant -> shape
    16: "Q4 KB1024 (r04 shape)", 21: "Q4 KB1024 buffer stores (r05 shipped)",
    23: "Q4 KB1024 buffer stores, next chunk's draws interleaved with the solves",
    22: "Q8 KB1024 buffer stores",
    25: "Q4 KB1024 buffer stores, engines write pool indices (binary64 remainder)",
    26: "23 with the engines writing pool indices",
    27: "Q8 KB1024 buffer stores, engines write pool indices",
}
if os.environ.get("KB_ALL"):
    VARIANTS.update({20: "Q4 KB768", 18: "Q8 KB768", 19: "Q8 KB512", 15: "Q8 KB1024 (6 VGPRs spilled)"})
if os.environ.get("KB_VARIANTS"):  # e.g. KB_VARIANTS=21,25: only these
    VARIANTS = {int(v): VARIANTS[int(v)] for v in os.environ["KB_VARIANTS"].split(",")}
NBUF = int(os.environ.get("KB_NBUF", "3"))  # output buffers per variant, used in turn: the
# 10 M figures move with where the 720 MB of H land (KERNEL_NOTES.md), so every variant is
# timed over the same number of distinct placements


def timeit(fns, loops):
    for f in fns.values():
        for _ in range(3):
            f()
    times = {k: [] for k in fns}
    keys = list(fns)
    for rnd in range(ROUNDS):
        # each round starts at another variant, so no variant always follows the same one
        for k in keys[rnd % len(keys):] + keys[:rnd % len(keys)]:
            f = fns[k]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(loops):
                f()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / loops)
    return {k: (round(statistics.median(v), 2), round(min(v), 2)) for k, v in times.items()}


def sustained(fns, keys, reps=3):
    """bench.py's launch_stats shape: per key 5 warm-up launches, then 10 groups of 10
    back-to-back launches (the clocks settle under this VALU-heavy load), median of the group
    means; keys in turn, `reps` times, median over the reps."""
    res = {k: [] for k in keys}
    for _ in range(reps):
        for k in keys:
            for _ in range(5):
                fns[k]()
            ts = []
            for _ in range(10):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fns[k]()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 10)
            res[k].append(statistics.median(ts))
    return {k: round(statistics.median(v), 2) for k, v in res.items()}


def main():
    pkg = ge.load_package()
    lib = pkg.lib()
    t = pkg._lib.tune()
    vp, i64, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64
    t.hg_tune_rand_gather_solve_f64.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp,
                                                ctypes.c_uint32, u64, vp, i64, vp]
    t.hg_tune_policy.argtypes = [ctypes.c_int, vp, vp, i64, vp]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev).cuda_stream
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(dev)
    out = {"pool": int(ps.shape[0]), "rounds": ROUNDS}
    n = int(os.environ.get("KB_N", "10000000"))
    for algo, aid in (("aca", 0), ("sks", 1)):
        keys = ["shipped", *VARIANTS]
        Hs = {k: [torch.empty((9, n), dtype=torch.float64, device=dev) for _ in range(NBUF)] for k in keys}
        H = {k: v[0] for k, v in Hs.items()}
        turn = {k: 0 for k in keys}

        def nxt(k):
            turn[k] = (turn[k] + 1) % NBUF
            return Hs[k][turn[k]].data_ptr()

        wsrc = torch.empty(n * 72 // 4, dtype=torch.float32, device=dev)
        wdst = torch.empty_like(wsrc)
        fns = {"shipped": lambda: lib.hg_rand_gather_solve_f64(aid, ps.data_ptr(), pt.data_ptr(),
                                                               ps.shape[0], 11, nxt("shipped"), n, 0, st),
               "write_only_72B": lambda: t.hg_tune_policy(0, wsrc.data_ptr(), wdst.data_ptr(), n * 72, st)}
        for v in VARIANTS:
            fns[v] = (lambda v=v: t.hg_tune_rand_gather_solve_f64(v, aid, ps.data_ptr(), pt.data_ptr(),
                                                                  ps.shape[0], 11, nxt(v), n, st))
        rc = {v: t.hg_tune_rand_gather_solve_f64(v, aid, ps.data_ptr(), pt.data_ptr(), ps.shape[0], 11,
                                                 H[v].data_ptr(), n, st) for v in VARIANTS}
        lib.hg_rand_gather_solve_f64(aid, ps.data_ptr(), pt.data_ptr(), ps.shape[0], 11,
                                     H["shipped"].data_ptr(), n, 0, st)
        torch.cuda.synchronize()
        same = {v: bool(torch.equal(H[v].view(torch.int64), H["shipped"].view(torch.int64)))
                for v in VARIANTS}
        r = timeit(fns, 6)
        if os.environ.get("KB_SUSTAINED"):
            sus = sustained(fns, ["shipped", *VARIANTS, "write_only_72B"])
            print(f"{algo} sustained (bench launch_stats shape)", sus, flush=True)
            out[f"{algo} sustained_us"] = sus
        w_us = r["write_only_72B"][0]
        for k, (us, best) in r.items():
            rec = {"us": us, "best_us": best, "ghyp_s": round(n / (us * 1e-6) / 1e9, 2),
                   "frac_of_write_only_stream": round(w_us / us, 4),
                   "frac_of_spec": round(n * 72 / (us * 1e-6) / 1e9 / 8000.0, 4)}
            if k in VARIANTS:
                rec["shape"] = VARIANTS[k]
                rec["rc"] = rc[k]
                rec["bit_exact_vs_shipped"] = same[k]
            out[f"{algo} {k}"] = rec
            print(f"{algo} {k}", rec, flush=True)
        del H, Hs, wsrc, wdst
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench_t8q.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
