"""The reference's Table-8 draw step and the pipeline around it (GPU_Runtime Test.cu:1443-1451),
timed on the MI355X (round 3):

  * draws: rocrand_generate (a fresh generator per call, as the harness makes one) against the
    hand-written generator (hg_rand_mrg32k3a_u32, and its split threshold through
    hg_tune_mrg_words), 4 M words (the 1 M-hypothesis call) and 40 M words (10 M);
  * pipeline: draws + fused gather + solve (two launches, the words through HBM) against the
    one-launch draws + gather + solve (hg_rand_gather_solve_f64, and its global-pool form),
    ACA and SKS on the reference's wall file, 1 M and 10 M hypotheses;
  * the write-only stream of the same bytes (hg_tune_policy variant 0: 16-B default stores)
    as the ceiling of a launch that only writes.

Device time per launch from event-bracketed back-to-back launches, interleaved rounds,
median.  Every variant is compared bit for bit with the shipped one.
    python tools/kbench_mrg.py   -> gpurun_out/kbench_mrg.json
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


def timeit(fns, loops):
    """fns: name -> callable; interleaved rounds; median us per call"""
    for f in fns.values():
        for _ in range(3):
            f()
    times = {k: [] for k in fns}
    for _ in range(ROUNDS):
        for k, f in fns.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(loops):
                f()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / loops)
    return {k: round(statistics.median(v), 2) for k, v in times.items()}


def main():
    pkg = ge.load_package()
    lib = pkg.lib()
    t = pkg._lib.tune()
    vp, i64, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64
    t.hg_tune_rocrand_mrg32k3a_u32.argtypes = [vp, i64, u64, vp]
    t.hg_tune_mrg_words.argtypes = [vp, i64, u64, i64, vp]
    t.hg_tune_rand_gather_solve_f64.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp,
                                                ctypes.c_uint32, u64, vp, i64, vp]
    t.hg_tune_policy.argtypes = [ctypes.c_int, vp, vp, i64, vp]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev).cuda_stream
    out = {}

    # ---- the draws alone ----
    for count in (4_000_000, 40_000_000):
        bufs = {k: torch.empty(count, dtype=torch.int32, device=dev)
                for k in ("rocrand", "shipped", "chunk4", "chunk8", "chunk32", "chunk64")}
        fns = {
            "rocrand": lambda: t.hg_tune_rocrand_mrg32k3a_u32(bufs["rocrand"].data_ptr(), count, 11, st),
            "shipped": lambda: lib.hg_rand_mrg32k3a_u32(bufs["shipped"].data_ptr(), count, 11, st),
        }
        for c in (4, 8, 32, 64):
            fns[f"chunk{c}"] = (lambda c=c: t.hg_tune_mrg_words(bufs[f"chunk{c}"].data_ptr(), count,
                                                                 11, c, st))
        r = timeit(fns, 5 if count > 10_000_000 else 20)
        for k in bufs:
            out[f"draws {count} {k}"] = {
                "us": r[k], "gbps_written": round(count * 4 / (r[k] * 1e-6) / 1e9, 1),
                "bit_exact_vs_rocrand": bool(torch.equal(bufs[k], bufs["rocrand"]))}
            print(f"draws {count} {k}", out[f"draws {count} {k}"], flush=True)
        del bufs

    # ---- the pipeline ----
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(dev)
    for algo, aid in (("aca", 0), ("sks", 1)):
        for n in (1_000_000, 10_000_000):
            rl = torch.empty((4, n), dtype=torch.int32, device=dev)
            H = {k: torch.empty((9, n), dtype=torch.float64, device=dev)
                 for k in ("two_launch", "fused", "fused_global", "gather_only")}
            wsrc = torch.empty(n * 72 // 4, dtype=torch.float32, device=dev)
            wdst = torch.empty_like(wsrc)
            lib.hg_rand_mrg32k3a_u32(rl.data_ptr(), 4 * n, 11, st)

            def two():
                lib.hg_rand_mrg32k3a_u32(rl.data_ptr(), 4 * n, 11, st)
                lib.hg_gather_solve_f64(aid, ps.data_ptr(), pt.data_ptr(), ps.shape[0], rl.data_ptr(),
                                        H["two_launch"].data_ptr(), n, 0, st)

            fns = {
                "two_launch": two,
                "gather_only": lambda: lib.hg_gather_solve_f64(aid, ps.data_ptr(), pt.data_ptr(),
                                                               ps.shape[0], rl.data_ptr(),
                                                               H["gather_only"].data_ptr(), n, 0, st),
                "fused": lambda: lib.hg_rand_gather_solve_f64(aid, ps.data_ptr(), pt.data_ptr(),
                                                              ps.shape[0], 11, H["fused"].data_ptr(),
                                                              n, 0, st),
                "fused_global": lambda: t.hg_tune_rand_gather_solve_f64(0, aid, ps.data_ptr(),
                                                                        pt.data_ptr(), ps.shape[0], 11,
                                                                        H["fused_global"].data_ptr(),
                                                                        n, st),
                # 72 B of H per hypothesis as a write-only stream (hg_tune_policy variant 0:
                # 16-B stores, default cache policy)
                "write_only_72B": lambda: t.hg_tune_policy(0, wsrc.data_ptr(), wdst.data_ptr(),
                                                           n * 72, st),
            }
            r = timeit(fns, 20 if n == 1_000_000 else 5)
            ref = H["two_launch"].view(torch.int64)
            for k, us in r.items():
                rec = {"us": us, "ghyp_s": round(n / (us * 1e-6) / 1e9, 2),
                       "gbps_H": round(n * 72 / (us * 1e-6) / 1e9, 1)}
                if k in H:
                    rec["bit_exact_vs_two_launch"] = bool(torch.equal(H[k].view(torch.int64), ref))
                out[f"{algo} n={n} {k}"] = rec
                print(f"{algo} n={n} {k}", rec, flush=True)
            del rl, H, wsrc, wdst
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench_mrg.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
