"""The pageable host path's staged ring (hg_host.cpp solve_staged) against its settings:
stage bytes x depth x copy threads, at 10 M f32 AoS ACA (BASELINE configs[1]'s batch in host
memory), beside the pinned zero-copy call, the HG_FLAG_HOST_REGISTER call and the H2D copy
alone.  Every staged result is checked bit for bit against the device solve.

    python tools/ring_probe.py [--n 10000000] [--out gpurun_out/ring_probe.json]
"""
import argparse
import ctypes
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_PINNED_MIN_XFER_SIZE", "65536")  # this process's own copies staged

import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402


def best_ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--out", default="gpurun_out/ring_probe.json")
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--no-numa", action="store_true")
    ap.add_argument("--stages", default="", help="MiB list, e.g. 16,32,64")
    ap.add_argument("--depths", default="")
    ap.add_argument("--threads", default="")
    ap.add_argument("--dma", type=int, default=-1,
                    help="1 device buffers by copy engines, 2 in by copy engines / H by the kernel, 0 kernel reads the stage")
    a = ap.parse_args()
    import bench  # the bench's own NUMA binding, before anything touches the GPU
    numa = bench.bind_numa(0) if not a.no_numa else None
    pkg = ge.load_package()
    lib = pkg.lib()
    p64 = ctypes.POINTER(ctypes.c_int64)
    lib.hg_internal_host_stage_stats.argtypes = [p64]

    def stats():
        st = (ctypes.c_int64 * 8)()
        lib.hg_internal_host_stage_stats(st)
        return list(st)
    lib.hg_internal_host_stage_config.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, p64]
    if a.dma in (0, 1, 2):
        lib.hg_internal_host_stage_dma(a.dma)
    dev = torch.device("cuda:0")
    n = a.n
    ds = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(n, 8)
    dt = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(n, 8)
    want = pkg.solve("aca", ds, dt).cpu()
    qs, qt = ds.cpu(), dt.cpu()
    qH = torch.empty((n, 9))
    ps, pt, pH = qs.pin_memory(), qt.pin_memory(), torch.empty((n, 9)).pin_memory()
    h2d_s, h2d_t = torch.empty_like(ds), torch.empty_like(dt)
    prev = (ctypes.c_int64 * 3)()
    lib.hg_internal_host_stage_config(0, 0, 0, prev)
    out = {"n": n, "default": list(prev), "cpus": len(os.sched_getaffinity(0)), "numa": numa,
           "dma": lib.hg_internal_host_stage_dma(-1)}

    def h2d():
        h2d_s.copy_(ps, non_blocking=True)
        h2d_t.copy_(pt, non_blocking=True)

    out["h2d_bound_ms"] = round(best_ms(h2d), 3)
    out["pinned_zero_copy_ms"] = round(best_ms(lambda: pkg.solve_host("aca", ps, pt, out=pH)), 3)
    out["registered_ms"] = round(best_ms(lambda: pkg.solve_host("aca", qs, qt, out=qH, register=True)), 3)
    sweep = []
    stages = [4 << 20, 8 << 20, 16 << 20] if a.quick else [2 << 20, 4 << 20, 8 << 20, 16 << 20, 32 << 20]
    depths = [3, 4] if a.quick else [2, 3, 4, 6]
    threads = [4, 8, 12] if a.quick else [1, 2, 4, 8, 12, 16]
    if a.stages:
        stages = [int(x) << 20 for x in a.stages.split(",")]
    if a.depths:
        depths = [int(x) for x in a.depths.split(",")]
    if a.threads:
        threads = [int(x) for x in a.threads.split(",")]
    for sb, dp, th in itertools.product(stages, depths, threads):
        assert lib.hg_internal_host_stage_config(sb, dp, th, None) == 0
        qH.fill_(float("nan"))
        s0 = stats()
        ms = best_ms(lambda: pkg.solve_host("aca", qs, qt, out=qH), reps=3)
        s1 = stats()
        calls = max(1, s1[1] - s0[1])
        ok = bool(torch.equal(qH.view(torch.int32), want.view(torch.int32)))
        sweep.append({"stage_MiB": sb >> 20, "depth": dp, "threads": th, "ms": round(ms, 3), "bit_exact": ok,
                      "copy_ms_per_call": round((s1[5] - s0[5]) / calls / 1e6, 3),
                      "wait_ms_per_call": round((s1[6] - s0[6]) / calls / 1e6, 3),
                      "copy_GBps": round((s1[7] - s0[7]) / max(1, s1[5] - s0[5]), 1)})
        print(json.dumps(sweep[-1]), flush=True)
    # the ring's two halves apart (timing only, wrong results): kernels without the host copies,
    # host copies without the kernels, at each stage size of the sweep with 8 threads
    parts = []
    for sb in stages:
        for dp in depths:
            assert lib.hg_internal_host_stage_config(sb, dp, 8, None) == 0
            rec = {"stage_MiB": sb >> 20, "depth": dp}
            for probe, name in ((1, "kernels_only_ms"), (2, "copies_only_ms")):
                lib.hg_internal_host_stage_probe(probe)
                rec[name] = round(best_ms(lambda: pkg.solve_host("aca", qs, qt, out=qH), reps=3), 3)
                lib.hg_internal_host_stage_probe(0)
            parts.append(rec)
            print(json.dumps(rec), flush=True)
    out["parts"] = parts
    lib.hg_internal_host_stage_config(prev[0], prev[1], prev[2], None)
    qH.fill_(float("nan"))
    out["default_staged_ms"] = round(best_ms(lambda: pkg.solve_host("aca", qs, qt, out=qH)), 3)
    # every call of a 12-call run apart (bench.py reports the mean of 5, this file the best)
    calls = []
    s0 = stats()
    for _ in range(12):
        t0 = time.perf_counter()
        pkg.solve_host("aca", qs, qt, out=qH)
        calls.append(round((time.perf_counter() - t0) * 1e3, 3))
    s1 = stats()
    out["default_staged_calls_ms"] = calls
    out["default_staged_copy_ms_per_call"] = round((s1[5] - s0[5]) / 12 / 1e6, 3)
    out["default_staged_wait_ms_per_call"] = round((s1[6] - s0[6]) / 12 / 1e6, 3)
    out["default_bit_exact"] = bool(torch.equal(qH.view(torch.int32), want.view(torch.int32)))
    out["sweep"] = sweep
    out["best"] = min(sweep, key=lambda r: r["ms"])
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "sweep"}))


if __name__ == "__main__":
    main()
