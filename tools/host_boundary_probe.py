"""bench.py's host_boundary section alone (one rank, the bench's NUMA binding), with the
library's ring counters around it: where the pageable path's time goes in the bench's own
process shape.  Output: one JSON line (gpurun_out/host_boundary_probe.json)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    numa = bench.bind_numa(0)  # before anything touches the GPU, as bench.py does
    import __graft_entry__ as ge
    pkg = ge.load_package()
    d = bench.Dist("nccl")
    lib = pkg.lib()
    p64 = ctypes.POINTER(ctypes.c_int64)
    lib.hg_internal_host_stage_stats.argtypes = [p64]
    pre = {}
    if os.environ.get("HBP_PREWARM"):  # one ring call (its helper threads made) well before
        import time
        import torch
        m = 2_000_000
        ws = pkg.fill_uniform(m * 8, 5, 0, device=d.dev).view(m, 8).cpu()
        wt = pkg.fill_uniform(m * 8, 5, m * 8, device=d.dev).view(m, 8).cpu()
        wH = torch.empty((m, 9))
        t0 = time.perf_counter()
        pkg.solve_host("aca", ws, wt, out=wH)
        pre["prewarm_call_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
        time.sleep(float(os.environ["HBP_PREWARM"]))
    st0 = (ctypes.c_int64 * 8)()
    lib.hg_internal_host_stage_stats(st0)
    out = bench.host_boundary_section(d, pkg, 10_000_000)
    out.update(pre)
    st1 = (ctypes.c_int64 * 8)()
    lib.hg_internal_host_stage_stats(st1)
    ring_calls = max(1, st1[4] - st0[4])
    out["ring_stats"] = {"ring_calls": st1[4] - st0[4],
                         "copy_ms_per_ring_call": round((st1[5] - st0[5]) / ring_calls / 1e6, 3),
                         "wait_ms_per_ring_call": round((st1[6] - st0[6]) / ring_calls / 1e6, 3)}
    # a fresh batch in this process, each call apart: wall, host-copy and event-wait times
    import time
    import torch
    n = 10_000_000
    ds = pkg.fill_uniform(n * 8, 11, 0, device=d.dev).view(n, 8)
    dt = pkg.fill_uniform(n * 8, 11, n * 8, device=d.dev).view(n, 8)
    qs, qt = ds.cpu(), dt.cpu()
    qH = torch.empty((n, 9))
    per_call = []
    for _ in range(10):
        a = (ctypes.c_int64 * 8)()
        lib.hg_internal_host_stage_stats(a)
        t0 = time.perf_counter()
        pkg.solve_host("aca", qs, qt, out=qH)
        wall = (time.perf_counter() - t0) * 1e3
        b = (ctypes.c_int64 * 8)()
        lib.hg_internal_host_stage_stats(b)
        per_call.append({"ms": round(wall, 2), "copy_ms": round((b[5] - a[5]) / 1e6, 2),
                         "wait_ms": round((b[6] - a[6]) / 1e6, 2), "stages_made": b[0] - a[0]})
    out["fresh_batch_calls"] = per_call
    out["numa"] = numa
    out["cpus"] = len(os.sched_getaffinity(0))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "host_boundary_probe.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
