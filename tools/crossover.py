"""Where the GPU-backed sks:: interface beats the reference's CPU code.

For batch sizes n = 1 ... 10 M of host-resident AoS f32 problems (the reference's own data
placement: std::vector / numpy, pageable), times
  * gpu_batch_pageable -- sks::runKernel_ACA_batch on the host arrays (hg_solve_host_f32:
    since 0.3 copied through the library's pinned stages; up to 0.2 registered for the call),
  * gpu_batch_pinned   -- the same on pinned arrays (no registration),
  * gpu_single_loop    -- n calls of the single-problem sks::runKernel_ACA (n <= 10 K),
  * cpu_1core / cpu_cores -- the reference's own ACA_SKS.cpp (oracle/_ref) over the same
    batch on one core and on `cores` pinned cores (the box's CPU quota),
each the median of several runs, and reports the crossover sizes.  Output:
gpurun_out/crossover.json (copied to profiles/r02/).
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import __graft_entry__ as ge  # noqa: E402


def med(f, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    pkg = ge.load_package()
    orc = ge.load_oracle()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lib = pkg.lib()
    batch = lib._ZN3sks19runKernel_ACA_batchEPKfS1_PflPv
    batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                      ctypes.c_void_p]
    batch.restype = ctypes.c_int
    one = lib._ZN3sks13runKernel_ACAEPfS0_S0_
    one.argtypes = [ctypes.c_void_p] * 3
    one.restype = ctypes.c_int
    ref = orc.RefOracle()
    gen = orc.Oracle()
    topo = bench.cpu_topology()
    quota = bench.cgroup_cpu_quota()
    cores = topo["cores"][:min(len(topo["cores"]), quota or len(topo["cores"]))]
    rows = []
    for n in (1, 10, 100, 1000, 10_000, 100_000, 1_000_000, 10_000_000):
        src = gen.fill_uniform(n * 8, 11, 0).reshape(n, 8)
        tar = gen.fill_uniform(n * 8, 11, n * 8).reshape(n, 8)
        H = np.empty((n, 9), np.float32)
        ps = torch.from_numpy(src).pin_memory()
        pt = torch.from_numpy(tar).pin_memory()
        pH = torch.empty((n, 9)).pin_memory()
        reps = 50 if n <= 100_000 else 7

        def gpu_pageable():
            assert batch(src.ctypes.data, tar.ctypes.data, H.ctypes.data, n, None) == 0

        def gpu_pinned():
            assert batch(ps.data_ptr(), pt.data_ptr(), pH.data_ptr(), n, None) == 0
            torch.cuda.synchronize(dev)  # pinned buffers are device-visible: the call is async

        for f in (gpu_pageable, gpu_pinned):
            f()
        rec = {"n": n,
               "gpu_batch_pageable_us": med(gpu_pageable, reps) * 1e6,
               "gpu_batch_pinned_us": med(gpu_pinned, reps) * 1e6}
        want = ref.solve("aca", src, tar)
        rec["gpu_bit_exact"] = bool(np.array_equal(H.view(np.uint32), want.view(np.uint32)) and
                                    np.array_equal(pH.numpy().view(np.uint32), want.view(np.uint32)))
        if n <= 10_000:
            h9 = np.empty(9, np.float32)

            def loop():
                for i in range(n):
                    one(src[i].ctypes.data, tar[i].ctypes.data, h9.ctypes.data)
            rec["gpu_single_loop_us"] = med(loop, 3 if n > 100 else 10) * 1e6
        r1 = max(1, int(2e5 / n))  # ~0.2 M problems per timing on CPU
        rec["cpu_1core_us"] = ref.time_pinned("aca", src, tar, cores[:1], r1) / r1 * 1e6
        rec["cpu_cores_us"] = min(ref.time_pinned("aca", src, tar, cores, r1) / r1 * 1e6
                                  for _ in range(3))
        rows.append({k: (round(v, 3) if isinstance(v, float) else v) for k, v in rec.items()})
        print(json.dumps(rows[-1]), flush=True)

    def first(key, cpu):
        for r in rows:
            if r[key] < r[cpu]:
                return r["n"]
        return None

    out = {"cores": len(cores), "cgroup_cpu_quota": quota, "rows": rows,
           "crossover_pageable_vs_1core": first("gpu_batch_pageable_us", "cpu_1core_us"),
           "crossover_pageable_vs_cores": first("gpu_batch_pageable_us", "cpu_cores_us"),
           "crossover_pinned_vs_cores": first("gpu_batch_pinned_us", "cpu_cores_us")}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "crossover.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "rows"}))


if __name__ == "__main__":
    main()
