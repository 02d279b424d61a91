"""Does the CPU binding set the eager autograd step's cost?  (bench `aca_vanilla_autograd`)

The eager step is host-bound: `.backward()` hands the graph to autograd's device thread and
waits for it, and the one-element floor (a mul and its backward) read 24-67 us a step in the
bench's NUMA-bound process against 26 us in `tools/autograd_cost.py` (unbound).  This runs the
floor and the full ACA_vanilla step (B = 64 K) in a fresh child process per CPU binding, the
binding applied before torch starts any thread (so autograd's device thread and HIP's threads
inherit it):
  all    the affinity the job was given
  node   the GPU's NUMA node (what bench.bind_numa does)
  node8  8 CPUs of that node          node2  2 CPUs          node1  1 CPU
Each child prints the best of 5 interleaved rounds of 2000 calls per variant.  The parent
makes no GPU call.  Run on the GPU box: python tools/handoff_probe.py
`--mimic` instead times the two steps in one process as bench's interleaved_ms does (rounds
of 40 or 400 calls inside bench.timed_region), then runs bench's section itself.
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(cpus):
    if cpus:
        os.sched_setaffinity(0, cpus)
    import torch
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    B = 65536
    torch.manual_seed(0)
    src, tar, *_ = pkg.adjust(dev, B)
    tar = (tar + torch.rand_like(tar)).contiguous()
    gH = torch.randn(B, 3, 3, device=dev)
    S, T = src.clone().requires_grad_(), tar.clone().requires_grad_()
    x1 = torch.ones(1, device=dev, requires_grad=True)
    g1 = torch.ones(1, device=dev)

    def ours():
        S.grad = None
        T.grad = None
        pkg.ACA_vanilla(B, S, T).backward(gH)

    def floor():
        x1.grad = None
        (x1 * 2.0).backward(g1)

    def fwd_only():
        pkg.ACA_vanilla(B, S, T)

    def per_call_us(fn, n=2000):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e6

    variants = {"ours": ours, "floor": floor, "fwd_only": fwd_only}
    for fn in variants.values():
        for _ in range(200):
            fn()
    runs = {k: [] for k in variants}
    for _ in range(5):
        for k, fn in variants.items():
            runs[k].append(per_call_us(fn))
    out = {k: {"best": round(min(v), 2), "median": round(sorted(v)[len(v) // 2], 2)}
           for k, v in runs.items()}
    out["cpus"] = len(os.sched_getaffinity(0))
    print(json.dumps(out), flush=True)


def mimic():
    """In one process: the same two steps timed as bench's interleaved_ms does (rounds of
    `steps` calls inside bench.timed_region, interleaved, median and best), for steps 40 and
    400, with and without the torch-composed step interleaved, against a plain 2000-call loop."""
    sys.path.insert(0, ROOT)
    import bench
    import torch
    pkg = bench.ge.load_package()
    d = bench.Dist("nccl")
    B = 65536
    torch.manual_seed(0)
    src, tar, *_ = pkg.adjust(d.dev, B)
    tar = (tar + torch.rand_like(tar)).contiguous()
    gH = torch.randn(B, 3, 3, device=d.dev)
    S, T = src.clone().requires_grad_(), tar.clone().requires_grad_()
    x1 = torch.ones(1, device=d.dev, requires_grad=True)
    g1 = torch.ones(1, device=d.dev)

    def ours():
        S.grad = None
        T.grad = None
        pkg.ACA_vanilla(B, S, T).backward(gH)

    def torch_step():
        S.grad = None
        T.grad = None
        bench.torch_aca_vanilla(S, T).backward(gH)

    def floor():
        x1.grad = None
        (x1 * 2.0).backward(g1)

    for _ in range(50):
        ours(), torch_step(), floor()
    res = {}
    for steps in (40, 400):
        for with_torch in (False, True):
            fns = {"ours": ours, "floor": floor}
            if with_torch:
                fns["torch"] = torch_step
            per = {k: [] for k in fns}
            for _ in range(7):
                for k, f in fns.items():
                    per[k].append(bench.timed_region(d, f, steps)[1] * 1e3)
            res[f"steps{steps}_torch{int(with_torch)}"] = {
                k: {"median": round(sorted(v)[3], 2), "best": round(min(v), 2)}
                for k, v in per.items() if k != "torch"}
    for k, f in (("ours", ours), ("floor", floor)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2000):
            f()
        torch.cuda.synchronize()
        res.setdefault("plain2000", {})[k] = round((time.perf_counter() - t0) / 2000 * 1e6, 2)
    print(json.dumps(res), flush=True)
    # bench's own section, alone in a fresh process (no headline or other section before it)
    sec = bench.vanilla_autograd_section(d, pkg, B)
    print(json.dumps({k: v for k, v in sec.items() if "us_per_call" in k or "eager" in k}),
          flush=True)


def main():
    sys.path.insert(0, ROOT)
    import bench  # /sys helpers only: no GPU call in this process
    orig = sorted(os.sched_getaffinity(0))
    gpus = bench._visible(bench._kfd_gpu_bdfs(), ("ROCR_VISIBLE_DEVICES",)) or []
    gpus = bench._visible(gpus, ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")) or []
    node_cpus = orig
    node = None
    if gpus:
        try:
            node = int(bench._read(f"/sys/bus/pci/devices/{gpus[0]}/numa_node"))
        except (TypeError, ValueError):
            node = -1
        if node >= 0:
            node_cpus = sorted(set(bench._cpu_list(bench._read(
                f"/sys/devices/system/node/node{node}/cpulist"))) & set(orig)) or orig
    configs = {"all": orig, "node": node_cpus, "node8": node_cpus[:8], "node2": node_cpus[:2],
               "node1": node_cpus[:1]}
    res = {"gpu_numa_node": node, "job_cpus": len(orig)}
    for name in ("all", "node", "node8", "node2", "node1", "all"):
        key = name if name not in res else name + "_again"
        p = subprocess.run([sys.executable, __file__, "--child", ",".join(map(str, configs[name]))],
                           capture_output=True, text=True, timeout=240)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        res[key] = json.loads(lines[-1]) if p.returncode == 0 and lines else {
            "rc": p.returncode, "err": p.stderr[-400:]}
        print(key, json.dumps(res[key]), file=sys.stderr, flush=True)
        if p.returncode not in (0, 1):
            break  # a crash or signal: no further GPU step
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--mimic":
        mimic()
    elif len(sys.argv) > 2 and sys.argv[1] == "--child":
        child([int(c) for c in sys.argv[2].split(",") if c])
    else:
        main()
