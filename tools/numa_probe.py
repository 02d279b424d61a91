"""Host-resident zero-copy vs NUMA placement (tools/gpu_round.sh numa_probe): for each NUMA
node, pin this process to the node's CPUs, allocate + first-touch a 10 M-problem host batch
(pageable and pinned), and time hg_solve_host_f32 on it.  Also reports the GPU's own NUMA
node (sysfs, via hipDeviceGetPCIBusId), so the two placements can be compared."""
import ctypes
import glob
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def parse_cpulist(text):
    cpus = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.extend(range(int(a), int(b or a) + 1))
    return cpus


def gpu_numa_node(dev_index=0):
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, dev_index) != 0:
        return None, None
    bdf = buf.value.decode().lower()
    for cand in (bdf, bdf[:-1] + "0"):
        p = f"/sys/bus/pci/devices/{cand}/numa_node"
        if os.path.exists(p):
            return bdf, int(open(p).read().strip())
    return bdf, None


def main():
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    n = 10_000_000
    ds = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(n, 8)
    dt = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(n, 8)
    want = pkg.solve("aca", ds, dt).cpu()
    bdf, gnode = gpu_numa_node(0)
    allowed = set(os.sched_getaffinity(0))
    nodes = {}
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        cpus = [c for c in parse_cpulist(open(os.path.join(d, "cpulist")).read()) if c in allowed]
        if cpus:
            nodes[int(d.rsplit("node", 1)[1])] = cpus
    res = {"gpu_pci": bdf, "gpu_numa_node": gnode, "nodes": {k: len(v) for k, v in nodes.items()}}
    for node, cpus in nodes.items():
        os.sched_setaffinity(0, cpus[:16])
        hs = torch.empty((n, 8)).copy_(ds.cpu())   # first touch on this node
        ht = torch.empty((n, 8)).copy_(dt.cpu())
        hH = torch.empty((n, 9)).fill_(0.0)
        rec = {}
        for name, (s, t, h) in (("pageable", (hs, ht, hH)),
                                ("pinned", (hs.pin_memory(), ht.pin_memory(), hH.pin_memory()))):
            pkg.solve_host("aca", s, t, out=h)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                pkg.solve_host("aca", s, t, out=h)
                ts.append(time.perf_counter() - t0)
            ok = torch.equal(h.view(torch.int32), want.view(torch.int32))
            rec[name] = {"ms": round(sorted(ts)[2] * 1e3, 3), "bit_exact": bool(ok)}
        res[f"node{node}"] = rec
        print(node, rec, flush=True)
    os.sched_setaffinity(0, allowed)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/numa_probe.json", "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
