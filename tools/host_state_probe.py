"""What is the host doing while a short host-bound step runs slowly?  (bench's eager rounds)

After the device-bound sections, and at a process's start, autograd's one-element floor
(a mul and its .backward(), which hands the graph to autograd's device thread and back)
runs ~1.7x slower for 0.5-3 s, then drops (profiles/r04/bench_r04t.log, bench_r04zb.log,
handoff_mimic_r04r.json).  This times the floor in passes of 1000 calls for `seconds` right
after a device-bound phase (10 M-problem solves for 2 s), and for every pass records which
CPU the main thread and each other thread of the process last ran on, those CPUs'
scaling_cur_freq, and the process's voluntary / involuntary context switches.
Run on the GPU box: python tools/host_state_probe.py [seconds]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def threads():
    """{tid: (comm, last cpu, voluntary, involuntary switches)} of this process."""
    out = {}
    for tid in os.listdir("/proc/self/task"):
        stat = _read(f"/proc/self/task/{tid}/stat")
        status = _read(f"/proc/self/task/{tid}/status") or ""
        if not stat:
            continue
        comm = stat[stat.index("(") + 1:stat.rindex(")")]
        fields = stat[stat.rindex(")") + 2:].split()
        cpu = int(fields[36])  # field 39 of stat
        vol = inv = 0
        for ln in status.splitlines():
            if ln.startswith("voluntary_ctxt_switches"):
                vol = int(ln.split()[1])
            elif ln.startswith("nonvoluntary_ctxt_switches"):
                inv = int(ln.split()[1])
        out[int(tid)] = (comm, cpu, vol, inv)
    return out


def freq(cpu):
    v = _read(f"/sys/devices/system/cpu/cpu{cpu}/cpufreq/scaling_cur_freq")
    return int(v) // 1000 if v else None


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    x1 = torch.ones(1, device=dev, requires_grad=True)
    g1 = torch.ones(1, device=dev)

    def floor():
        x1.grad = None
        (x1 * 2.0).backward(g1)

    for _ in range(50):
        floor()
    n = 10_000_000
    src = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(n, 8)
    tar = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(n, 8)
    H = torch.empty((n, 9), device=dev)
    info = {"governor": (_read("/sys/devices/system/cpu/cpu0/cpufreq/scaling_governor") or "").strip(),
            "idle_governor": (_read("/sys/devices/system/cpu/cpuidle/current_governor_ro") or
                              _read("/sys/devices/system/cpu/cpuidle/current_governor") or "").strip(),
            "cpus": len(os.sched_getaffinity(0))}
    for phase in ("fresh", "after_device_bound", "pinned_l3"):
        if phase == "pinned_l3":  # the main thread and autograd's device threads on one L3
            cur = int(_read("/proc/self/stat").rsplit(")", 1)[1].split()[36])
            l3 = _read(f"/sys/devices/system/cpu/cpu{cur}/cache/index3/shared_cpu_list")
            cpus = set()
            for part in (l3 or str(cur)).strip().split(","):
                a, _, b = part.partition("-")
                cpus |= set(range(int(a), int(b or a) + 1))
            cpus &= os.sched_getaffinity(0)
            os.sched_setaffinity(0, cpus)
            for tid, (comm, *_r) in threads().items():
                if comm.startswith("pt_autograd"):
                    os.sched_setaffinity(tid, cpus)
            info["pinned_cpus"] = sorted(cpus)
        if phase != "fresh":  # 2 s of back-to-back 10 M solves, host waiting
            t_end = time.perf_counter() + 2.0
            while time.perf_counter() < t_end:
                for _ in range(20):
                    pkg.solve("aca", src, tar, normalize=True, out=H)
                torch.cuda.synchronize()
        rows = []
        t0 = time.perf_counter()
        before = threads()
        while time.perf_counter() - t0 < seconds:
            ta = time.perf_counter()
            for _ in range(1000):
                floor()
            dt = (time.perf_counter() - ta) / 1000 * 1e6
            now = threads()
            busy = []
            for tid, (comm, cpu, vol, inv) in now.items():
                b = before.get(tid)
                if b and (vol - b[2] or inv - b[3]):
                    busy.append([comm, cpu, freq(cpu), vol - b[2], inv - b[3]])
            rows.append({"t_s": round(ta - t0, 3), "us": round(dt, 1), "active_threads": busy})
            before = now
        info[phase] = rows
    print(json.dumps(info), flush=True)


if __name__ == "__main__":
    main()
