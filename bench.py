"""bench.py -- headline benchmark: batched ACA (and SKS) homographies on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 it is
launched by torch.distributed.run, one process per GPU.  A *step* is one pass of
the hot path over one batch: one ACA launch over the rank's 10 M-problem block
(BASELINE.json configs[1]; configs[4] = 80 M over 8 GPUs = the same 10 M per GPU,
weak scaling).  Inputs are generated on each device before the timed region
(counter-based stream, seed 11), so they are resident in HBM when timing starts.
Rank 0 prints ONE JSON line.

Extra fields: SKS on the same inputs (configs[2]), TensorACA rect at B = 64 K
(configs[3]) against the torch-composed formulation on the same GPU, a streaming
copy yardstick, the roofline of the dominant kernel and the CPU baseline (the
reference's own C++ solver bodies, timed on this host's cores).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import threading
import time

# HIP maps pageable host buffers of >= 2 MB in place for its copies and KFD keeps those mappings;
# such a copy writing a reused heap page is the one GPU fault this project's runs ever had
# (DESIGN.md section 10).  This process's own .cpu() / .to() copies of pageable memory go through
# HIP's staging buffers instead (read when the runtime starts; no timed region copies pageable
# memory: the staged host-boundary baseline uses pinned buffers).
os.environ.setdefault("GPU_PINNED_MIN_XFER_SIZE", "65536")  # MiB

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
SEED = 11
# exit status of a run a watchdog ended (a stalled collective or extras section): the JSON
# line is printed first, but torchrun / CI can tell the stall from a clean finish
EXIT_STALLED = 3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--problems-per-gpu", "--n", dest="n", type=int, default=10_000_000,
                    help="problems per GPU (--n is ambiguous under torchrun: use the long name)")
    ap.add_argument("--algo", default="aca", choices=["aca", "sks", "ge", "gpt"],
                    help="the headline solver (aca: BASELINE configs[1]; sks: configs[2])")
    ap.add_argument("--layout", default="aos", choices=["aos", "soa"],
                    help="aos: (n,8) -> (n,9), normalised as sks::runKernel_*; soa: (8,n) -> "
                         "(9,n), unnormalised as cal_Homo_*")
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--seed", type=int, default=SEED, help="input stream seed")
    ap.add_argument("--rect-batch", type=int, default=65536)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--no-extras", action="store_true", help="ACA headline only")
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: skip the timed split (scatter) / gather through rank 0")
    ap.add_argument("--gather-deadline", type=float, default=180.0,
                    help="N>1: seconds the split / gather may take before the job ends without it")
    ap.add_argument("--extras-deadline", type=float, default=420.0,
                    help="seconds everything after the headline may take before the line is "
                         "printed without the rest")
    ap.add_argument("--inject-extras-failure", type=int, default=-1, metavar="RANK",
                    help="testing only: this rank raises as the extras start (the guard's rehearsal)")
    ap.add_argument("--no-host-shard", action="store_true",
                    help="skip the shared-memory host-resident batch (per-rank zero-copy)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo only to rehearse N>1 on a one-GPU box")
    return ap.parse_args()


def launch_plan(gpus: int, env) -> tuple[str, str]:
    """What ``--gpus N`` means for this process, decided before anything touches a GPU:
    ("self", "") -- run as this rank: N = 1 alone, or a torch.distributed.run rank whose
    WORLD_SIZE equals N; ("spawn", why) -- N > 1 and no WORLD_SIZE: start N ranks under
    torch.distributed.run as a child process; ("refuse", why) -- WORLD_SIZE is set and is not
    N, or N < 1 (a job that would report a GPU count it did not run on)."""
    if gpus < 1:
        return "refuse", f"--gpus {gpus}: at least one GPU"
    ws = env.get("WORLD_SIZE")
    if ws is None or ws == "":
        if gpus == 1:
            return "self", ""
        return "spawn", f"--gpus {gpus} without WORLD_SIZE: starting {gpus} ranks"
    try:
        world = int(ws)
    except ValueError:
        return "refuse", f"WORLD_SIZE={ws!r} is not an integer"
    if world != gpus:
        return "refuse", f"WORLD_SIZE={world} but --gpus {gpus}: the line would misreport n_gpus"
    return "self", ""


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def torchrun_cmd(gpus: int, argv, port: int) -> list:
    """The child command of launch_plan's "spawn": one process per GPU on this node, the
    rendezvous on the loopback address (the container's hostname may not resolve)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__), *argv]


def spawn_ranks(gpus: int, argv) -> int:
    """Runs torch.distributed.run as a CHILD (never exec: see the process rules in DESIGN
    §7) and passes its stdout through line by line -- rank 0's JSON line among it -- then
    returns its exit status.  No GPU call happens in this process."""
    import subprocess
    cmd = torchrun_cmd(gpus, argv, _free_port())
    print(f"bench.py: {' '.join(cmd[1:5])} ... (--gpus {gpus}, no WORLD_SIZE)", file=sys.stderr,
          flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    # a SIGTERM / SIGINT / SIGHUP meant for this process (a driver's time limit) goes on to the
    # child -- torch.distributed.run passes it to the ranks -- instead of leaving the ranks
    # running on the GPUs without a parent; the child's exit then ends this process too
    import signal
    forwarded = (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)
    previous = {sig: signal.signal(sig, lambda signum, _f: proc.send_signal(signum))
                for sig in forwarded}
    try:
        for text in proc.stdout:
            sys.stdout.write(text)
            sys.stdout.flush()
        rc = proc.wait()
    finally:
        for sig, handler in previous.items():
            signal.signal(sig, handler)
    return 128 - rc if rc < 0 else rc  # a child ended by signal N exits 128 + N, as a shell reports


def _kfd_gpu_bdfs(base: str = "/sys/class/kfd/kfd/topology/nodes"):
    """PCI addresses of the node's GPUs in KFD topology order (the order the HIP runtime
    numbers them), read from /sys without touching the GPU."""
    out = []
    try:
        nodes = sorted(int(x) for x in os.listdir(base) if x.isdigit())
    except OSError:
        return out
    for nd in nodes:
        props = {}
        for line in (_read(f"{base}/{nd}/properties") or "").splitlines():
            k, _, v = line.partition(" ")
            props[k] = v.strip()
        try:
            if int(props.get("simd_count", "0")) == 0:
                continue  # a CPU node
            loc, dom = int(props["location_id"]), int(props.get("domain", "0"))
        except (KeyError, ValueError):
            continue
        out.append(f"{dom:04x}:{loc >> 8 & 0xff:02x}:{loc >> 3 & 0x1f:02x}.{loc & 7}")
    return out


def _visible(items, env_names):
    for name in env_names:
        v = os.environ.get(name)
        if v is None or v == "":
            continue
        try:
            return [items[int(x)] for x in v.split(",")]
        except (ValueError, IndexError):
            return None  # UUIDs or out of range: mapping unknown
    return items


def bind_numa(local_index: int):
    """Binds this process to the CPUs of its GPU's NUMA node -- BEFORE any GPU call, so the
    threads the HIP runtime and torch create afterwards inherit the binding -- and returns
    what it did.  The GPU is found from /sys (KFD topology order, the visible-devices
    variables applied), its node from /sys/bus/pci/devices/<bdf>/numa_node.  A host batch's
    pages then first-touch on the GPU's node (SharedHostBatch), and the PCIe traffic of
    hg_solve_host_* crosses no socket link.  The pre-binding affinity is kept for the CPU
    baseline (_ORIGINAL_AFFINITY)."""
    global _ORIGINAL_AFFINITY
    _ORIGINAL_AFFINITY = sorted(os.sched_getaffinity(0))
    rec = {"gpu_index": local_index, "bdf": None, "node": None, "bound_cpus": None}
    gpus = _visible(_kfd_gpu_bdfs(), ("ROCR_VISIBLE_DEVICES",))
    gpus = _visible(gpus, ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")) if gpus else gpus
    if not gpus or local_index >= len(gpus):
        rec["note"] = "GPU not found in /sys/class/kfd: not bound"
        return rec
    bdf = gpus[local_index]
    rec["bdf"] = bdf
    try:
        node = int(_read(f"/sys/bus/pci/devices/{bdf}/numa_node"))
    except (TypeError, ValueError):
        node = -1
    rec["node"] = node
    if node < 0:
        rec["note"] = "no NUMA node for the GPU: not bound"
        return rec
    cpus = sorted(set(_cpu_list(_read(f"/sys/devices/system/node/node{node}/cpulist"))) &
                  set(_ORIGINAL_AFFINITY))
    if cpus:
        os.sched_setaffinity(0, cpus)
        rec["bound_cpus"] = len(cpus)
    return rec


_ORIGINAL_AFFINITY = None


class Dist:
    """One process per GPU (torch.distributed.run sets RANK/LOCAL_RANK/WORLD_SIZE).
    Backend "nccl" (= RCCL over xGMI) by default.  --dist-backend gloo exists only to
    rehearse the N > 1 control path on a one-GPU box (RCCL refuses two ranks on one
    device): ranks then share cuda:(LOCAL_RANK % device_count) and reduce on the host."""

    def __init__(self, backend: str = "nccl"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.backend = backend
        ndev = torch.cuda.device_count()
        idx = self.local if backend == "nccl" else self.local % max(ndev, 1)
        self.dev = torch.device("cuda", idx)
        torch.cuda.set_device(self.dev)
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            # a process-group timeout past bench.py's own deadlines, so a stalled collective
            # ends through bench's watchdogs (which print the line) and not an abort
            timeout = datetime.timedelta(minutes=20)
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev, timeout=timeout)
            else:
                dist.init_process_group(backend, timeout=timeout)
            self.pg = dist

    def barrier(self):
        if self.pg:
            if self.backend == "nccl":
                self.pg.barrier(device_ids=[self.dev.index])
            else:
                self.pg.barrier()

    def max(self, x: float) -> float:
        if not self.pg:
            return x
        dev = self.dev if self.backend == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def gather_rows(self, row):
        """Every rank's equal-length list of numbers, on every rank (a SUM all-reduce of a
        zero matrix holding each rank's row: small, control path only)."""
        if not self.pg:
            return [list(row)]
        dev = self.dev if self.backend == "nccl" else "cpu"
        t = torch.zeros((self.world, len(row)), dtype=torch.float64, device=dev)
        t[self.rank] = torch.tensor(row, dtype=torch.float64, device=dev)
        self.pg.all_reduce(t)
        return t.cpu().tolist()

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


START_MARGIN_S = 0.003


def timed_region(d: Dist, fn, steps: int):
    """barrier + sync, K steps, sync + barrier; returns (the job's wall seconds, mean
    per-launch device time in ms from HIP events on the launch stream).  After the opening
    barrier the ranks agree on a start instant a few ms ahead on CLOCK_MONOTONIC
    (time.perf_counter on Linux: one clock for every process of the node) and each waits
    for it, so the barrier's release skew between processes is not charged to the job; each
    rank stamps its start when it begins and its end after its final synchronize, and the
    job's time is the latest end minus the earliest start over ranks (a rank that missed
    the common start is counted late; the closing barrier's own latency is not work; at
    N = 1 it is the rank's own span)."""
    stream = torch.cuda.current_stream(d.dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    d.barrier()
    torch.cuda.synchronize(d.dev)
    t_start = d.max(time.perf_counter()) + START_MARGIN_S
    while time.perf_counter() < t_start:
        pass
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize(d.dev)
    t1 = time.perf_counter()
    d.barrier()
    return d.max(t1) + d.max(-t0), e0.elapsed_time(e1) / steps


def interleaved_ms(d: Dist, fns: dict, rounds: int = 7, steps=40) -> dict:
    """Host-bound per-call figures (eager autograd steps): `rounds` rounds, each timing
    `steps` calls of every function in turn (timed_region), and per function the median of
    its rounds' ms per call, and under "best" the fastest round's.  One mean over a single
    long run took every host stall of the box (its CPU quota's throttling, another process)
    at full weight: the same build's eager autograd step read 30-140 us from run to run that
    way, its device work 5 us.  The fastest round is the cost with the fewest such stalls.
    `steps` may be a dict (calls per round for each function): a round of a short step
    must be long -- 40 calls of a 33 us step read 60 us a call in a fresh process (about
    1 ms per round that 400 calls do not show: tools/handoff_probe.py --mimic,
    profiles/r04/handoff_mimic_r04r.json)."""
    per = {k: [] for k in fns}
    thr0 = cgroup_throttle()
    for _ in range(rounds):
        for k, f in fns.items():
            n = steps[k] if isinstance(steps, dict) else steps
            per[k].append(timed_region(d, f, n)[1])
    thr1 = cgroup_throttle()
    out = {k: float(np.median(v)) for k, v in per.items()}
    out["best"] = {k: float(np.min(v)) for k, v in per.items()}
    out["rounds"] = per
    # the job's CPU quota stopping its threads meanwhile (cgroup v2 cpu.stat), if readable
    out["throttled"] = ({k: thr1[k] - thr0[k] for k in thr0} if thr0 and thr1 else None)
    return out


def card_vram_used(dev):
    """Card-wide device memory in use (the amdgpu driver's mem_info_vram_used, what rocm-smi
    shows) for `dev`, or None when /sys does not say."""
    import glob
    try:
        pr = torch.cuda.get_device_properties(dev)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
    except (AttributeError, RuntimeError):
        return None
    for card in glob.glob("/sys/class/drm/card*/device"):
        try:
            if os.path.basename(os.path.realpath(card)).startswith(bdf):
                return int(_read(os.path.join(card, "mem_info_vram_used")))
        except (OSError, TypeError, ValueError):
            continue
    return None


def wait_quiet_card(dev, limit_s: float = 30.0) -> dict:
    """Waits (up to limit_s) until no more than 4 GB of the card is held outside this
    process's allocator -- on a box handed over while a previous process's memory is still
    being released (r04: 200-267 GB in use at the start of a call, gone seconds later;
    tests/test_gpu_large.py) -- and says what it found."""
    t0 = time.monotonic()
    first = None
    while True:
        used = card_vram_used(dev)
        if used is None:
            return {"vram_in_use_by_others_gb": None, "waited_s": 0.0}
        others = used - torch.cuda.memory_reserved(dev)
        first = others if first is None else first
        if others <= (4 << 30) or time.monotonic() - t0 >= limit_s:
            return {"vram_in_use_by_others_gb": round(first / 1e9, 1),
                    "waited_s": round(time.monotonic() - t0, 1),
                    "still_in_use_gb": round(max(others, 0) / 1e9, 1)}
        time.sleep(0.5)


def warm_host(calls: dict, seconds: float) -> dict:
    """Runs each function its number of calls in turn, over and over, for `seconds` of wall
    time (at least one pass), then waits for the device; returns the first function's first
    and last pass time (allocator and autograd caches warm before the eager rounds)."""
    t0 = time.perf_counter()
    first = next(iter(calls))
    passes = []
    while True:
        for f, n in calls.items():
            ta = time.perf_counter()
            for _ in range(n):
                f()
            if f is first:
                passes.append((time.perf_counter() - ta) / n)
        if time.perf_counter() - t0 >= seconds:
            break
    torch.cuda.synchronize()
    return {"s": round(time.perf_counter() - t0, 2), "passes": len(passes),
            "first_pass_us": round(passes[0] * 1e6, 1), "last_pass_us": round(passes[-1] * 1e6, 1)}


def pin_host_threads_l3(prefixes=("pt_autograd",)):
    """Puts the calling thread and this process's threads named `prefixes` (autograd's device
    threads) on the CPUs of one L3 domain (the calling thread's current one, within its
    allowed CPUs), and returns (cpus, restore) -- or (None, no-op) when /sys does not say.
    A short eager step hands the graph from the main thread to autograd's device thread and
    back; on two CPUs of different L3 domains that round trip costs up to 3x what it costs
    within one (tools/host_state_probe.py: the floor's passes 27-29 us with the two threads
    on one CCD, 44-82 us across CCDs or sockets; pinned, median 27.4 / p90 31.6 us,
    profiles/r04/host_state_r04zc.json) -- the scheduler's placement, not the code."""
    try:
        stat = _read("/proc/thread-self/stat")
        cur = int(stat.rsplit(")", 1)[1].split()[36])
        allowed = os.sched_getaffinity(0)
        cpus = set(_cpu_list(_read(f"/sys/devices/system/cpu/cpu{cur}/cache/index3/"
                                   "shared_cpu_list"))) & allowed
    except (AttributeError, TypeError, ValueError, IndexError, OSError):
        return None, lambda: None
    if not cpus:
        return None, lambda: None
    saved = [(0, allowed)]
    os.sched_setaffinity(0, cpus)
    for tid in os.listdir("/proc/self/task"):
        comm = (_read(f"/proc/self/task/{tid}/comm") or "").strip()
        if comm.startswith(prefixes):
            try:
                saved.append((int(tid), os.sched_getaffinity(int(tid))))
                os.sched_setaffinity(int(tid), cpus)
            except OSError:
                pass

    def restore():
        for tid, mask in saved:
            try:
                os.sched_setaffinity(tid, mask)
            except OSError:
                pass
    return sorted(cpus), restore


def cgroup_throttle():
    """cgroup v2 cpu.stat's throttling counters for this job (nr_periods, nr_throttled,
    throttled_usec), or None."""
    text = _read("/sys/fs/cgroup/cpu.stat")
    if not text:
        return None
    vals = {}
    for ln in text.splitlines():
        parts = ln.split()
        if len(parts) == 2 and parts[0] in ("nr_periods", "nr_throttled", "throttled_usec"):
            vals[parts[0]] = int(parts[1])
    return vals if len(vals) == 3 else None


def launch_stats(d: Dist, fn, groups: int = 40, per_group: int = 10):
    """Per-launch device-time distribution (the median beside the mean):
    HIP events bracket groups of `per_group` back-to-back launches on the launch stream,
    and each group's mean is one sample.  (An event pair around every single launch
    adds its own ~5 us to each sample -- tools/prof_agree.py against rocprofv3.)"""
    stream = torch.cuda.current_stream(d.dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(groups)]
    torch.cuda.synchronize(d.dev)
    for a, b in ev:
        a.record(stream)
        for _ in range(per_group):
            fn()
        b.record(stream)
    torch.cuda.synchronize(d.dev)
    ts = np.sort(np.array([a.elapsed_time(b) for a, b in ev])) / per_group * 1e3
    return {"launches": groups * per_group, "groups": groups, "median_us": round(float(np.median(ts)), 2),
            "p10_us": round(float(ts[groups // 10]), 2),
            "p90_us": round(float(ts[(9 * groups) // 10]), 2),
            "min_us": round(float(ts[0]), 2)}


def settle(d: Dist, fn, ms: float = 80.0, cap: int = 2000) -> int:
    """Back-to-back launches of `fn` until `ms` of device time have run (at most `cap`
    launches); returns the launches made.  Under a VALU-heavy load the card's clock takes a few
    hundred launches to settle after any change of load: 10 M SKS Table-8 launches go
    186 -> 133 us over ~300 launches, again after a 2 s idle gap (tools/t8_ramp_probe.py,
    profiles/r06/t8_ramp_r06z.json).  The reference's own statistic is a ~10 s mean
    (cal_ACA, GPU_Runtime Test.cu:1183-1200), i.e. the settled rate."""
    stream = torch.cuda.current_stream(d.dev)
    done_ms, n = 0.0, 0
    while done_ms < ms and n < cap:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            fn()
        e1.record(stream)
        e1.synchronize()
        done_ms += e0.elapsed_time(e1)
        n += 20
    return n


def reference_statistic(d: Dist, fn):
    """cal_ACA's own statistic (GPU_Runtime Test.cu:1183-1200): time one launch,
    loops = 10000 / ms (about 10 s of back-to-back launches), report the mean."""
    _, ms1 = timed_region(d, fn, 1)
    loops = max(1, int(10000.0 / max(ms1, 1e-3)))
    _, ms = timed_region(d, fn, loops)
    return {"loops": loops, "mean_us": round(ms * 1e3, 2)}


def _read(path: str):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _cpu_list(text: str):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out = []
    for part in (text or "").split(","):
        if part:
            a, _, b = part.partition("-")
            out.extend(range(int(a), int(b or a) + 1))
    return out


def cpu_topology():
    """The logical CPUs this process may run on, one per physical core (the lowest-numbered
    of each core's hardware threads), ordered so that any prefix spreads evenly over the
    NUMA nodes; plus each core's node.  From /sys (topology/thread_siblings_list,
    /sys/devices/system/node)."""
    allowed = _ORIGINAL_AFFINITY or sorted(os.sched_getaffinity(0))  # before bind_numa
    node_of = {}
    for nd in sorted(int(x[4:]) for x in os.listdir("/sys/devices/system/node")
                     if x.startswith("node") and x[4:].isdigit()) if os.path.isdir(
                         "/sys/devices/system/node") else []:
        for c in _cpu_list(_read(f"/sys/devices/system/node/node{nd}/cpulist")):
            node_of[c] = nd
    first = {}
    for c in allowed:
        sib = _cpu_list(_read(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list"))
        key = min(sib) if sib else c
        first.setdefault(key, c)
    per_node = {}
    for c in sorted(first.values()):
        per_node.setdefault(node_of.get(c, 0), []).append(c)
    order = []
    for i in range(max((len(v) for v in per_node.values()), default=0)):
        for nd in sorted(per_node):
            if i < len(per_node[nd]):
                order.append(per_node[nd][i])
    return {"cores": order, "node_of": {c: node_of.get(c, 0) for c in order},
            "nodes": len(per_node)}


def cgroup_cpu_quota():
    """CPUs of time per period this job may use (cgroup v2 cpu.max), or None if unlimited."""
    text = _read("/sys/fs/cgroup/cpu.max")
    try:
        q, period = text.split()
        return None if q == "max" else max(1, int(-(-int(q) // int(period))))
    except (AttributeError, ValueError):
        return None


def host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    tpc = None
    try:  # "0,128" or "0-1" -> 2 hardware threads per core
        tpc = len(_cpu_list(_read("/sys/devices/system/cpu/cpu0/topology/thread_siblings_list")))
    except (TypeError, ValueError):
        pass
    topo = cpu_topology()
    return {"cpu_model": model, "nproc": os.cpu_count(),
            "usable_cpus": len(os.sched_getaffinity(0)), "threads_per_core": tpc,
            "physical_cores_usable": len(topo["cores"]), "numa_nodes": topo["nodes"],
            # a cgroup CPU quota ("max" = none) caps what many threads can get
            "cgroup_cpu_max": _read("/sys/fs/cgroup/cpu.max")}


def graph_of(d: Dist, fn, calls: int):
    """HIP graph of `calls` back-to-back invocations (captured on a side stream)."""
    s = torch.cuda.Stream(d.dev)
    s.wait_stream(torch.cuda.current_stream(d.dev))
    with torch.cuda.stream(s):
        fn()  # warm the allocator on the capture stream
        g = torch.cuda.CUDAGraph()
        # thread-local capture: under RCCL (N > 1) the process group's watchdog thread
        # queries events while we capture, which a global-mode capture would reject
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            for _ in range(calls):
                fn()
    torch.cuda.current_stream(d.dev).wait_stream(s)
    g.replay()
    torch.cuda.synchronize(d.dev)
    return g


PMC_TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def traffic_source() -> dict:
    """Where `roofline.traffic` comes from: the committed rocprofv3 PMC summary, the run it
    was reduced from, and whether the headline kernels' gfx950 machine code in the library
    loaded now is the code that was measured (build_lib.kernel_code_digest: a changed kernel
    makes the committed figure stale, and traffic is then reported as null until the PMC
    passes are re-run).  The source digest of the files around it is reported beside it."""
    sys.path.insert(0, os.path.join(ROOT, "sks-homography_amd"))
    try:
        import build_lib
        now_src = build_lib.sources_digest("aos")
        try:
            now_code = build_lib.kernel_code_digest()
        except Exception:  # noqa: BLE001 -- unreadable library: no code match, traffic null
            now_code = None
    finally:
        sys.path.pop(0)
    try:
        with open(PMC_TRAFFIC) as f:
            prov = json.load(f).get("provenance", {})
    except (OSError, ValueError):
        prov = {}
    measured_src = prov.get("sources_aos", {}).get("sha256")
    measured_code = prov.get("kernel_code")
    return {"file": os.path.relpath(PMC_TRAFFIC, ROOT), "pmc_run": prov.get("pmc_run"),
            "kernel_code_measured": measured_code, "kernel_code_now": now_code,
            "kernel_code_match": bool(measured_code) and measured_code == now_code,
            "sources_sha256_measured": measured_src, "sources_sha256_now": now_src["sha256"],
            "sources_match": measured_src == now_src["sha256"]}


def pmc_traffic(kernel_key: str):
    """Per-launch HBM bytes of `kernel_key` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, produced by tools/pmc_traffic.py), or None -- also None when
    the kernel's machine code changed since it was measured (traffic_source)."""
    if not traffic_source()["kernel_code_match"]:
        return None
    try:
        with open(PMC_TRAFFIC) as f:
            rec = json.load(f)
        return rec[kernel_key]
    except (OSError, KeyError, ValueError):
        return None


_FAMILY_CODE = {}


def pmc_detail(key: str, note: str = None) -> dict:
    """The committed PMC figure (profiles/pmc_traffic.json "detail") for one kernel family,
    reported beside the section's `frac`: HBM bytes per launch and their ratio to the
    section's algorithmic bytes, while the library loaded now holds the machine code that
    was measured (build_lib.kernel_family_digest); otherwise traffic null with the reason.
    The PMC workload (tools/pmc_run.py) runs each kernel at the bench's own size."""
    try:
        with open(PMC_TRAFFIC) as f:
            rec = json.load(f)["detail"][key]
    except (OSError, KeyError, ValueError):
        return {"traffic_bytes": None, "reason": f"no PMC record for {key}"}
    prefix = rec.get("prefix")
    if prefix not in _FAMILY_CODE:
        sys.path.insert(0, os.path.join(ROOT, "sks-homography_amd"))
        try:
            import build_lib
            _FAMILY_CODE[prefix] = build_lib.kernel_family_digest(prefix) if prefix else None
        except Exception:  # noqa: BLE001 -- unreadable library or no demangler: no match
            _FAMILY_CODE[prefix] = None
        finally:
            sys.path.pop(0)
    if not rec.get("code") or _FAMILY_CODE[prefix] != rec["code"]:
        return {"traffic_bytes": None,
                "reason": "the kernel's machine code changed since the PMC run (tools/gpu_round.sh pmc)"}
    out = {"traffic_bytes": int(rec["hbm_bytes"]), "pmc_key": key}
    if rec.get("traffic_over_algorithmic") is not None:
        out["traffic_over_algorithmic"] = rec["traffic_over_algorithmic"]
    if note:
        out["note"] = note
    return out


# Table 5 (imgs/CPU-runtime.png): one 4-point set solved 10 M times on one core,
# MSVC /O2, us per H (main.cpp:87-114)
TABLE5_US = {"aca": 0.0145, "sks": 0.0252, "aca_f64": 0.0171, "sks_f64": 0.0256}


def cpu_baseline(n_sample: int):
    """The reference's own C++ solver bodies (oracle/_ref) on this host's cores, SURVEY 8(d):
    (iii) the streaming AoS f32 batch of n_sample problems on ALL physical cores -- one thread
    per core, pinned, each thread first-touching its own slice so its pages are NUMA-local
    -- is `value`; the sweep 1, 2, 4 ... all cores is methodology (ii)/(iii); (i) is the
    reference's own single-core same-points method (main.cpp:87-114) in f32 and f64 beside
    Table 5.  About 10-30 s of CPU time.  If oracle/_ref did not travel to this box the
    builder's C restatement is timed instead (kind "port") and the record says so loudly."""
    orc = ge.load_oracle()
    topo = cpu_topology()
    cores = topo["cores"]
    P = len(cores)
    # A cgroup CPU quota caps the CPU time all threads together get: the GPU boxes give a
    # one-GPU job 16 CPUs of time (cpu.max 1600000 100000) on a 2 x 64-core host.  `value` is
    # then measured on that many physical cores (spread over both sockets); the sweep still
    # runs up to every physical core to show it, and a linear all-core bound is reported.
    quota = cgroup_cpu_quota()
    P_eff = min(P, quota) if quota else P
    gen = orc.Oracle()
    src = gen.fill_uniform(n_sample * 8, SEED, 0).reshape(n_sample, 8)
    tar = gen.fill_uniform(n_sample * 8, SEED, n_sample * 8).reshape(n_sample, 8)
    H = np.empty((n_sample, 9), dtype=np.float32)
    warning = None
    if orc.RefOracle.available():
        engine, kind = orc.RefOracle(), "reference"

        def timed(algo, eng, k, reps):
            return eng.time_pinned(algo, src, tar, cores[:k], reps)
    else:
        engine, kind = orc.Oracle(), "port"
        warning = ("oracle/_ref (the reference's own compiled C++) is missing on this box: the "
                   "CPU baseline times the builder's C restatement instead, unpinned")
        print(f"bench.py: WARNING: {warning}", file=sys.stderr, flush=True)

        def timed(algo, eng, k, reps):
            return eng.time_batch(algo, src, tar, H, k, reps)

    def rate(algo, eng, k, seconds, tries=1):
        """Best of `tries` timed runs of about `seconds` each (the host is shared: another
        tenant's load only ever slows a run down)."""
        t1 = timed(algo, eng, k, 1)
        reps = max(1, int(seconds / max(t1, 1e-6)))
        best = max(n_sample * reps / timed(algo, eng, k, reps) / 1e6 for _ in range(tries))
        return best, reps

    # methodology (ii)/(iii) of SURVEY 8(d): the streaming batch on 1, 2, 4 ... all cores
    counts = sorted({min(1 << i, P) for i in range(P.bit_length() + 1)} | {P_eff})
    sweep_f = {k: rate("aca", engine, k, 0.3, tries=2)[0] for k in counts}
    sweep = {str(k): round(v, 1) for k, v in sweep_f.items()}
    k_best = max(counts, key=lambda k: (sweep_f[k], -k))  # fastest thread count (fewest on ties)
    out = {}
    algos = ("aca", "sks", "ge") if kind == "reference" else ("aca", "sks")
    for algo in algos:
        out[algo], out[algo + "_reps"] = rate(algo, engine, k_best, 0.5, tries=3)
    out["aca"] = max(out["aca"], sweep_f[k_best])
    verified = None
    if kind == "reference":  # the timed multi-core path computes what the reference computes
        Hp = np.empty_like(H)
        engine.time_pinned("aca", src, tar, cores[:k_best], 1, Hp)
        verified = bool(np.array_equal(Hp.view(np.uint32), engine.solve("aca", src, tar).view(np.uint32)))
    native = None
    if kind == "reference" and os.path.exists(orc.REF_NATIVE_SO) and orc.cpu_has_avx512():
        # the reference built for speed (not bit-exact): a stronger CPU yardstick beside the
        # bit-exact one; the GPU is never compared with anything but both
        fast = orc.RefOracle(orc.REF_NATIVE_SO)
        native = {"flags": "g++ -O3 -march=x86-64-v4 -ffp-contract=fast -flto (not bit-exact)",
                  "threads": k_best}
        for algo in ("aca", "sks"):
            native[algo + "_value"] = round(rate(algo, fast, k_best, 0.5, tries=2)[0], 1)
    single = {}
    if kind == "reference":
        # the reference's own CPU methodology (main.cpp:87-114): one set, 10 M calls, one core
        for algo in algos:
            single[algo] = engine.time_repeat(algo, src[0], tar[0], 10_000_000) / 1e7 * 1e6
        for algo in ("aca", "sks"):
            single[algo + "_f64"] = engine.time_repeat(
                algo, src[0].astype(np.float64), tar[0].astype(np.float64), 10_000_000) / 1e7 * 1e6
        single = {k: round(v, 5) for k, v in single.items()}
        single["table5_us_msvc_O2"] = TABLE5_US
    quota_note = (f"the fastest point of the sweep 1 ... {P} threads; this job's cgroup CPU quota "
                  f"(cpu.max) is {P_eff} CPUs of time on a host of {P} physical cores, so more "
                  f"threads share the same time (a run may briefly burst past it)"
                  ) if P_eff < P else f"the fastest point of the sweep 1 ... all {P} physical cores"
    rec = {
        "value": out["aca"], "unit": "M homographies/s", "cores": k_best, "kind": kind,
        "sks_value": out["sks"], "ge_value": out.get("ge"),
        "sample": (f"AoS f32 normalised batch of {n_sample} problems (seed {SEED}, U[0,1024)), "
                   f"best of 3 runs of {out['aca_reps']} passes ACA / {out['sks_reps']} SKS, one "
                   f"std::thread per physical core, pinned, spread over the NUMA nodes, NUMA-local "
                   f"first-touch slices; cores: {quota_note}"),
        "physical_cores": P, "cgroup_cpu_quota": quota,
        # every physical core at the measured per-core rate: an upper bound, not a measurement
        # (it ignores the DRAM bandwidth 100 B/H would need at that rate)
        "all_physical_cores_linear_bound": round(sweep_f[P_eff] / P_eff * P, 1),
        "all_core_output_bit_exact": verified,
        "single_core_same_points_us_per_H": single or None,
        "aca_thread_sweep_M_per_s": sweep,
        "sixteen_thread_aca_value": sweep.get("16"),
        "native_march": native,
        "host": host_info(),
    }
    if warning:
        rec["warning"] = warning
    return rec


def config0_check(pkg, dev, n: int = 1000) -> dict:
    """BASELINE configs[0]: ACA on 1 000 problems (seed SEED), the reference's own compiled
    C++ (oracle/_ref, the checker of the cpu_baseline leg) against the GPU kernel's bits."""
    orc = ge.load_oracle()
    gen = orc.Oracle()
    s = gen.fill_uniform(n * 8, SEED, 0).reshape(n, 8)
    t = gen.fill_uniform(n * 8, SEED, n * 8).reshape(n, 8)
    got = pkg.solve("aca", torch.from_numpy(s).to(dev), torch.from_numpy(t).to(dev),
                    normalize=True).cpu().numpy()
    ref = orc.RefOracle() if orc.RefOracle.available() else None
    want = ref.solve("aca", s, t) if ref else gen.solve("aca", s, t)
    return {"n": n, "checker": "reference" if ref else "port",
            "bit_exact": bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))}


def baseline_configs(line: dict, args, world: int) -> dict:
    """One compact entry per BASELINE.json config, drawn from the sections above, printed at
    the END of the line so that a tail of it shows all five."""
    def get(*path):
        x = line
        for k in path:
            if not isinstance(x, dict) or k not in x:
                return None
            x = x[k]
        return x

    def tb(tr):
        return tr.get("traffic_bytes") if isinstance(tr, dict) else tr

    head = get("config", "algo") == "aca" and get("config", "layout") == "aos" and get("dtype") == "f32"
    c0 = get("cpu_baseline", "config0_n1000")
    return {
        "c0_aca_n1000_cpu": ({"bit_exact": c0.get("bit_exact"), "checker": c0.get("checker"),
                              "ref_cpu_M_H_s": get("cpu_baseline", "value")} if c0 else
                             {"bit_exact": None, "reason": "cpu leg runs at N=1 on rank 0 only"}),
        "c1_aca_10M": ({"M_H_s": get("value"), "frac": get("roofline", "frac"),
                        "traffic_B": tb(get("roofline", "traffic"))} if head else None),
        "c2_sks_10M": {"M_H_s": get("sks", "value"), "frac": get("sks", "frac"),
                       "traffic_B": tb(get("sks", "traffic")),
                       "sks_over_aca_time": get("sks", "sks_over_aca_time")},
        "c3_tensor_aca_64K": {"us": get("tensor_aca_rect", "us_per_call"),
                              "torch_us": get("tensor_aca_rect", "torch_composed_us_per_call"),
                              "graph_us": get("tensor_aca_rect", "graph_us_per_call"),
                              "torch_graph_us": get("tensor_aca_rect", "torch_composed_graph_us_per_call"),
                              "large_16M_frac": get("tensor_aca_rect", "large_frac")},
        "c4_aca_80M_8gpu": ({"n_gpus": world, "M_H_s": get("value"), "global_batch": get("config", "global_batch")}
                            if world == 8 else
                            {"n_gpus": world, "M_H_s": None,
                             "reason": f"configs[4] is the 8-GPU run (driver's SCALE); this run has {world}"}),
    }


def torch_tensor_aca_rect(src, tar, scale, div):
    """The reference's composed ATen formulation (Modules_Runtime_Test.py:294-302),
    restated for timing on the same GPU (the comparison the survey asks for)."""
    bs = tar.shape[0]
    H = torch.zeros((bs, 3, 3), device=tar.device)
    d = tar[:, :, 1:] - tar[:, :, 0:1]
    q = torch.cross(d[:, 1:2, :], d[:, 0:1, :], dim=2)
    b = torch.sum(q, dim=2, keepdim=True) * tar[:, :, 0:1]
    H[:, :, 0:1] = tar[:, :, 1:2] * q[:, :, 0:1] - b
    H[:, :, 1:2] = torch.mul(div, tar[:, :, 2:3] * q[:, :, 1:2] - b)
    H[:, :, 2:3] = scale * b - src[:, 0:1, 0:1] * H[:, :, 0:1] - src[:, 1:2, 0:1] * H[:, :, 1:2]
    return H


def torch_aca_vanilla(src, tar):
    """The reference's composed ACA_vanilla (Modules_Runtime_Test.py:322-382) as the same
    sequence of tensor operations -- the same selects, products, differences and column
    writes in the same order, so autograd builds the same graph (the CPU suite pins its H
    and gradients to tests/golden/torch_vanilla_grad.npz).  For timing on the same GPU and
    as the GPU tests' autograd checker on the box's CPU.  Names follow hg_solvers.hpp."""
    bs = src.shape[0]
    sn_x = src[:, 1, 0] - src[:, 0, 0]                       # :322-329
    sn_y = src[:, 1, 1] - src[:, 0, 1]
    sp_x = src[:, 2, 0] - src[:, 0, 0]
    sp_y = src[:, 2, 1] - src[:, 0, 1]
    sq_x = src[:, 3, 0] - src[:, 0, 0]
    sq_y = src[:, 3, 1] - src[:, 0, 1]
    det_s = sn_x * sp_y - sn_y * sp_x                        # :331-333
    qs_x = sp_y * sq_x - sp_x * sq_y
    qs_y = sn_x * sq_y - sn_y * sq_x
    tn_x = tar[:, 1, 0] - tar[:, 0, 0]                       # :335-342
    tn_y = tar[:, 1, 1] - tar[:, 0, 1]
    tp_x = tar[:, 2, 0] - tar[:, 0, 0]
    tp_y = tar[:, 2, 1] - tar[:, 0, 1]
    tq_x = tar[:, 3, 0] - tar[:, 0, 0]
    tq_y = tar[:, 3, 1] - tar[:, 0, 1]
    det_t = tn_x * tp_y - tn_y * tp_x                        # :344-346
    qt_x = tp_y * tq_x - tp_x * tq_y
    qt_y = tn_x * tq_y - tn_y * tq_x
    r = det_s - qs_x - qs_y                                  # :348-353
    c11 = qs_y * qt_x * r
    c22 = qs_x * qt_y * r
    c33 = qs_x * qs_y * (det_t - qt_x - qt_y)
    c31 = c11 - c33
    c32 = c22 - c33
    m0 = tar[:, 0, 0] * c33                                  # :355-360
    m1 = tar[:, 0, 1] * c33
    a11 = tar[:, 1, 0] * c11 - m0
    a12 = tar[:, 2, 0] * c22 - m0
    a21 = tar[:, 1, 1] * c11 - m1
    a22 = tar[:, 2, 1] * c22 - m1
    h0 = a11 * sp_y - a12 * sn_y                             # :362-370
    h1 = a12 * sn_x - a11 * sp_x
    h3 = a21 * sp_y - a22 * sn_y
    h4 = a22 * sn_x - a21 * sp_x
    h6 = c31 * sp_y - c32 * sn_y
    h7 = c32 * sn_x - c31 * sp_x
    h2 = m0 * det_s - h0 * src[:, 0, 0] - h1 * src[:, 0, 1]
    h5 = m1 * det_s - h3 * src[:, 0, 0] - h4 * src[:, 0, 1]
    h8 = c33 * det_s - h6 * src[:, 0, 0] - h7 * src[:, 0, 1]
    H = torch.ones((bs, 9), device=src.device)   # :372-382 (torch's default dtype)
    for k, v in enumerate((h0, h1, h2, h3, h4, h5, h6, h7, h8)):
        H[:, k] = v
    return H.reshape(bs, 3, 3)


# TensorACA rect in the reference's (B,3,4) layout: 48 B tar + 48 B src (whole records: the
# two floats used, src[:,0,0] and src[:,1,0], touch every 32-B sector) + 36 B H
RECT_LAYOUT_MIN_BYTES = 132
# the backwards' floors in the same layout: every 32-B sector of the 48-B src records is fetched
# for M's two coordinates (16 B apart), so src costs 48 B, not 8.  dL/dtar alone: src 48 + tar
# 48 + dL/dH 36 in, dL/dtar 48 out; everything: + dL/dsrc 48 and the (problem, row) scale / div
# terms 24 out.  PMC reads 183.7 / 256.2 B (profiles/pmc_traffic.json)
RECT_BWD_TAR_LAYOUT_MIN_BYTES = 180
RECT_BWD_ALL_LAYOUT_MIN_BYTES = 252
# the fused all-gradient op (round 6: hg_tensor_aca_rect_backward_sum_f32) writes no terms:
# algorithmic src M 8 + tar 48 + dL/dH 36 in, dL/dtar 48 + dL/dsrc 48 out; layout floor with
# src's whole 48-B records (the level-0 block sums it leaves are 24 / step B, ~1.5 B)
RECT_BWD_SUM_BYTES = 188
RECT_BWD_SUM_LAYOUT_MIN_BYTES = 228

# imgs/GPU-runtime.png (Table 8), N = 1M, FP64 SoA, unnamed CUDA GPU
TABLE8_US = {"aca": 245.0, "sks": 436.0, "gpt": 8390.0, "ge": 589.0}
# the same table's full rows, N = 1 .. 1M
TABLE8_ROWS = {"aca": [3.11, 3.16, 3.19, 3.20, 5.26, 29.3, 245.0],
               "sks": [4.20, 4.26, 4.31, 4.83, 7.45, 49.9, 436.0]}
TABLE8_N = [1, 10, 100, 1000, 10_000, 100_000, 1_000_000]


def table8_sweep(d: Dist, pkg):
    """Table 8 row by row: ACA and SKS, f64 SoA unnormalised (cal_Homo_ACA/SKS), N = 1 ..
    1M.  `native`: cal_ACA's own method (.cu:1183-1200) -- back-to-back launches from a
    C++ loop (hg_tune_launch_loop), event-timed, mean per launch; host-launch-bound at
    small N on both GPUs.  `python`: the same through pkg.solve.  `graph`: device time per
    launch from a HIP graph of 100 launches."""
    import ctypes
    loop = pkg._lib.tune().hg_tune_launch_loop
    loop.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                     ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                     ctypes.c_void_p]
    loop.restype = ctypes.c_double
    stream = torch.cuda.current_stream(d.dev).cuda_stream
    w = torch.zeros((8, 1024), dtype=torch.float64, device=d.dev)
    wh = torch.empty((9, 1024), dtype=torch.float64, device=d.dev)
    loop(0, 8, w.data_ptr(), w.data_ptr(), wh.data_ptr(), 1024, 1, 0, 20000, stream)  # clocks up
    out = {}
    for algo in ("aca", "sks"):
        rows = []
        for n, ref_us in zip(TABLE8_N, TABLE8_ROWS[algo]):
            src = pkg.fill_uniform(n * 8, SEED, 0, device=d.dev).view(8, n).double()
            tar = pkg.fill_uniform(n * 8, SEED, n * 8, device=d.dev).view(8, n).double()
            H = torch.empty((9, n), dtype=torch.float64, device=d.dev)
            f = lambda: pkg.solve(algo, src, tar, normalize=False, layout="soa", out=H)  # noqa
            for _ in range(20):
                f()
            _, ms1 = timed_region(d, f, 20)
            loops = max(20, min(20000, int(300.0 / max(ms1, 1e-3))))
            _, ms = timed_region(d, f, loops)
            native = loop(0 if algo == "aca" else 1, 8, src.data_ptr(), tar.data_ptr(),
                          H.data_ptr(), n, 1, 0, loops, stream)
            g = graph_of(d, f, 100)
            _, ms_g = timed_region(d, g.replay, 5)
            del g
            rows.append({"n": n, "native_us_per_launch": round(native, 2),
                         "python_us_per_launch": round(ms * 1e3, 2),
                         "graph_us_per_launch": round(ms_g * 1e3 / 100, 2),
                         "table8_us": ref_us, "speedup_vs_table8": round(ref_us / native, 2)})
        out[algo] = rows
    return out


def vanilla_autograd_section(d: Dist, pkg, batch: int, big: int = 16 * 1024 * 1024):
    """ACA_vanilla as a differentiable loss term (deep homography with general quads):
    forward + backward of the reference's ATen composition (torch_aca_vanilla: the same
    graph, so the same gradient bits) against ours (torch.ops.sks_amd.aca + one
    hg_aca_backward_f32 launch) at the config-4 batch -- eager (against autograd's own floor
    for a one-element op on this host) and 100 steps per HIP graph; the same for
    TensorACA_rect with tar requiring grad; and the backward kernel alone at 16 M problems
    against its 164 B per problem (32 + 32 + 36 in, 32 + 32 out)."""
    torch.manual_seed(0)
    src, tar, *_ = pkg.adjust(d.dev, batch)
    tar = (tar + torch.rand_like(tar)).contiguous()
    gH = torch.randn(batch, 3, 3, device=d.dev)
    S, T = src.clone().requires_grad_(), tar.clone().requires_grad_()

    def step(fn):
        def f():
            S.grad = None
            T.grad = None
            fn(S, T).backward(gH)
        return f

    f_ours = step(lambda a, b: pkg.ACA_vanilla(batch, a, b))
    f_torch = step(torch_aca_vanilla)
    f_ours()
    ours = (S.grad.clone(), T.grad.clone())
    f_torch()
    same = bool(torch.equal(ours[0], S.grad) and torch.equal(ours[1], T.grad))
    # autograd's own per-step floor on this host: a one-element mul and its .backward()
    x1 = torch.ones(1, device=d.dev, requires_grad=True)
    g1 = torch.ones(1, device=d.dev)

    def f_floor():
        x1.grad = None
        (x1 * 2.0).backward(g1)

    # unpinned, a host-bound loop ran 1.7x slower for 0.5-3 s at a time depending on where
    # the scheduler put the two threads (profiles/r04/bench_r04t.log: rounds 50, 50, 50, 29,
    # 29 ... us; bench_r04zb.log: six slow rounds), with no CPU-quota throttling (cpu.stat)
    # the eager rounds with the main thread and autograd's device thread on one L3 domain
    # (pin_host_threads_l3: across domains the hand-off round trip costs up to 3x), after a
    # short host warm-up; the affinities come back after the TensorACA rounds below
    l3_cpus, unpin = pin_host_threads_l3()
    try:
        warm = warm_host({f_ours: 400, f_floor: 400, f_torch: 10}, seconds=1.0)
        eager = interleaved_ms(d, {"ours": f_ours, "torch": f_torch, "floor": f_floor},
                               steps={"ours": 400, "torch": 40, "floor": 400})
        ms_o, ms_t, ms_floor = eager["ours"], eager["torch"], eager["floor"]
        # 100 fwd + bwd steps (torch.autograd.grad: no .grad accumulation) in one HIP graph
        ops = torch.ops.sks_amd
        g_o = graph_of(d, lambda: torch.autograd.grad(ops.aca.default(S, T, False), (S, T), gH), 100)
        g_t = graph_of(d, lambda: torch.autograd.grad(torch_aca_vanilla(S, T), (S, T), gH), 100)
        _, ms_go = timed_region(d, g_o.replay, 10)
        _, ms_gt = timed_region(d, g_t.replay, 3)
        del g_o, g_t
        # the same for TensorACA_rect with tar requiring grad (deep-homography training)
        _, _, sh, th, sc, dv = pkg.adjust(d.dev, batch)
        Th = th.clone().requires_grad_()

        def r_ours():
            Th.grad = None
            pkg.TensorACA_rect(batch, sh, Th, sc, dv).backward(gH)

        def r_torch():
            Th.grad = None
            torch_tensor_aca_rect(sh, Th, sc, dv).backward(gH)

        warm_host({r_ours: 400, r_torch: 10}, seconds=0.5)
        eager_r = interleaved_ms(d, {"ours": r_ours, "torch": r_torch}, steps={"ours": 400, "torch": 40})
    finally:
        unpin()  # a failure in the rounds must not leave the process pinned
    ms_ro, ms_rt = eager_r["ours"], eager_r["torch"]
    # the same rounds with the threads where the scheduler puts them -- what a caller who does
    # not pin gets; floor measured the same way, in the same rounds
    warm_host({f_ours: 400, f_floor: 400}, seconds=0.5)
    eager_u = interleaved_ms(d, {"ours": f_ours, "floor": f_floor}, steps={"ours": 400, "floor": 400})
    g_ro = graph_of(d, lambda: torch.autograd.grad(ops.tensor_aca_rect.default(sh, Th, sc, dv), (Th,), gH), 100)
    g_rt = graph_of(d, lambda: torch.autograd.grad(torch_tensor_aca_rect(sh, Th, sc, dv), (Th,), gH), 100)
    _, ms_gro = timed_region(d, g_ro.replay, 10)
    _, ms_grt = timed_region(d, g_rt.replay, 3)
    del g_ro, g_rt, S, T, src, tar, gH, sh, th, Th
    n = big
    s = torch.rand(n, 8, device=d.dev) * 1024
    t = torch.rand(n, 8, device=d.dev) * 1024
    g = torch.randn(n, 9, device=d.dev)
    gs, gt = torch.empty_like(s), torch.empty_like(t)
    stream = torch.cuda.current_stream(d.dev).cuda_stream
    f_k = lambda: pkg._lib.call("hg_aca_backward_f32", s.data_ptr(), t.data_ptr(),  # noqa: E731
                                g.data_ptr(), n, gs.data_ptr(), gt.data_ptr(), stream)
    for _ in range(5):
        f_k()
    _, ms_k = timed_region(d, f_k, 50)
    del s, t, g, gs, gt
    gbps = n * 164 / (ms_k * 1e-3) / 1e9
    return {"batch": batch, "fwd_bwd_us_per_call": round(ms_o * 1e3, 2),
            "torch_composed_fwd_bwd_us_per_call": round(ms_t * 1e3, 2),
            "speedup_vs_torch": round(ms_t / ms_o, 2),
            "autograd_floor_us_per_call": round(ms_floor * 1e3, 2),
            "above_floor_us_per_call": round((ms_o - ms_floor) * 1e3, 2),
            "graph_fwd_bwd_us_per_call": round(ms_go * 1e3 / 100, 2),
            "torch_composed_graph_fwd_bwd_us_per_call": round(ms_gt * 1e3 / 100, 2),
            "rect_fwd_bwd_us_per_call": round(ms_ro * 1e3, 2),
            "rect_torch_composed_fwd_bwd_us_per_call": round(ms_rt * 1e3, 2),
            "rect_graph_fwd_bwd_us_per_call": round(ms_gro * 1e3 / 100, 2),
            "rect_torch_composed_graph_fwd_bwd_us_per_call": round(ms_grt * 1e3 / 100, 2),
            "eager_best_round_us_per_call": {"ours": round(eager["best"]["ours"] * 1e3, 2),
                                             "floor": round(eager["best"]["floor"] * 1e3, 2),
                                             "torch": round(eager["best"]["torch"] * 1e3, 2),
                                             "rect_ours": round(eager_r["best"]["ours"] * 1e3, 2)},
            "eager_rounds_us_per_call": {k: [round(x * 1e3, 1) for x in eager["rounds"][k]]
                                         for k in ("ours", "floor")},
            "eager_cgroup_throttling": eager["throttled"],
            "eager_host_warmup": warm,
            "eager_threads_on_l3_cpus": l3_cpus,
            "eager_method": "median (and fastest) of 7 interleaved rounds of 400 calls (ours, floor) / 40 (torch), main and autograd device threads on one L3 domain",
            "eager_unpinned": {"fwd_bwd_us_per_call": round(eager_u["ours"] * 1e3, 2),
                               "autograd_floor_us_per_call": round(eager_u["floor"] * 1e3, 2),
                               "above_floor_us_per_call": round((eager_u["ours"] - eager_u["floor"]) * 1e3, 2),
                               "rounds_us_per_call": {k: [round(x * 1e3, 1) for x in eager_u["rounds"][k]]
                                                      for k in ("ours", "floor")},
                               "method": "the same interleaved rounds with no thread pinning (the scheduler's placement)"},
            "gradients_bit_identical_to_torch_composed_on_gpu": same,
            "backward_large_batch": n, "backward_large_us_per_launch": round(ms_k * 1e3, 2),
            "backward_large_gbps": round(gbps, 1), "backward_large_frac": round(gbps / HBM_PEAK_GBPS, 4),
            "backward_large_traffic": pmc_detail("aca_vanilla_backward"),
            "backward_bytes_per_problem": 164}


def grouped_section(d: Dist, pkg, k: int = 64, m: int = 1000):
    """A caller with many of Table 8's N = 1000 batches (f64 SoA, unnormalised, cal_Homo_ACA's
    contract): hg_solve_grouped_f64 (32 batches per launch) called as a native caller would,
    with its pointer arrays built once, against one launch per batch (`table8_sweep`'s native
    C++ loop at n = 1000 is the per-launch figure; `one_launch_each` here goes through
    ops.solve from Python) and against ops.solve_grouped, whose per-tensor checks cost more
    host time than the launches.  Device time per batch from HIP events."""
    import ctypes
    srcs, tars, outs = [], [], []
    for i in range(k):
        srcs.append(pkg.fill_uniform(m * 8, SEED, 2 * i * m * 8, device=d.dev).view(8, m).double())
        tars.append(pkg.fill_uniform(m * 8, SEED, (2 * i + 1) * m * 8, device=d.dev).view(8, m).double())
        outs.append(torch.empty((9, m), dtype=torch.float64, device=d.dev))
    each = [torch.empty_like(o) for o in outs]

    P = ctypes.c_void_p * k
    ps, pt, ph = (P(*[x.data_ptr() for x in v]) for v in (srcs, tars, outs))
    ns = (ctypes.c_int64 * k)(*([m] * k))
    grouped = pkg.lib().hg_solve_grouped_f64
    stream = torch.cuda.current_stream(d.dev).cuda_stream

    def f_group():
        rc = grouped(0, ps, pt, ph, ns, k, 1, 0, stream)
        if rc:
            raise pkg.HipError("hg_solve_grouped_f64", rc)

    def f_group_py():
        pkg.solve_grouped("aca", srcs, tars, normalize=False, layout="soa", outs=outs)

    def f_each():
        for s, t, o in zip(srcs, tars, each):
            pkg.solve("aca", s, t, normalize=False, layout="soa", out=o)

    for _ in range(5):
        f_group()
        f_group_py()
        f_each()
    _, ms_g = timed_region(d, f_group, 200)
    _, ms_gp = timed_region(d, f_group_py, 20)
    _, ms_e = timed_region(d, f_each, 20)
    same = all(torch.equal(a.view(torch.int64), b.view(torch.int64)) for a, b in zip(outs, each))
    us_g, us_e = ms_g * 1e3 / k, ms_e * 1e3 / k
    return {"batches": k, "n_per_batch": m, "layout": "soa f64, unnormalised",
            "grouped_us_per_batch": round(us_g, 3),
            "grouped_python_wrapper_us_per_batch": round(ms_gp * 1e3 / k, 3),
            "one_launch_each_us_per_batch": round(us_e, 3),
            "grouped_speedup": round(us_e / us_g, 1), "table8_us_n1000": 3.20,
            "speedup_vs_table8": round(3.20 / us_g, 1), "bit_identical": bool(same)}


def reference_layout(d: Dist, pkg):
    """Like-for-like with the reference GPU harness (cal_Homo_ACA/SKS,
    GPU_Runtime Test.cu:81-240, timed as cal_ACA does at :1166-1206): FP64, SoA
    (8,N)/(9,N), unnormalised, N = 1M and 10M, mean per-launch time over ~1 s of
    back-to-back launches.  Table 8's numbers are from an unnamed CUDA GPU."""
    out = {}
    for n in (1_000_000, 10_000_000):
        src = pkg.fill_uniform(n * 8, SEED, 0, device=d.dev).view(8, n).double()
        tar = pkg.fill_uniform(n * 8, SEED, n * 8, device=d.dev).view(8, n).double()
        H = torch.empty((9, n), dtype=torch.float64, device=d.dev)
        algos = ("aca", "sks", "gpt", "ge") if n == 1_000_000 else ("aca", "sks")
        for algo in algos:  # all four in binary64, as Table 8 (cal_Homo_GE is f64 too)
            f = lambda: pkg.solve(algo, src, tar, normalize=False, layout="soa", out=H)  # noqa
            for _ in range(10):
                f()
            _, ms1 = timed_region(d, f, 10)
            loops = max(10, min(5000, int(1000.0 / max(ms1, 1e-3))))  # ~1 s, like .cu:1188
            _, ms = timed_region(d, f, loops)
            bpp = 200
            rec = {"us_per_launch": round(ms * 1e3, 2), "launches": loops,
                   "achieved_gbps": round(n * bpp / (ms * 1e-3) / 1e9, 1),
                   "frac": round(n * bpp / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                   "G_homographies_per_s": round(n / (ms * 1e-3) / 1e9, 2)}
            if n == 10_000_000:
                rec["traffic"] = pmc_detail(f"{algo}_f64_soa")
            if n == 1_000_000:
                rec["table8_us"] = TABLE8_US[algo]
                rec["speedup_vs_table8"] = round(TABLE8_US[algo] / (ms * 1e3), 2)
            out[f"{algo}_f64_soa_n{n}"] = rec
        del src, tar, H
    return out


def table8_pipeline_section(d: Dist, pkg, n: int = 1_000_000):
    """The reference harness's sampling flow in its own formats (GPU_Runtime Test.cu:
    1443-1451) on its own point file, N = 1M: 4N MRG32K3A words (seed 11), get_rand_list,
    cal_Homo_ACA/SKS.  Draws: the hand-written generator (rocRAND's host-API words, bit for
    bit) against rocrand_generate itself with a fresh generator per call, as the harness
    creates one.  Pipeline: draws + gather + solve in ONE launch (hg_rand_gather_solve_f64:
    72 B of H per hypothesis, no words in memory) against the two launches (draws, then
    hg_gather_solve_f64: +16 B of words written and read) and the unfused gather-then-solve;
    at 1 M and 10 M, beside a write-only stream of the same 72 B per hypothesis (the ceiling
    of a launch that only writes).  Table 8 times cal_Homo_* alone (245 / 436 us at 1M)."""
    import ctypes
    tune = pkg._lib.tune()
    tune.hg_tune_rocrand_mrg32k3a_u32.argtypes = [ctypes.c_void_p, ctypes.c_int64,
                                                  ctypes.c_uint64, ctypes.c_void_p]
    wr = tune.hg_tune_copy
    wr.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    stream = torch.cuda.current_stream(d.dev).cuda_stream
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"]).to(d.dev).double()  # Point2f -> Point2d (.cu:1414-1416)
    pt = torch.from_numpy(g["pool_tar"]).to(d.dev).double()
    words = torch.empty(4 * n, dtype=torch.int32, device=d.dev)
    f_draw = lambda: pkg._lib.call("hg_rand_mrg32k3a_u32", words.data_ptr(), 4 * n, SEED, stream)  # noqa: E731
    for _ in range(5):
        f_draw()
    ms_draw = launch_stats(d, f_draw, groups=20)["median_us"] * 1e-3
    ref_words = torch.empty_like(words)
    f_roc = lambda: tune.hg_tune_rocrand_mrg32k3a_u32(ref_words.data_ptr(), 4 * n, SEED, stream)  # noqa: E731
    f_roc()
    _, ms_roc = timed_region(d, f_roc, 5)
    f_draw()
    # the launch's yardstick: a write-only stream of the same 16 B per hypothesis (16-B stores)
    wsmall = torch.empty(4 * n, dtype=torch.int32, device=d.dev)
    f_wsmall = lambda: wr(5, None, wsmall.data_ptr(), 4 * n * 4, stream)  # noqa: E731
    for _ in range(5):
        f_wsmall()
    ms_wsmall = launch_stats(d, f_wsmall, groups=20)["median_us"] * 1e-3
    del wsmall
    rl = words.view(4, n)
    out = {"n": n, "pool": int(ps.shape[0]),
           "draws": {"words": 4 * n, "us": round(ms_draw * 1e3, 2),
                     "gbps_written": round(4 * n * 4 / (ms_draw * 1e-3) / 1e9, 1),
                     "write_only_stream_us": round(ms_wsmall * 1e3, 2),
                     "frac_of_write_only_stream": round(ms_wsmall / ms_draw, 4),
                     "traffic": pmc_detail("mrg_words", "PMC at 40 M words (10 x this launch)"),
                     "rocrand_generate_us": round(ms_roc * 1e3, 1),
                     "speedup_vs_rocrand": round(ms_roc / ms_draw, 1),
                     "bit_identical_to_rocrand": bool(torch.equal(words, ref_words))}}
    del ref_words
    for algo in ("aca", "sks"):
        aid = {"aca": 0, "sks": 1}[algo]
        H = torch.empty((9, n), dtype=torch.float64, device=d.dev)
        H1 = torch.empty((9, n), dtype=torch.float64, device=d.dev)
        f_fused = lambda: pkg.gather_solve(ps, pt, rl, algo)  # noqa: E731
        f_one = lambda: pkg._lib.call("hg_rand_gather_solve_f64", aid, ps.data_ptr(), pt.data_ptr(),  # noqa: E731
                                      ps.shape[0], SEED, H1.data_ptr(), n, 0, stream)

        def f_two():
            f_draw()
            pkg._lib.call("hg_gather_solve_f64", aid, ps.data_ptr(), pt.data_ptr(), ps.shape[0],
                          words.data_ptr(), H.data_ptr(), n, 0, stream)

        def f_split():
            s_, t_ = pkg.get_rand_list(rl, ps, pt)
            pkg.solve(algo, s_, t_, normalize=False, layout="soa", out=H)

        for _ in range(10):
            f_fused()
            f_split()
            f_one()
        ms_fused = launch_stats(d, f_fused, groups=20)["median_us"] * 1e-3
        ms_one = launch_stats(d, f_one, groups=20)["median_us"] * 1e-3
        _, ms_two = timed_region(d, f_two, 100)
        _, ms_split = timed_region(d, f_split, 100)
        f_split()
        same = bool(torch.equal(f_fused().view(torch.int64), H.view(torch.int64)))
        f_one()
        same_one = bool(torch.equal(H1.view(torch.int64), H.view(torch.int64)))
        out[algo] = {"draws_gather_solve_one_launch_us": round(ms_one * 1e3, 2),
                     "draws_then_gather_solve_us": round(ms_two * 1e3, 2),
                     "gather_solve_from_words_us": round(ms_fused * 1e3, 2),
                     "fused_gbps": round(n * 88 / (ms_fused * 1e-3) / 1e9, 1),
                     "gather_then_solve_us": round(ms_split * 1e3, 2),
                     "table8_solver_us": TABLE8_US[algo],
                     "one_launch_speedup_vs_table8_solver": round(TABLE8_US[algo] / (ms_one * 1e3), 2),
                     "fused_bit_identical_to_unfused": same,
                     "one_launch_bit_identical_to_draws_then_fused": same_one}
        del H, H1
    del words, rl
    # 10 M hypotheses (the headline's batch): the one-launch pipeline against a write-only
    # stream of its 72 B per hypothesis, and the two-launch form
    big = 10 * n
    wbuf = torch.empty(big * 18, dtype=torch.float32, device=d.dev)
    f_write = lambda: wr(5, None, wbuf.data_ptr(), big * 72, stream)  # noqa: E731
    wb = torch.empty(4 * big, dtype=torch.int32, device=d.dev)
    for algo in ("aca", "sks"):
        aid = {"aca": 0, "sks": 1}[algo]
        # three output buffers used in turn: the 10 M figure moves by up to +-10 % with where
        # the 720 MB of H land (KERNEL_NOTES.md, tools/kbench_t8q.py), so the launch is timed
        # over three placements rather than one
        Hbs = [torch.empty((9, big), dtype=torch.float64, device=d.dev) for _ in range(3)]
        Hb = Hbs[0]
        turn = [0]

        def f_one():
            turn[0] = (turn[0] + 1) % len(Hbs)
            pkg._lib.call("hg_rand_gather_solve_f64", aid, ps.data_ptr(), pt.data_ptr(),
                          ps.shape[0], SEED, Hbs[turn[0]].data_ptr(), big, 0, stream)

        def f_two():
            pkg._lib.call("hg_rand_mrg32k3a_u32", wb.data_ptr(), 4 * big, SEED, stream)
            pkg._lib.call("hg_gather_solve_f64", aid, ps.data_ptr(), pt.data_ptr(), ps.shape[0],
                          wb.data_ptr(), Hb.data_ptr(), big, 0, stream)

        for _ in range(5):
            f_one()
            f_two()
            f_write()
        settled = settle(d, f_one)
        ms_one = launch_stats(d, f_one, groups=10)["median_us"] * 1e-3
        ms_write = launch_stats(d, f_write, groups=10)["median_us"] * 1e-3
        _, ms_two = timed_region(d, f_two, 20)
        out[f"{algo}_large"] = {
            "n": big, "draws_gather_solve_one_launch_us": round(ms_one * 1e3, 2),
            "G_hyp_per_s": round(big / (ms_one * 1e-3) / 1e9, 2),
            "gbps_H": round(big * 72 / (ms_one * 1e-3) / 1e9, 1),
            "frac": round(big * 72 / (ms_one * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "traffic": pmc_detail(f"rand_gather_solve_f64_{algo}"),
            "write_only_stream_gbps": round(big * 72 / (ms_write * 1e-3) / 1e9, 1),
            "frac_of_write_only_stream": round(ms_write / ms_one, 4),
            "draws_then_gather_solve_us": round(ms_two * 1e3, 2),
            "placements": len(Hbs), "settle_launches": settled}
        del Hb, Hbs
    del wbuf, wb
    return out


def host_boundary_section(d: Dist, pkg, n: int):
    """What the host-buffer side of the boundary costs (reported, never `value`):
    (1) the reference's single-problem C++ call sks::runKernel_ACA on host pointers
    (the points ride in the launch, H comes back through mapped memory; synchronous like
    ACA_SKS.cpp:24); (2) a host-resident n-problem batch, the PCIe-inclusive rate of a
    caller whose data lives in host memory: `staged` = pinned H2D of src/tar + the kernel
    + D2H of H on one stream; `zero_copy_pinned` = hg_solve_host_f32 on pinned buffers, the
    kernel reading and writing them over PCIe itself; `pageable_staged` = hg_solve_host_f32 on
    pageable buffers, the default since 0.3 -- host threads copy them through the library's
    ring of pinned stages while the kernel reads the stage before, and the caller's pages are
    never mapped for the GPU; `pageable_registered` = the same with HG_FLAG_HOST_REGISTER (the
    pages registered for the call, zero-copy -- what round 5 did by default);
    `h2d_bound` = the 64 B/problem H2D copy alone."""
    import ctypes
    lib = pkg.lib()
    f = lib._ZN3sks13runKernel_ACAEPfS0_S0_
    f.restype = ctypes.c_int
    s8 = (ctypes.c_float * 8)(*[0, 0, 200, 0, 50, 139, 181, 93])
    t8 = (ctypes.c_float * 8)(*[10, 12, 220, 5, 40, 160, 190, 110])
    h9 = (ctypes.c_float * 9)()
    for _ in range(100):
        f(s8, t8, h9)
    reps = 2000
    t0 = time.perf_counter()
    for _ in range(reps):
        f(s8, t8, h9)
    single_us = (time.perf_counter() - t0) / reps * 1e6
    ds = pkg.fill_uniform(n * 8, SEED, 0, device=d.dev).view(n, 8)
    dt = pkg.fill_uniform(n * 8, SEED, n * 8, device=d.dev).view(n, 8)
    hs = torch.empty((n, 8), dtype=torch.float32).pin_memory()
    ht = torch.empty((n, 8), dtype=torch.float32).pin_memory()
    hH = torch.empty((n, 9), dtype=torch.float32).pin_memory()
    hs.copy_(ds.cpu())
    ht.copy_(dt.cpu())
    dH = torch.empty((n, 9), device=d.dev)
    want = pkg.solve("aca", ds, dt, out=dH).cpu()

    def staged():
        ds.copy_(hs, non_blocking=True)
        dt.copy_(ht, non_blocking=True)
        pkg.solve("aca", ds, dt, out=dH)
        hH.copy_(dH, non_blocking=True)

    def h2d():
        ds.copy_(hs, non_blocking=True)
        dt.copy_(ht, non_blocking=True)

    qs, qt = hs.clone(), ht.clone()  # pageable copies
    qH = torch.empty((n, 9), dtype=torch.float32)
    out = {"single_problem_host_ptr_us": round(single_us, 2), "batch": n,
           "pcie_bytes_per_problem": 100}
    for name, fn, res in (("staged", staged, hH),
                          ("zero_copy_pinned", lambda: pkg.solve_host("aca", hs, ht, out=hH), hH),
                          ("pageable_staged", lambda: pkg.solve_host("aca", qs, qt, out=qH), qH),
                          ("pageable_registered",
                           lambda: pkg.solve_host("aca", qs, qt, out=qH, register=True), qH),
                          ("h2d_bound", h2d, None)):
        fn()
        torch.cuda.synchronize(d.dev)
        # seven calls timed one by one (each a timed region of its own: the synchronous host
        # calls and the async pinned ones alike end synchronised); the median is `ms`.  Three
        # at N > 1, where every rank's host copies share the node's memory and CPU quota
        calls = [timed_region(d, fn, 1)[0] * 1e3 for _ in range(7 if d.world == 1 else 3)]
        ms = float(np.median(calls))
        rec = {"ms": round(ms, 3), "M_homographies_per_s": round(n / ms / 1e3, 1),
               "calls_ms": [round(c, 2) for c in calls]}
        if res is not None:
            rec["bit_exact"] = bool(torch.equal(res.view(torch.int32), want.view(torch.int32)))
        out[name] = rec
    out["zero_copy_speedup_vs_staged"] = round(out["staged"]["ms"] / out["zero_copy_pinned"]["ms"], 2)
    prev = (ctypes.c_int64 * 3)()
    lib.hg_internal_host_stage_config.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                  ctypes.POINTER(ctypes.c_int64)]
    if lib.hg_internal_host_stage_config(0, 0, 0, prev) == 0:
        out["pageable_ring"] = {"stage_bytes": prev[0], "depth": prev[1], "copy_threads": prev[2]}
    del hs, ht, hH, qs, qt, qH, ds, dt, dH
    return out


def host_sharded_section(d: Dist, pkg, src, tar, H, n: int, n_total: int):
    """The whole n_total-problem batch in HOST memory (one /dev/shm file every rank maps,
    shard.SharedHostBatch); every rank's GPU reads its block and writes its H rows over its
    own PCIe link (hg_solve_host_f32, zero-copy): the end-to-end rate of a host-resident
    batch, with N links working at once and no xGMI traffic.  Each rank fills its block
    with its own device inputs and checks the H rows it wrote against its device solve."""
    from importlib import import_module
    shard = import_module("sks_homography_amd.shard")
    need = n_total * 100
    try:
        st = os.statvfs("/dev/shm")
        room = st.f_bavail * st.f_frsize
    except OSError:
        room = 0
    if d.max(0.0 if room >= 1.25 * need else 1.0) != 0.0:  # every rank takes the same branch
        return {"skipped": f"/dev/shm too small for {need} B"}
    name = f"sks_hg_bench_{os.environ.get('MASTER_PORT', '0')}_{n_total}"
    batch, err = None, None
    try:
        # every rank allocates the pages of its own block (NUMA-local: the rank is bound to
        # its GPU's node, bind_numa); a failure anywhere reaches every rank through `agree`
        batch = shard.SharedHostBatch(name, n_total, d.rank, d.barrier, world=d.world,
                                      agree=lambda ok: d.max(0.0 if ok else 1.0) == 0.0)
    except OSError as e:
        err = str(e)
    if d.max(0.0 if batch is not None else 1.0) != 0.0:  # all ranks leave together
        if batch is not None:
            batch.close()
        return {"error": err or "another rank could not map the shared batch"}
    try:
        lo, hi = batch.block(d.world)
        batch.src[lo:hi].copy_(src)
        batch.tar[lo:hi].copy_(tar)
        batch.solve_block(d.world, device=d.dev)  # warm: registration path, clocks
        ts = []
        for _ in range(3):
            d.barrier()
            t0 = time.perf_counter()
            batch.solve_block(d.world, device=d.dev)
            d.barrier()
            ts.append(d.max(time.perf_counter() - t0))
        ms = sorted(ts)[1] * 1e3
        ok = torch.equal(batch.H[lo:hi].view(torch.int32), H.cpu().view(torch.int32))
        verified = d.max(0.0 if ok else 1.0) == 0.0
    finally:
        batch.close()
    return {"batch": n_total, "ms": round(ms, 3),
            "M_homographies_per_s": round(n_total / ms / 1e3, 1),
            "pcie_gbps_per_gpu": round(n * 100 / ms / 1e6, 1), "verified": bool(verified),
            "note": "shared-memory host batch, per-rank zero-copy over its own PCIe link"}


def ransac_section(d: Dist, pkg, hyps: int = 1 << 20, thresh: float = 3.0):
    """1M random 4-point hypotheses over the reference's own
    correspondence file (orig_pts_wall.txt, 2540 pairs, committed in tests/golden):
    draw + fused gather/solve (HBM-bound: 16 B idx + 36 B H per hypothesis) and the
    inlier scorer (VALU-bound: every hypothesis x every pair)."""
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"]).to(d.dev)
    pt = torch.from_numpy(g["pool_tar"]).to(d.dev)
    idx = pkg.fill_bits(hyps * 4, SEED, 0, d.dev).view(hyps, 4)
    H = pkg.sample_solve(ps, pt, idx)
    f_solve = lambda: pkg.sample_solve(ps, pt, idx)  # noqa: E731
    f_score = lambda: pkg.ransac_score(H, ps, pt, thresh)  # noqa: E731
    for _ in range(3):
        f_solve()
    _, ms_solve = timed_region(d, f_solve, 20)
    # the scorer is VALU-bound (~0.7 ms a launch): settled clock (`settle`), then the median
    # of 10 three-launch groups
    for _ in range(3):
        f_score()
    settle(d, f_score)
    ms_score = launch_stats(d, f_score, groups=10, per_group=3)["median_us"] * 1e-3
    counts = pkg.ransac_score(H, ps, pt, thresh)
    pairs = hyps * ps.shape[0]
    big = 16 * hyps  # the sampler's HBM-rate figure (16 B idx + 36 B H per hypothesis)
    idx_b = pkg.fill_bits(big * 4, SEED, 0, d.dev).view(big, 4)
    f_big = lambda: pkg.sample_solve(ps, pt, idx_b)  # noqa: E731
    # the box's clocks wander under these VALU-heavy launches for the first ~100 of them
    # (135 -> 190 -> 131 us per seeded launch in one rocprofv3 trace): warm, then take the
    # median of 20 ten-launch groups instead of one short mean
    for _ in range(30):
        f_big()
    ms_big = launch_stats(d, f_big, groups=20)["median_us"] * 1e-3
    # the two-launch form a caller of the reference pipeline runs (draws, then gather+solve)
    # against the seeded fused sampler (draws made in the kernel: 36 B per hypothesis)
    f_two = lambda: pkg.sample_solve(ps, pt, pkg.fill_bits(big * 4, SEED, 0, d.dev).view(big, 4))  # noqa: E731
    f_seed = lambda: pkg.sample_solve_seeded(ps, pt, big, SEED, 0)  # noqa: E731
    for _ in range(30):
        f_two()
        f_seed()
    ms_two = launch_stats(d, f_two, groups=20)["median_us"] * 1e-3
    settled_seed = settle(d, f_seed)
    ms_seed = launch_stats(d, f_seed, groups=20)["median_us"] * 1e-3
    seeded_same = bool(torch.equal(pkg.sample_solve_seeded(ps, pt, hyps, SEED, 0).view(torch.int32),
                                   H.view(torch.int32)))
    del idx_b
    # the seeded launch is a write-only stream (36 B of H per hypothesis, the pool stays in
    # LDS): its own ceiling is a plain write-only stream of the same bytes on this box
    # (tune library's 16-B store kernel, hg_tune_copy variant 5), interleaved with it
    import ctypes
    wr = pkg._lib.tune().hg_tune_copy
    wr.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    wr.restype = ctypes.c_int
    wbuf = torch.empty(big * 9, dtype=torch.float32, device=d.dev)
    wstream = torch.cuda.current_stream(d.dev).cuda_stream
    f_write = lambda: wr(5, None, wbuf.data_ptr(), big * 36, wstream)  # noqa: E731
    for _ in range(30):
        f_write()
    ms_write = launch_stats(d, f_write, groups=20)["median_us"] * 1e-3
    del wbuf
    return {
        "hypotheses": hyps, "pool": int(ps.shape[0]), "thresh_px": thresh,
        "sample_solve_us": round(ms_solve * 1e3, 2),
        "sample_solve_G_hyp_per_s": round(hyps / (ms_solve * 1e-3) / 1e9, 2),
        "sample_solve_gbps": round(hyps * 52 / (ms_solve * 1e-3) / 1e9, 1),
        "sample_solve_large": {"hypotheses": big, "us": round(ms_big * 1e3, 2),
                               "G_hyp_per_s": round(big / (ms_big * 1e-3) / 1e9, 2),
                               "achieved_gbps": round(big * 52 / (ms_big * 1e-3) / 1e9, 1),
                               "frac": round(big * 52 / (ms_big * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                               "traffic": pmc_detail("sample_solve_indexed")},
        "sample_solve_seeded_large": {
            "hypotheses": big, "us": round(ms_seed * 1e3, 2),
            "G_hyp_per_s": round(big / (ms_seed * 1e-3) / 1e9, 2),
            "achieved_gbps": round(big * 36 / (ms_seed * 1e-3) / 1e9, 1),
            "frac": round(big * 36 / (ms_seed * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "traffic": pmc_detail("sample_solve_seeded"),
            "write_only_stream_gbps": round(big * 36 / (ms_write * 1e-3) / 1e9, 1),
            "frac_of_write_only_stream": round(ms_write / ms_seed, 4),
            "draws_then_indexed_us": round(ms_two * 1e3, 2),
            "speedup_vs_two_launch": round(ms_two / ms_seed, 2),
            "bit_identical_to_indexed": seeded_same, "settle_launches": settled_seed},
        "score_ms": round(ms_score, 3),
        "score_G_pairs_per_s": round(pairs / (ms_score * 1e-3) / 1e9, 1),
        "best_inliers": int(counts.max().item()),
    }


def split_gather_section(d: Dist, pkg, src, tar, H, n: int, n_total: int, step_ms: float):
    """SURVEY 8(e)'s second number: the split / gather a caller whose batch lives on one
    rank pays, outside the timed steps.  Split: rank 0 holds the whole (n_total, 8)
    src/tar and scatter_blocks hands each rank its block (paired send/recv; RCCL over
    xGMI, bound by rank 0's egress); every rank checks the bytes it received against the
    block it generated itself.  Gather: every H block to rank 0 (ingress-bound); rank 0
    re-solves a slice of the last rank's block and checks the gathered bits.  Over gloo
    (one-GPU rehearsal) the blocks go through the host."""
    host = d.backend != "nccl"
    mv = (lambda t: t.cpu()) if host else (lambda t: t)  # noqa: E731
    full_s = full_t = None
    if d.rank == 0:
        full_s = mv(pkg.fill_uniform(n_total * 8, SEED, 0, device=d.dev).view(n_total, 8))
        full_t = mv(pkg.fill_uniform(n_total * 8, SEED, n_total * 8, device=d.dev).view(n_total, 8))
    like = mv(src[:1])
    warm = pkg.scatter_blocks(full_s[:1024 * d.world] if d.rank == 0 else None, 1024 * d.world,
                              d.world, d.rank, like)  # open the p2p connections
    del warm
    torch.cuda.synchronize(d.dev)
    d.barrier()
    t0 = time.perf_counter()
    got_s = pkg.scatter_blocks(full_s, n_total, d.world, d.rank, like)
    got_t = pkg.scatter_blocks(full_t, n_total, d.world, d.rank, like)
    torch.cuda.synchronize(d.dev)
    d.barrier()
    t_split = d.max(time.perf_counter() - t0)
    ok = (torch.equal(got_s.to(d.dev).view(torch.int32), src.view(torch.int32)) and
          torch.equal(got_t.to(d.dev).view(torch.int32), tar.view(torch.int32)))
    split_ok = d.max(0.0 if ok else 1.0) == 0.0
    del full_s, full_t, got_s, got_t

    blk = mv(H)
    pkg.gather_blocks(blk[:1024].contiguous(), 1024 * d.world, d.world, d.rank)
    torch.cuda.synchronize(d.dev)
    d.barrier()
    t0 = time.perf_counter()
    full = pkg.gather_blocks(blk, n_total, d.world, d.rank)
    torch.cuda.synchronize(d.dev)
    d.barrier()
    t_gather = d.max(time.perf_counter() - t0)
    out = {"split_from_rank0_ms": round(t_split * 1e3, 3), "split_bytes": n_total * 64,
           "rank0_egress_gbps": round((n_total - n) * 64 / t_split / 1e9, 1),
           "split_verified": bool(split_ok),
           "gather_to_rank0_ms": round(t_gather * 1e3, 3), "gathered_bytes": n_total * 36,
           "rank0_ingress_gbps": round((n_total - n) * 36 / t_gather / 1e9, 1),
           "end_to_end_M_homographies_per_s": round(
               n_total / (t_split + step_ms * 1e-3 + t_gather) / 1e6, 1)}
    if d.rank == 0:
        lo, m = (d.world - 1) * n, min(n, 1 << 20)
        s = pkg.fill_uniform(m * 8, SEED, lo * 8, device=d.dev).view(m, 8)
        t = pkg.fill_uniform(m * 8, SEED, (n_total + lo) * 8, device=d.dev).view(m, 8)
        want = pkg.solve("aca", s, t, normalize=True)
        got = full[lo:lo + m].to(d.dev)
        out["gather_verified"] = bool(torch.equal(want.view(torch.int32), got.view(torch.int32)))
    del full
    return out


def rank_block_inputs(pkg, dev, n: int, n_total: int, rank: int):
    """Rank `rank`'s block of the global batch (weak scaling: every rank owns n problems of
    n_total = n * world, rows [rank*n, (rank+1)*n)).  The global batch is src = the stream's
    values [0, 8 n_total) and tar = values [8 n_total, 16 n_total) (seed SEED), so the
    blocks of all ranks concatenate to exactly the batch one device would generate whole
    (tests/test_gpu_config5.py checks this for the 80 M batch of BASELINE configs[4])."""
    lo = rank * n
    src = pkg.fill_uniform(n * 8, SEED, lo * 8, device=dev).view(n, 8)
    tar = pkg.fill_uniform(n * 8, SEED, (n_total + lo) * 8, device=dev).view(n, 8)
    return src, tar


def main():
    args = parse()
    # --gpus N is authoritative: a bare `bench.py --gpus 8` starts the 8 ranks itself, and a
    # rank whose WORLD_SIZE disagrees with --gpus refuses to run (before any GPU call)
    plan, why = launch_plan(args.gpus, os.environ)
    if plan == "refuse":
        print(f"bench.py: {why}", file=sys.stderr, flush=True)
        sys.exit(2)
    if plan == "spawn":
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    # before anything touches the GPU: this rank's CPUs and first-touch pages on its GPU's
    # NUMA node (the device index is LOCAL_RANK, as Dist picks it)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "nccl":  # one GPU per rank: device index = LOCAL_RANK
        numa = bind_numa(local)
    else:  # gloo rehearsal: ranks share the devices (device_count does not initialise HIP here)
        numa = bind_numa(local % max(torch.cuda.device_count(), 1))
    d = Dist(args.dist_backend)
    assert d.world == args.gpus, f"n_gpus {d.world} != --gpus {args.gpus}"
    numa["rank"] = d.rank
    try:  # the device HIP gave this rank is the one bound to
        pr = torch.cuda.get_device_properties(d.dev)
        got = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
        numa["bdf_matches_device"] = bool(numa["bdf"]) and numa["bdf"].startswith(got)
        if not numa["bdf_matches_device"]:
            # /sys and HIP numbered the GPUs differently: bind this thread (and every thread
            # started from now on) to the node of the device HIP actually gave the rank
            node = _read(f"/sys/bus/pci/devices/{got}.0/numa_node")
            cpus = sorted(set(_cpu_list(_read(f"/sys/devices/system/node/node{node}/cpulist")))
                          & set(_ORIGINAL_AFFINITY or [])) if node and int(node) >= 0 else []
            if cpus:
                os.sched_setaffinity(0, cpus)
                numa.update(node=int(node), bound_cpus=len(cpus), bdf=f"{got}.0",
                            note="rebound after GPU init: /sys order differed from HIP's")
    except (AttributeError, RuntimeError, ValueError):
        numa["bdf_matches_device"] = None
    pkg = ge.load_package()
    # a card handed over while a previous process's device memory is still coming back:
    # wait for it before allocating and timing (one rank per GPU only -- gloo rehearsal ranks
    # share a card, and each other's memory is not foreign)
    card = wait_quiet_card(d.dev) if d.backend == "nccl" else None
    global SEED
    SEED = args.seed
    n = args.n
    n_total = n * d.world
    src, tar = rank_block_inputs(pkg, d.dev, n, n_total, d.rank)
    H = torch.empty((n, 9), dtype=torch.float32, device=d.dev)
    bpp = pkg.BYTES_PER_PROBLEM["f32"]

    def run(algo):
        return lambda: pkg.solve(algo, src, tar, normalize=True, out=H)

    # the headline: BASELINE configs[1] by default (ACA, AoS f32, normalised); --algo /
    # --layout / --dtype pick another solver or the reference GPU harness's layout over the
    # same rank block (the sections after the headline keep the default buffers)
    head_algo, head_layout, head_dtype = args.algo, args.layout, args.dtype
    head_norm = head_layout == "aos"
    default_head = (head_algo, head_layout, head_dtype) == ("aca", "aos", "f32")
    if default_head:
        run_head = run("aca")
    else:
        hs = src.double() if head_dtype == "f64" else src
        ht = tar.double() if head_dtype == "f64" else tar
        if head_layout == "soa":
            hs, ht = hs.t().contiguous(), ht.t().contiguous()
        hH = torch.empty((9, n) if head_layout == "soa" else (n, 9), dtype=hs.dtype, device=d.dev)

        def run_head():
            pkg.solve(head_algo, hs, ht, normalize=head_norm, layout=head_layout, out=hH)
    bpp_head = pkg.BYTES_PER_PROBLEM[head_dtype]

    for _ in range(args.warmup):
        run_head()
    wall, ms_launch = timed_region(d, run_head, args.steps)
    value = n_total * args.steps / wall / 1e6
    per_launch = launch_stats(d, run_head)
    achieved = n * bpp_head / (ms_launch * 1e-3) / 1e9
    # the committed PMC figures are per launch at the bench's 10 M; another size has none
    traffic = (pmc_traffic(f"{head_algo}_{head_dtype}_{head_layout}_norm")
               if n == 10_000_000 and head_norm else None)
    if default_head:
        workload = ("ACA general-quad 4-point homography, AoS f32, normalised (H[8]=1), "
                    "batch=10M per GPU (BASELINE configs[1]; configs[4] at 8 GPUs)")
        kernel = "hg::solve_aos<ACA,NORM,f32,P=2,nt|lds-dma> (hg_aos.hpp)"
    else:
        workload = (f"{head_algo.upper()} 4-point homography, {head_layout.upper()} {head_dtype}, "
                    + ("normalised (H[8]=1)" if head_norm else "unnormalised (cal_Homo_* contract)")
                    + f", batch={n / 1e6:g}M per GPU"
                    + (" (BASELINE configs[2])" if (head_algo, head_layout, head_dtype, n) ==
                       ("sks", "aos", "f32", 10_000_000) else ""))
        kernel = (f"hg::solve_aos<{head_algo.upper()},NORM,{head_dtype},P={2 if head_dtype == 'f32' else 1},"
                  "nt|lds-dma> (hg_aos.hpp)" if head_layout == "aos" else
                  f"hg::solve_soa_narrow / solve_soa_vec <{head_algo.upper()},{head_dtype}> "
                  "(hg_soa.hpp; the dispatcher picks by size and alignment)")
    line = {
        "metric": "M homographies/sec (ACA & SKS) at batch=10M; achieved HBM GB/s vs roofline",
        "value": round(value, 2),
        "unit": "M homographies/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": head_dtype,
        "data": f"synthetic (on-device counter-based U[0,1024) coordinates, seed {SEED})",
        "config": {
            "workload": workload,
            "algo": head_algo, "batch_per_gpu": n, "global_batch": n_total, "layout": head_layout,
            "parallelism": f"dp{d.world} (contiguous shards, no data-path collective)",
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_source(),
            "kernel": kernel,
            "algorithmic_bytes_per_launch": n * bpp_head,
            "launch_ms": round(ms_launch, 5),
        },
        "launch_stats": per_launch,
    }
    m = numa.get("bdf_matches_device")
    rows = d.gather_rows([numa["node"] if numa["node"] is not None else -1,
                          numa["bound_cpus"] or 0, -1 if m is None else int(m)])
    line["numa"] = {
        "per_rank": [{"rank": r, "node": int(a), "bound_cpus": int(b),
                      "bdf_matches_device": None if c < 0 else bool(c)}
                     for r, (a, b, c) in enumerate(rows)],
        "rank0_gpu_bdf": numa["bdf"],
        "note": numa.get("note", "each rank bound to its GPU's NUMA node before GPU init"),
    }
    if card is not None:
        line["card_at_start_rank0"] = card  # wait_quiet_card: a handed-over card's memory

    # Everything after the headline is reported beside it.  A global watchdog and a
    # per-section guard keep any failure there from costing the measured line: an
    # exception is recorded and the job moves on to printing; a stall (say, a rank left
    # waiting in a collective after a peer failed) ends every rank after the deadline,
    # rank 0 printing the line first.
    printed = threading.Lock()

    def emit():
        if d.rank == 0 and printed.acquire(blocking=False):
            for _ in range(50):  # the watchdog may race a section still filling `line`
                try:
                    text = json.dumps(line)
                    break
                except RuntimeError:
                    time.sleep(0.01)
            else:
                text = json.dumps({k: line[k] for k in list(line)})
            print(text, flush=True)

    all_done = threading.Event()

    def extras_watchdog(limit=args.extras_deadline):
        if all_done.wait(limit):
            return
        line["extras_error"] = f"extras did not finish within {limit} s"
        emit()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(EXIT_STALLED)  # the line is out; the exit code still says the run stalled

    threading.Thread(target=extras_watchdog, daemon=True).start()
    if not args.no_extras:
        try:
            if d.rank == args.inject_extras_failure:
                raise RuntimeError("injected failure (--inject-extras-failure)")
            line["reference_statistic"] = reference_statistic(d, run_head)
            # the ratios below are against ACA f32 AoS, the default headline
            ms_aca = ms_launch if default_head else timed_region(d, run("aca"), args.steps)[1]
            for _ in range(args.warmup):
                run("sks")()
            wall_s, ms_s = timed_region(d, run("sks"), args.steps)
            line["sks"] = {
                "value": round(n_total * args.steps / wall_s / 1e6, 2), "unit": "M homographies/s",
                "ms_per_step": round(wall_s / args.steps * 1e3, 5),
                "achieved_gbps": round(n * bpp / (ms_s * 1e-3) / 1e9, 1),
                "frac": round(n * bpp / (ms_s * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "sks_over_aca_time": round(ms_s / ms_aca, 3),
                "traffic": pmc_detail("sks_f32_aos_norm") if n == 10_000_000 else None,
            }
            # the reference's RHO-GE comparison baseline on the same inputs
            for _ in range(args.warmup):
                run("ge")()
            wall_g, ms_g = timed_region(d, run("ge"), args.steps)
            line["ge_baseline"] = {
                "value": round(n_total * args.steps / wall_g / 1e6, 2), "unit": "M homographies/s",
                "ms_per_step": round(wall_g / args.steps * 1e3, 5),
                "achieved_gbps": round(n * bpp / (ms_g * 1e-3) / 1e9, 1),
                "aca_speedup_over_ge": round(ms_g / ms_aca, 3),
                "note": "all three closed forms are HBM-bound on MI355X: FLOP savings no longer "
                        "show at 10M; the CPU baseline shows them",
            }
            # streaming-copy yardstick over the same byte count
            nb = (n * bpp) // 2 // 16 * 16
            a = torch.empty(nb // 4, dtype=torch.float32, device=d.dev)
            b = torch.empty_like(a)
            a.fill_(1.0)
            for _ in range(5):
                pkg.stream_copy(a, b)
            _, ms_c = timed_region(d, lambda: pkg.stream_copy(a, b), 50)
            line["copy_yardstick_gbps"] = round(2 * nb / (ms_c * 1e-3) / 1e9, 1)
            line["roofline"]["frac_of_copy"] = round(achieved / line["copy_yardstick_gbps"], 4)
            del a, b
            # TensorACA rect, B = 64 K x 128 x 128 (reference generator, torch seed 0)
            torch.manual_seed(0)
            _, _, src_h, tar_h, scale, div = pkg.adjust(d.dev, args.rect_batch)
            Hr = torch.empty((args.rect_batch, 3, 3), device=d.dev)
            f_ours = lambda: pkg.ops.tensor_aca_rect(src_h, tar_h, scale, div, out=Hr)  # noqa: E731
            f_torch = lambda: torch_tensor_aca_rect(src_h, tar_h, scale, div)  # noqa: E731
            for _ in range(100):
                f_ours()
                f_torch()
            _, ms_o = timed_region(d, f_ours, 1000)
            _, ms_t = timed_region(d, f_torch, 1000)
            g_ours = graph_of(d, f_ours, 100)
            g_torch = graph_of(d, f_torch, 100)
            _, ms_go = timed_region(d, g_ours.replay, 20)
            _, ms_gt = timed_region(d, g_torch.replay, 20)
            del g_ours, g_torch
            big = 16 * 1024 * 1024
            torch.manual_seed(0)
            _, _, bs_h, bt_h, bsc, bdv = pkg.adjust(d.dev, big)
            Hb = torch.empty((big, 3, 3), device=d.dev)
            for _ in range(5):
                pkg.ops.tensor_aca_rect(bs_h, bt_h, bsc, bdv, out=Hb)
            _, ms_b = timed_region(d, lambda: pkg.ops.tensor_aca_rect(bs_h, bt_h, bsc, bdv, out=Hb), 50)
            # per-problem (B,1,1) scale / div (the reference composition's broadcast, .py:301-302)
            psc = torch.full((big, 1, 1), 128.0, device=d.dev) + torch.rand(big, 1, 1, device=d.dev)
            pdv = torch.ones((big, 1, 1), device=d.dev)
            f_pp = lambda: pkg.ops.tensor_aca_rect(bs_h, bt_h, psc, pdv, out=Hb)  # noqa: E731
            for _ in range(5):
                f_pp()
            _, ms_pp = timed_region(d, f_pp, 50)
            del psc, pdv
            gHb = torch.randn(big, 3, 3, device=d.dev)
            f_bt = lambda: pkg.tensor_aca_rect_backward(bs_h, bt_h, gHb, bsc, bdv, False, False)  # noqa
            f_ba = lambda: pkg.tensor_aca_rect_backward(bs_h, bt_h, gHb, bsc, bdv, True, True)  # noqa
            for _ in range(5):
                f_bt()
                f_ba()
            _, ms_bt = timed_region(d, f_bt, 20)
            _, ms_ba = timed_region(d, f_ba, 20)
            # the all-gradient op's kernels apart (raw C ABI, no allocation): the fused backward
            # kernel alone (rect_backward_sum_l0: gradients + the sum's level 0), and the round-5
            # two-launch form (the terms kernel, then hg_sum_aten_f32 over its 24 B of terms)
            gs_k, gt_k = torch.empty_like(bs_h), torch.empty_like(bt_h)
            terms_k = torch.empty((2, big, 3), device=d.dev)
            sd_k = torch.empty(2, device=d.dev)
            stream_k = torch.cuda.current_stream(d.dev).cuda_stream
            T_bw = torch.get_num_threads()
            import ctypes
            lib_k = pkg.lib()
            lib_k.hg_internal_rect_backward_sum_l0.argtypes = (
                [ctypes.c_void_p] * 3 + [ctypes.c_int64] + [ctypes.c_void_p] * 5
                + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p])
            f_bk = lambda: lib_k.hg_internal_rect_backward_sum_l0(  # noqa: E731
                bs_h.data_ptr(), bt_h.data_ptr(), gHb.data_ptr(), big, bsc.data_ptr(),
                bdv.data_ptr(), gs_k.data_ptr(), gt_k.data_ptr(), terms_k.data_ptr(), 8, T_bw,
                stream_k)

            def f_b2():
                pkg._lib.call("hg_tensor_aca_rect_backward_terms_f32", bs_h.data_ptr(),
                              bt_h.data_ptr(), gHb.data_ptr(), big, bsc.data_ptr(), bdv.data_ptr(),
                              gs_k.data_ptr(), gt_k.data_ptr(), terms_k.data_ptr(), stream_k)
                pkg._lib.call("hg_sum_aten_f32", terms_k.data_ptr(), 2, 3 * big, 3 * big, 1, 8,
                              T_bw, sd_k.data_ptr(), stream_k)
            for _ in range(5):
                f_bk()
                f_b2()
            _, ms_bk = timed_region(d, f_bk, 20)
            _, ms_b2 = timed_region(d, f_b2, 20)
            del gs_k, gt_k, terms_k, sd_k
            # a plain copy of the same 228 B per problem (half read, half written): what the
            # box's HBM gives this read/write mix with two streams instead of the layout's seven
            cpy_src = torch.empty(big * RECT_BWD_SUM_LAYOUT_MIN_BYTES // 8, dtype=torch.float32,
                                  device=d.dev)
            cpy_dst = torch.empty_like(cpy_src)
            f_cp = lambda: pkg._lib.call(  # noqa: E731
                "hg_stream_copy", cpy_src.data_ptr(), cpy_dst.data_ptr(),
                big * RECT_BWD_SUM_LAYOUT_MIN_BYTES // 2, stream_k)
            for _ in range(5):
                f_cp()
            _, ms_cp = timed_region(d, f_cp, 20)
            del cpy_src, cpy_dst
            # the opt-in torch-ROCm evaluation order (order="rocm"): the same kernels' forms with
            # the GPU's 3-term sums -- forward, dL/dtar alone, everything
            f_rf = lambda: pkg.ops.tensor_aca_rect(bs_h, bt_h, bsc, bdv, out=Hb, order="rocm")  # noqa
            f_rbt = lambda: pkg.tensor_aca_rect_backward(bs_h, bt_h, gHb, bsc, bdv, False, False,  # noqa
                                                         order="rocm")
            f_rba = lambda: pkg.tensor_aca_rect_backward(bs_h, bt_h, gHb, bsc, bdv, True, True,  # noqa
                                                         order="rocm")
            for _ in range(5):
                f_rf()
                f_rbt()
                f_rba()
            _, ms_rf = timed_region(d, f_rf, 50)
            _, ms_rbt = timed_region(d, f_rbt, 20)
            _, ms_rba = timed_region(d, f_rba, 20)
            del gHb
            rect_backward_large = {
                "large_backward_tar_us": round(ms_bt * 1e3, 2),
                "large_backward_tar_frac": round(big * 140 / (ms_bt * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "large_backward_tar_traffic": pmc_detail("rect_backward_tar"),
                # everything (dL/dsrc, dL/dtar, the (1,) scale / div in ATen-CPU's order): one
                # fused backward kernel (the sum's level 0 in LDS) + the sum's small upper levels
                "large_backward_all_us": round(ms_ba * 1e3, 2),
                "large_backward_all_frac": round(big * RECT_BWD_SUM_BYTES / (ms_ba * 1e-3) / 1e9
                                                 / HBM_PEAK_GBPS, 4),
                "large_backward_all_traffic": pmc_detail(
                    "rect_backward_sum", "the fused backward kernel alone (rect_backward_sum_l0)"),
                "large_backward_all_kernel_us": round(ms_bk * 1e3, 2),
                "large_backward_all_op_over_kernel": round(ms_ba / ms_bk, 4),
                "large_backward_all_two_launch_us": round(ms_b2 * 1e3, 2),
                "large_backward_all_aten_threads": T_bw,
                # against the (B,3,4) layout's own floors (RECT_BWD_*_LAYOUT_MIN_BYTES)
                "large_backward_tar_layout_min_bytes_per_problem": RECT_BWD_TAR_LAYOUT_MIN_BYTES,
                "large_backward_tar_layout_min_frac": round(
                    big * RECT_BWD_TAR_LAYOUT_MIN_BYTES / (ms_bt * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "large_backward_all_layout_min_bytes_per_problem": RECT_BWD_SUM_LAYOUT_MIN_BYTES,
                "large_backward_all_layout_min_frac": round(
                    big * RECT_BWD_SUM_LAYOUT_MIN_BYTES / (ms_ba * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "large_backward_all_kernel_layout_min_frac": round(
                    big * RECT_BWD_SUM_LAYOUT_MIN_BYTES / (ms_bk * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "large_backward_all_copy_yardstick_us": round(ms_cp * 1e3, 2),
                # > 1: the kernel moves its layout's bytes faster than a plain copy of them
                "large_backward_all_kernel_vs_copy": round(ms_cp / ms_bk, 4),
                "rocm_order": {
                    "large_us_per_call": round(ms_rf * 1e3, 2),
                    "large_frac": round(big * RECT_LAYOUT_MIN_BYTES / (ms_rf * 1e-3) / 1e9
                                        / HBM_PEAK_GBPS, 4),
                    "large_backward_tar_us": round(ms_rbt * 1e3, 2),
                    "large_backward_tar_frac": round(big * 140 / (ms_rbt * 1e-3) / 1e9
                                                     / HBM_PEAK_GBPS, 4),
                    "large_backward_all_us": round(ms_rba * 1e3, 2),
                    "large_backward_all_frac": round(big * 212 / (ms_rba * 1e-3) / 1e9
                                                     / HBM_PEAK_GBPS, 4),
                    "note": "order='rocm' (the reference's device='cuda' bits); frac of the "
                            "(B,3,4) layout floor forward, of 140 / 212 B backward",
                },
            }
            # compact form (corner + 4 offsets) on the same big batch
            corner = bs_h[:, 0:2, 0].contiguous()
            offs = (bt_h[:, 0:2, :] - bs_h[:, 0:2, :]).transpose(1, 2).contiguous()
            Ho = torch.empty((big, 3, 3), device=d.dev)
            f_off = lambda: pkg.ops.tensor_aca_offsets(corner, offs, 128.0, 128.0, out=Ho)  # noqa
            for _ in range(5):
                f_off()
            _, ms_ob = timed_region(d, f_off, 50)
            c64, o64 = corner[:args.rect_batch].contiguous(), offs[:args.rect_batch].contiguous()
            Hs = torch.empty((args.rect_batch, 3, 3), device=d.dev)
            f_os = lambda: pkg.ops.tensor_aca_offsets(c64, o64, 128.0, 128.0, out=Hs)  # noqa
            for _ in range(100):
                f_os()
            _, ms_os = timed_region(d, f_os, 1000)
            # the torch-composed deep-homography path from the same corner + offsets: build
            # the (B,3,4) target as getTar/adjust do (.py:19-37), then TensorACA_rect's ATen ops
            s64 = src_h  # the batch's static (B,3,4) rectangle, as above

            def f_ot():
                t = s64.clone()
                t[:, 0:2, :] += o64.transpose(1, 2)
                return torch_tensor_aca_rect(s64, t, scale, div)

            for _ in range(100):
                f_ot()
            _, ms_ot = timed_region(d, f_ot, 1000)
            g_os = graph_of(d, f_os, 100)
            g_ot = graph_of(d, f_ot, 100)
            _, ms_gos = timed_region(d, g_os.replay, 20)
            _, ms_got = timed_region(d, g_ot.replay, 20)
            del g_os, g_ot
            del corner, offs, Ho
            rb = pkg.RECT_BYTES_PER_PROBLEM
            line["tensor_aca_offsets"] = {
                "batch": args.rect_batch, "us_per_call": round(ms_os * 1e3, 3),
                "torch_composed_us_per_call": round(ms_ot * 1e3, 3),
                "speedup_vs_torch": round(ms_ot / ms_os, 2),
                "graph_us_per_call": round(ms_gos * 1e3 / 100, 3),
                "torch_composed_graph_us_per_call": round(ms_got * 1e3 / 100, 3),
                "graph_speedup_vs_torch": round(ms_got / ms_gos, 2),
                "large_batch": big, "large_us_per_call": round(ms_ob * 1e3, 2),
                "large_achieved_gbps": round(big * 76 / (ms_ob * 1e-3) / 1e9, 1),
                "large_frac": round(big * 76 / (ms_ob * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "large_traffic": pmc_detail("tensor_aca_offsets"),
                "bytes_per_problem": 76,
            }
            line["tensor_aca_rect"] = {
                "batch": args.rect_batch, "us_per_call": round(ms_o * 1e3, 3),
                "torch_composed_us_per_call": round(ms_t * 1e3, 3),
                "speedup_vs_torch": round(ms_t / ms_o, 2),
                "graph_us_per_call": round(ms_go * 1e3 / 100, 3),
                "torch_composed_graph_us_per_call": round(ms_gt * 1e3 / 100, 3),
                "graph_speedup_vs_torch": round(ms_gt / ms_go, 2),
                "large_batch": big, "large_us_per_call": round(ms_b * 1e3, 2),
                "large_achieved_gbps": round(big * rb / (ms_b * 1e-3) / 1e9, 1),
                "large_frac": round(big * rb / (ms_b * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "large_traffic": pmc_detail("tensor_aca_rect"),
                # the (B,3,4) contract's floor: the 2 src floats used sit 16 B apart in every
                # 48-B record, so every 32-B sector of src is fetched (PMC: 1.0x of this count)
                "layout_min_bytes_per_problem": RECT_LAYOUT_MIN_BYTES,
                "large_layout_min_frac": round(
                    big * RECT_LAYOUT_MIN_BYTES / (ms_b * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                # (B,1,1) scale and div: 8 B more per problem
                "large_per_problem_scale_div_us_per_call": round(ms_pp * 1e3, 2),
                "large_per_problem_layout_min_frac": round(
                    big * (RECT_LAYOUT_MIN_BYTES + 8) / (ms_pp * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "large_per_problem_traffic": pmc_detail("tensor_aca_rect_bcast"),
                # the backward at 16 M: dL/dtar alone (140 B per problem) and everything
                # (dL/dsrc, dL/dtar, the (1,) scale / div through hg_sum_aten_f32: 212 B)
                **rect_backward_large,
            }
            del bs_h, bt_h, Hb
            line["aca_vanilla_autograd"] = vanilla_autograd_section(d, pkg, args.rect_batch)
            line["reference_layout"] = reference_layout(d, pkg)
            line["table8_sweep"] = table8_sweep(d, pkg)
            line["table8_pipeline"] = table8_pipeline_section(d, pkg)
            line["grouped_small"] = grouped_section(d, pkg)
            line["ransac"] = ransac_section(d, pkg)
            line["host_boundary"] = host_boundary_section(d, pkg, n)
            # f64 AoS (sks::runKernel_ACA_double semantics) on the same inputs
            s64, t64 = src.double(), tar.double()
            H64 = torch.empty((n, 9), dtype=torch.float64, device=d.dev)
            f64 = lambda: pkg.solve("aca", s64, t64, normalize=True, out=H64)  # noqa: E731
            for _ in range(5):
                f64()
            _, ms64 = timed_region(d, f64, 50)
            line["aca_f64_aos"] = {"us_per_launch": round(ms64 * 1e3, 2),
                                   "G_homographies_per_s": round(n / (ms64 * 1e-3) / 1e9, 2),
                                   "achieved_gbps": round(n * 200 / (ms64 * 1e-3) / 1e9, 1),
                                   "frac": round(n * 200 / (ms64 * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                                   "traffic": pmc_detail("aca_f64_aos_norm") if n == 10_000_000
                                   else {"traffic_bytes": None, "reason": "PMC measured at 10 M"}}
            del s64, t64, H64
            if not args.no_host_shard:
                run("aca")()  # H = this rank's device result again (the f64 step used other buffers)
                torch.cuda.synchronize(d.dev)
                line["host_sharded"] = host_sharded_section(d, pkg, src, tar, H, n, n_total)
        except Exception as e:  # noqa: BLE001 -- recorded, the headline still prints
            line["extras_error"] = f"{type(e).__name__}: {e}"

    if d.world > 1 and not args.no_gather and "extras_error" not in line:
        run("aca")()
        # The split / gather is reported beside the measurement, never part of it: should its
        # point-to-point traffic stall, every rank's watchdog ends the job after the deadline
        # and rank 0 still prints the measured line (with the stall recorded).
        done = threading.Event()

        def watchdog(limit=args.gather_deadline):
            if done.wait(limit):
                return
            line["split_gather"] = {"error": f"no completion within {limit} s"}
            emit()
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(EXIT_STALLED)

        threading.Thread(target=watchdog, daemon=True).start()
        try:
            line["split_gather"] = split_gather_section(d, pkg, src, tar, H, n, n_total,
                                                        wall / args.steps * 1e3)
        except Exception as e:  # noqa: BLE001
            line["split_gather"] = {"error": f"{type(e).__name__}: {e}"}
        done.set()

    if d.rank == 0 and d.world == 1 and not args.no_cpu:
        try:
            line["cpu_baseline"] = cpu_baseline(min(n, 10_000_000))
            line["cpu_baseline"]["config0_n1000"] = config0_check(pkg, d.dev)
            # the speed-up is quoted against the multi-threaded host baseline
            line["cpu_baseline"]["gpu_speedup"] = round(
                line["value"] / line["cpu_baseline"]["value"], 1)
            line["cpu_baseline"]["gpu_speedup_vs_all_core_linear_bound"] = round(
                line["value"] / line["cpu_baseline"]["all_physical_cores_linear_bound"], 1)
            nat = line["cpu_baseline"].get("native_march")
            if nat:
                nat["gpu_speedup"] = round(line["value"] / nat["aca_value"], 1)
        except Exception as e:  # noqa: BLE001
            line["cpu_baseline"] = {"error": f"{type(e).__name__}: {e}"}
    line["baseline_configs"] = baseline_configs(line, args, d.world)  # last: the driver's tail
    all_done.set()
    emit()
    d.close()


if __name__ == "__main__":
    main()
