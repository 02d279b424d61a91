"""Kernel-variant sweep for the AoS solver (tools/kbench.py).

Interleaved rounds in ONE process (cdna_hip_programming.md rule 24): every variant
of hg_tune_aos_f32 is timed with HIP events on the launch stream, round-robin, and
the median / min per-launch time is reported with the achieved algorithmic GB/s.
Each variant's output is compared bit for bit with the shipped kernel's.
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def main():
    n = int(os.environ.get("KB_N", 10_000_000))
    rounds = int(os.environ.get("KB_ROUNDS", 7))
    iters = int(os.environ.get("KB_ITERS", 30))
    pkg = ge.load_package()
    lib = pkg._lib.tune()
    lib.hg_tune_num_variants.restype = ctypes.c_int
    lib.hg_tune_variant_name.restype = ctypes.c_char_p
    lib.hg_tune_variant_name.argtypes = [ctypes.c_int]
    lib.hg_tune_aos_f32.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    lib.hg_tune_aos_f32.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    src = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(n, 8)
    tar = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(n, 8)
    H = torch.empty(n, 9, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    nv = lib.hg_tune_num_variants()
    cases = []
    only = os.environ.get("KB_VARIANTS")
    keep = set(int(x) for x in only.split(",")) if only else set(range(nv))
    for v in range(nv):
        if v not in keep:
            continue
        name = lib.hg_tune_variant_name(v).decode()
        per = [8] if "persist" not in name else [2, 4, 8, 16]
        for pc in per:
            for algo in (0, 1):
                cases.append((v, name + (f" x{pc}/CU" if "persist" in name else ""), pc, algo))

    ref = {a: pkg.solve("aca" if a == 0 else "sks", src, tar).clone() for a in (0, 1)}
    times = {c: [] for c in cases}
    bad = {}
    for c in cases:
        v, _, pc, algo = c
        H.zero_()
        rc = lib.hg_tune_aos_f32(algo, v, src.data_ptr(), tar.data_ptr(), H.data_ptr(), n, pc, sp)
        assert rc == 0, rc
        torch.cuda.synchronize()
        same = torch.equal(H.view(torch.int32), ref[algo].view(torch.int32))
        if not same:
            bad[c] = True
    # copy yardstick (same byte count)
    nb = n * 100 // 2 // 16 * 16
    a = torch.ones(nb // 4, device=dev)
    b = torch.empty_like(a)
    copy_t = []
    for r in range(rounds):
        for c in cases:
            v, _, pc, algo = c
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(iters):
                lib.hg_tune_aos_f32(algo, v, src.data_ptr(), tar.data_ptr(), H.data_ptr(), n, pc, sp)
            e1.record(stream)
            e1.synchronize()
            times[c].append(e0.elapsed_time(e1) / iters)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(iters):
            pkg.stream_copy(a, b)
        e1.record(stream)
        e1.synchronize()
        copy_t.append(e0.elapsed_time(e1) / iters)
    # copy-yardstick variants (hg_tune_copy), same byte count, interleaved
    lib.hg_tune_copy.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                 ctypes.c_void_p]
    lib.hg_tune_copy.restype = ctypes.c_int
    nbc = nb // 32768 * 32768
    ctimes = {v: [] for v in range(4)}
    for v in range(4):
        assert lib.hg_tune_copy(v, a.data_ptr(), b.data_ptr(), nbc, sp) == 0
    torch.cuda.synchronize()
    for r in range(rounds):
        for v in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(iters):
                lib.hg_tune_copy(v, a.data_ptr(), b.data_ptr(), nbc, sp)
            e1.record(stream)
            e1.synchronize()
            ctimes[v].append(e0.elapsed_time(e1) / iters)
    copy_variants = {}
    for v, name in enumerate(["U4 nt", "U8 nt", "U4 plain", "LDS-DMA 8K/wave"]):
        med = statistics.median(ctimes[v])
        copy_variants[name] = round(2 * nbc / (med * 1e-3) / 1e9, 1)
        print(f"copy variant {name}: {copy_variants[name]} GB/s")
    out = []
    cmed = statistics.median(copy_t)
    print(f"copy yardstick: {2 * nb / (cmed * 1e-3) / 1e9:.1f} GB/s ({cmed * 1e3:.1f} us)")
    for c in cases:
        v, name, pc, algo = c
        med = statistics.median(times[c])
        mn = min(times[c])
        gbps = n * 100 / (med * 1e-3) / 1e9
        rec = {"variant": v, "name": name, "algo": "aca" if algo == 0 else "sks",
               "median_us": round(med * 1e3, 2), "min_us": round(mn * 1e3, 2),
               "gbps": round(gbps, 1), "bit_exact": c not in bad}
        out.append(rec)
        print(json.dumps(rec))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench.json"), "w") as f:
        json.dump({"n": n, "copy_gbps": 2 * nb / (cmed * 1e-3) / 1e9,
                   "copy_variants_gbps": copy_variants, "cases": out}, f, indent=1)


if __name__ == "__main__":
    main()
