"""SoA (reference GPU layout) kernel-variant sweep, interleaved in one process.
Each variant's output is compared bit for bit with the shipped path (pkg.solve)."""
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
    rounds, iters = 5, 20
    pkg = ge.load_package()
    lib = pkg._lib.tune()
    lib.hg_tune_num_soa_variants.restype = ctypes.c_int
    lib.hg_tune_soa_variant_name.restype = ctypes.c_char_p
    lib.hg_tune_soa_variant_name.argtypes = [ctypes.c_int]
    lib.hg_tune_soa.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    lib.hg_tune_soa.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    base = pkg.fill_uniform(n * 8 * 2, 11, 0, device=dev)
    data = {"f32": (base[:n * 8].view(8, n), base[n * 8:].view(8, n))}
    data["f64"] = tuple(x.double() for x in data["f32"])
    out = {k: torch.empty(9, n, dtype=v[0].dtype, device=dev) for k, v in data.items()}
    sp = torch.cuda.current_stream(dev).cuda_stream
    cases = []
    for v in range(lib.hg_tune_num_soa_variants()):
        name = lib.hg_tune_soa_variant_name(v).decode()
        dt = name.split()[0]
        for pc in ([8] if "persist" not in name else [4, 8, 16]):
            for algo in (0, 1):
                cases.append((v, f"{name} x{pc}" if "persist" in name else name, dt, pc, algo))
    ok = {}
    for c in cases:
        v, name, dt, pc, algo = c
        s, t = data[dt]
        want = pkg.solve("aca" if algo == 0 else "sks", s, t, normalize=False, layout="soa")
        out[dt].zero_()
        assert lib.hg_tune_soa(algo, v, s.data_ptr(), t.data_ptr(), out[dt].data_ptr(), n, pc,
                               sp) == 0
        torch.cuda.synchronize()
        ok[c] = torch.equal(out[dt].view(torch.uint8), want.view(torch.uint8))
    times = {c: [] for c in cases}
    for _ in range(rounds):
        for c in cases:
            v, name, dt, pc, algo = c
            s, t = data[dt]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                lib.hg_tune_soa(algo, v, s.data_ptr(), t.data_ptr(), out[dt].data_ptr(), n, pc, sp)
            e1.record()
            e1.synchronize()
            times[c].append(e0.elapsed_time(e1) / iters)
    res = []
    for c in cases:
        v, name, dt, pc, algo = c
        med = statistics.median(times[c])
        bpp = 100 if dt == "f32" else 200
        rec = {"name": name, "algo": "aca" if algo == 0 else "sks", "median_us": round(med * 1e3, 2),
               "gbps": round(n * bpp / (med * 1e-3) / 1e9, 1), "bit_exact": ok[c]}
        res.append(rec)
        print(json.dumps(rec))
    with open(os.path.join(ROOT, "gpurun_out", "kbench_soa.json"), "w") as f:
        json.dump({"n": n, "cases": res}, f, indent=1)


if __name__ == "__main__":
    main()
