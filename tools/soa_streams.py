"""How much does the NUMBER of concurrent row streams cost?  (tools/gpu_round.sh soa_streams)
row_streams<RI,RO,U> (hg_tune.hip) reads RI rows and writes RO rows with no arithmetic; the
total read is held at 640 MB (RI=16: the f32 10 M SoA batch) so only the stream count and the
row pitch change.  Median of 7 interleaved rounds of 20 launches, bytes = (RI+RO)*row."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

SHAPES = {0: (16, 9, 1), 1: (16, 8, 1), 2: (8, 4, 1), 3: (4, 2, 1), 4: (2, 1, 1), 5: (16, 9, 4),
          6: (32, 16, 1)}


def main():
    pkg = ge.load_package()
    f = pkg._lib.tune().hg_tune_streams
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                  ctypes.c_void_p]
    f.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    # SOA_READ_TOTAL=1280000000 SOA_SHAPES=0: the binary64 10 M batch's 25 rows (80 MB each)
    read_total = int(os.environ.get("SOA_READ_TOTAL", 640_000_000))
    slack = 32 * (1 << 20)
    inb = torch.empty(read_total + slack, dtype=torch.uint8, device=dev).fill_(7)
    outb = torch.empty(read_total * 9 // 16 + slack * 2, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    cases = []
    shapes = ({int(v): SHAPES[int(v)] for v in os.environ["SOA_SHAPES"].split(",")}
              if os.environ.get("SOA_SHAPES") else SHAPES)
    for v, (ri, ro, u) in shapes.items():
        row = read_total // ri
        cases.append((f"RI={ri} RO={ro} U={u} pitch=row", v, row, row))
    row = read_total // 16
    for extra in ((256, 4096, 65536, (1 << 21) - row % (1 << 21)) if shapes is SHAPES else ()):
        cases.append((f"RI=16 RO=9 U=1 pitch=row+{extra}", 0, row, row + extra))
    for name, v, row, pitch in cases:
        ri, ro, _ = SHAPES[v]
        assert (ri - 1) * pitch + row <= inb.numel() and (ro - 1) * pitch + row <= outb.numel()
        assert f(v, inb.data_ptr(), outb.data_ptr(), row, pitch, st) == 0
    torch.cuda.synchronize()
    runs = {name: (lambda v=v, row=row, pitch=pitch: f(v, inb.data_ptr(), outb.data_ptr(), row, pitch, st))
            for name, v, row, pitch in cases}
    solver = {}
    if os.environ.get("SOA_SOLVE"):  # the shipped SoA solvers on the matching batch, interleaved
        dt = torch.float64 if read_total // 16 >= 8 * 10_000_000 else torch.float32
        nprob = read_total // 16 // (8 if dt is torch.float64 else 4)
        ss = pkg.fill_uniform(nprob * 8, 11, 0, device=dev).view(8, nprob).to(dt)
        tt = pkg.fill_uniform(nprob * 8, 11, nprob * 8, device=dev).view(8, nprob).to(dt)
        hh = torch.empty((9, nprob), dtype=dt, device=dev)
        for algo in ("aca", "sks"):
            name = f"shipped {algo} SoA {'f64' if dt is torch.float64 else 'f32'} n={nprob}"
            runs[name] = lambda algo=algo: pkg.solve(algo, ss, tt, normalize=False, layout="soa", out=hh)
            solver[name] = nprob * (200 if dt is torch.float64 else 100)
    times = {name: [] for name in runs}
    for _ in range(7):
        for name, fn in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 20 * 1e3)
    out = {}
    for name, v, row, pitch in cases:
        ri, ro, _ = SHAPES[v]
        us = statistics.median(times[name])
        out[name] = {"us": round(us, 2), "gbps": round((ri + ro) * row / us / 1e3, 1)}
        print(name, out[name], flush=True)
    for name, nbytes in solver.items():
        us = statistics.median(times[name])
        out[name] = {"us": round(us, 2), "gbps": round(nbytes / us / 1e3, 1)}
        print(name, out[name], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "soa_streams.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
