"""Does a large AoS batch run faster as several back-to-back launches over consecutive slices?
(tools/gpu_round.sh chunk_probe).  At 20 M problems (2 GB) the headline kernel ran at 6.33 TB/s
against 6.54 at 10 M on another box; this measures, interleaved in one process on one box,
one launch over N against k launches over N/k contiguous slices (same bits: problems are
independent), for N = 10 M and 20 M f32 and 10 M f64.  Median per batch of 7 rounds x 10 reps."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    out = {}
    for dtype, n in ((torch.float32, 10_000_000), (torch.float32, 20_000_000), (torch.float64, 10_000_000)):
        src = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(n, 8).to(dtype)
        tar = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(n, 8).to(dtype)
        H = torch.empty((n, 9), dtype=dtype, device=dev)
        want = pkg.solve("aca", src, tar).clone()
        cases = {}
        for k in (1, 2, 4):
            step = -(-n // k)
            sl = [(a, min(a + step, n)) for a in range(0, n, step)]

            def run(sl=sl):
                for a, b in sl:
                    pkg.solve("aca", src[a:b], tar[a:b], out=H[a:b])
            cases[k] = run
        bits = {}
        for k, f in cases.items():
            H.zero_()
            f()
            torch.cuda.synchronize()
            bits[k] = bool(torch.equal(H.view(torch.int64 if dtype is torch.float64 else torch.int32),
                                       want.view(torch.int64 if dtype is torch.float64 else torch.int32)))
        times = {k: [] for k in cases}
        for _ in range(7):
            for k, f in cases.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / 10 * 1e3)
        bpp = 100 if dtype is torch.float32 else 200
        rec = {}
        for k in cases:
            us = statistics.median(times[k])
            rec[f"{k} launch(es)"] = {"us_per_batch": round(us, 2), "gbps": round(n * bpp / us / 1e3, 1),
                                      "bit_exact": bits[k]}
        key = f"{'f32' if dtype is torch.float32 else 'f64'} n={n}"
        out[key] = rec
        print(key, json.dumps(rec), flush=True)
        del src, tar, H, want
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "chunk_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
