"""The standalone MRG32K3A words kernel (hg_rand_mrg32k3a_u32) against variants of its split
and store policy (hg_tune_mrg_words: min_chunk c = positions per thread; 2^21 + c the same with
non-temporal stores), beside a write-only stream of the same bytes; every variant compared bit
for bit with the shipped kernel.  Interleaved rounds, median us per launch.
    python tools/kbench_mrg_words.py   -> gpurun_out/kbench_mrg_words.json"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import __graft_entry__ as ge  # noqa: E402
from kbench_mrg import timeit  # noqa: E402


def main():
    pkg = ge.load_package()
    lib = pkg.lib()
    t = pkg._lib.tune()
    vp, i64, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64
    t.hg_tune_mrg_words.argtypes = [vp, i64, u64, i64, vp]
    t.hg_tune_policy.argtypes = [ctypes.c_int, vp, vp, i64, vp]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev).cuda_stream
    out = {}
    variants = {"shipped": None, "c16": 16, "c32": 32, "c128": 128, "nt": (1 << 20) + 4,
                "nt_c16": (1 << 21) + 16, "nt_c8": (1 << 21) + 8}
    for count in (4_000_000, 40_000_000):
        bufs = {k: torch.empty(count, dtype=torch.int32, device=dev) for k in variants}
        wsrc = torch.empty(count, dtype=torch.int32, device=dev)
        wdst = torch.empty_like(wsrc)
        fns = {}
        for k, c in variants.items():
            if c is None:
                fns[k] = lambda b=bufs[k]: lib.hg_rand_mrg32k3a_u32(b.data_ptr(), count, 11, st)
            else:
                fns[k] = lambda b=bufs[k], c=c: t.hg_tune_mrg_words(b.data_ptr(), count, 11, c, st)
        fns["write_only"] = lambda: t.hg_tune_policy(0, wsrc.data_ptr(), wdst.data_ptr(), count * 4, st)
        r = timeit(fns, 5 if count > 10_000_000 else 20)
        rec = {k: {"us": us, "bit_exact": bool(torch.equal(bufs[k], bufs["shipped"])) if k in bufs else None}
               for k, us in r.items()}
        out[f"words {count}"] = rec
        print("words", count, rec, flush=True)
        del bufs, wsrc, wdst
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench_mrg_words.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
