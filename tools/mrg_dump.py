"""Dumps rocrand_generate(ROCRAND_RNG_PSEUDO_MRG32K3A) words on the GPU box (round 3).

The words come from rocRAND's host API through the library's rocRAND-backed path
(``hg_rand_mrg32k3a_u32`` before the hand-written generator replaced it, or
``hg_rand_mrg32k3a_rocrand_u32`` after), and are written to an npz under gpurun_out/.
They are the data that pins the MRG32K3A restatement (tests/restate_mrg32k3a.py) and
the hand-written kernel to rocRAND's host-API word order: fixtures, not source.

    python tools/mrg_dump.py gpurun_out/mrg_dump.npz
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

SEEDS = [11, 3, 0, 1, (1 << 32) + 7, (1 << 64) - 1, 0x0123456789ABCDEF]
COUNTS = [1, 37, 131071, 131072, 131073, 300001]


def main(out: str) -> None:
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    lib = pkg._lib
    fn = "hg_rand_mrg32k3a_rocrand_u32" if hasattr(lib.lib(), "hg_rand_mrg32k3a_rocrand_u32") \
        else "hg_rand_mrg32k3a_u32"

    def gen(count, seed):
        o = torch.empty(count, dtype=torch.int32, device=dev)
        lib.call(fn, o.data_ptr(), count, seed, torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize()
        return o.cpu().numpy().view(np.uint32)

    rec = {"fn": np.array(fn)}
    for seed in SEEDS:
        for c in COUNTS:
            rec[f"s{seed}_n{c}"] = gen(c, seed)
        print("seed", seed, "done", flush=True)
    big = (1 << 22) + 3
    rec[f"s11_n{big}"] = gen(big, 11)
    t0 = time.perf_counter()
    for _ in range(20):
        gen(1 << 22, 11)
    rec["rocrand_4M_ms_incl_copy"] = np.array((time.perf_counter() - t0) / 20 * 1e3)
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    np.savez(out, **rec)
    print("wrote", out, flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mrg_dump.npz")
