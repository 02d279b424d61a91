"""Where the one-launch draws + gather + solve spends its time (hg_rand_gather_solve_f64,
Table-8 formats, the reference's wall file): the shipped kernel against itself with the
solve, the engine starts' table jumps and the engine steps removed, alone and together
(hg_tune_rand_gather_solve_f64 variants 2 ... 8; wrong bits, timing only), beside a
write-only stream of the same 72 B per hypothesis.  Interleaved rounds, median us per launch.
    python tools/kbench_mrg_ablate.py   -> gpurun_out/kbench_mrg_ablate.json
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import __graft_entry__ as ge  # noqa: E402
from kbench_mrg import timeit  # noqa: E402

NAMES = {1: "shipped", 2: "no_solve", 3: "no_start", 4: "no_draws", 5: "no_solve_no_start",
         6: "no_solve_no_draws", 7: "no_start_no_draws", 8: "gather_and_stores_only",
         9: "stores_only", 10: "shipped_st16", 11: "stores_only_st16",
         12: "stores_only_2_blocks_per_cu", 13: "shipped_default_stores",
         14: "shipped_st16_default_stores"}


def main():
    pkg = ge.load_package()
    t = pkg._lib.tune()
    vp, i64, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64
    t.hg_tune_rand_gather_solve_f64.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp,
                                                ctypes.c_uint32, u64, vp, i64, vp]
    t.hg_tune_policy.argtypes = [ctypes.c_int, vp, vp, i64, vp]
    t.hg_tune_mrg_pattern.argtypes = [ctypes.c_int, vp, i64, vp]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev).cuda_stream
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"].astype(np.float64)).to(dev)
    pt = torch.from_numpy(g["pool_tar"].astype(np.float64)).to(dev)
    sizes = [int(x) for x in os.environ.get("KB_SIZES", "1000000,10000000").split(",")]
    out = {}
    # the standalone words kernel: shipped, without the table jumps, without the engine steps,
    # without both (hg_tune_mrg_words min_chunk 2^20 + 1 / 2 / 3), and a write-only stream of
    # the same bytes (hg_tune_copy variant 5)
    t.hg_tune_mrg_words.argtypes = [vp, i64, u64, i64, vp]
    t.hg_tune_copy.argtypes = [ctypes.c_int, vp, vp, i64, vp]
    for count in (4 * s_ for s_ in sizes):
        wb = torch.empty(count, dtype=torch.int32, device=dev)
        fns = {name: (lambda a=a: t.hg_tune_mrg_words(wb.data_ptr(), count, 11, a, st))
               for name, a in (("words_shipped", 64), ("words_no_start", (1 << 20) + 1),
                               ("words_no_steps", (1 << 20) + 2), ("words_neither", (1 << 20) + 3))}
        fns["write_only"] = lambda: t.hg_tune_copy(5, None, wb.data_ptr(), count * 4, st)
        for f in fns.values():
            assert f() == 0
        r = timeit(fns, 20)
        out[f"words {count}"] = r
        print("words", count, r, flush=True)
        del wb
    for algo, aid in (("aca", 0), ("sks", 1)):
        for n in sizes:
            H = torch.empty((9, n), dtype=torch.float64, device=dev)
            w = torch.empty(n * 18, dtype=torch.float32, device=dev)
            fns = {}
            for v, name in NAMES.items():
                fns[name] = (lambda v=v: t.hg_tune_rand_gather_solve_f64(
                    v, aid, ps.data_ptr(), pt.data_ptr(), ps.shape[0], 11, H.data_ptr(), n, st))
            fns["write_only_72B"] = lambda: t.hg_tune_policy(0, w.data_ptr(), w.data_ptr(), n * 72, st)
            for cls in (64, 128, 256, 512, 1024):  # the store pattern alone, C classes x 1024/C positions
                fns[f"pattern_{cls}x{1024 // cls}"] = (lambda cls=cls: t.hg_tune_mrg_pattern(
                    cls, H.data_ptr(), n, st))
            fns["pattern_9_rows_in_order"] = lambda: t.hg_tune_mrg_pattern(0, H.data_ptr(), n, st)
            for code, name in ((1, "one_row_8B_nt"), (2, "one_row_16B_nt"), (3, "one_row_8B"),
                               (4, "one_row_16B"), (5, "9_rows_in_order_16B_nt"),
                               (6, "9_rows_in_order_16B"), (7, "9_rows_in_order_8B")):
                fns[f"pattern_{name}"] = (lambda code=code: t.hg_tune_mrg_pattern(code, H.data_ptr(), n, st))
            for f in fns.values():
                assert f() == 0
            r = timeit(fns, 20 if n <= 1_000_000 else 5)
            fns["shipped"]()
            ref = H.clone()
            fns["shipped_st16"]()
            r["st16_bit_exact"] = bool(torch.equal(H.view(torch.int64), ref.view(torch.int64)))
            del ref
            out[f"{algo} n={n}"] = r
            print(algo, n, r, flush=True)
            del H, w
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kbench_mrg_ablate.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
