"""Reduces tools/mrg_dump.py's rocrand_generate words (dumped on the MI355X box) to the
committed fixture tests/golden/mrg32k3a_rocrand.npz: for every seed the whole 37-word call,
and index/value samples of the 300001-word call (the first and last 512 words, both sides
of the 2^17 and 2^18 subsequence wraps, and every 97th word); for seed 11 also samples of
a (2^22 + 3)-word call.  Data only: rocRAND's words, no source.

    python tools/make_mrg_fixture.py gpurun_out/mrg_dump.npz
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden", "mrg32k3a_rocrand.npz")


def sample_idx(n: int, step: int) -> np.ndarray:
    idx = [np.arange(min(n, 512)), np.arange(max(0, n - 512), n), np.arange(0, n, step)]
    for w in (1 << 17, 1 << 18):
        if n > w:
            idx.append(np.arange(w - 64, min(n, w + 64)))
    return np.unique(np.concatenate(idx)).astype(np.int64)


def main(src: str) -> None:
    d = np.load(src)
    rec = {"source": np.array(f"rocrand_generate via {d['fn']} on MI355X (tools/mrg_dump.py)")}
    seeds = sorted({int(k[1:k.index("_n")]) for k in d.files if k.startswith("s")})
    rec["seeds"] = np.array(seeds, dtype=np.uint64)
    for seed in seeds:
        rec[f"s{seed}_n37"] = d[f"s{seed}_n37"]
        w = d[f"s{seed}_n300001"]
        idx = sample_idx(w.size, 97)
        rec[f"s{seed}_n300001_idx"] = idx
        rec[f"s{seed}_n300001_val"] = w[idx]
        # the shorter calls' words are the longer call's prefix (counts change nothing)
        for c in (1, 131071, 131072, 131073):
            assert np.array_equal(d[f"s{seed}_n{c}"], w[:c]), (seed, c)
    big = [k for k in d.files if k.startswith("s11_n") and int(k.split("_n")[1]) > 300001][0]
    w = d[big]
    idx = sample_idx(w.size, 4099)
    rec["s11_big_n"] = np.array(w.size)
    rec["s11_big_idx"] = idx
    rec["s11_big_val"] = w[idx]
    np.savez_compressed(OUT, **rec)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "mrg_dump.npz"))
