"""Seeded sampler timing probe: the bench route (pkg.sample_solve_seeded, fresh output
per call) against a preallocated output through the same C ABI, interleaved with the
indexed sampler, at 16M hypotheses over the committed wall pool."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def ev_time(fn, reps=10):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"]).to(dev)
    pt = torch.from_numpy(g["pool_tar"]).to(dev)
    n = 1 << 24
    out = torch.empty((n, 9), device=dev)
    lib = pkg._lib.lib()
    fn = lib.hg_sample_solve_seeded_f32
    st = torch.cuda.current_stream(dev).cuda_stream

    def direct():
        assert fn(ctypes.c_void_p(ps.data_ptr()), ctypes.c_void_p(pt.data_ptr()),
                  ctypes.c_uint32(ps.shape[0]), ctypes.c_uint64(11), ctypes.c_uint64(0),
                  ctypes.c_void_p(out.data_ptr()), ctypes.c_int64(n), 0, 1,
                  ctypes.c_void_p(st)) == 0

    idx = pkg.fill_bits(n * 4, 11, 0, dev).view(n, 4)
    routes = {"bench_route": lambda: pkg.sample_solve_seeded(ps, pt, n, 11, 0),
              "direct_prealloc": direct,
              "indexed": lambda: pkg.sample_solve(ps, pt, idx)}
    for f in routes.values():
        for _ in range(3):
            f()
    res = {k: [] for k in routes}
    for _ in range(5):
        for k, f in routes.items():
            res[k].append(round(ev_time(f), 2))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
