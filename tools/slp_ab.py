"""A/B of the product library built with and without the SLP vectoriser, in one process on
one box (tools/gpu_round.sh slp_ab): lib/libsks_homography_amd.so (shipped flags) against
tools/_build/slp/libsks_homography_amd.so (the same sources with SLP; built by
tools/sample_flags_probe.sh slp).  Interleaved rounds, median us per launch, and the output
bits of both compared."""
import ctypes
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def load(path):
    lib = ctypes.CDLL(path)
    pkg = ge.load_package()
    for name, (argtypes, restype) in pkg._lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes, fn.restype = argtypes, restype
    return lib


def main():
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    libs = {"noslp": load(os.path.join(ROOT, "sks-homography_amd", "lib", "libsks_homography_amd.so")),
            "slp": load(os.path.join(ROOT, "tools", "_build", "slp", "libsks_homography_amd.so"))}
    st = torch.cuda.current_stream().cuda_stream
    n = 10_000_000
    s = pkg.fill_uniform(n * 8, 11, 0, device=dev)
    t = pkg.fill_uniform(n * 8, 11, n * 8, device=dev)
    H = torch.empty(n * 9, device=dev)
    s64, t64 = s.double(), t.double()
    H64 = torch.empty(n * 9, dtype=torch.float64, device=dev)
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"]).to(dev).contiguous()
    pt = torch.from_numpy(g["pool_tar"]).to(dev).contiguous()
    npool = ps.shape[0]
    m = 1 << 24
    Hs = torch.empty(m * 9, device=dev)
    idx = pkg.fill_bits(m * 4, 11, 0, dev)
    hyp = 1 << 20
    Hh = torch.empty(hyp * 9, device=dev)
    cnt = torch.empty(hyp, dtype=torch.int32, device=dev)
    torch.manual_seed(0)
    _, _, rs, rt, _, _ = pkg.adjust(dev, m)
    Hr = torch.empty(m * 9, device=dev)
    cases = {
        "aca_f32_aos_10M": (lambda L: L.hg_aca_f32(s.data_ptr(), t.data_ptr(), H.data_ptr(), n, 0, 1, st), H),
        "sks_f32_aos_10M": (lambda L: L.hg_sks_f32(s.data_ptr(), t.data_ptr(), H.data_ptr(), n, 0, 1, st), H),
        "sks_f64_soa_10M": (lambda L: L.hg_sks_f64(s64.data_ptr(), t64.data_ptr(), H64.data_ptr(), n, 1, 0, st), H64),
        "seeded_16M": (lambda L: L.hg_sample_solve_seeded_f32(ps.data_ptr(), pt.data_ptr(), npool, 11, 0,
                                                              Hs.data_ptr(), m, 0, 1, st), Hs),
        "indexed_16M": (lambda L: L.hg_sample_solve_f32(ps.data_ptr(), pt.data_ptr(), npool, idx.data_ptr(),
                                                        Hs.data_ptr(), m, 0, 1, st), Hs),
        "score_1Mx2540": (lambda L: L.hg_ransac_score_f32(Hh.data_ptr(), hyp, ps.data_ptr(), pt.data_ptr(),
                                                          npool, 3.0, cnt.data_ptr(), st), cnt),
        "rect_16M": (lambda L: L.hg_tensor_aca_rect_f32_hostscalar(rs.data_ptr(), rt.data_ptr(), Hr.data_ptr(),
                                                                  m, 128.0, 1.0, st), Hr),
    }
    libs["noslp"].hg_sample_solve_f32(ps.data_ptr(), pt.data_ptr(), npool, idx.data_ptr(), Hh.data_ptr(),
                                      hyp, 0, 1, st)
    res = {}
    for name, (fn, out) in cases.items():
        times = {k: [] for k in libs}
        outs = {}
        for k, L in libs.items():
            for _ in range(5):
                assert fn(L) == 0
        for _ in range(5):
            for k, L in libs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(20):
                    fn(L)
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / 20 * 1e3)
                outs[k] = out.clone()
        same = bool(torch.equal(outs["noslp"].view(torch.int32) if outs["noslp"].dtype != torch.float64
                                else outs["noslp"].view(torch.int64),
                                outs["slp"].view(torch.int32) if outs["slp"].dtype != torch.float64
                                else outs["slp"].view(torch.int64)))
        res[name] = {k: round(statistics.median(v), 2) for k, v in times.items()}
        res[name]["same_bits"] = same
        print(name, res[name], flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/slp_ab.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
