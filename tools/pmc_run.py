"""Workload for the rocprofv3 PMC passes (tools/gpu_round.sh pmc): each kernel whose
HBM traffic bench.py or DESIGN.md quotes, launched a few times at its measured size,
nothing else -- a short, fixed dispatch list (the full bench under --pmc is tens of
thousands of serialized dispatches).  tools/pmc_traffic.py reduces the counters."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

REPS = 5


def main():
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    n = 10_000_000
    src = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(n, 8)
    tar = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(n, 8)
    H = torch.empty((n, 9), device=dev)
    for algo in ("aca", "sks"):
        for _ in range(REPS):
            pkg.solve(algo, src, tar, normalize=True, out=H)
    nb = (n * 100) // 2 // 16 * 16
    a = torch.ones(nb // 4, device=dev)
    b = torch.empty_like(a)
    for _ in range(REPS):
        pkg.stream_copy(a, b)
    del a, b
    s64, t64 = src.view(8, n).double(), tar.view(8, n).double()
    H64 = torch.empty((9, n), dtype=torch.float64, device=dev)
    for algo in ("aca", "sks"):
        for _ in range(REPS):
            pkg.solve(algo, s64, t64, normalize=False, layout="soa", out=H64)
    del s64, t64, H64
    # binary64 AoS, normalised (sks::runKernel_ACA_double semantics; bench aca_f64_aos)
    sd, td = src.double(), tar.double()
    Hd = torch.empty((n, 9), dtype=torch.float64, device=dev)
    for _ in range(REPS):
        pkg.solve("aca", sd, td, normalize=True, out=Hd)
    del sd, td, Hd, src, tar, H
    big = 16 * 1024 * 1024
    # ACA_vanilla's backward alone at 16 M (bench aca_vanilla_autograd.backward_large)
    vs = torch.rand(big, 8, device=dev) * 1024
    vt = torch.rand(big, 8, device=dev) * 1024
    vg = torch.randn(big, 9, device=dev)
    for _ in range(REPS):
        pkg.aca_backward(vs, vt, vg)
    del vs, vt, vg
    torch.manual_seed(0)
    _, _, bs, bt, sc, dv = pkg.adjust(dev, big)
    Hb = torch.empty((big, 3, 3), device=dev)
    for _ in range(REPS):
        pkg.ops.tensor_aca_rect(bs, bt, sc, dv, out=Hb)
    # per-problem (B,1,1) scale / div: the staged broadcast kernel
    psc = torch.full((big, 1, 1), 128.0, device=dev) + torch.rand(big, 1, 1, device=dev)
    pdv = torch.ones((big, 1, 1), device=dev)
    for _ in range(REPS):
        pkg.ops.tensor_aca_rect(bs, bt, psc, pdv, out=Hb)
    del psc, pdv
    # the rect backward: dL/dtar alone (deep-homography training), then everything (src,
    # tar, and the batch-uniform scale / div through hg_sum_aten_f32)
    gHb = torch.randn(big, 3, 3, device=dev)
    for _ in range(REPS):
        pkg.tensor_aca_rect_backward(bs, bt, gHb, sc, dv, False, False)
    for _ in range(REPS):
        pkg.tensor_aca_rect_backward(bs, bt, gHb, sc, dv, True, True, aten_threads=16)
    corner = bs[:, 0:2, 0].contiguous()
    offs = (bt[:, 0:2, :] - bs[:, 0:2, :]).transpose(1, 2).contiguous()
    del bs, bt
    for _ in range(REPS):
        pkg.ops.tensor_aca_offsets(corner, offs, 128.0, 128.0, out=Hb)
    for _ in range(REPS):
        pkg.tensor_aca_offsets_backward(corner, offs, gHb, 128.0, 128.0, False)
    del corner, offs, Hb, gHb
    g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
    ps = torch.from_numpy(g["pool_src"]).to(dev)
    pt = torch.from_numpy(g["pool_tar"]).to(dev)
    idx = pkg.fill_bits(big * 4, 11, 0, dev).view(big, 4)
    for _ in range(REPS):
        pkg.sample_solve(ps, pt, idx)
    del idx
    for _ in range(REPS):
        pkg.sample_solve_seeded(ps, pt, big, 11, 0)
    # the fused binary64 gather + cal_Homo_ACA in the reference's formats (hg_gather.hpp),
    # 10 M hypotheses on the wall file: 16 B of words in, 72 B of H out per hypothesis
    rl = pkg.rand_mrg32k3a(4 * n, 11, dev).view(4, n)
    ps64, pt64 = ps.double(), pt.double()
    for _ in range(REPS):
        pkg.gather_solve(ps64, pt64, rl, "aca")
    # round 3: the hand-written MRG32K3A draws (40 M words = 4 x 10 M) and the draws fused
    # into the gather + solve (no words in memory: 72 B of H per hypothesis)
    for _ in range(REPS):
        pkg.rand_mrg32k3a(4 * n, 11, dev)
    del rl
    for algo in ("aca", "sks"):
        for _ in range(REPS):
            pkg.rand_gather_solve(ps64, pt64, n, 11, algo)
    torch.cuda.synchronize()
    print("pmc workload done")


if __name__ == "__main__":
    main()
