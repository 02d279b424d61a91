"""Workload for a counter pass over the seeded RANSAC sampler (tools/gpu_round.sh
pmc_sample): 16 M hypotheses over the 2540-pair wall pool, 3 launches."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
dev = torch.device("cuda:0")
g = np.load(os.path.join(ROOT, "tests", "golden", "cpp_wall.npz"))
ps = torch.from_numpy(g["pool_src"]).to(dev)
pt = torch.from_numpy(g["pool_tar"]).to(dev)
n = 1 << 24
for _ in range(3):
    pkg.sample_solve_seeded(ps, pt, n, 11, 0)
torch.cuda.synchronize()
print("pmc_sample done")
