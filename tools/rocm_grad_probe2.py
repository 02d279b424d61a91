"""Probe (GPU box): where torch-ROCm's autograd through TensorACA_rect's statements departs from
ATen-CPU's.  The statements run on the GPU and on the CPU (the CPU forward with the GPU's cross-term
order, ((0 + c0) + c2) + c1, so both forwards are the same bits); hooks capture the gradient of every
intermediate; the first intermediate whose gradient differs names the backward op that evaluates
differently.  Candidate orders for the 3-term reductions are then tried on the CPU gradients.
Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(src, tar, scale, div, gH):
    grads = {}

    def keep(name, t):
        t.register_hook(lambda g: grads.__setitem__(name, g.detach().cpu().clone()))
        return t

    bs = tar.shape[0]
    tar = tar.clone().requires_grad_()
    H = torch.zeros((bs, 3, 3), device=tar.device)
    d = keep("d", tar[:, :, 1:] - tar[:, :, 0:1])
    a, b = keep("a", d[:, 1:2, :]), keep("b", d[:, 0:1, :])
    q = keep("q", torch.cross(a, b, dim=2))
    z = torch.zeros_like(q[:, :, 0:1])
    s = keep("s", ((z + q[:, :, 0:1]) + q[:, :, 2:3]) + q[:, :, 1:2])
    ht = keep("ht", s * tar[:, :, 0:1])
    h0 = keep("h0", tar[:, :, 1:2] * q[:, :, 0:1] - ht)
    H[:, :, 0:1] = h0
    x = keep("x", tar[:, :, 2:3] * q[:, :, 1:2] - ht)
    H[:, :, 1:2] = torch.mul(div, x)
    H[:, :, 2:3] = scale * ht - src[:, 0:1, 0:1] * H[:, :, 0:1] - src[:, 1:2, 0:1] * H[:, :, 1:2]
    H.backward(gH)
    grads["tar"] = tar.grad.detach().cpu().clone()
    return grads


def same(a, b):
    a, b = a.numpy(), b.numpy()
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def main():
    rng = np.random.default_rng(11)
    B = 100_003
    s_np = rng.uniform(0, 160, (B, 3, 4)).astype(np.float32)
    t_np = rng.uniform(0, 160, (B, 3, 4)).astype(np.float32)
    t_np[:, 2, :] = 1.0
    g_np = rng.standard_normal((B, 3, 3)).astype(np.float32)
    sc, dv = torch.tensor([50.0]), torch.tensor([1.25])
    dev = torch.device("cuda:0")
    gpu = run(torch.from_numpy(s_np).to(dev), torch.from_numpy(t_np).to(dev), sc.to(dev), dv.to(dev),
              torch.from_numpy(g_np).to(dev))
    cpu = run(torch.from_numpy(s_np), torch.from_numpy(t_np), sc, dv, torch.from_numpy(g_np))
    out = {k: float(same(gpu[k], cpu[k]).mean()) for k in gpu}
    # candidate orders for the 3-term reductions on the GPU, restated on the CPU values
    ght = cpu["ht"].reshape(B, 3)
    tr0 = torch.from_numpy(t_np[:, :, 0])
    terms = ght * tr0  # (B,3): the (B,3,1) -> (B,1,1) sum gives dL/ds
    cand = {
        "cpu_((0+t0)+t1)+t2": ((torch.zeros(B) + terms[:, 0]) + terms[:, 1]) + terms[:, 2],
        "((0+t0)+t2)+t1": ((torch.zeros(B) + terms[:, 0]) + terms[:, 2]) + terms[:, 1],
        "((0+t2)+t1)+t0": ((torch.zeros(B) + terms[:, 2]) + terms[:, 1]) + terms[:, 0],
        "((0+t1)+t2)+t0": ((torch.zeros(B) + terms[:, 1]) + terms[:, 2]) + terms[:, 0],
        "(0+t0)+(t1+t2)": (torch.zeros(B) + terms[:, 0]) + (terms[:, 1] + terms[:, 2]),
    }
    gs_gpu = gpu["s"].reshape(B)
    out["gs_candidates"] = {k: float(same(v, gs_gpu).mean()) for k, v in cand.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
