"""Probe: the order in which ROCm's ATen sums a (B,1,3) tensor over its last dimension (the
`torch.sum(Q4, dim=2, keepdim=True)` of TensorACA_rect, .py:299) -- against every association of
three binary32 terms, with and without a +0 start, and ATen-CPU's -- and whether torch.cross on
the GPU equals the CPU's FMA-contracted cross.  Prints one JSON line.
    python tools/rocm_sum_probe.py"""
import json

import numpy as np
import torch


def main():
    rng = np.random.default_rng(5)
    B = 1 << 20
    x = (rng.standard_normal((B, 1, 3)) * 10.0 ** rng.integers(-3, 4, (B, 1, 3))).astype(np.float32)
    g = torch.sum(torch.from_numpy(x).cuda(), dim=2, keepdim=True).cpu().numpy().reshape(B)
    c = torch.sum(torch.from_numpy(x), dim=2, keepdim=True).numpy().reshape(B)
    a, b, d = (x[:, 0, k] for k in range(3))
    cand = {"(a+b)+c": (a + b) + d, "a+(b+c)": a + (b + d), "(a+c)+b": (a + d) + b,
            "aten_cpu": c}
    out = {k: float(np.mean(v.view(np.uint32) == g.view(np.uint32))) for k, v in cand.items()}
    u = torch.from_numpy((rng.standard_normal((B, 1, 3))).astype(np.float32))
    v = torch.from_numpy((rng.standard_normal((B, 1, 3))).astype(np.float32))
    out["cross_gpu_eq_cpu"] = float((torch.cross(u.cuda(), v.cuda(), dim=2).cpu() == torch.cross(u, v, dim=2)).float().mean())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
