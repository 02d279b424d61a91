"""Probe (GPU box): the reference's TensorACA_rect statements as torch-ROCm evaluates them on the
GPU -- the reference's own default run (Modules_Runtime_Test.py:393, device='cuda') -- against
candidate restatements, forward and backward.

Forward: the GPU composition equals the CPU statements with the three cross terms summed as
(c0 + c2) + c1 (profiles/r03/rocm_sum_probe.json); this checks that on special values too
(all-(-0) cross terms: does the GPU sum start from +0?).  Backward: ATen autograd on the GPU
against our op (the CPU order) element by element -- which of dL/dtar's 12 components differ,
and how often -- and the batch-uniform dL/dscale, dL/ddiv.  Prints one JSON object.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402


def statements(src, tar, scale, div, order):
    """TensorACA_rect's statements (.py:296-302) with the cross-term sum in `order`."""
    bs = tar.shape[0]
    H = torch.zeros((bs, 3, 3), device=tar.device)
    d = tar[:, :, 1:] - tar[:, :, 0:1]
    q = torch.cross(d[:, 1:2, :], d[:, 0:1, :], dim=2)
    if order == "aten":
        s = torch.sum(q, dim=2, keepdim=True)
    elif order == "c0c2c1":
        s = (q[:, :, 0:1] + q[:, :, 2:3]) + q[:, :, 1:2]
    elif order == "0c0c2c1":
        s = ((torch.zeros_like(q[:, :, 0:1]) + q[:, :, 0:1]) + q[:, :, 2:3]) + q[:, :, 1:2]
    else:
        raise ValueError(order)
    ht = s * tar[:, :, 0:1]
    H[:, :, 0:1] = tar[:, :, 1:2] * q[:, :, 0:1] - ht
    H[:, :, 1:2] = torch.mul(div, tar[:, :, 2:3] * q[:, :, 1:2] - ht)
    H[:, :, 2:3] = scale * ht - src[:, 0:1, 0:1] * H[:, :, 0:1] - src[:, 1:2, 0:1] * H[:, :, 1:2]
    return H


def same(a, b):
    a, b = a.detach().cpu().numpy(), b.detach().cpu().numpy()
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def main():
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(7)
    B = 200_003
    out = {}
    vals = np.array([0.0, -0.0, 1.0, -1.0, 2.0, 0.5, 3.0, 1024.0, np.inf, -np.inf, 1e-45,
                     -1.2e-40, 3e38, -3e38], np.float32)
    cases = {
        "fractional": (rng.uniform(0, 160, (B, 3, 4)).astype(np.float32),
                       rng.uniform(0, 160, (B, 3, 4)).astype(np.float32)),
        "special": (rng.choice(vals, (B, 3, 4)).astype(np.float32),
                    rng.choice(vals, (B, 3, 4)).astype(np.float32)),
    }
    for name, (s_np, t_np) in cases.items():
        t_np[:, 2, :] = 1.0
        s = torch.from_numpy(s_np).to(dev)
        t = torch.from_numpy(t_np).to(dev)
        sc = torch.tensor([50.0], device=dev)
        dv = torch.tensor([1.25], device=dev)
        gpu = bench.torch_tensor_aca_rect(s, t, sc, dv)
        rec = {"ours_cpu_order_equal": float(same(pkg.tensor_aca_rect(s, t, sc, dv), gpu).mean())}
        for order in ("aten", "c0c2c1", "0c0c2c1"):
            cpu = statements(s.cpu(), t.cpu(), sc.cpu(), dv.cpu(), order)
            rec[f"cpu_{order}_equal"] = float(same(cpu, gpu).mean())
        # backward: GPU autograd through the statements vs the op
        gH = torch.from_numpy(rng.standard_normal((B, 3, 3)).astype(np.float32)).to(dev)
        tg = t.clone().requires_grad_()
        sg, dg = sc.clone().requires_grad_(), dv.clone().requires_grad_()
        bench.torch_tensor_aca_rect(s, tg, sg, dg).backward(gH)
        _, g_tar, g_sc, g_dv = pkg.tensor_aca_rect_backward(s, t, gH, sc, dv, False, True)
        ok = same(g_tar, tg.grad)
        rec["gtar_equal"] = float(ok.mean())
        rec["gtar_equal_per_component"] = [round(float(x), 6) for x in ok.reshape(B, 12).mean(0)]
        rec["gscale_gpu_vs_ours"] = [float(sg.grad.item()), float(g_sc.item())]
        rec["gdiv_gpu_vs_ours"] = [float(dg.grad.item()), float(g_dv.item())]
        # the CPU statements with the GPU's forward order, under CPU autograd
        tc = t.cpu().clone().requires_grad_()
        statements(s.cpu(), tc, sc.cpu(), dv.cpu(), "c0c2c1").backward(gH.cpu())
        rec["gtar_cpu_c0c2c1_equal_gpu"] = float(same(tc.grad, tg.grad).mean())
        out[name] = rec
    print(json.dumps(out))


if __name__ == "__main__":
    main()
