"""Deep-homography usage of the compact TensorACA op with autograd: recover the 4-corner
offsets that map a 128x128 patch onto known target quads by gradient descent on the
normalised H -- the loss a deep homography net puts behind its offset head
(PyTorch Codes/Modules_Runtime_Test.py:9-37 builds the same rectangle / offset inputs).

    python examples/fit_offsets.py          # on cuda:0; prints the final corner error

Returns the max corner error in pixels from fit(); tests/test_gpu_offsets.py runs it.
"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sks = importlib.import_module("sks-homography_amd")


def fit(batch: int = 4096, steps: int = 300, device: str = "cuda:0", seed: int = 0) -> float:
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)
    w = h = 128.0
    corner = (torch.rand(batch, 2, device=dev, generator=g) * 20 + 10).floor()
    true_off = torch.rand(batch, 4, 2, device=dev, generator=g) * 32 - 16
    # a 3x3 grid of patch points (homogeneous); the loss is their mean reprojection error
    u = torch.tensor([0.0, 0.5, 1.0], device=dev)
    gx, gy = torch.meshgrid(u * w, u * h, indexing="xy")
    pts = torch.stack([gx.reshape(-1), gy.reshape(-1), torch.ones(9, device=dev)])  # (3,9)
    pts = pts.unsqueeze(0) + torch.cat([corner, torch.zeros(batch, 1, device=dev)], 1)[:, :, None]
    pts[:, 2, :] = 1.0

    def project(H):
        q = H @ pts                                            # (B,3,9)
        return q[:, 0:2, :] / q[:, 2:3, :]

    with torch.no_grad():
        target = project(sks.tensor_aca_offsets(corner, true_off, w, h))
    off = torch.zeros(batch, 4, 2, device=dev, requires_grad=True)
    opt = torch.optim.Adam([off], lr=0.5)
    for _ in range(steps):
        opt.zero_grad()
        H = sks.tensor_aca_offsets(corner, off, w, h)          # differentiable, one HIP kernel
        loss = ((project(H) - target) ** 2).sum(1).mean()
        loss.backward()                                        # one HIP kernel for dL/doffsets
        opt.step()
    return float((off.detach() - true_off).abs().max())


if __name__ == "__main__":
    err = fit()
    print(f"max corner error after fitting: {err:.4f} px")
