"""The reference's PyTorch interface for this path, served by the HIP kernels.

Mirrors "PyTorch Codes/Modules_Runtime_Test.py" (names, argument meaning, tensor
layouts).  Differences, all deliberate:
  * the reference functions time a loop and return the mean time; these return H
    (the value the reference computes and discards, .py:294-302 / :330-383);
  * no `loops`/warm-up arguments (timing lives in bench.py);
  * CPU tensors raise (the product path is GPU-only).
The input generators reproduce the reference's draws call for call, so the same
torch seed yields the same batch.
"""
from __future__ import annotations

import torch

from . import ops


def getInput(bS: int, device) -> torch.Tensor:
    """(bS,4,2) axis-aligned 128x128 squares M,N,P,Q with integer top-left corner in
    [10,30)^2 (Modules_Runtime_Test.py:9-16)."""
    corner = torch.randint(low=10, high=30, size=[bS, 2], device=device).float()
    offs = torch.tensor([[0.0, 0.0], [128.0, 0.0], [0.0, 128.0], [128.0, 128.0]], device=device)
    return corner[:, None, :] + offs[None, :, :]


def getTar(bs: int, src: torch.Tensor) -> torch.Tensor:
    """Target quad = source + integer perturbation in [0,32) (.py:19-21)."""
    jitter = torch.randint(low=0, high=32, size=[bs, 4, 2], device=src.device).float()
    return src + jitter


def adjust(device, bs: int):
    """Builds (src, tar, src_h, tar_h, scale, div) like .py:24-37: src/tar (bs,4,2),
    homogeneous (bs,3,4) copies, and the batch-uniform rectangle width `scale` and
    width/height ratio `div` read from sample 0 as (1,)-shaped tensors."""
    src = getInput(bs, device)
    tar = getTar(bs, src)
    ones = torch.ones((bs, 1, 4), device=src.device)
    src_h = torch.cat((src.transpose(1, 2), ones), dim=1)
    tar_h = torch.cat((tar.transpose(1, 2), ones), dim=1)
    scale = src_h[0, 0, 1:2] - src_h[0, 0, 0:1]
    div = scale / (src_h[0, 1, 2:3] - src_h[0, 1, 0:1])
    return src, tar, src_h, tar_h, scale, div


def TensorACA_rect(bs: int, src: torch.Tensor, tar: torch.Tensor, scale, div, *,
                   order: str = "cpu") -> torch.Tensor:
    """TensorACA for a source rectangle (.py:286-309): src/tar (bs,3,4) homogeneous,
    returns the unnormalised (bs,3,3) H.  Differentiable (w.r.t. tar, src, scale, div)
    when an input requires grad, as the reference's ATen composition is; the backward
    is one HIP kernel (hg_tensor_aca_rect_backward_terms_f32) and a device-side batch sum.
    ``order`` (keyword only, not in the reference's signature): "cpu" gives the bits of the
    statements run on ATen-CPU, "rocm" those of the reference's default device='cuda' run on
    a ROCm GPU (.py:393), forward and gradients (ops.tensor_aca_rect).

    Host dependence (order="cpu"): ATen-CPU sums a batch-uniform scale / div gradient of
    >= 32768 terms (B >= 10923) in chunks, one per ATen thread, so its bits depend on
    torch.get_num_threads() of the process running the reference.  This op follows the
    forward caller's torch.get_num_threads() the same way: a plain `python` run and a
    torchrun rank (OMP_NUM_THREADS=1) give different dL/dscale, dL/ddiv bits, each equal to
    what ATen-CPU gives in that process.  To pin them, call torch.set_num_threads(T) first,
    or use ops.tensor_aca_rect_backward(..., aten_threads=T).  H and dL/dtar, dL/dsrc never
    depend on it; order="rocm" does not either (the GPU's reduction shape is fixed)."""
    if src.shape[0] != bs or tar.shape[0] != bs:
        raise ValueError(f"batch size {bs} does not match tensors {tuple(src.shape)}")
    needs_grad = torch.is_grad_enabled() and any(
        isinstance(x, torch.Tensor) and x.requires_grad for x in (src, tar, scale, div))
    if needs_grad:  # differentiable like the reference's ATen composition
        return ops.tensor_aca_rect_autograd(src, tar, scale, div, order=order)
    return ops.tensor_aca_rect(src, tar, scale, div, order=order)


def ACA_vanilla(bs: int, src: torch.Tensor, tar: torch.Tensor, loops=None) -> torch.Tensor:
    """General-quad ACA (.py:312-388): src/tar (bs,4,2), returns unnormalised (bs,3,3) in
    torch's default dtype, as the reference's statements do (computed in src's dtype).
    Differentiable w.r.t. src and tar, as the reference's statements are under ATen
    autograd, with the same gradient bits (one HIP kernel, hg_aca_backward_*).
    ``loops`` (the reference's timing-loop count) is accepted so its call sites run
    unchanged, and ignored: timing is bench.py's job."""
    if src.shape[0] != bs or tar.shape[0] != bs:
        raise ValueError(f"batch size {bs} does not match tensors {tuple(src.shape)}")
    H = ops.aca_vanilla(src, tar)
    # the statements write their results into torch.ones((bs, 9)), i.e. torch's default dtype
    # (.py:372): binary64 inputs give a float32 H unless the default dtype is float64, each
    # value rounded once (and differentiably: the cast's backward widens the gradient)
    dt = torch.get_default_dtype()
    return H if H.dtype is dt else H.to(dt)
