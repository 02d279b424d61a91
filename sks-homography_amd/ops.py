"""Torch-facing entry points over the C ABI (device memory, torch's current stream).

PyTorch is plumbing here: tensors own the HBM buffers and name the stream; every
computation is one of the library's HIP kernels.  CPU tensors are rejected -- the
product has no CPU path.

Also registers the ops with torch.library as ``torch.ops.sks_amd.{aca, sks,
tensor_aca_rect}`` (the op contract of SURVEY.md section 8(b)).
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import torch

from . import _lib
from ._lib import HG_FLAG_NORMALIZE, HG_LAYOUT_AOS, HG_LAYOUT_SOA

_DTYPES = {torch.float32: "f32", torch.float64: "f64"}


def _require_device(*tensors: torch.Tensor) -> torch.device:
    dev = tensors[0].device
    for t in tensors:
        if t.device.type != "cuda":
            raise ValueError("sks_homography_amd kernels run on the GPU only; got a "
                             f"{t.device} tensor (no CPU fallback by design)")
        if t.device != dev:
            raise ValueError(f"tensors on different devices: {dev} vs {t.device}")
    return dev


def _stream(dev: torch.device) -> int:
    """Raw hipStream_t of torch's current stream on `dev` (0 = the default stream)."""
    return torch._C._cuda_getCurrentRawStream(dev.index if dev.index is not None
                                              else torch.cuda.current_device())


class _NoGuard:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NO_GUARD = _NoGuard()


def _guard(dev: torch.device):
    """Device guard only when `dev` is not already current: a launch on the default
    stream goes to the current device, and the guard costs microseconds per call."""
    if dev.index is None or dev.index == torch.cuda.current_device():
        return _NO_GUARD
    return torch.cuda.device(dev)


def _scalar_ptr(x, dev: torch.device):
    """Device pointer of a batch-uniform scalar kept on the device (no copy when it
    already is a float32 CUDA tensor there), plus the tensor that owns it."""
    if (isinstance(x, torch.Tensor) and x.dtype == torch.float32 and x.device == dev
            and x.numel() >= 1):
        return x.data_ptr(), x
    t = torch.as_tensor(x, dtype=torch.float32, device=dev).reshape(-1)[:1].contiguous()
    return t.data_ptr(), t


def _as_problems(x: torch.Tensor, layout: str) -> torch.Tensor:
    """AoS accepts (n,8) or (n,4,2) (the ACA_vanilla layout, .py:312); SoA (8,n)."""
    if layout == "aos":
        if x.dim() == 3 and x.shape[1:] == (4, 2):
            x = x.reshape(x.shape[0], 8)
        if x.dim() != 2 or x.shape[1] != 8:
            raise ValueError(f"AoS problems must be (n,8) or (n,4,2), got {tuple(x.shape)}")
    elif layout == "soa":
        if x.dim() != 2 or x.shape[0] != 8:
            raise ValueError(f"SoA problems must be (8,n), got {tuple(x.shape)}")
    else:
        raise ValueError(f"layout must be 'aos' or 'soa', got {layout!r}")
    return x.contiguous()


def solve(algo: str, src: torch.Tensor, tar: torch.Tensor, normalize: bool = True,
          layout: str = "aos", out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Batched 4-point homography, ``algo`` in {"aca", "sks", "ge", "gpt"}.  "ge" and
    "gpt" are the reference's comparison baselines: RHO Gaussian elimination (f32,
    cv::runKernel_GE) and 8x8 pivoted LU (f64, cal_Homo_GPT).

    AoS: src/tar (n,8) or (n,4,2) -> H (n,9); SoA: (8,n) -> (9,n).
    ``normalize=True`` returns H/H[8] exactly as sks::runKernel_* (ACA_SKS.cpp:94-98);
    False returns H up to scale as cal_Homo_* / ACA_vanilla do.
    """
    if algo not in ("aca", "sks", "ge", "gpt"):
        raise ValueError(f"algo must be 'aca', 'sks', 'ge' or 'gpt', got {algo!r}")
    dev = _require_device(src, tar)
    if algo == "ge" and src.dtype != torch.float32:
        raise TypeError("the GE baseline (cv::runKernel_GE) is float32 only")
    if algo == "gpt" and src.dtype != torch.float64:
        raise TypeError("the GPT-LU baseline (cal_Homo_GPT) is float64 only")
    if src.dtype not in _DTYPES or tar.dtype != src.dtype:
        raise TypeError(f"src/tar must both be float32 or float64, got {src.dtype}/{tar.dtype}")
    src = _as_problems(src, layout)
    tar = _as_problems(tar, layout)
    if src.shape != tar.shape:
        raise ValueError(f"src {tuple(src.shape)} and tar {tuple(tar.shape)} differ")
    n = src.shape[0] if layout == "aos" else src.shape[1]
    shape = (n, 9) if layout == "aos" else (9, n)
    if out is None:
        out = torch.empty(shape, dtype=src.dtype, device=dev)
    elif out.shape != shape or out.dtype != src.dtype or not out.is_contiguous() or out.device != dev:
        raise ValueError(f"out must be a contiguous {shape} {src.dtype} tensor on {dev}")
    fn = f"hg_{algo}_{_DTYPES[src.dtype]}"
    with _guard(dev):
        _lib.call(fn, src.data_ptr(), tar.data_ptr(), out.data_ptr(), n,
                  HG_LAYOUT_AOS if layout == "aos" else HG_LAYOUT_SOA,
                  HG_FLAG_NORMALIZE if normalize else 0, _stream(dev))
    return out


def aca(src, tar, normalize: bool = True, layout: str = "aos", out=None) -> torch.Tensor:
    return solve("aca", src, tar, normalize, layout, out)


def sks(src, tar, normalize: bool = True, layout: str = "aos", out=None) -> torch.Tensor:
    return solve("sks", src, tar, normalize, layout, out)


Scalar = Union[float, int, torch.Tensor]


def tensor_aca_rect(src: torch.Tensor, tar: torch.Tensor, scale: Scalar, div: Scalar,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """TensorACA rectangle->quad (Modules_Runtime_Test.py:286-309), unnormalised.

    src, tar: (B,3,4) float32 homogeneous (rows x, y, 1; columns M, N, P, Q).
    scale, div: batch-uniform width and width/height -- Python numbers or one-element
    float32 tensors (kept on device, as the reference keeps them).  Returns (B,3,3).
    """
    dev = _require_device(src, tar)
    for name, t in (("src", src), ("tar", tar)):
        if t.dtype != torch.float32 or t.dim() != 3 or t.shape[1:] != (3, 4):
            raise ValueError(f"{name} must be a (B,3,4) float32 tensor, got "
                             f"{tuple(t.shape)} {t.dtype}")
    if src.shape[0] != tar.shape[0]:
        raise ValueError("src and tar batch sizes differ")
    src = src.contiguous()
    tar = tar.contiguous()
    B = tar.shape[0]
    if out is None:
        out = torch.empty((B, 3, 3), dtype=torch.float32, device=dev)
    stream = _stream(dev)
    with _guard(dev):
        if isinstance(scale, torch.Tensor) or isinstance(div, torch.Tensor):
            sp, _sc = _scalar_ptr(scale, dev)
            dp, _dv = _scalar_ptr(div, dev)
            _lib.call("hg_tensor_aca_rect_f32", src.data_ptr(), tar.data_ptr(), out.data_ptr(),
                      B, sp, dp, stream)
        else:
            _lib.call("hg_tensor_aca_rect_f32_hostscalar", src.data_ptr(), tar.data_ptr(),
                      out.data_ptr(), B, float(scale), float(div), stream)
    return out


def tensor_aca_rect_backward(src: torch.Tensor, tar: torch.Tensor, grad: torch.Tensor,
                             scale: torch.Tensor, div: torch.Tensor, need_src: bool = True,
                             need_scale_div: bool = True):
    """Gradients of tensor_aca_rect: (dL/dsrc (B,3,4) or empty, dL/dtar (B,3,4),
    [dL/dscale, dL/ddiv] (2,) or empty).  The per-problem scale/div partials from the
    kernel are summed here (deterministically, in float32)."""
    dev = _require_device(src, tar, grad)
    src, tar, grad = src.contiguous(), tar.contiguous(), grad.contiguous()
    B = tar.shape[0]
    sc = torch.as_tensor(scale, dtype=torch.float32, device=dev).reshape(-1)[:1].contiguous()
    dv = torch.as_tensor(div, dtype=torch.float32, device=dev).reshape(-1)[:1].contiguous()
    g_tar = torch.empty((B, 3, 4), dtype=torch.float32, device=dev)
    g_src = torch.empty((B, 3, 4) if need_src else (0,), dtype=torch.float32, device=dev)
    part = torch.empty((B, 2) if need_scale_div else (0,), dtype=torch.float32, device=dev)
    with _guard(dev):
        _lib.call("hg_tensor_aca_rect_backward_f32", src.data_ptr(), tar.data_ptr(),
                  grad.data_ptr(), B, sc.data_ptr(), dv.data_ptr(),
                  g_src.data_ptr() if need_src and B else None, g_tar.data_ptr(),
                  part.data_ptr() if need_scale_div and B else None, _stream(dev))
    g_sd = part.sum(0) if need_scale_div else part
    return g_src, g_tar, g_sd


def _check_offsets(corner: torch.Tensor, offsets: torch.Tensor) -> torch.device:
    dev = _require_device(corner, offsets)
    if offsets.dtype != torch.float32 or tuple(offsets.shape[1:]) not in ((4, 2), (8,)):
        raise ValueError(f"offsets must be (B,4,2) or (B,8) float32, got {tuple(offsets.shape)}")
    if corner.dtype != torch.float32 or tuple(corner.shape) != (offsets.shape[0], 2):
        raise ValueError(f"corner must be (B,2) float32, got {tuple(corner.shape)}")
    return dev


def tensor_aca_offsets(corner: torch.Tensor, offsets: torch.Tensor, width: float, height: float,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Compact TensorACA: source = the width x height rectangle at
    ``corner`` (B,2), target = source + ``offsets`` (B,4,2) in M,N,P,Q order.  Same bits
    as building the (B,3,4) tensors and calling tensor_aca_rect(scale=width,
    div=width/height).  Returns the unnormalised (B,3,3) H."""
    dev = _check_offsets(corner, offsets)
    corner, offsets = corner.contiguous(), offsets.contiguous()
    B = offsets.shape[0]
    if out is None:
        out = torch.empty((B, 3, 3), dtype=torch.float32, device=dev)
    with _guard(dev):
        _lib.call("hg_tensor_aca_offsets_f32", corner.data_ptr(), offsets.data_ptr(),
                  out.data_ptr(), B, float(width), float(height), _stream(dev))
    return out


def tensor_aca_offsets_backward(corner, offsets, grad, width: float, height: float,
                                need_corner: bool = True):
    dev = _check_offsets(corner, offsets)
    corner, offsets, grad = corner.contiguous(), offsets.contiguous(), grad.contiguous()
    B = offsets.shape[0]
    g_off = torch.empty(offsets.shape, dtype=torch.float32, device=dev)
    g_cor = torch.empty((B, 2) if need_corner else (0,), dtype=torch.float32, device=dev)
    with _guard(dev):
        _lib.call("hg_tensor_aca_offsets_backward_f32", corner.data_ptr(), offsets.data_ptr(),
                  grad.data_ptr(), B, float(width), float(height), g_off.data_ptr(),
                  g_cor.data_ptr() if need_corner and B else None, _stream(dev))
    return g_off, g_cor


def tensor_aca_rect_autograd(src: torch.Tensor, tar: torch.Tensor, scale: Scalar,
                             div: Scalar) -> torch.Tensor:
    """Differentiable TensorACA (torch.ops.sks_amd.tensor_aca_rect): gradients flow to
    tar, src (M's coordinates), and scale/div when they are tensors requiring grad."""
    dev = _require_device(src, tar)
    sc = scale if isinstance(scale, torch.Tensor) else torch.tensor([float(scale)], device=dev)
    dv = div if isinstance(div, torch.Tensor) else torch.tensor([float(div)], device=dev)
    return torch.ops.sks_amd.tensor_aca_rect(src, tar, sc.to(torch.float32),
                                             dv.to(torch.float32))


def fill_uniform(count: int, seed: int, offset: int = 0, lo: float = 0.0, hi: float = 1024.0,
                 device: Union[str, torch.device] = "cuda", out=None) -> torch.Tensor:
    """Counter-based U[lo,hi) float32 stream generated on the device."""
    dev = torch.device(device)
    if out is None:
        out = torch.empty(count, dtype=torch.float32, device=dev)
    with _guard(dev):
        _lib.call("hg_fill_uniform_f32", out.data_ptr(), count, seed, offset, lo, hi, _stream(dev))
    return out


def stream_copy(src: torch.Tensor, dst: torch.Tensor) -> None:
    dev = _require_device(src, dst)
    nbytes = src.numel() * src.element_size()
    with _guard(dev):
        _lib.call("hg_stream_copy", src.data_ptr(), dst.data_ptr(), nbytes, _stream(dev))


# ----------------------------------------------------------------- torch.library
_NS = "sks_amd"


def _register_ops() -> None:
    if hasattr(torch.ops, _NS) and hasattr(getattr(torch.ops, _NS), "aca"):
        return

    @torch.library.custom_op(f"{_NS}::aca", mutates_args=())
    def _aca(src: torch.Tensor, tar: torch.Tensor, normalize: bool = False) -> torch.Tensor:
        return aca(src, tar, normalize).reshape(-1, 3, 3)

    @_aca.register_fake
    def _(src, tar, normalize=False):
        return src.new_empty((src.shape[0], 3, 3))

    @torch.library.custom_op(f"{_NS}::sks", mutates_args=())
    def _sks(src: torch.Tensor, tar: torch.Tensor, normalize: bool = False) -> torch.Tensor:
        return sks(src, tar, normalize).reshape(-1, 3, 3)

    @_sks.register_fake
    def _(src, tar, normalize=False):
        return src.new_empty((src.shape[0], 3, 3))

    @torch.library.custom_op(f"{_NS}::tensor_aca_rect", mutates_args=())
    def _rect(src: torch.Tensor, tar: torch.Tensor, scale: torch.Tensor,
              div: torch.Tensor) -> torch.Tensor:
        return tensor_aca_rect(src, tar, scale, div)

    @_rect.register_fake
    def _(src, tar, scale, div):
        return tar.new_empty((tar.shape[0], 3, 3))

    @torch.library.custom_op(f"{_NS}::tensor_aca_rect_backward", mutates_args=())
    def _rect_bwd(src: torch.Tensor, tar: torch.Tensor, grad: torch.Tensor, scale: torch.Tensor,
                  div: torch.Tensor, need_src: bool,
                  need_scale_div: bool) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        return tensor_aca_rect_backward(src, tar, grad, scale, div, need_src, need_scale_div)

    @_rect_bwd.register_fake
    def _(src, tar, grad, scale, div, need_src, need_scale_div):
        B = tar.shape[0]
        return (tar.new_empty((B, 3, 4) if need_src else (0,)), tar.new_empty((B, 3, 4)),
                tar.new_empty((2,) if need_scale_div else (0,)))

    def _setup(ctx, inputs, output):
        src, tar, scale, div = inputs
        ctx.save_for_backward(src, tar, scale, div)

    def _backward(ctx, grad):
        src, tar, scale, div = ctx.saved_tensors
        need_src = ctx.needs_input_grad[0]
        need_sd = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        g_src, g_tar, g_sd = torch.ops.sks_amd.tensor_aca_rect_backward(
            src, tar, grad.contiguous(), scale, div, need_src, need_sd)
        g_scale = g_sd[0:1].reshape(scale.shape) if ctx.needs_input_grad[2] else None
        g_div = g_sd[1:2].reshape(div.shape) if ctx.needs_input_grad[3] else None
        return (g_src if need_src else None, g_tar if ctx.needs_input_grad[1] else None,
                g_scale, g_div)

    _rect.register_autograd(_backward, setup_context=_setup)

    @torch.library.custom_op(f"{_NS}::tensor_aca_offsets", mutates_args=())
    def _offs(corner: torch.Tensor, offsets: torch.Tensor, width: float,
              height: float) -> torch.Tensor:
        return tensor_aca_offsets(corner, offsets, width, height)

    @_offs.register_fake
    def _(corner, offsets, width, height):
        return offsets.new_empty((offsets.shape[0], 3, 3))

    @torch.library.custom_op(f"{_NS}::tensor_aca_offsets_backward", mutates_args=())
    def _offs_bwd(corner: torch.Tensor, offsets: torch.Tensor, grad: torch.Tensor, width: float,
                  height: float, need_corner: bool) -> Tuple[torch.Tensor, torch.Tensor]:
        return tensor_aca_offsets_backward(corner, offsets, grad, width, height, need_corner)

    @_offs_bwd.register_fake
    def _(corner, offsets, grad, width, height, need_corner):
        return (offsets.new_empty(offsets.shape),
                offsets.new_empty((offsets.shape[0], 2) if need_corner else (0,)))

    def _offs_setup(ctx, inputs, output):
        corner, offsets, width, height = inputs
        ctx.save_for_backward(corner, offsets)
        ctx.wh = (width, height)

    def _offs_backward(ctx, grad):
        corner, offsets = ctx.saved_tensors
        need_c = ctx.needs_input_grad[0]
        g_off, g_cor = torch.ops.sks_amd.tensor_aca_offsets_backward(
            corner, offsets, grad.contiguous(), ctx.wh[0], ctx.wh[1], need_c)
        return (g_cor if need_c else None,
                g_off if ctx.needs_input_grad[1] else None, None, None)

    _offs.register_autograd(_offs_backward, setup_context=_offs_setup)


_register_ops()
