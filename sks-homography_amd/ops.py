"""Torch-facing entry points over the C ABI (device memory, torch's current stream).

PyTorch is plumbing here: tensors own the HBM buffers and name the stream; every
computation is one of the library's HIP kernels.  CPU tensors are rejected -- the
product has no CPU path.

The op contract of SURVEY.md section 8(b) -- ``torch.ops.sks_amd.{aca, sks,
tensor_aca_rect, tensor_aca_offsets}`` with autograd -- is native C++
(csrc/hg_torch_ops.cpp), loaded here.
"""
from __future__ import annotations

import os
from typing import Optional, Union

import torch

from . import _lib

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


_ALGO_ID = {"aca": 0, "sks": 1, "ge": 2, "gpt": 3}
_LAYOUT_ID = {"aos": 0, "soa": 1}


def solve(algo: str, src: torch.Tensor, tar: torch.Tensor, normalize: bool = True,
          layout: str = "aos", out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Batched 4-point homography, ``algo`` in {"aca", "sks", "ge", "gpt"}.  "ge" and
    "gpt" are the reference's comparison baselines: RHO Gaussian elimination (f32 as
    cv::runKernel_GE, f64 as cal_Homo_GE) and 8x8 pivoted LU (f64, cal_Homo_GPT).

    AoS: src/tar (n,8) or (n,4,2) -> H (n,9); SoA: (8,n) -> (9,n).
    ``normalize=True`` returns H/H[8] exactly as sks::runKernel_* (ACA_SKS.cpp:94-98);
    False returns H up to scale as cal_Homo_* / ACA_vanilla do.  Runs the native
    torch.ops.sks_amd.solve (shape/dtype checks there; no CPU path).
    """
    algo_id = _ALGO_ID.get(algo)
    if algo_id is None:
        raise ValueError(f"algo must be 'aca', 'sks', 'ge' or 'gpt', got {algo!r}")
    lay = _LAYOUT_ID.get(layout)
    if lay is None:
        raise ValueError(f"layout must be 'aos' or 'soa', got {layout!r}")
    _gpu_only(src)
    _gpu_only(tar)
    if src.dtype not in _DTYPES or tar.dtype is not src.dtype:
        raise TypeError(f"src/tar must both be float32 or float64, got {src.dtype}/{tar.dtype}")
    if algo_id == 3 and src.dtype is not torch.float64:
        raise TypeError("the GPT-LU baseline (cal_Homo_GPT) is float64 only")
    if out is None:
        return _OPS.solve.default(src, tar, algo_id, normalize, lay)
    return _OPS.solve.out(src, tar, algo_id, normalize, lay, out=out)


def solve_host(algo: str, src: torch.Tensor, tar: torch.Tensor, normalize: bool = True,
               layout: str = "aos", out: Optional[torch.Tensor] = None,
               device: Union[int, str, torch.device, None] = None,
               register: bool = False) -> torch.Tensor:
    """``solve`` for a batch that lives in HOST memory (CPU tensors, pinned or not)
    (hg_solve_host_*).  Pinned tensors are read and written by the GPU kernel in place over
    PCIe (zero-copy); pageable tensors go through the library's ring of pinned stages, copied
    by host threads, so their pages are never mapped for the GPU.  ``register=True``
    (HG_FLAG_HOST_REGISTER) registers pageable tensors for the call instead -- zero-copy, but
    the driver keeps those pages GPU-mapped afterwards: only for memory that is never handed
    back to the heap.  Returns when H is complete.  ``device``
    picks the GPU (default: the current one).  The computation is the same HIP kernel with
    the same bits -- there is no CPU solver."""
    algo_id = _ALGO_ID.get(algo)
    if algo_id is None:
        raise ValueError(f"algo must be 'aca', 'sks', 'ge' or 'gpt', got {algo!r}")
    lay = _LAYOUT_ID.get(layout)
    if lay is None:
        raise ValueError(f"layout must be 'aos' or 'soa', got {layout!r}")
    for t in (src, tar) + ((out,) if out is not None else ()):
        if t.device.type != "cpu":
            raise ValueError(f"solve_host takes host tensors, got a {t.device} tensor (use solve)")
        if not t.is_contiguous():
            raise ValueError("solve_host needs contiguous tensors (the kernel reads raw memory)")
    if src.dtype not in _DTYPES or tar.dtype is not src.dtype:
        raise TypeError(f"src/tar must both be float32 or float64, got {src.dtype}/{tar.dtype}")
    if algo_id == 3 and src.dtype is not torch.float64:
        raise TypeError("the GPT-LU baseline (cal_Homo_GPT) is float64 only")
    if lay == 0:
        n = src.shape[0] if src.dim() else -1
        ok = (src.dim() == 2 and src.shape[1] == 8) or (src.dim() == 3 and tuple(src.shape[1:]) == (4, 2))
        want_out = (n, 9)
    else:
        n = src.shape[1] if src.dim() == 2 else -1
        ok = src.dim() == 2 and src.shape[0] == 8
        want_out = (9, n)
    if not ok or tar.shape != src.shape:
        raise ValueError(f"{layout} src/tar must be {'(n,8) or (n,4,2)' if lay == 0 else '(8,n)'} "
                         f"and equal, got {tuple(src.shape)} / {tuple(tar.shape)}")
    if out is None:
        out = torch.empty(want_out, dtype=src.dtype)
    elif tuple(out.shape) != want_out or out.dtype is not src.dtype:
        raise ValueError(f"out must be {want_out} {src.dtype}, got {tuple(out.shape)} {out.dtype}")
    dev = _gpu_device("cuda" if device is None else
                      (torch.device("cuda", device) if isinstance(device, int) else device))
    fn = "hg_solve_host_f32" if src.dtype is torch.float32 else "hg_solve_host_f64"
    with _guard(dev):
        _lib.call(fn, algo_id, src.data_ptr(), tar.data_ptr(), out.data_ptr(), n, lay,
                  (_lib.HG_FLAG_NORMALIZE if normalize else 0)
                  | (_lib.HG_FLAG_HOST_REGISTER if register else 0), None)
    return out


def solve_grouped(algo: str, srcs, tars, normalize: bool = True, layout: str = "aos",
                  outs=None):
    """Many small batches in as few launches as possible (hg_solve_grouped_*: up to 32
    batches per launch): ``srcs[i]``, ``tars[i]`` -> H_i, each batch shaped as for
    ``solve``.  Returns the list of H (or fills ``outs``).  Same bits as ``solve`` on each
    batch; for workloads of many small batches, where one launch each costs more than the
    work."""
    import ctypes

    algo_id = _ALGO_ID.get(algo)
    if algo_id is None:
        raise ValueError(f"algo must be 'aca', 'sks', 'ge' or 'gpt', got {algo!r}")
    lay = _LAYOUT_ID.get(layout)
    if lay is None:
        raise ValueError(f"layout must be 'aos' or 'soa', got {layout!r}")
    srcs, tars = list(srcs), list(tars)
    if len(srcs) != len(tars):
        raise ValueError(f"{len(srcs)} src batches but {len(tars)} tar batches")
    if not srcs:
        return []
    dev = _require_device(*srcs, *tars)
    dt = srcs[0].dtype
    if dt not in _DTYPES:
        raise TypeError(f"batches must be float32 or float64, got {dt}")
    if algo_id == 3 and dt is not torch.float64:
        raise TypeError("the GPT-LU baseline (cal_Homo_GPT) is float64 only")
    ns = []
    for s, t in zip(srcs, tars):
        if s.dtype is not dt or t.dtype is not dt:
            raise TypeError("every batch must have the same dtype")
        if not (s.is_contiguous() and t.is_contiguous()) or s.shape != t.shape:
            raise ValueError("each src/tar pair must be contiguous and of equal shape")
        if lay == 0 and not ((s.dim() == 2 and s.shape[1] == 8) or
                             (s.dim() == 3 and tuple(s.shape[1:]) == (4, 2))):
            raise ValueError(f"AoS batches must be (n,8) or (n,4,2), got {tuple(s.shape)}")
        if lay == 1 and not (s.dim() == 2 and s.shape[0] == 8):
            raise ValueError(f"SoA batches must be (8,n), got {tuple(s.shape)}")
        ns.append(s.shape[0] if lay == 0 else s.shape[1])
    if outs is None:
        outs = [torch.empty((m, 9) if lay == 0 else (9, m), dtype=dt, device=dev) for m in ns]
    else:
        outs = list(outs)
        if len(outs) != len(srcs):
            raise ValueError("one out tensor per batch")
        if _require_device(*outs) != dev:
            # a kernel launched on `dev` writing another GPU's memory is a peer write or a fault
            raise ValueError(f"out tensors must be on {dev}, the inputs' device")
        for o, m in zip(outs, ns):
            want = (m, 9) if lay == 0 else (9, m)
            if tuple(o.shape) != want or o.dtype is not dt or not o.is_contiguous():
                raise ValueError(f"out must be a contiguous {want} {dt} tensor, got {tuple(o.shape)}")
    k = len(srcs)
    P = ctypes.c_void_p * k
    fn = "hg_solve_grouped_f32" if dt is torch.float32 else "hg_solve_grouped_f64"
    with _guard(dev):
        _lib.call(fn, algo_id, P(*[x.data_ptr() for x in srcs]), P(*[x.data_ptr() for x in tars]),
                  P(*[x.data_ptr() for x in outs]), (ctypes.c_int64 * k)(*ns), k, lay,
                  _lib.HG_FLAG_NORMALIZE if normalize else 0, _stream(dev))
    return outs


def aca(src, tar, normalize: bool = True, layout: str = "aos", out=None) -> torch.Tensor:
    return solve("aca", src, tar, normalize, layout, out)


def sks(src, tar, normalize: bool = True, layout: str = "aos", out=None) -> torch.Tensor:
    return solve("sks", src, tar, normalize, layout, out)


def aca_vanilla(src: torch.Tensor, tar: torch.Tensor) -> torch.Tensor:
    """ACA_vanilla's contract (Modules_Runtime_Test.py:312-388): src, tar (B,4,2) or (B,8),
    float32 or float64 -> the unnormalised (B,3,3) H.  Runs torch.ops.sks_amd.aca, which is
    differentiable w.r.t. src and tar as the reference's statements are under ATen autograd,
    with the same gradient bits (hg_aca_backward_*)."""
    _gpu_only(src)
    _gpu_only(tar)
    return _OPS.aca.default(src, tar, False)


def aca_backward(src: torch.Tensor, tar: torch.Tensor, grad: torch.Tensor,
                 need_src: bool = True, need_tar: bool = True):
    """Gradients of aca_vanilla: (dL/dsrc, dL/dtar) shaped like src / tar (or empty)."""
    _gpu_only(tar)
    return _OPS.aca_backward.default(src, tar, grad, need_src, need_tar)


Scalar = Union[float, int, torch.Tensor]


def _dev_scalar(x, dev: torch.device) -> torch.Tensor:
    """scale / div as a float32 GPU tensor: kept as it is when it already is one (the
    reference keeps them in (1,)-shaped tensors, .py:33-35), else converted (differentiably).
    Any shape the reference composition broadcasts against the (B,3,1) columns -- one value,
    (B,1,1) per problem, (3,1) per row, (B,3,1) -- is accepted; the native op checks it."""
    if type(x) is torch.Tensor and x.dtype is torch.float32 and x.is_cuda:
        return x
    return torch.as_tensor(x, dtype=torch.float32, device=dev)


def _gpu_device(device) -> torch.device:
    """A `device=` argument resolved to a GPU device (kernels must never see host memory)."""
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("sks_homography_amd kernels run on the GPU only; got device "
                         f"{dev} (no CPU fallback by design)")
    return dev


def _gpu_only(t: torch.Tensor) -> None:
    if not t.is_cuda:
        raise ValueError("sks_homography_amd kernels run on the GPU only; got a "
                         f"{t.device} tensor (no CPU fallback by design)")


_ORDERS = {"cpu": 0, "rocm": 1}


def _order(order: str) -> int:
    """Whose evaluation of the reference's statements to reproduce bit for bit (HG_ORDER_*)."""
    try:
        return _ORDERS[order]
    except KeyError:
        raise ValueError(f"order must be 'cpu' (ATen-CPU) or 'rocm' (torch-ROCm), got {order!r}") \
            from None


def tensor_aca_rect(src: torch.Tensor, tar: torch.Tensor, scale: Scalar, div: Scalar,
                    out: Optional[torch.Tensor] = None, order: str = "cpu") -> torch.Tensor:
    """TensorACA rectangle->quad (Modules_Runtime_Test.py:286-309), unnormalised.

    src, tar: (B,3,4) float32 homogeneous (rows x, y, 1; columns M, N, P, Q).
    scale, div: width and width/height -- Python numbers, or tensors of any shape the
    reference composition broadcasts against the (B,3,1) columns it scales (.py:301-302):
    one value (the reference's own (1,) tensors, .py:33-35), (B,1,1) per problem, (3,1)
    per row, (B,3,1); taken as float32 on tar's device.  Returns (B,3,3).
    Runs torch.ops.sks_amd.tensor_aca_rect (native, csrc/hg_torch_ops.cpp); with tensor
    scale/div and no ``out`` it is differentiable in all four inputs.

    Which bits (``order``): "cpu" (default) -- the reference's statements as ATen-CPU
    evaluates them (FMA-contracted cross, the three cross terms summed ((c0 + c1) + c2) + 0),
    bit for bit, as the golden fixtures pin.  "rocm" -- as torch-ROCm evaluates them on the
    GPU, the reference's own default run (Modules_Runtime_Test.py:393, device='cuda'): every
    three-term sum, forward and backward, is ((0 + t0) + t2) + t1
    (profiles/r04/rocm_grad_probe_r04j.json), and a (1,) / (3,1) scale or div gradient is
    summed over the batch in ATen-ROCm's reduction order (hg_sum_rocm_f32); H, dL/dtar and
    dL/dscale, dL/ddiv of every shape then equal that run's bits (dL/dsrc, which the
    reference cannot take, follows the same sums).  The two orders differ by ~1e-5 relative
    on fractional inputs and agree exactly on the reference's integer batches.
    """
    _gpu_only(tar)  # the op checks that src (and out) share tar's device
    o = _order(order)
    if o or isinstance(scale, torch.Tensor) or isinstance(div, torch.Tensor):
        sc, dv = _dev_scalar(scale, tar.device), _dev_scalar(div, tar.device)
        if out is None:
            return _OPS.tensor_aca_rect.default(src, tar, sc, dv, o)
        return _OPS.tensor_aca_rect.out(src, tar, sc, dv, o, out=out)
    if out is None:
        return _OPS.tensor_aca_rect.scalar(src, tar, float(scale), float(div))
    return _OPS.tensor_aca_rect.scalar_out(src, tar, float(scale), float(div), out=out)


def tensor_aca_rect_backward(src: torch.Tensor, tar: torch.Tensor, grad: torch.Tensor,
                             scale: Scalar, div: Scalar, need_src: bool = True,
                             need_scale_div: bool = True, aten_threads: int = 0,
                             order: str = "cpu"):
    """Gradients of tensor_aca_rect: (dL/dsrc (B,3,4) or empty, dL/dtar (B,3,4), dL/dscale,
    dL/ddiv shaped like scale and div, or empty).  The kernel's (problem, row) terms are
    summed over the dimensions scale / div were broadcast along, on the device, in the
    float32 order ATen-CPU's autograd sums them through the reference's statements
    (hg_sum_aten_f32): for a batch-uniform scale / div of >= 32768 terms that order depends
    on ATen's thread count -- this process's (torch.get_num_threads()) unless
    ``aten_threads`` names another.  ``order`` as tensor_aca_rect's."""
    _gpu_only(tar)
    return _OPS.tensor_aca_rect_backward.default(
        src, tar, grad, _dev_scalar(scale, tar.device), _dev_scalar(div, tar.device),
        need_src, need_scale_div, aten_threads, _order(order))


def tensor_aca_offsets(corner: torch.Tensor, offsets: torch.Tensor, width: float, height: float,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Compact TensorACA: source = the width x height rectangle at
    ``corner`` (B,2), target = source + ``offsets`` (B,4,2) in M,N,P,Q order.  Same bits
    as building the (B,3,4) tensors and calling tensor_aca_rect(scale=width,
    div=width/height).  Returns the unnormalised (B,3,3) H; differentiable without
    ``out``."""
    _gpu_only(offsets)  # the op checks that corner (and out) share its device
    if out is None:
        return _OPS.tensor_aca_offsets.default(corner, offsets, float(width), float(height))
    return _OPS.tensor_aca_offsets.out(corner, offsets, float(width), float(height), out=out)


def tensor_aca_offsets_backward(corner, offsets, grad, width: float, height: float,
                                need_corner: bool = True):
    _gpu_only(offsets)
    return _OPS.tensor_aca_offsets_backward.default(corner, offsets, grad, float(width),
                                                    float(height), need_corner)


def tensor_aca_rect_autograd(src: torch.Tensor, tar: torch.Tensor, scale: Scalar,
                             div: Scalar, order: str = "cpu") -> torch.Tensor:
    """Differentiable TensorACA (torch.ops.sks_amd.tensor_aca_rect): gradients flow to
    tar, src (M's coordinates), and scale/div when they are tensors requiring grad.
    ``order`` as tensor_aca_rect's (the backward follows the forward's).

    With order="cpu", a batch-uniform scale / div gradient of >= 32768 terms is summed in
    ATen-CPU's order FOR THE FORWARD CALLER'S torch.get_num_threads() (ATen chunks such sums
    per thread): the bits then differ between, e.g., a plain python run and a torchrun rank
    with OMP_NUM_THREADS=1, exactly as the reference's own CPU autograd does.  Pin them with
    torch.set_num_threads(T) before the forward, or call tensor_aca_rect_backward with
    aten_threads=T.  Other gradients, H, and order="rocm" do not depend on it."""
    _gpu_only(tar)
    return _OPS.tensor_aca_rect.default(src, tar, _dev_scalar(scale, tar.device),
                                        _dev_scalar(div, tar.device), _order(order))


def fill_uniform(count: int, seed: int, offset: int = 0, lo: float = 0.0, hi: float = 1024.0,
                 device: Union[str, torch.device] = "cuda", out=None) -> torch.Tensor:
    """Counter-based U[lo,hi) float32 stream generated on the device."""
    if count < 0:
        raise ValueError(f"count must be >= 0, got {count}")
    if out is None:
        dev = _gpu_device(device)
        out = torch.empty(count, dtype=torch.float32, device=dev)
    else:
        dev = _require_device(out)
        if out.dtype != torch.float32 or not out.is_contiguous() or out.numel() < count:
            raise ValueError(f"out must be a contiguous float32 tensor of >= {count} elements, "
                             f"got {out.dtype} {tuple(out.shape)}")
    with _guard(dev):
        _lib.call("hg_fill_uniform_f32", out.data_ptr(), count, seed, offset, lo, hi, _stream(dev))
    return out


def stream_copy(src: torch.Tensor, dst: torch.Tensor) -> None:
    dev = _require_device(src, dst)
    nbytes = src.numel() * src.element_size()
    if not (src.is_contiguous() and dst.is_contiguous()) or dst.numel() * dst.element_size() < nbytes:
        raise ValueError("stream_copy needs contiguous tensors and dst at least as large as src")
    with _guard(dev):
        _lib.call("hg_stream_copy", src.data_ptr(), dst.data_ptr(), nbytes, _stream(dev))


# ----------------------------------------------------------------- torch.library
def _load_native_ops():
    """torch.ops.sks_amd.* are native (csrc/hg_torch_ops.cpp -> lib/libsks_homography_torch.so):
    CUDA/HIP, Meta and C++ autograd kernels registered with the dispatcher.  Missing
    library = ImportError (no Python or CPU substitute)."""
    if not os.path.exists(_lib.TORCH_LIB_PATH):
        raise ImportError(f"{_lib.TORCH_LIB_PATH} not built: run `python -c 'import "
                          "__graft_entry__ as g; g.build()'` (the MI355X kernels have no CPU "
                          "fallback)")
    if not hasattr(torch.ops.sks_amd, "tensor_aca_offsets_backward"):
        _lib.lib()  # the product library first (the op library links it)
        torch.ops.load_library(_lib.TORCH_LIB_PATH)
    return torch.ops.sks_amd


_OPS = _load_native_ops()
