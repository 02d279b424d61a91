"""sks-homography_amd -- MI355X-native batched 4-point homography (ACA / SKS / TensorACA).

Import as ``importlib.import_module("sks-homography_amd")`` (the directory name
carries a hyphen); ``load()`` below also aliases it as ``sks_homography_amd``.

Layers:
  include/sks_homography.h   C ABI (device pointers, hipStream_t, hipError_t codes;
                             hg_solve_host_*: host-resident batches, zero-copy)
  include/sks_aca_sks.hpp    the reference's sks::runKernel_* C++ interface
  csrc/                      HIP kernels for gfx950 + the C ABI + the sks:: API
  ops.py                     torch-facing wrappers, torch.ops.sks_amd.*
  reference_api.py           TensorACA_rect / ACA_vanilla / getInput / adjust mirrors
  shard.py                   per-GPU block sharding, optional RCCL split / gather
  ransac.py                  fused hypothesis sampling + solve + inlier scoring
"""
from __future__ import annotations

from . import _lib
from ._lib import HG_FLAG_NORMALIZE, HG_LAYOUT_AOS, HG_LAYOUT_SOA, HipError, lib, version
from .ops import (aca, aca_backward, aca_vanilla, fill_uniform, sks, solve, solve_grouped, solve_host, stream_copy, tensor_aca_rect,
                  tensor_aca_rect_autograd, tensor_aca_rect_backward,
                  tensor_aca_offsets, tensor_aca_offsets_backward)
from .ransac import (RansacResult, fill_bits, gather_solve, get_rand_list, mrg32k3a_state,
                     rand_gather_solve, rand_mrg32k3a, ransac, read_points, sample_solve,
                     sample_solve_seeded)
from .ransac import score as ransac_score
from .reference_api import ACA_vanilla, TensorACA_rect, adjust, getInput, getTar
from .shard import gather_blocks, scatter_blocks, shard_range

BYTES_PER_PROBLEM = {"f32": 64 + 36, "f64": 128 + 72}   # algorithmic HBM bytes per H
RECT_BYTES_PER_PROBLEM = 48 + 8 + 36                     # tar + src M + H

__all__ = [
    "aca", "aca_vanilla", "aca_backward", "sks", "solve", "solve_grouped", "solve_host", "tensor_aca_rect", "tensor_aca_rect_autograd",
    "tensor_aca_rect_backward", "tensor_aca_offsets", "tensor_aca_offsets_backward",
    "fill_uniform", "sample_solve", "sample_solve_seeded", "fill_bits", "ransac", "ransac_score", "RansacResult", "stream_copy",
    "read_points", "rand_mrg32k3a", "get_rand_list", "gather_solve", "rand_gather_solve",
    "mrg32k3a_state",
    "TensorACA_rect", "ACA_vanilla", "getInput", "getTar", "adjust", "shard_range",
    "gather_blocks", "scatter_blocks", "lib", "version", "HipError", "HG_LAYOUT_AOS", "HG_LAYOUT_SOA",
    "HG_FLAG_NORMALIZE", "BYTES_PER_PROBLEM", "RECT_BYTES_PER_PROBLEM",
]
