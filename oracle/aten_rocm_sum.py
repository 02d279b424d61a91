"""ATen's float32 GPU sum on ROCm, restated: the order in which torch-ROCm's autograd sums a
(B,3,1) gradient to a (1,) or (3,1) parameter (at::sum_to -> sum over dims {0,1} / {0},
keepdim), as the reference's default device='cuda' run (Modules_Runtime_Test.py:301-302,
:393) reduces TensorACA_rect's batch-uniform scale / div gradients.

TEST INFRASTRUCTURE ONLY (tests/, tools/): the checker for hg_sum_rocm_f32, never the product.

Algorithm restated from torch 2.10.0+rocm7.0's ATen/native/hip/Reduce.cuh (the ROCm
translation of Reduce.cuh; the header ships with the wheel), for a float32 input with
float32 accumulation (sum_functor: vt0 = 4, input_vec_size = 4, MAX_NUM_THREADS = 512):
  * setReduceConfig: block (bw, bh) from set_block_dimension, the input / output splits,
    the ROCm rules for the CTA split (the chained `grid().x == grid().y == grid().z == 1`
    comparison included, as C++ evaluates it), the device's multiProcessorCount and
    maxThreadsPerMultiProcessor;
  * ReduceOp::run: each thread's strided sum (vectorised by 4 with four accumulators along a
    contiguous reduced dimension, else four strided accumulators), accumulators folded
    ((a0 + a1) + a2) + a3; block_x_reduce (a shared-memory halving down to the wave, then
    the ROCm wave tree: offsets 1, 2, 4, ... with shfl_down, a lane past the wave keeping its
    own value); block_y_reduce (shared-memory halving over y); global_reduce (the CTA
    partials summed from 0 by the last block's threads, then the block trees again).
Pinned by tests/golden/rocm_sum.npz (tools/make_rocm_sum_golden.py: torch.sum on the GPU
box, the device properties recorded beside) in tests/test_rocm_sum_order.py.

Scope: a contiguous, 16-B aligned float32 (B,3,1) tensor reduced over {0,1} ("full": the (1,)
parameter) or over {0} ("cols": the (3,1) parameter) -- what autograd hands at::sum_to there.
"""
from __future__ import annotations

import numpy as np

WARP = 64
MAX_THREADS = 512
VT0 = 4
VEC = 4


def div_up(a: int, b: int) -> int:
    return (a + b - 1) // b


def last_pow2(n: int) -> int:
    """ATen's last_pow2: the largest power of two <= n (1 for n <= 1)."""
    if n <= 1:
        return 1
    return 1 << (int(n).bit_length() - 1)


class Config:
    """setReduceConfig for the two iterator shapes above."""

    def __init__(self, kind: str, B: int, num_mp: int, max_tpm: int):
        if kind == "full":
            self.ndim, self.num_outputs, self.num_inputs = 1, 1, 3 * B
            fastest = True
            dim0, dim1 = self.num_inputs, self.num_outputs
            self.vectorize = dim0 >= 128
            if self.vectorize:
                dim0 //= VEC
        elif kind == "cols":
            assert B >= 2, "B = 1 leaves no reduced dimension"
            self.ndim, self.num_outputs, self.num_inputs = 2, 3, B
            fastest = False
            dim0, dim1 = self.num_outputs, self.num_inputs
            self.vectorize = False  # output vectors: 3 outputs give output_vec_size 1
        else:
            raise ValueError(kind)
        self.kind, self.fastest = kind, fastest
        # set_block_dimension
        d0 = last_pow2(dim0) if dim0 < MAX_THREADS else MAX_THREADS
        d1 = last_pow2(dim1) if dim1 < MAX_THREADS else MAX_THREADS
        bw = min(d0, WARP)
        bh = min(d1, MAX_THREADS // bw)
        bw = min(d0, MAX_THREADS // bh)
        self.bw, self.bh = bw, bh
        self.step_input, self.step_output = 1, 1
        self.input_mult = [0, 0, 0]
        self.output_mult = [0, 0]

        def split_input(p):
            s = self.step_input
            self.step_input *= p
            return s

        def split_output(p):
            s = self.step_output
            self.step_output *= p
            return s

        if fastest:
            self.input_mult[0] = split_input(bw)
        else:
            self.output_mult[0] = split_output(bw)
        vpt = div_up(self.num_inputs, self.step_input)
        if vpt >= min(bh * 16, 256):  # ROCm's force_splitting_output needs < 100 CUs
            self.input_mult[1] = split_input(bh)
        else:
            self.output_mult[1] = split_output(bh)
        self.ctas = 1
        gx = div_up(self.num_outputs, self.step_output)
        single = int(gx == self.ctas) == 1  # (gx == gy) == gz, then == 1, with gz = 1
        tpm = max_tpm
        if not single:
            tpm = 512 if self.ndim in (1, 3) else 256
        target = num_mp * (tpm // (bw * bh))
        vpt = div_up(self.num_inputs, self.step_input)
        if self.input_mult[1] != 0 and vpt >= 256 and gx <= target:
            c = max(min(div_up(target, gx), div_up(vpt, 16)), div_up(vpt, 256))
            if c > num_mp:
                c = num_mp * (4 if c > 512 else 2) if num_mp < 128 else num_mp
            elif c > div_up(num_mp, 2):
                c = div_up(num_mp, 2)
            elif c < 16:
                c = 1
            self.ctas = c
            if c > 1:
                self.input_mult[2] = split_input(c)
        self.grid_x = div_up(self.num_outputs, self.step_output)

    def as_tuple(self):
        return (self.bw, self.bh, self.ctas, tuple(self.input_mult), tuple(self.output_mult),
                self.step_input, self.step_output, self.vectorize, self.grid_x)


def _wave_tree(v: np.ndarray, dim_x: int) -> np.ndarray:
    """ROCm's in-wave reduction over the block's lanes (linear thread order, waves of 64):
    for offset 1, 2, 4, ... < dim_x every lane adds the pre-step value of lane + offset
    (shfl_down; a source past its wave leaves the lane its own value)."""
    n = v.shape[0]
    v = v.copy()
    lane = np.arange(n) % WARP
    offset = 1
    while offset < dim_x:
        src = np.arange(n) + offset
        ok = (lane + offset) < WARP
        other = np.where(ok, v[np.minimum(src, n - 1)], v)
        v = (v + other).astype(np.float32)
        offset <<= 1
    return v


def _block_x(v: np.ndarray, bw: int, bh: int) -> np.ndarray:
    """block_x_reduce over a block's (bh * bw) thread values, linear index x + y bw."""
    v = v.astype(np.float32).copy()
    dim_x = bw
    if dim_x > WARP:
        s = v.reshape(bh, bw).copy()
        offset = dim_x // 2
        while offset >= WARP:
            s[:, :offset] = (s[:, :offset] + s[:, offset:2 * offset]).astype(np.float32)
            offset >>= 1
        v = s.reshape(-1)
        dim_x = WARP
    return _wave_tree(v, dim_x)


def _block_y(v: np.ndarray, bw: int, bh: int) -> np.ndarray:
    s = v.reshape(bh, bw).astype(np.float32).copy()
    offset = bh // 2
    while offset > 0:
        s[:offset] = (s[:offset] + s[offset:2 * offset]).astype(np.float32)
        offset >>= 1
    return s.reshape(-1)


def rocm_sum(terms, kind: str, num_mp: int, max_tpm: int) -> np.ndarray:
    """terms: (B,3) float32 -- the contiguous (B,3,1) tensor -- summed as ATen-ROCm sums it to
    (1,) ("full") or to (3,1) ("cols"); returns (1,) or (3,) float32."""
    t = np.ascontiguousarray(terms, np.float32).reshape(-1, 3)
    B = t.shape[0]
    if B == 0:
        return np.zeros(1 if kind == "full" else 3, np.float32)
    if kind == "cols" and B == 1:
        return (np.float32(0) + t[0]).astype(np.float32)
    cfg = Config(kind, B, num_mp, max_tpm)
    flat = t.reshape(-1)
    bw, bh = cfg.bw, cfg.bh
    nt = bw * bh
    xs = np.arange(nt) % bw
    ys = np.arange(nt) // bw
    outs = np.zeros(cfg.num_outputs, np.float32)
    z = np.float32(0)
    for bx in range(cfg.grid_x):
        out_idx = xs * cfg.output_mult[0] + ys * cfg.output_mult[1] + bx * cfg.step_output
        partial = np.zeros(cfg.ctas, np.float32)
        finals = None
        for cta in range(cfg.ctas):
            in_idx = xs * cfg.input_mult[0] + ys * cfg.input_mult[1] + cta * cfg.input_mult[2]
            vals = np.zeros(nt, np.float32)
            for t_ in range(nt):
                o, i = int(out_idx[t_]), int(in_idx[t_])
                if not (o < cfg.num_outputs and i < cfg.num_inputs):
                    continue  # (ATen leaves these uninitialised; no stored value reads them)
                if cfg.kind == "full":
                    get = lambda e: flat[e]  # noqa: E731
                else:
                    get = lambda e, o=o: flat[e * 3 + o]  # noqa: E731
                acc = [z, z, z, z]
                end = cfg.num_inputs
                stride = cfg.step_input
                if cfg.vectorize:
                    idx = i
                    while idx * VEC + VEC - 1 < end:
                        for k in range(VEC):
                            acc[k] = np.float32(acc[k] + get(idx * VEC + k))
                        idx += stride
                    tail = end - end % VEC
                    tail_ok = (cfg.input_mult[1] == 0 or ys[t_] == 0) and \
                              (cfg.input_mult[2] == 0 or cta == 0)
                    e = tail + int(xs[t_])
                    if tail_ok and e < end:
                        acc[0] = np.float32(acc[0] + get(e))
                else:
                    idx = i
                    while idx + (VT0 - 1) * stride < end:
                        for k in range(VT0):
                            acc[k] = np.float32(acc[k] + get(idx + k * stride))
                        idx += stride * VT0
                    for k in range(VT0):
                        if idx >= end:
                            break
                        acc[k] = np.float32(acc[k] + get(idx))
                        idx += stride
                v = acc[0]
                for k in range(1, 4):
                    v = np.float32(v + acc[k])
                vals[t_] = v
            if cfg.input_mult[0] != 0:
                vals = _block_x(vals, bw, bh)
            if cfg.input_mult[1] != 0:
                vals = _block_y(vals, bw, bh)
            if cfg.input_mult[2] != 0:
                partial[cta] = vals[0]
            else:
                finals = vals
        if cfg.input_mult[2] != 0:
            vals = np.zeros(nt, np.float32)
            for t_ in range(nt):
                v = z
                o = t_ if cfg.input_mult[0] != 0 else int(ys[t_])
                step = nt if cfg.input_mult[0] != 0 else bh
                while o < cfg.ctas:
                    v = np.float32(v + partial[o])
                    o += step
                vals[t_] = v
            vals = _block_y(vals, bw, bh)
            if cfg.input_mult[0] != 0:
                vals = _block_x(vals, bw, bh)
            finals = vals
        for t_ in range(nt):
            o = int(out_idx[t_])
            store = o < cfg.num_outputs and (cfg.input_mult[0] == 0 or xs[t_] == 0) and \
                (cfg.input_mult[1] == 0 or ys[t_] == 0)
            if store:
                outs[o] = finals[t_]
    return outs


def rocm_sum_case(kind: str, B: int, seed: int, flavour: str = "mixed") -> np.ndarray:
    """The (B,3) float32 terms of a fixture case (regenerated identically on any host)."""
    rng = np.random.default_rng(seed)
    if flavour == "mixed":
        mag = 10.0 ** rng.integers(-3, 4, (B, 1))
        t = rng.standard_normal((B, 3)) * mag
    elif flavour == "uniform":
        t = rng.uniform(-1, 1, (B, 3))
    elif flavour == "zeros":
        t = np.where(rng.random((B, 3)) < 0.5, -0.0, 0.0)
    else:
        raise ValueError(flavour)
    return np.ascontiguousarray(t, np.float32)
