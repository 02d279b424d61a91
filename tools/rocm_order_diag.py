"""Diagnostic (GPU box): the elements where order="rocm"'s dL/dtar differs from torch-ROCm's
autograd through the reference's statements, on tests/test_gpu_rect_rocm_order.py's
special-value batch -- with each problem's inputs, dL/dH and both gradients, and the
intermediate gradients torch computed for that problem.  Prints one JSON object."""
import json
import os
import sys
import zlib

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import __graft_entry__ as ge  # noqa: E402
import test_gpu_rect_rocm_order as T  # noqa: E402


def hooked(src, tar, scale, div, gH):
    """bench.torch_tensor_aca_rect with hooks on the intermediates (same statements)."""
    g = {}

    def keep(name, t):
        t.register_hook(lambda x: g.__setitem__(name, x.detach().cpu().numpy().copy()))
        return t

    bs = tar.shape[0]
    tar = tar.clone().requires_grad_()
    H = torch.zeros((bs, 3, 3), device=tar.device)
    d = keep("d", tar[:, :, 1:] - tar[:, :, 0:1])
    q = keep("q", torch.cross(d[:, 1:2, :], d[:, 0:1, :], dim=2))
    s = keep("s", torch.sum(q, dim=2, keepdim=True))
    b = keep("b", s * tar[:, :, 0:1])
    h0 = keep("h0", tar[:, :, 1:2] * q[:, :, 0:1] - b)
    H[:, :, 0:1] = h0
    x = keep("x", tar[:, :, 2:3] * q[:, :, 1:2] - b)
    H[:, :, 1:2] = torch.mul(div, x)
    H[:, :, 2:3] = scale * b - src[:, 0:1, 0:1] * H[:, :, 0:1] - src[:, 1:2, 0:1] * H[:, :, 1:2]
    H.backward(gH)
    g["tar"] = tar.grad.detach().cpu().numpy()
    return g


def main():
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    s_np, t_np, g_np, rng = T._batch("special", zlib.crc32(repr(("bwd", "special", "one")).encode()))
    sc_np, dv_np = T._params("one", rng)
    s, t, gH = (torch.from_numpy(x).to(dev) for x in (s_np, t_np, g_np))
    sc, dv = torch.from_numpy(sc_np).to(dev), torch.from_numpy(dv_np).to(dev)
    g = hooked(s, t, sc, dv, gH)
    _, g_tar, _, _ = pkg.tensor_aca_rect_backward(s, t, gH, sc, dv, False, False, order="rocm")
    got = g_tar.cpu().numpy()
    want = g["tar"]
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    out = {"differ": int((~same).sum()), "cases": []}
    for b, r, c in np.argwhere(~same)[:8].tolist():
        out["cases"].append({
            "at": [b, r, c], "got": float(got[b, r, c]), "want": float(want[b, r, c]),
            "got_bits": hex(int(got[b, r, c:c + 1].view(np.uint32)[0])),
            "want_bits": hex(int(want[b, r, c:c + 1].view(np.uint32)[0])),
            "src": s_np[b].tolist(), "tar": t_np[b].tolist(), "gH": g_np[b].tolist(),
            "got_row": got[b].tolist(), "want_row": want[b].tolist(),
            **{f"g_{k}": g[k][b].tolist() for k in ("d", "q", "s", "b", "h0", "x")},
        })
    print(json.dumps(out, default=str))


if __name__ == "__main__":
    main()
