"""GPU box: fixtures of ATen-ROCm's float32 sum for the two shapes autograd's at::sum_to takes
for TensorACA_rect's batch-uniform scale / div (a (B,3,1) gradient to (1,) and to (3,1)):
torch.sum on the GPU (and Tensor.sum_to_size, the same at::sum_to autograd calls, checked to
agree), the device properties the reduction's launch configuration reads, and -- live -- the
restatement oracle/aten_rocm_sum.py against them.  Writes gpurun_out/rocm_sum.npz (copied to
tests/golden/) and prints one JSON summary.  Inputs are regenerated from seeds
(aten_rocm_sum.rocm_sum_case), so the fixture holds only the cases and the output bits."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import aten_rocm_sum as ars  # noqa: E402

SIZES = [1, 2, 3, 5, 10, 21, 42, 43, 64, 100, 128, 170, 171, 200, 341, 342, 500, 1000, 1365,
         1366, 2000, 2731, 5000, 10922, 10923, 20000, 43690, 43691, 65536, 100003, 174762,
         174763, 262144]


def main():
    dev = torch.device("cuda:0")
    props = torch.cuda.get_device_properties(dev)
    num_mp = props.multi_processor_count
    max_tpm = props.max_threads_per_multi_processor
    cases, bits, ok, first_bad = [], [], 0, []
    seed = 0
    for kind in ("full", "cols"):
        for B in SIZES:
            for flavour in ("mixed", "uniform", "zeros"):
                seed += 1
                t = ars.rocm_sum_case(kind, B, seed, flavour)
                x = torch.from_numpy(t).to(dev).view(B, 3, 1)
                if kind == "full":
                    got = x.sum((0, 1), keepdim=True).reshape(1)
                    via = x.sum_to_size(1)
                else:
                    got = x.sum((0,), keepdim=True).reshape(3)
                    via = x.sum_to_size(3, 1).reshape(3)
                g = got.cpu().numpy()
                assert (g.view(np.uint32) == via.cpu().numpy().view(np.uint32)).all(), (kind, B)
                want = ars.rocm_sum(t, kind, num_mp, max_tpm) if B <= 262144 else None
                match = want is not None and (want.view(np.uint32) == g.view(np.uint32)).all()
                ok += int(match)
                if not match and len(first_bad) < 12:
                    cfg = ars.Config(kind, B, num_mp, max_tpm).as_tuple() if (kind == "full" or B > 1) else None
                    first_bad.append({"kind": kind, "B": B, "flavour": flavour, "torch": g.tolist(),
                                      "restated": None if want is None else want.tolist(),
                                      "config": str(cfg)})
                cases.append((kind, B, seed, flavour))
                bits.append(np.pad(g.view(np.uint32), (0, 3 - g.size)))
    out = os.path.join(ROOT, "gpurun_out", "rocm_sum.npz")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    np.savez_compressed(out, kind=np.array([c[0] for c in cases]), B=np.array([c[1] for c in cases]),
                        seed=np.array([c[2] for c in cases]), flavour=np.array([c[3] for c in cases]),
                        bits=np.array(bits, np.uint32), num_mp=num_mp, max_tpm=max_tpm,
                        warp=props.warp_size if hasattr(props, "warp_size") else 64,
                        torch=torch.__version__, device=props.name)
    print(json.dumps({"cases": len(cases), "restatement_equal": ok, "num_mp": num_mp,
                      "max_threads_per_mp": max_tpm, "torch": torch.__version__,
                      "first_mismatches": first_bad}))


if __name__ == "__main__":
    main()
