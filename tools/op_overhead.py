"""Host cost per call of the torch-facing TensorACA entry points at B = 64 K (the
reference's launch-bound config): host-side wall per call (no sync inside the loop) and
the device-event time per call, for each way of reaching the kernel."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B = 65536
    _, _, src, tar, scale, div = pkg.adjust(dev, B)
    corner = src[:, 0:2, 0].contiguous()
    offs = (tar[:, 0:2, :] - src[:, 0:2, :]).transpose(1, 2).contiguous()
    out = torch.empty((B, 3, 3), device=dev)
    ops = torch.ops.sks_amd
    lib = pkg.lib()
    st = torch._C._cuda_getCurrentRawStream(0)
    cands = {
        "pkg.tensor_aca_rect(tensor scale/div, out=)": lambda: pkg.ops.tensor_aca_rect(src, tar, scale, div, out=out),
        "pkg.tensor_aca_rect(float, out=)": lambda: pkg.ops.tensor_aca_rect(src, tar, 128.0, 1.0, out=out),
        "ops.tensor_aca_rect.out": lambda: ops.tensor_aca_rect.out(src, tar, scale, div, out=out),
        "ops.tensor_aca_rect.default": lambda: ops.tensor_aca_rect.default(src, tar, scale, div),
        "ops.tensor_aca_rect (packet)": lambda: ops.tensor_aca_rect(src, tar, scale, div),
        "ops.tensor_aca_rect.scalar_out": lambda: ops.tensor_aca_rect.scalar_out(src, tar, 128.0, 1.0, out=out),
        "pkg.tensor_aca_offsets(out=)": lambda: pkg.ops.tensor_aca_offsets(corner, offs, 128.0, 128.0, out=out),
        "ops.tensor_aca_offsets.default": lambda: ops.tensor_aca_offsets.default(corner, offs, 128.0, 128.0),
        "ctypes hg_tensor_aca_rect_f32 (raw ptrs)": lambda: lib.hg_tensor_aca_rect_f32(
            src.data_ptr(), tar.data_ptr(), out.data_ptr(), B, scale.data_ptr(), div.data_ptr(), st),
        "empty kernel-free torch op (x.add_(0))": lambda: out.add_(0),
    }
    res = {}
    for name, f in cands.items():
        for _ in range(200):
            f()
        torch.cuda.synchronize()
        n = 2000
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        for _ in range(n):
            f()
        host = (time.perf_counter() - t0) / n * 1e6
        e1.record()
        torch.cuda.synchronize()
        res[name] = {"host_us": round(host, 2), "device_us": round(e0.elapsed_time(e1) / n * 1e3, 2)}
        print(name, res[name], flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/op_overhead.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
