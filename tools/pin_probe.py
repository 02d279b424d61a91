"""Which host<->device copies of pageable memory does HIP pin in place, and does a pin outlive
the copy?  (Round 5, the write-to-read-only GPU fault on a heap address: DESIGN.md section 10.)

For each size: a pageable tensor is copied to the device (H2D, the host pages are the source),
then a device tensor into a FRESH pageable tensor (D2H, the host pages are the destination --
never into a buffer an earlier copy read from).  After each copy hipPointerGetAttributes says
what HIP believes the host pages are (0 unregistered, 1 host/pinned).  HIP's own copy log
(AMD_LOG_LEVEL=4, set before the runtime starts) goes to stderr: its "Pinned resource" lines
name the copies that pinned the user's pages instead of staging them.
    AMD_LOG_LEVEL=4 python tools/pin_probe.py 2> gpurun_out/pin_probe.log
"""
import ctypes
import json
import os
import sys

import torch

SIZES_MB = [0.0625, 1, 2, 4, 5.76, 8, 16, 33, 64, 129]


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipPointerGetAttributes.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    attrs = ctypes.create_string_buffer(256)

    def kind(p):
        rc = hip.hipPointerGetAttributes(attrs, ctypes.c_void_p(p))
        hip.hipGetLastError()
        return -1 if rc else int.from_bytes(attrs.raw[:4], "little")

    dev = torch.device("cuda:0")
    torch.ones(1, device=dev)
    out = []
    keep = []  # nothing freed during the probe: no address is reused
    for mb in SIZES_MB:
        n = int(mb * 2**20) // 4
        a = torch.arange(n, dtype=torch.float32)
        print(f"--- H2D {mb} MB from {a.data_ptr():#x}", file=sys.stderr, flush=True)
        d = a.to(dev)
        torch.cuda.synchronize()
        ka = kind(a.data_ptr())
        b = torch.empty(n, dtype=torch.float32)
        print(f"--- D2H {mb} MB into {b.data_ptr():#x}", file=sys.stderr, flush=True)
        b.copy_(d)
        torch.cuda.synchronize()
        kb = kind(b.data_ptr())
        ok = bool(torch.equal(a, b))
        rec = {"mb": mb, "h2d_src_kind_after": ka, "d2h_dst_kind_after": kb, "equal": ok,
               "src": hex(a.data_ptr()), "dst": hex(b.data_ptr())}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        keep += [a, b, d]
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/pin_probe.json", "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
