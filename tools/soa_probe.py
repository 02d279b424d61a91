"""SoA f64 10 M: per-launch time vs the relative placement of the src / tar / H buffers
(the 25 component rows of a (8,n)+(8,n)+(9,n) batch are 25 concurrent streams)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
dev = torch.device("cuda:0")
n = 10_000_000


def timeit(f, it=30):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


pool = torch.empty(3 * (n * 9 + (1 << 20)), dtype=torch.float64, device=dev)
gen = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(8, n).double()
for so, to, ho in ((0, 0, 0), (0, 4096, 8192), (0, 65536, 131072), (512, 1024, 2048),
                   (0, 256 * 1024, 512 * 1024), (0, 1 << 20, 2 << 20), (4096, 0, 0), (0, 0, 4096)):
    # three buffers carved from one pool at chosen byte offsets past 2 MiB-aligned bases
    stride = n * 9 + (1 << 20)  # elements
    src = pool[so // 8: so // 8 + 8 * n].view(8, n)
    tar = pool[stride + to // 8: stride + to // 8 + 8 * n].view(8, n)
    H = pool[2 * stride + ho // 8: 2 * stride + ho // 8 + 9 * n].view(9, n)
    src.copy_(gen)
    tar.copy_(gen)
    us = timeit(lambda: pkg.solve("aca", src, tar, normalize=False, layout="soa", out=H))
    print(f"offsets src {so:>8} tar {to:>8} H {ho:>8}: {us:7.1f} us = {n * 200 / us / 1e3:6.0f} GB/s",
          flush=True)
