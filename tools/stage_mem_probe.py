"""Why the staged ring is slower than the pinned zero-copy call: the kernel alone reading and
writing pinned host buffers of each kind -- hipHostMalloc fine-grained (coherent), coarse-
grained (non-coherent), torch's pin_memory -- at 10 M f32 AoS ACA, with and without host
threads copying other memory at the same time; then the ring with coherent and with
non-coherent stages (hg_internal_host_stage_coherent).

    python tools/stage_mem_probe.py [--out gpurun_out/stage_mem_probe.json]
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_PINNED_MIN_XFER_SIZE", "65536")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

COHERENT, NONCOHERENT, MAPPED, PORTABLE = 0x40000000, 0x80000000, 0x2, 0x1


def best_ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/stage_mem_probe.json")
    a = ap.parse_args()
    import bench
    numa = bench.bind_numa(0)
    pkg = ge.load_package()
    lib = pkg.lib()
    hip = ctypes.CDLL("libamdhip64.so")
    n = 10_000_000
    dev = torch.device("cuda:0")
    ds = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(n, 8)
    dt = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(n, 8)
    want = pkg.solve("aca", ds, dt).cpu()
    hs, ht = ds.cpu(), dt.cpu()
    out = {"numa": numa}

    def alloc(flags, nbytes):
        p = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flags)) == 0
        return p.value

    # background load: 8 threads memcpy-ing 256 MB pageable buffers back and forth (numpy
    # releases the GIL for large copies)
    stop = threading.Event()
    bufs = [(np.ones(1 << 26, np.float32), np.empty(1 << 26, np.float32)) for _ in range(8)]

    def load(i):
        a_, b_ = bufs[i]
        while not stop.is_set():
            np.copyto(b_, a_)

    kinds = {"coherent": MAPPED | PORTABLE | COHERENT, "noncoherent": MAPPED | PORTABLE | NONCOHERENT}
    for name, flags in kinds.items():
        ps, pt, pH = alloc(flags, n * 32), alloc(flags, n * 32), alloc(flags, n * 36)
        ctypes.memmove(ps, hs.data_ptr(), n * 32)
        ctypes.memmove(pt, ht.data_ptr(), n * 32)
        f = lambda: lib.hg_solve_host_f32(0, ps, pt, pH, n, 0, 1, None)  # noqa: E731
        out[f"{name}_kernel_ms"] = round(best_ms(f), 3)
        got = np.ctypeslib.as_array((ctypes.c_int32 * (n * 9)).from_address(pH))
        out[f"{name}_bit_exact"] = bool(np.array_equal(got, want.view(torch.int32).numpy().ravel()))
        th = [threading.Thread(target=load, args=(i,)) for i in range(8)]
        stop.clear()
        for x in th:
            x.start()
        out[f"{name}_kernel_under_copy_load_ms"] = round(best_ms(f), 3)
        stop.set()
        for x in th:
            x.join()
        for p in (ps, pt, pH):
            hip.hipHostFree(ctypes.c_void_p(p))
    ps, pt, pH = hs.pin_memory(), ht.pin_memory(), torch.empty((n, 9)).pin_memory()
    out["torch_pinned_kernel_ms"] = round(best_ms(lambda: pkg.solve_host("aca", ps, pt, out=pH)), 3)
    qH = torch.empty((n, 9))
    for coh in (1, 0):
        lib.hg_internal_host_stage_coherent(coh)
        qH.fill_(float("nan"))
        ms = best_ms(lambda: pkg.solve_host("aca", hs, ht, out=qH))
        out[f"ring_{'coherent' if coh else 'noncoherent'}_ms"] = round(ms, 3)
        out[f"ring_{'coherent' if coh else 'noncoherent'}_bit_exact"] = bool(
            torch.equal(qH.view(torch.int32), want.view(torch.int32)))
    lib.hg_internal_host_stage_coherent(1)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
