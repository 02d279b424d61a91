"""Host-resident batches: what a caller whose src/tar/H live in host memory pays per
10 M-problem ACA batch (the reference's C++ API is host-pointer based, ACA_SKS.hpp:17-20).

  seq       pinned H2D src, H2D tar, kernel, D2H H -- one stream (bench.py host_boundary)
  zerocopy  the kernel reads src/tar from pinned host memory and writes H there directly
            (device pointers from hipHostGetDevicePointer): PCIe traffic both ways at once
  chunk/C   C-problem chunks over three streams (H2D, solve, D2H) with events between
            them: copy engines run both directions while the previous chunk solves

Each candidate's H is compared bit for bit with the device-resident solve."""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

SEED = 11


def dev_ptr(hip, t):
    p = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(t.data_ptr()), 0)
    if rc != 0:
        raise RuntimeError(f"hipHostGetDevicePointer rc={rc}")
    return p.value


def main():
    pkg = ge.load_package()
    lib = pkg.lib()
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda:0")
    n = int(os.environ.get("HP_N", 10_000_000))
    ds = pkg.fill_uniform(n * 8, SEED, 0, device=dev).view(n, 8)
    dt = pkg.fill_uniform(n * 8, SEED, n * 8, device=dev).view(n, 8)
    want = pkg.solve("aca", ds, dt, normalize=True).cpu()
    hs = torch.empty((n, 8), dtype=torch.float32).pin_memory()
    ht = torch.empty((n, 8), dtype=torch.float32).pin_memory()
    hH = torch.empty((n, 9), dtype=torch.float32).pin_memory()
    hs.copy_(ds.cpu())
    ht.copy_(dt.cpu())
    dH = torch.empty((n, 9), device=dev)
    cur = torch.cuda.current_stream(dev)
    res = {"n": n}

    def timed(name, fn, reps=5):
        hH.zero_()
        fn()
        torch.cuda.synchronize(dev)
        ok = bool(torch.equal(hH.view(torch.int32), want.view(torch.int32)))
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        ms = ts[len(ts) // 2] * 1e3
        res[name] = {"ms": round(ms, 3), "M_per_s": round(n / ms / 1e3, 1),
                     "pcie_gbps": round(n * 100 / ms / 1e6, 1), "bit_exact": ok}
        print(name, res[name], flush=True)

    # H2D / D2H alone: the per-direction ceilings
    def h2d():
        ds.copy_(hs, non_blocking=True)
        dt.copy_(ht, non_blocking=True)

    def d2h():
        hH.copy_(dH, non_blocking=True)

    for name, fn, nbytes in (("h2d_only", h2d, 64), ("d2h_only", d2h, 36)):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / 5 * 1e3
        res[name] = {"ms": round(ms, 3), "gbps": round(n * nbytes / ms / 1e6, 1)}
        print(name, res[name], flush=True)

    def seq():
        ds.copy_(hs, non_blocking=True)
        dt.copy_(ht, non_blocking=True)
        pkg.solve("aca", ds, dt, normalize=True, out=dH)
        hH.copy_(dH, non_blocking=True)

    timed("seq", seq)

    ps, pt, pH = dev_ptr(hip, hs), dev_ptr(hip, ht), dev_ptr(hip, hH)
    st = cur.cuda_stream

    def zerocopy():
        rc = lib.hg_aca_f32(ps, pt, pH, n, 0, 1, st)
        if rc:
            raise RuntimeError(rc)

    timed("zerocopy", zerocopy)

    s_in, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for chunk in (1 << 19, 1 << 20, 1 << 21):
        nb = 3  # device ring of chunk buffers
        bs = [torch.empty((chunk, 8), device=dev) for _ in range(nb)]
        bt = [torch.empty((chunk, 8), device=dev) for _ in range(nb)]
        bH = [torch.empty((chunk, 9), device=dev) for _ in range(nb)]

        def pipe():
            done_out = [None] * nb
            for k, lo in enumerate(range(0, n, chunk)):
                hi = min(n, lo + chunk)
                m, b = hi - lo, k % nb
                with torch.cuda.stream(s_in):
                    if done_out[b] is not None:
                        s_in.wait_event(done_out[b])  # ring slot free again
                    bs[b][:m].copy_(hs[lo:hi], non_blocking=True)
                    bt[b][:m].copy_(ht[lo:hi], non_blocking=True)
                    e_in = torch.cuda.Event()
                    e_in.record(s_in)
                cur.wait_event(e_in)
                pkg.solve("aca", bs[b][:m], bt[b][:m], normalize=True, out=bH[b][:m])
                e_sv = torch.cuda.Event()
                e_sv.record(cur)
                with torch.cuda.stream(s_out):
                    s_out.wait_event(e_sv)
                    hH[lo:hi].copy_(bH[b][:m], non_blocking=True)
                    e_o = torch.cuda.Event()
                    e_o.record(s_out)
                done_out[b] = e_o
            cur.wait_stream(s_out)

        timed(f"chunk_{chunk}", pipe)
        del bs, bt, bH

    # pageable (plain malloc'd) host buffers: driver-staged copies vs registering the
    # buffers for the call (hipHostRegister mapped), zero-copy, unregister
    qs, qt = hs.clone(), ht.clone()  # pageable CPU tensors
    qH = torch.empty((n, 9), dtype=torch.float32)
    hipHostRegister, hipHostUnregister = hip.hipHostRegister, hip.hipHostUnregister
    hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hipHostUnregister.argtypes = [ctypes.c_void_p]

    def timed_q(name, fn, reps=3):
        qH.zero_()
        fn()
        torch.cuda.synchronize(dev)
        ok = bool(torch.equal(qH.view(torch.int32), want.view(torch.int32)))
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        ms = ts[len(ts) // 2] * 1e3
        res[name] = {"ms": round(ms, 3), "M_per_s": round(n / ms / 1e3, 1), "bit_exact": ok}
        print(name, res[name], flush=True)

    def pageable_seq():
        ds.copy_(qs)
        dt.copy_(qt)
        pkg.solve("aca", ds, dt, normalize=True, out=dH)
        qH.copy_(dH)

    timed_q("pageable_seq", pageable_seq)

    reg_ms = {}

    def pageable_register():
        t0 = time.perf_counter()
        for t in (qs, qt, qH):
            rc = hipHostRegister(t.data_ptr(), t.numel() * 4, 2)  # hipHostRegisterMapped
            if rc:
                raise RuntimeError(f"hipHostRegister rc={rc}")
        t1 = time.perf_counter()
        p = [dev_ptr(hip, t) for t in (qs, qt, qH)]
        rc = lib.hg_aca_f32(p[0], p[1], p[2], n, 0, 1, st)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        for t in (qs, qt, qH):
            hipHostUnregister(t.data_ptr())
        t3 = time.perf_counter()
        reg_ms.update(register=round((t1 - t0) * 1e3, 3), solve=round((t2 - t1) * 1e3, 3),
                      unregister=round((t3 - t2) * 1e3, 3))
        if rc:
            raise RuntimeError(rc)

    timed_q("pageable_register_zerocopy", pageable_register)
    res["pageable_register_zerocopy"]["split_ms"] = dict(reg_ms)
    print(reg_ms, flush=True)

    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/host_probe.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
