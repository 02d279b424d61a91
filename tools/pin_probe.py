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


def svm_query():
    """KFD's SVM access attribute of the page holding a host address (tests/fault_probe.c),
    or None when the probe library is not built."""
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests",
                        "_build", "libfault_probe.so")
    if not os.path.exists(path):
        return None
    fp = ctypes.CDLL(path)
    u64 = ctypes.c_uint64
    fp.hg_fault_probe_svm.argtypes = [u64, u64] + [ctypes.POINTER(u64)] * 3
    if fp.hg_fault_probe_install() != 0:
        return None

    def q(p):
        acc, ro, gf = u64(), u64(), u64()
        rc = fp.hg_fault_probe_svm(p // 4096 * 4096, 4096, ctypes.byref(acc), ctypes.byref(ro),
                                   ctypes.byref(gf))
        return hex(acc.value) if rc == 0 else f"rc {rc}"
    return q


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
    svm = svm_query()
    out = [{"GPU_PINNED_MIN_XFER_SIZE": os.environ.get("GPU_PINNED_MIN_XFER_SIZE")}]
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
        if svm is not None:  # 0x202: no GPU access; 0x201: the GPU maps the page in place
            rec["svm_src_after"] = svm(a.data_ptr() + a.numel() * 2)
            rec["svm_dst_after"] = svm(b.data_ptr() + b.numel() * 2)
        print(json.dumps(rec), flush=True)
        out.append(rec)
        keep += [a, b, d]
    if not os.environ.get("PIN_PROBE_SIZES_ONLY"):
        out += interplay(kind, dev)
    os.makedirs("gpurun_out", exist_ok=True)
    tag = os.environ.get("PIN_PROBE_TAG", "")
    with open(f"gpurun_out/pin_probe{tag}.json", "w") as fh:
        json.dump(out, fh, indent=1)


def interplay(kind, dev):
    """HIP's own pins beside the library's registrations of the same pages (hg_solve_host:
    hipHostRegister of page-rounded ranges).  The GPU only READS pages shared with an earlier
    pin here (H2D copies, the solver's src/tar reads), and every step asks ROCr itself what it
    holds at the buffers (tests/fault_probe.c: hsa_amd_pointer_info, a host-side query) --
    HIP's cached copy pins are invisible to hipPointerGetAttributes."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    fp = ctypes.CDLL(os.path.join(root, "tests", "_build", "libfault_probe.so"))
    u32, u64 = ctypes.c_uint32, ctypes.c_uint64
    fp.hg_fault_probe_pointer.argtypes = [u64, ctypes.POINTER(u32), ctypes.POINTER(u64),
                                          ctypes.POINTER(u64), ctypes.POINTER(u64)]
    fp.hg_fault_probe_svm.argtypes = [u64, u64] + [ctypes.POINTER(u64)] * 3
    assert fp.hg_fault_probe_install() == 0

    def rocr(p):
        t, hb, ab, nb = u32(), u64(), u64(), u64()
        rc = fp.hg_fault_probe_pointer(p, ctypes.byref(t), ctypes.byref(hb), ctypes.byref(ab),
                                       ctypes.byref(nb))
        acc, ro, gf = u64(), u64(), u64()
        src = fp.hg_fault_probe_svm(p // 4096 * 4096, 4096, ctypes.byref(acc), ctypes.byref(ro),
                                    ctypes.byref(gf))
        return {"rc": rc, "type": t.value, "host_base": hex(hb.value), "agent_base": hex(ab.value),
                "bytes": hex(nb.value), "svm_rc": src, "svm_access": hex(acc.value),
                "svm_read_only": ro.value, "svm_global_flag": gf.value}

    n = 200_003  # 6.4 MB of src: HIP pins its copies in place (>= 2 MB)
    ds = pkg.fill_uniform(n * 8, 3, 0, device=dev).view(n, 8)
    dt = pkg.fill_uniform(n * 8, 3, n * 8, device=dev).view(n, 8)
    want = pkg.solve("aca", ds, dt).cpu()
    recs = []
    keep = []
    src, tar = None, None

    def step(tag, fn):
        print(f"--- {tag}", file=sys.stderr, flush=True)
        fn()
        torch.cuda.synchronize()
        rec = {"step": tag, "src_hip_kind": kind(src.data_ptr()),
               "rocr_src": rocr(src.data_ptr()), "rocr_src_slice": rocr(src[1000].data_ptr()),
               "rocr_tar": rocr(tar.data_ptr())}
        print(json.dumps(rec), flush=True)
        recs.append(rec)

    def d2h():
        nonlocal src, tar
        src, tar = ds.cpu(), dt.cpu()

    step("D2H into fresh src, tar (HIP pins their pages for the copy)", d2h)
    step("library solve_host on slices inside those pages (registers, releases)",
         lambda: keep.append(pkg.solve_host("aca", src[1000:150_000], tar[1000:150_000])))
    # no further GPU access to src / tar: if the release above took HIP's pin with it, HIP's
    # next copy through that pin would fault -- the ROCr queries answer without one
    ok = torch.equal(keep[0], want[1000:150_000])
    recs.append({"solve_host_bits_equal_device_solve": bool(ok)})
    print(json.dumps(recs[-1]), flush=True)

    # registration and release alone (no GPU access), against a fresh HIP copy pin each time:
    # the same page range, a range inside it, a range around it
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    page = 4096
    for case in ("same range", "inside", "around"):
        x = ds.cpu()  # fresh pageable memory: HIP pins it for the copy
        keep.append(x)
        lo, hi = x.data_ptr() // page * page, -(-(x.data_ptr() + x.numel() * 4) // page) * page
        pin = rocr(x.data_ptr())
        if case == "same range":
            r_lo, r_hi = int(pin["host_base"], 16), int(pin["host_base"], 16) + int(pin["bytes"], 16)
        elif case == "inside":
            r_lo, r_hi = lo + 16 * page, hi - 16 * page
        else:
            r_lo, r_hi = lo - 4 * page, hi + 4 * page  # the neighbours' pages too (heap)
        rc_r = hip.hipHostRegister(r_lo, r_hi - r_lo, 3)
        during = rocr(x.data_ptr() + 20 * page)
        rc_u = hip.hipHostUnregister(r_lo)
        hip.hipGetLastError()
        rec = {"case": case, "pin_before": pin, "registered": [hex(r_lo), hex(r_hi - r_lo), rc_r],
               "during": during, "unregister_rc": rc_u, "after": rocr(x.data_ptr() + 20 * page)}
        print(json.dumps(rec), flush=True)
        recs.append(rec)

    # pages no HIP copy ever touched: CPU-filled memory, registered and released directly
    y = torch.arange(2_000_000, dtype=torch.float32) + 1  # 8 MB, written by the CPU only
    keep.append(y)
    y_lo = -(-y.data_ptr() // page) * page
    y_n = (y.numel() * 4 - page) // page * page
    before = rocr(y_lo + 8 * page)
    rc_r = hip.hipHostRegister(y_lo, y_n, 3)
    during = rocr(y_lo + 8 * page)
    rc_u = hip.hipHostUnregister(y_lo)
    hip.hipGetLastError()
    rec = {"case": "fresh CPU pages, register + unregister", "before": before,
           "register_rc": rc_r, "during": during, "unregister_rc": rc_u,
           "after": rocr(y_lo + 8 * page)}
    print(json.dumps(rec), flush=True)
    recs.append(rec)
    # the same through the library: a batch whose src / tar / H are CPU-filled pages
    m = 100_000
    s2 = src[:m].clone()
    t2 = tar[:m].clone()
    h2 = torch.full((m, 9), float("nan"))
    keep += [s2, t2, h2]
    b2 = {"src": rocr(s2.data_ptr() + 8 * page), "H": rocr(h2.data_ptr() + 8 * page)}
    pkg.solve_host("aca", s2, t2, out=h2)
    rec = {"case": "library solve_host on CPU-filled pages", "before": b2,
           "after": {"src": rocr(s2.data_ptr() + 8 * page), "H": rocr(h2.data_ptr() + 8 * page)},
           "bits_equal": bool(torch.equal(h2, want[:m]))}
    print(json.dumps(rec), flush=True)
    recs.append(rec)
    return recs


if __name__ == "__main__":
    main()
