"""Child process of tests/test_gpu_host_nomap.py (test infrastructure; run as a program).

Runs with HIP's default copy policy -- GPU_PINNED_MIN_XFER_SIZE unset, unlike the test
process -- and touches the GPU only through the library's C ABI (ctypes on
libsks_homography_amd.so, no torch):

1. hg_solve_host_f32/_f64 on fresh pageable numpy buffers of 256 KiB, 2 MB and 64 MB per
   input, AoS and SoA: H's bits against the oracle, read from the caller's own buffer on the
   CPU (no HIP copy), and KFD's attribute of every page of src, tar and H after the call
   (tests/fault_probe.c hg_fault_probe_svm_pages): 0x202, no GPU access, as before the call.
2. The ADVICE r05 sequence: those buffers freed, the same sizes allocated again (malloc and
   mmap hand the pages back), and HIP's own in-place device-to-host copy of 2 MB and 64 MB
   into them -- data checked, the device synchronised, no fault event.
3. A positive control, last (its pages are never reused): one HG_FLAG_HOST_REGISTER call, whose
   pages KFD keeps mapped after the unregistration -- the count shows the probe sees mappings.

Prints one JSON line; exits 0 only when every check of 1 and 2 holds.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as orc  # noqa: E402  (the checker)

NO_ACCESS = 0x202
PAGE = 4096


def main():
    out = {"knob": os.environ.get("GPU_PINNED_MIN_XFER_SIZE"), "cases": [], "ok": False}
    if out["knob"] is not None:
        print(json.dumps(out))
        return 2
    lib = ctypes.CDLL(os.path.join(ROOT, "sks-homography_amd", "lib", "libsks_homography_amd.so"))
    vp, i64, cint = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    for f in ("hg_solve_host_f32", "hg_solve_host_f64"):
        getattr(lib, f).argtypes = [cint, vp, vp, vp, i64, cint, cint, vp]
        getattr(lib, f).restype = cint
    fp = ctypes.CDLL(os.path.join(ROOT, "tests", "_build", "libfault_probe.so"))
    u64 = ctypes.c_uint64
    fp.hg_fault_probe_svm_pages.argtypes = [u64, u64, u64, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    fp.hg_fault_probe_svm_pages.restype = ctypes.c_int64
    fp.hg_fault_probe_read.argtypes = [ctypes.POINTER(cint), ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_uint32)]
    assert fp.hg_fault_probe_install() == 0
    hip = ctypes.CDLL("libamdhip64.so")
    o = orc.Oracle()

    def mapped(a):
        """Pages of array `a` whose first-GPU access is not 'no access'."""
        bad_va, bad_acc = u64(), u64()
        k = fp.hg_fault_probe_svm_pages(a.ctypes.data, a.nbytes, PAGE, NO_ACCESS,
                                        ctypes.byref(bad_va), ctypes.byref(bad_acc))
        assert k >= 0, f"SVM query failed ({k})"
        return int(k), bad_va.value, bad_acc.value

    sizes = {"256KiB": 256 << 10, "2MB": 2 << 20, "64MB": 64 << 20}
    keep = []
    ok = True
    for dt in (np.float32, np.float64):
        fn = lib.hg_solve_host_f32 if dt == np.float32 else lib.hg_solve_host_f64
        for layout in ("aos", "soa"):
            for label, nbytes in sizes.items():
                n = nbytes // (8 * np.dtype(dt).itemsize)
                s = o.fill_uniform(n * 8, 11, 0).reshape(n, 8).astype(dt)
                t = o.fill_uniform(n * 8, 11, n * 8).reshape(n, 8).astype(dt)
                if layout == "soa":
                    s, t = np.ascontiguousarray(s.T), np.ascontiguousarray(t.T)
                H = np.full((9, n) if layout == "soa" else (n, 9), np.nan, dtype=dt)
                before = [mapped(x)[0] for x in (s, t, H)]
                for algo, aid in (("aca", 0), ("sks", 1)):
                    if algo == "sks" and label != "2MB":
                        continue
                    rc = fn(aid, s.ctypes.data, t.ctypes.data, H.ctypes.data, n,
                            0 if layout == "aos" else 1, 1, None)
                    want = o.solve(algo, s, t, normalize=True, layout=layout)
                    bits = bool(rc == 0 and np.array_equal(H.view(np.uint8), want.view(np.uint8)))
                    after = [mapped(x) for x in (s, t, H)]
                    case = {"dtype": np.dtype(dt).name, "layout": layout, "size": label, "algo": algo,
                            "n": n, "rc": rc, "bits": bits, "mapped_before": before,
                            "mapped_after": [a[0] for a in after],
                            "first_mapped": [hex(a[1]) if a[0] else None for a in after]}
                    out["cases"].append(case)
                    ok &= bits and all(a[0] == 0 for a in after)
                keep.append((s, t, H))
    # 2: free, reallocate, HIP's own in-place device-to-host copies into the reused pages
    del keep, s, t, H
    reuse = []
    dptr = ctypes.c_void_p()
    big = 64 << 20
    assert hip.hipMalloc(ctypes.byref(dptr), ctypes.c_size_t(big)) == 0
    assert hip.hipMemset(dptr, 0x3F, ctypes.c_size_t(big)) == 0
    for nbytes in (2 << 20, 64 << 20, 2 << 20, 64 << 20):
        dst = np.zeros(nbytes, np.uint8)
        rc = hip.hipMemcpy(ctypes.c_void_p(dst.ctypes.data), dptr, ctypes.c_size_t(nbytes), 2)  # D2H
        reuse.append({"bytes": nbytes, "rc": rc, "data": bool(rc == 0 and (dst == 0x3F).all())})
        ok &= reuse[-1]["data"]
        del dst
    sync = hip.hipDeviceSynchronize()
    t_, va_, why_ = cint(), u64(), ctypes.c_uint32()
    events = fp.hg_fault_probe_read(ctypes.byref(t_), ctypes.byref(va_), ctypes.byref(why_))
    out["reuse_copies"] = reuse
    out["sync_rc"], out["fault_events"] = sync, events
    ok &= sync == 0 and events == 0
    hip.hipFree(dptr)
    # 3: the positive control (HG_FLAG_HOST_REGISTER = 2), pages kept until exit
    n = (2 << 20) // 32
    cs = o.fill_uniform(n * 8, 11, 0).reshape(n, 8)
    ct = o.fill_uniform(n * 8, 11, n * 8).reshape(n, 8)
    cH = np.empty((n, 9), np.float32)
    rc = lib.hg_solve_host_f32(0, cs.ctypes.data, ct.ctypes.data, cH.ctypes.data, n, 0, 1 | 2, None)
    out["control_register"] = {"rc": rc, "mapped_after": [mapped(x)[0] for x in (cs, ct, cH)],
                               "pages": [x.nbytes // PAGE for x in (cs, ct, cH)]}
    ok &= rc == 0
    out["ok"] = bool(ok)
    print(json.dumps(out))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
