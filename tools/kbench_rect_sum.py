"""The TensorACA all-gradient backward at B = 16 M three ways (hg_rect_sum.hpp): the op
(fused kernel + the sum's upper levels), the fused kernel alone, and the round-5 two-launch
form (terms kernel + hg_sum_aten_f32), best of 5 x 20 calls each; bits compared.

    python tools/kbench_rect_sum.py [--out gpurun_out/kbench_rect_sum.json]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402


def time_us(fn, reps=20, tries=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(tries):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/kbench_rect_sum.json")
    ap.add_argument("--B", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--T", type=int, default=16)
    a = ap.parse_args()
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    B, T = a.B, a.T
    torch.manual_seed(0)
    _, _, bs, bt, sc, dv = pkg.adjust(dev, B)
    gH = torch.randn(B, 3, 3, device=dev)
    gs, gt = torch.empty_like(bs), torch.empty_like(bt)
    ws = torch.empty(6 * B, device=dev)
    sd = torch.empty(2, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    lib = pkg.lib()
    lib.hg_internal_rect_backward_sum_l0.argtypes = ([ctypes.c_void_p] * 3 + [ctypes.c_int64]
                                                     + [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p])
    f_l0 = lambda: lib.hg_internal_rect_backward_sum_l0(  # noqa: E731
        bs.data_ptr(), bt.data_ptr(), gH.data_ptr(), B, sc.data_ptr(), dv.data_ptr(), gs.data_ptr(),
        gt.data_ptr(), ws.data_ptr(), 8, T, st)
    f_fused = lambda: pkg._lib.call(  # noqa: E731
        "hg_tensor_aca_rect_backward_sum_f32", bs.data_ptr(), bt.data_ptr(), gH.data_ptr(), B,
        sc.data_ptr(), dv.data_ptr(), gs.data_ptr(), gt.data_ptr(), ws.data_ptr(), 8, T, sd.data_ptr(), st)

    def f_two():
        pkg._lib.call("hg_tensor_aca_rect_backward_terms_f32", bs.data_ptr(), bt.data_ptr(), gH.data_ptr(),
                      B, sc.data_ptr(), dv.data_ptr(), gs.data_ptr(), gt.data_ptr(), ws.data_ptr(), st)
        pkg._lib.call("hg_sum_aten_f32", ws.data_ptr(), 2, 3 * B, 3 * B, 1, 8, T, sd.data_ptr(), st)

    f_op = lambda: pkg.tensor_aca_rect_backward(bs, bt, gH, sc, dv, True, True, aten_threads=T)  # noqa: E731
    out = {"B": B, "T": T}
    f_two()
    ref = (gs.clone(), gt.clone(), sd.clone())
    f_fused()
    out["bit_exact"] = bool(torch.equal(gs.view(torch.int32), ref[0].view(torch.int32))
                            and torch.equal(gt.view(torch.int32), ref[1].view(torch.int32))
                            and torch.equal(sd.view(torch.int32), ref[2].view(torch.int32)))
    lib.hg_internal_rect_sum_config.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    prev = (ctypes.c_int * 2)()
    lib.hg_internal_rect_sum_config(-1, -1, prev)
    sweep = []
    for budget in (1024, 2048, 4096):
        for gdma in (0,):
            assert lib.hg_internal_rect_sum_config(budget, gdma, None) == 0
            f_fused()
            ok = bool(torch.equal(gt.view(torch.int32), ref[1].view(torch.int32))
                      and torch.equal(sd.view(torch.int32), ref[2].view(torch.int32)))
            sweep.append({"budget": budget, "gdma": gdma, "l0_us": round(time_us(f_l0), 2),
                          "fused_us": round(time_us(f_fused), 2), "bit_exact": ok})
            print(json.dumps(sweep[-1]), flush=True)
    lib.hg_internal_rect_sum_config(prev[0], prev[1], None)
    out["sweep"] = sweep
    for name, fn in (("l0_kernel_us", f_l0), ("fused_cabi_us", f_fused), ("two_launch_us", f_two),
                     ("op_us", f_op)):
        out[name] = round(time_us(fn), 2)
    out["op_over_kernel"] = round(out["op_us"] / out["l0_kernel_us"], 4)
    out["fused_frac_188"] = round(B * 188 / (out["op_us"] * 1e-6) / 8e12, 4)
    print(json.dumps(out))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
