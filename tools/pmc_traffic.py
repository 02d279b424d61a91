"""HBM traffic per launch from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> [out.json]

Corrections (MI355X_MICROARCH.md "HBM" + cdna_hip_programming.md section 7):
  * both counters are in KiB -> x1024;
  * on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read
    -> x2.  Verified here on hg::stream_copy_kernel, whose byte count is known
    exactly: the x2-corrected fetch must equal the bytes copied (check printed and
    stored as "calibration");
  * WRITE_SIZE reads exact for 16-B-per-lane streaming stores.
Counters were collected in separate passes (FETCH_SIZE and WRITE_SIZE cannot share
one), with no tracing domains, as the guide prescribes.
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import statistics
import sys

M10, M16 = 10_000_000, 16 * 1024 * 1024
# key: (a substring of the kernel name -- every kernel containing it counts --, algorithmic
# bytes per launch at the pmc_run.py size, or None).  Each key names the figure bench.py
# quotes beside it (a section's `frac`); the layout-floor bytes of the (B,3,4) contract are
# bench's RECT_LAYOUT_MIN_BYTES.
KEYS = {
    "aca_f32_aos_norm": ("void hg::solve_aos<0, true, float", M10 * 100),
    "sks_f32_aos_norm": ("void hg::solve_aos<1, true, float", M10 * 100),
    "stream_copy": ("hg::stream_copy_kernel", None),
    "aca_f64_aos_norm": ("void hg::solve_aos<0, true, double", M10 * 200),
    "aca_f64_soa": ("void hg::solve_soa_narrow<0, false, double, 8, true>", M10 * 200),
    "sks_f64_soa": ("void hg::solve_soa_narrow<1, false, double, 8, true>", M10 * 200),
    "aca_vanilla_backward": ("void hg::aca_vanilla_backward_staged<true, true, true>", M16 * 164),
    # (B,3,4) contract: tar 48 + src M 8 + H 36 (the 8 B of src sit in 32-B sectors)
    "tensor_aca_rect": ("void hg::tensor_aca_rect_kernel", M16 * 92),
    "tensor_aca_rect_bcast": ("void hg::tensor_aca_rect_bcast_staged<true, 0>", M16 * 100),
    # dL/dtar alone: src M 8 + tar 48 + dL/dH 36 in, dL/dtar 48 out
    "rect_backward_tar": ("void hg::tensor_aca_rect_backward_staged<false, 0, true, 0, false>", M16 * 140),
    "aten_sum_l1": ("hg::aten_sum_l1", None),
    # the fused all-gradient backward (round 6): no terms out, the sum's level 0 in LDS
    "rect_backward_sum": ("void hg::rect_backward_sum_l0<true, true>", M16 * 188),
    "tensor_aca_offsets": ("void hg::tensor_aca_offsets_kernel", M16 * 76),
    # corner 8 + offsets 32 + dL/dH 36 in, dL/doffsets 32 out
    "offsets_backward": ("void hg::tensor_aca_offsets_backward_staged<false, true>", M16 * 108),
    # 16 B of indices + 36 B of H per hypothesis (the pool stays in LDS)
    "sample_solve_indexed": ("void hg::sample_solve_lds_kernel<0, true, 2, 1", M16 * 52),
    "sample_solve_seeded": ("void hg::sample_solve_lds_kernel<0, true, 2, 0, 4, 1", M16 * 36),
    "gather_solve_f64_aca": ("void hg::gather_solve_f64_kernel<0", M10 * 88),
    "mrg_words": ("hg::mrg_words_kernel<0>", 40_000_000 * 4),
    "rand_gather_solve_f64_aca": ("void hg::mrg_gather_solve_f64_kernel<0, false, true, 320", M10 * 72),
    "rand_gather_solve_f64_sks": ("void hg::mrg_gather_solve_f64_kernel<1, false, true, 320", M10 * 72),
}


def load(d):
    path = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        per[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return per


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    out_path = sys.argv[3] if len(sys.argv) > 3 else None
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "sks-homography_amd"))
    import build_lib
    res = {}
    for key, (prefix, algo_bytes) in KEYS.items():
        groups = sorted({g for (k, g) in fetch if prefix in k})
        for g in groups:
            f = [v for (k, gg), vs in fetch.items() if prefix in k and gg == g for v in vs]
            w = [v for (k, gg), vs in write.items() if prefix in k and gg == g for v in vs]
            if not f or not w:
                continue
            fb = statistics.median(f) * 1024 * 2
            wb = statistics.median(w) * 1024
            name = key if len(groups) == 1 else f"{key}@grid{g}"
            res[name] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                         "fetch_kib_raw": statistics.median(f), "write_kib_raw": statistics.median(w),
                         "launches": len(f), "grid": g, "prefix": prefix,
                         "kernels": sorted({k for (k, gg) in fetch if prefix in k and gg == g}),
                         # the machine code measured: bench.py quotes the figure only while
                         # the library it runs holds the same code for this family
                         "code": build_lib.kernel_family_digest(prefix)}
            if algo_bytes:
                res[name]["algorithmic_bytes"] = algo_bytes
                res[name]["traffic_over_algorithmic"] = round((fb + wb) / algo_bytes, 4)
    # calibration on the copy kernel: bytes copied == bytes written (exact counter)
    cp = next((v for k, v in res.items() if k.startswith("stream_copy")), None)
    if cp:
        cp["calibration"] = {"fetch_x2_over_written": round(cp["fetch_bytes"] / cp["write_bytes"], 4)}
    # flat per-launch numbers bench.py reads
    flat = {k: round(v["hbm_bytes"]) for k, v in res.items() if k in ("aca_f32_aos_norm",
                                                                      "sks_f32_aos_norm")}
    doc = dict(flat)
    doc["detail"] = res
    # provenance: which run, and the kernels it was measured on -- the gfx950 machine code of
    # the headline entry points in the library that ran (reduce right after the run, before
    # rebuilding); bench.py reports the figure only while the library still holds that code
    # (tests/test_capi.py checks), the source digest is kept for reference
    doc["provenance"] = {
        "pmc_run": {"fetch_dir": sys.argv[1], "write_dir": sys.argv[2],
                    "tag": os.environ.get("PMC_TAG", "")},
        "kernel_code": build_lib.kernel_code_digest(),
        "compiler": build_lib.compiler_id(),
        "sources_aos": build_lib.sources_digest("aos"),
    }
    doc["method"] = ("rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, csv; "
                     "bytes = KiB*1024, FETCH x2 (gfx950 wide-read correction, calibrated on "
                     "stream_copy); median over the launches of `python3 tools/pmc_run.py` (each kernel 5x at "
                     "its bench size)")
    print(json.dumps(doc, indent=1))
    if out_path:
        with open(out_path, "w") as fh:
            json.dump(doc, fh, indent=1)


if __name__ == "__main__":
    main()
