"""Workload for a translation-cache PMC pass (tools/gpu_round.sh pmc_tlb): the headline kernel
over 10 M problems (1 GB, repeated on the same buffers) and over 20 M (2 GB), 10 launches
each, nothing else.  The 2 GB sweep runs ~5 % slower per byte (profiles/r02/chunk_probe.json);
counting UTCL1 misses and UTCL2 busy cycles per launch says whether address translation is
why.  Reduced by the same script with `--reduce <counter_collection.csv>`."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run():
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    dev = torch.device("cuda:0")
    for n in (10_000_000, 20_000_000):
        src = pkg.fill_uniform(n * 8, 11, 0, device=dev).view(n, 8)
        tar = pkg.fill_uniform(n * 8, 11, n * 8, device=dev).view(n, 8)
        H = torch.empty((n, 9), device=dev)
        for _ in range(10):
            pkg.solve("aca", src, tar, out=H)
        torch.cuda.synchronize()
        del src, tar, H
    print("pmc tlb workload done")


def reduce(path):
    rows = [r for r in csv.DictReader(open(path)) if "solve_aos" in r.get("Kernel_Name", "")]
    per = {}
    for r in rows:
        key = (r["Dispatch_Id"], r["Grid_Size"])
        per.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    out = {}
    for (_, grid), c in per.items():
        out.setdefault(grid, []).append(c)
    res = {}
    for grid, lst in out.items():
        keys = sorted(set().union(*lst))
        res[grid] = {k: sorted(x[k] for x in lst)[len(lst) // 2] for k in keys}
    print(json.dumps(res, indent=1))
    return res


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--reduce":
        res = reduce(sys.argv[2])
        if len(sys.argv) > 3:
            json.dump(res, open(sys.argv[3], "w"), indent=1)
    else:
        run()
