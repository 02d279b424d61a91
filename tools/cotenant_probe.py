"""Does hipMemGetInfo count another process's device memory?  (tests/test_gpu_large.py)

A child process allocates GB_OTHER GB on cuda:0 and holds it; this process (which allocates
nothing large) then prints torch.cuda.mem_get_info beside the driver's card-wide
mem_info_vram_used.  Nothing here allocates past the card.  Answer (r04,
profiles/r04/cotenant_probe_r04w.json): yes -- with 150 GB held by the child, HIP's free
figure drops by 150 GB, so the >2^31 tests' free-memory check already sees other processes.  Run on the GPU box: python tools/cotenant_probe.py [GB_OTHER]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def holder(gb):
    import torch
    x = torch.empty(int(gb) << 30, dtype=torch.uint8, device="cuda:0")
    x.fill_(1)
    torch.cuda.synchronize()
    print("held", flush=True)
    time.sleep(float(os.environ.get("HOLD_S", "40")))
    del x


def card_used():
    """The driver's card-wide VRAM in use (what rocm-smi shows) for the first card, or None."""
    import glob
    for path in sorted(glob.glob("/sys/class/drm/card*/device/mem_info_vram_used")):
        try:
            with open(path) as f:
                return int(f.read())
        except (OSError, ValueError):
            continue
    return None


def main():
    gb = int(sys.argv[1]) if len(sys.argv) > 1 else 150
    import torch
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    out = {"before": {"hip_free": torch.cuda.mem_get_info(dev)[0], "card_used": card_used()}}
    p = subprocess.Popen([sys.executable, __file__, "--hold", str(gb)], stdout=subprocess.PIPE,
                         text=True)
    line = p.stdout.readline()
    out["holder"] = line.strip()
    time.sleep(1.0)
    out["during"] = {"hip_free": torch.cuda.mem_get_info(dev)[0], "card_used": card_used(),
                     "total": torch.cuda.mem_get_info(dev)[1], "other_gb": gb}
    p.wait(timeout=120)
    out["holder_rc"] = p.returncode
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--hold":
        holder(sys.argv[2])
    else:
        main()
