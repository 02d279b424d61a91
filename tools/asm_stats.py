"""Per-kernel instruction census of a hipcc -S output (FMA contraction, division
sequences, vector memory ops).  Usage: python tools/asm_stats.py file.s [substr]"""
import re
import sys

text = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
parts = re.split(r"\n(?=_Z\w+:\s*;)", text)
pats = {
    "fma": r"\bv_(?:pk_)?fma(?:c|mk|ak)?_f(?:32|64)\b",
    "div_scale": r"\bv_div_scale_f(?:32|64)\b",
    "rcp": r"\bv_rcp_f(?:32|64)\b",
    "ld_x4": r"\bglobal_load_dwordx4\b",
    "ld_x2": r"\bglobal_load_dwordx2\b",
    "ld_x1": r"\bglobal_load_dword\b",
    "st_x4": r"\bglobal_store_dwordx4\b",
    "st_x1": r"\bglobal_store_dword\b",
    "ds_w": r"\bds_write",
    "ds_r": r"\bds_read",
    "pk": r"\bv_pk_\w+",
    "nt": r"\bnt\b",
}
for part in parts:
    m = re.match(r"(_Z\w+):", part)
    if not m or flt not in m.group(1):
        continue
    body = part.split(".Lfunc_end")[0]
    vg = re.search(r"\.vgpr_count:\s+(\d+)", text[text.find(m.group(1) + ":"):])
    stats = {k: len(re.findall(p, body)) for k, p in pats.items()}
    print(m.group(1)[:70], " ".join(f"{k}={v}" for k, v in stats.items()))
