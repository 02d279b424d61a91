"""Per-dispatch-group kernel durations from a rocprofv3 SQLite trace (rocpd `kernels` view):
consecutive dispatches of one kernel with one grid form a group; prints count, median and
min duration (us).   python tools/prof_db.py gpurun_out/prof_x/run_results.db [substring]"""
import sqlite3
import sys


def groups(db, sub=""):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end, grid_x, grid_y, workgroup_x from kernels "
                          "order by start"))
    out, prev, cur = [], None, []
    for r in rows:
        if sub not in r[0]:
            continue
        key = (r[0], r[3], r[4], r[5])
        if key != prev and cur:
            out.append((prev, cur))
            cur = []
        prev = key
        cur.append((r[2] - r[1]) / 1000.0)
    if cur:
        out.append((prev, cur))
    return out


if __name__ == "__main__":
    for (name, gx, gy, wg), d in groups(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""):
        d = sorted(d)
        print(f"{name[:60]:60s} grid {gx}x{gy} wg {wg}: n={len(d)} median {d[len(d) // 2]:.2f} "
              f"min {d[0]:.2f} us")
