#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 kernel trace written as a rocpd SQLite database (the default
output format of `rocprofv3 --kernel-trace --stats -d DIR -o NAME`): one CSV row per (kernel, grid)
with calls, total / average / min / max duration in microseconds.

    python3 tools/rocpd_stats.py gpurun_out/r02a/prof/prof_results.db > profiles/r02_kernel_stats.csv
"""
import csv
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    depth, out = 0, []
    for ch in name:  # drop the parameter list, keep template arguments
        if ch == "(" and depth == 0 and out and not "".join(out).endswith("operator"):
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).replace("void ", "").strip()


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, duration, vgpr_count, lds_size "
                     "from kernels").fetchall()
    agg = {}
    for name, gx, gy, gz, wx, dur, vgpr, lds in rows:
        k = (short(name), gx, gy, gz, wx, vgpr, lds)
        agg.setdefault(k, []).append(dur / 1e3)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid_x", "grid_y", "grid_z", "workgroup_x", "vgpr", "lds_bytes", "calls", "total_us",
                "avg_us", "min_us", "max_us"])
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        w.writerow(list(k) + [len(v), round(sum(v), 3), round(sum(v) / len(v), 3), round(min(v), 3),
                              round(max(v), 3)])


if __name__ == "__main__":
    main(sys.argv[1])
