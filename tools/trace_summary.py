#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 --kernel-trace csv, including the last-N window
(the back-to-back launches bench.py brackets with HIP events), for comparing with bench.py's
roofline.kernel_us.

    python tools/trace_summary.py kernel_trace.csv out.json [substr=N ...]
"""
import csv
import json
import sys

import numpy as np


def main():
    path, out = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    res = {}
    for spec in sys.argv[3:]:
        sub, n = spec.split("=")
        n = int(n)
        sel = [r for r in rows if sub in r["Kernel_Name"]]
        d = np.array([int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel]) / 1e3
        res[sub] = {
            "launches": int(d.size), "mean_us": float(d.mean()), "median_us": float(np.median(d)),
            "min_us": float(d.min()), f"last_{n}_mean_us": float(d[-n:].mean()),
            f"last_{n}_median_us": float(np.median(d[-n:])),
            "kernel_name": sel[0]["Kernel_Name"][:120], "grid": sel[0].get("Grid_Size_X"),
            "vgpr": sel[0].get("VGPR_Count"), "lds": sel[0].get("LDS_Block_Size"),
            "scratch": sel[0].get("Scratch_Size"),
        }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
