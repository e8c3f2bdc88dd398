#!/usr/bin/env python3
"""Per-launch means of the counters in a tools/gpu/top2_pmc.sh output directory for one kernel.
    python tools/pmc_top2_summary.py gpurun_out/DIR k_top2_mfma [out.json]"""
import collections
import csv
import glob
import json
import sys


def main():
    d, sub = sys.argv[1], sys.argv[2]
    res = {}
    for f in sorted(glob.glob(f"{d}/*/*_counter_collection.csv")):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            res[k] = sum(v) / len(v)
    kc = res.get("GRBM_GUI_ACTIVE", 0) / 8.0
    out = {"kernel": sub, "counters_mean_per_launch": res, "kernel_cycles": kc}
    if kc:
        simd = kc * 1024
        if "SQ_VALU_MFMA_BUSY_CYCLES" in res:
            out["mfma_busy_frac"] = res["SQ_VALU_MFMA_BUSY_CYCLES"] / simd
        for k in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_ADDR_CONFLICT", "SQ_LDS_DATA_FIFO_FULL",
                  "SQ_LDS_CMD_FIFO_FULL", "SQ_BUSY_CU_CYCLES"):
            if k in res:
                out[k + "_per_cu_frac"] = res[k] / 256 / kc
        if "SQ_WAVE_CYCLES" in res:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_VALU"):
                if k in res:
                    out[k + "_of_wave_cycles"] = res[k] / res["SQ_WAVE_CYCLES"]
    for k in ("FETCH_SIZE", "WRITE_SIZE"):
        if k in res:
            out[k + "_bytes"] = res[k] * 1024 * (2 if k == "FETCH_SIZE" else 1)
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s)
    print(s)


if __name__ == "__main__":
    main()
