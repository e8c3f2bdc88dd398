#!/usr/bin/env python3
"""VALU issue utilisation of a kernel from one rocprofv3 --pmc pass (no traces in that pass):

    rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
        --output-format csv -d DIR -o valu -- python3 bench.py ...
    python tools/pmc_valu.py DIR/.../valu_counter_collection.csv k_top2_batch out.json

Per launch of the kernel (averaged over its launches):
  * kernel_cycles  = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs; MI355X_MICROARCH.md, DVFS note)
  * simd_cycles    = kernel_cycles x 1024 SIMDs (256 CUs x 4)
  * cycles_per_valu_inst = simd_cycles / SQ_INSTS_VALU: what one wave-instruction cost a SIMD when the
    kernel keeps every SIMD issuing VALU; 4.0 = 16 lanes / clk, 2.0 = the guide's 32 lanes / clk
  * valu_issue_util_16 = 4 SQ_INSTS_VALU / simd_cycles (1.0 = every SIMD issuing a wave64 VALU
    instruction every 4 cycles), valu_issue_util_32 = the same at 2 cycles per instruction
  * valu_active_frac = 4 SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES x 4 (quad-cycle counters): the share of
    the waves' lifetime spent in VALU instructions
  * eff_clock_ghz = kernel_cycles / kernel duration (the dispatch's own timestamps)
"""
import csv
import json
import sys
from collections import defaultdict

SIMDS = 256 * 4


def main():
    path, substr, out_path = sys.argv[1], sys.argv[2], sys.argv[3]
    by = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if substr not in name:
                continue
            key = f"{name}|grid={row.get('Grid_Size', '?')}"
            by[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
            if row["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur[key].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    out = {}
    for key, c in by.items():
        m = {k: sum(v) / len(v) for k, v in c.items()}
        n = len(c.get("SQ_INSTS_VALU", []))
        kc = m["GRBM_GUI_ACTIVE"] / 8.0
        sc = kc * SIMDS
        d_ns = sum(dur[key]) / len(dur[key]) if dur[key] else None
        r = {"launches": n, "counters_mean": m, "kernel_cycles": kc, "simd_cycles": sc,
             "kernel_ns": d_ns, "eff_clock_ghz": (kc / d_ns) if d_ns else None,
             "cycles_per_valu_inst": sc / m["SQ_INSTS_VALU"],
             "valu_issue_util_16": 4.0 * m["SQ_INSTS_VALU"] / sc,
             "valu_issue_util_32": 2.0 * m["SQ_INSTS_VALU"] / sc}
        if "SQ_ACTIVE_INST_VALU" in m and m.get("SQ_WAVE_CYCLES"):
            r["valu_active_frac"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]
        if "SQ_BUSY_CYCLES" in m:
            r["sq_busy_frac"] = m["SQ_BUSY_CYCLES"] / kc
        out[key] = r
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    for k, r in out.items():
        print(json.dumps({"kernel": k[:80], "cycles_per_valu_inst": round(r["cycles_per_valu_inst"], 3),
                          "valu_issue_util_16": round(r["valu_issue_util_16"], 4),
                          "eff_clock_ghz": r["eff_clock_ghz"]}))


if __name__ == "__main__":
    main()
