#!/usr/bin/env python3
"""Per-kernel PMC summary for the LBA engine (profiles/r02_schur_pmc.json): from separate rocprofv3
--pmc passes over `tools/lba_batch_bench.py` (B = 64 windows), the per-launch averages of the
largest-grid launches of each kernel, with
  mfma_busy_frac       = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x launch duration x clock)
  hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B; gfx950 FETCH_SIZE half-count,
                         MI355X_MICROARCH.md HBM/rocprofv3 section)
    python3 tools/pmc_kernel_summary.py OUT.json SQ.csv [FETCH.csv WRITE.csv]"""
import collections
import csv
import json
import re
import sys

SIMDS = 256 * 4
CLOCK_GHZ = 2.4


def short(name):
    m = re.search(r"(k_[a-z0-9_]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name


def load(path):
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        grid = int(r["Grid_Size"].split(",")[0]) if r["Grid_Size"].split(",")[0].isdigit() else 0
        by[(k, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[(k, grid)][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for (k, grid), d in by.items():
        prev = out.get(k)
        if prev and prev["grid"] >= grid:
            continue
        ds = list(dur[(k, grid)].values())
        out[k] = {"grid": grid, "launches": len(ds), "duration_us": 1e6 * sum(ds) / len(ds),
                  "counters": {c: sum(v) / len(v) for c, v in d.items()}}
    return out


def main():
    out_path, sq = sys.argv[1], sys.argv[2]
    res = load(sq)
    extra = [load(p) for p in sys.argv[3:5]]
    summary = {}
    for k, v in res.items():
        c = v["counters"]
        e = {"grid": v["grid"], "launches": v["launches"], "duration_us": round(v["duration_us"], 2),
             "counters": {n: round(x, 1) for n, x in c.items()}}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and v["duration_us"] > 0:
            e["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * v["duration_us"] * 1e3 * CLOCK_GHZ), 5)
        if len(extra) == 2 and k in extra[0] and k in extra[1]:
            f = extra[0][k]["counters"].get("FETCH_SIZE")
            w = extra[1][k]["counters"].get("WRITE_SIZE")
            if f is not None and w is not None:
                e["hbm_bytes_per_launch"] = round((2 * f + w) * 1024)
        summary[k] = e
    summary["_note"] = ("rocprofv3 --pmc passes (counters only) over tools/lba_batch_bench.py TS=1 BS=64; per kernel "
                        "the largest-grid launches (64 windows); durations are profiled-clock launch times")
    json.dump(summary, open(out_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
