#!/usr/bin/env python3
"""Global-BA A/B probe (bench infrastructure): wall time per call and the per-kernel device time
(osg_lba_kernel_times) of Optimizer::BundleAdjustment on bench.py's maps -- a 150-KF map and the
1500-KF loop-closed map -- with whichever library OSG_LIB_PATH selects.  One JSON line per map.

    python tools/gba_kernel_probe.py [--label cur]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_comments_ghr_amd import Context, optimizer as op  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default=os.environ.get("OSG_LIB_PATH", "cur"))
    a = ap.parse_args()
    maps = [("gba150", op.synth_gba_graph(np.random.default_rng(0x0B5EED30), n_kf=150, n_points=20000)),
            ("loop1500", op.synth_map_graph(np.random.default_rng(0x0B5EED31), n_kf=1500, n_points=150000,
                                            loop=True))]
    for name, G in maps:
        ctx = Context(0)
        opt = op.Optimizer(ctx)
        opt.BundleAdjustment(G)
        ctx.synchronize()
        t = time.perf_counter()
        reps = 3
        for _ in range(reps):
            r = opt.BundleAdjustment(G)
        el = (time.perf_counter() - t) / reps
        op.lba_kernel_times(ctx, True)
        opt.BundleAdjustment(G)
        kt = op.lba_kernel_times(ctx, False)
        print(json.dumps({"label": a.label, "map": name, "ms_per_call": round(el * 1e3, 3), "iterations": r.iterations,
                          "trials": r.trials, "device_bytes": ctx.device_bytes(),
                          "kernel_ms": {k: round(v[0], 3) for k, v in kt.items() if v[1]}}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
