"""Batched LocalBundleAdjustment throughput (SURVEY.md §8d C4, B windows per GPU in lockstep):
LM iterations per wall second for B = 1 .. 64.  Run on the GPU box:  python tools/lba_batch_bench.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_comments_ghr_amd import Context, optimizer as op  # noqa: E402


def main():
    ctx = Context(0)
    opt = op.Optimizer(ctx)
    rng = np.random.default_rng(0x0B5EED04)
    pool = [op.synth_lba_graph(rng, n_kf=50, n_points=10000) for _ in range(8)]
    for B in [int(x) for x in os.environ.get("BS", "1,4,16,32,64").split(",")]:
        graphs = [pool[i % len(pool)] for i in range(B)]
        opt.LocalBundleAdjustmentBatch(graphs)
        reps = max(1, 8 // B)
        t = time.perf_counter()
        it = 0
        for _ in range(reps):
            t1 = time.perf_counter()
            res = opt.LocalBundleAdjustmentBatch(graphs)
            if os.environ.get("OSG_LBA_PROFILE"):
                print(f"  python call {1e3 * (time.perf_counter() - t1):.2f} ms", flush=True)
            it += sum(r.iterations for r in res)
        el = time.perf_counter() - t
        print(f"B={B:3d}  {it / el:10.1f} LM iters/s   {el / reps * 1e3:8.2f} ms per batch   "
              f"{el / reps / B * 1e3:6.3f} ms per window", flush=True)


if __name__ == "__main__":
    main()
