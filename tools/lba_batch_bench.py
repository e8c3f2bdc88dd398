"""Batched LocalBundleAdjustment throughput (SURVEY.md §8d C4, B windows per GPU in lockstep):
LM iterations per wall second for B = 1 .. 64, and with T host threads each driving its own context
(own HIP stream) so that one thread's structure build / packing overlaps another's device steps.
Run on the GPU box:  BS=1,64 TS=1,2,3 python tools/lba_batch_bench.py  (REPS: calls per thread)"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_comments_ghr_amd import Context, optimizer as op  # noqa: E402


def main():
    import torch
    torch.cuda.init()
    rng = np.random.default_rng(0x0B5EED04)
    pool = [op.synth_lba_graph(rng, n_kf=50, n_points=10000) for _ in range(8)]
    tmax = max(int(x) for x in os.environ.get("TS", "1").split(","))
    opts = [op.Optimizer(Context(0)) for _ in range(tmax)]
    for T in [int(x) for x in os.environ.get("TS", "1").split(",")]:
        for B in [int(x) for x in os.environ.get("BS", "1,4,16,32,64").split(",")]:
            graphs = [pool[i % len(pool)] for i in range(B)]
            for o in opts[:T]:
                o.LocalBundleAdjustmentBatch(graphs)
            reps = int(os.environ.get("REPS", max(2, 8 // B)))
            its = [0] * T

            def run(t):
                for _ in range(reps):
                    t1 = time.perf_counter()
                    res = opts[t].LocalBundleAdjustmentBatch(graphs)
                    if os.environ.get("OSG_LBA_PROFILE"):
                        print(f"  thread {t} python call {1e3 * (time.perf_counter() - t1):.2f} ms", flush=True)
                    its[t] += sum(r.iterations for r in res)
            t0 = time.perf_counter()
            th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            el = time.perf_counter() - t0
            print(f"T={T} B={B:3d}  {sum(its) / el:10.1f} LM iters/s   {el / reps * 1e3:8.2f} ms per round of "
                  f"{T} batches   {el / reps / B / T * 1e3:6.3f} ms per window", flush=True)
            if T == 1 and os.environ.get("KT"):  # per-kernel device time of one batch (HIP events)
                op.lba_kernel_times(opts[0].ctx, True)
                opts[0].LocalBundleAdjustmentBatch(graphs)
                kt = op.lba_kernel_times(opts[0].ctx, False)
                print("   kernels (ms, launch groups): " + ", ".join(f"{k} {v[0]:.3f}/{v[1]}" for k, v in kt.items()),
                      flush=True)


if __name__ == "__main__":
    main()
