"""Batched matcher throughput (SURVEY.md §8d C3 / C5 shapes): kernel time per frame for B problems per
launch vs one problem per launch.  Run on the GPU box:  python tools/match_batch_bench.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_comments_ghr_amd import Context, frames as fr  # noqa: E402
from orb_slam3_comments_ghr_amd.matcher import ORBmatcher  # noqa: E402


def main():
    ctx = Context(0)
    m = ORBmatcher(ctx, 0.7, True)
    rng = np.random.default_rng(3)
    nb = int(os.environ.get("NB", "64"))
    pairs = [fr.synth_bow_pair(rng, n_kf=1200, n_f=1200, n_nodes=100) for _ in range(nb)]
    KFs, Fs = [p[0] for p in pairs], [p[1] for p in pairs]
    for B in [1, 8, 64, 256, 1024]:
        reps = (B + nb - 1) // nb
        KB = (KFs * reps)[:B]
        FB = (Fs * reps)[:B]
        m.SearchByBoWBatch(KB, FB)
        t = time.perf_counter()
        n = 3
        ks = []
        for _ in range(n):
            m.SearchByBoWBatch(KB, FB)
            ks.append(ctx.match_last_stats()["kernel_ms"])
        wall = (time.perf_counter() - t) / n
        k = min(ks)
        print(f"bow kf-f  B={B:5d}  kernel {k * 1e3 / B:8.2f} us/frame ({k:.3f} ms)  wall {wall * 1e6 / B:8.2f} us/frame",
              flush=True)
    F = fr.synth_frame(rng, n=1200)
    Q = fr.synth_mp_queries(rng, F, m=3000)
    L = fr.synth_last_queries(rng, F, n_last=1100)
    sm, tk = fr.synth_slots(rng, F.n)
    for name, q, args in [("mps", Q, (3.0, False, 20.0)), ("last", L, (7.0, False))]:
        for B in [1, 64, 256, 1024]:
            m.SearchByProjectionBatch([F] * B, [q] * B, *args, slot_mps=[sm.copy() for _ in range(B)],
                                      slot_takens=[tk] * B)
            ks = []
            for _ in range(3):
                m.SearchByProjectionBatch([F] * B, [q] * B, *args, slot_mps=[sm.copy() for _ in range(B)],
                                          slot_takens=[tk] * B)
                ks.append(ctx.match_last_stats()["kernel_ms"])
            k = min(ks)
            print(f"{name:8s}  B={B:5d}  kernel {k * 1e3 / B:8.2f} us/frame ({k:.3f} ms)", flush=True)


if __name__ == "__main__":
    main()
