"""Fuse search throughput (LocalMapping::SearchInNeighbors shape): one MapPoint list of ~1000
points fused into B keyframes of 1200 keypoints, th 3; kernel device time vs the C oracle.
python tools/fuse_bench.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_comments_ghr_amd import Context, frames as fr  # noqa: E402
from orb_slam3_comments_ghr_amd.matcher import ORBmatcher  # noqa: E402
from tests import oracle_calls as oc  # noqa: E402


def main():
    ctx = Context(0)
    rng = np.random.default_rng(5)
    pool = [fr.synth_frame(rng, n=1200) for _ in range(16)]
    qs = [fr.synth_fuse_queries(rng, F, m=1000) for F in pool]
    m = ORBmatcher(ctx)
    for B in (1, 20, 256, 2048):
        KF = [pool[i % 16] for i in range(B)]
        Q = [qs[i % 16] for i in range(B)]
        m.FuseBatch(KF, Q)
        ks = []
        t = time.perf_counter()
        for _ in range(3):
            m.FuseBatch(KF, Q)
            ks.append(ctx.last_kernel_ms())
        wall = (time.perf_counter() - t) / 3
        k = min(ks)
        print(f"B={B:5d}  kernel {k * 1e3 / B:8.2f} us/keyframe ({k:.3f} ms)  wall {wall * 1e6 / B:8.2f} us/keyframe",
              flush=True)
    o = oc.load()
    t = time.perf_counter()
    for i in range(32):
        oc.fuse(o, pool[i % 16], qs[i % 16], 3.0)
    print(f"oracle {(time.perf_counter() - t) / 32 * 1e6:.1f} us/keyframe (1 thread)")


if __name__ == "__main__":
    main()
