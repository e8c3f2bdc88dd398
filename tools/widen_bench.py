"""Kernel device time of the §8(f) matchers built this round, at their reference call shapes, beside the
C oracle on one host thread (bounded samples).  python tools/widen_bench.py

  triang    SearchForTriangulation, 1200 x 1200 keypoints, batches of B keyframe pairs
  sim3      SearchByProjection(KeyFrame*, Sim3f&, ...), 1200 keypoints, 3000 / 9000 MapPoints (th 8, 1.5)
  distinct  ComputeDistinctiveDescriptors, 1000 / 100 000 MapPoints, N ~ U{1..30} rows
  init      SearchForInitialization, 2 x 5000 keypoints (22 % level 0), windowSize 100, nnratio 0.9
  stereo    ComputeStereoMatches, EuRoC 752 x 480 x 8 levels, 1200 keypoints per side (`... stereo` alone)
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_comments_ghr_amd import Context, frames as fr, mappoint as mp  # noqa: E402
from orb_slam3_comments_ghr_amd.matcher import ORBmatcher  # noqa: E402
from tests import oracle_calls as oc  # noqa: E402


def best_of(fn, ctx, n=3):
    fn()
    ks = []
    for _ in range(n):
        fn()
        ks.append(ctx.last_kernel_ms())
    return min(ks)


def cpu(fn, n):
    t = time.perf_counter()
    for i in range(n):
        fn(i)
    return (time.perf_counter() - t) / n * 1e3


def stereo_bench(ctx, o):
    """ComputeStereoMatches, EuRoC stereo 752 x 480, 8 levels, 1200 keypoints per side."""
    from orb_slam3_comments_ghr_amd import stereo as st
    rng = np.random.default_rng(13)
    pool = [st.synth_stereo_frame(rng, n=1200) for _ in range(16)]
    dev = [f.to_device() for f in pool]
    for B in (1, 16, 256, 1024):
        frames = [dev[i % 16] for i in range(B)]
        k = best_of(lambda: st.ComputeStereoMatchesBatch(ctx, frames), ctx)
        t = time.perf_counter()
        st.ComputeStereoMatchesBatch(ctx, frames)
        w = time.perf_counter() - t
        print(f"stereo   B={B:4d}  kernel {k * 1e3 / B:8.2f} us/frame  wall {w * 1e6 / B:8.1f} us/frame "
              f"(pyramids in HBM)", flush=True)
    k = best_of(lambda: st.ComputeStereoMatchesBatch(ctx, pool), ctx)
    t = time.perf_counter()
    st.ComputeStereoMatchesBatch(ctx, pool)
    w = time.perf_counter() - t
    print(f"stereo   B=  16  kernel {k * 1e3 / 16:8.2f} us/frame  wall {w * 1e6 / 16:8.1f} us/frame "
          f"(host pyramids packed + uploaded)", flush=True)
    c = cpu(lambda i: oc.stereo(o, pool[i % 16]), 48)
    print(f"stereo   oracle {c * 1e3:8.2f} us/frame (1 thread)", flush=True)


def orb_bench(ctx, o):
    """IC_Angle + rBRIEF for one EuRoC frame's keypoints (752 x 480, 8 levels), and a large batch of
    keypoints in one call (the kernels' throughput)."""
    from orb_slam3_comments_ghr_amd import orb
    rng = np.random.default_rng(14)
    raw, blur, x, y, level = orb.synth_orb_frame(rng, n=1200)
    pat = orb.synth_pattern(rng)
    rp, bp = orb.ImagePyramid(raw).to_device(), orb.ImagePyramid(blur).to_device()
    for n in (1200, 12000, 120000):
        idx = np.arange(n) % 1200
        args = (x[idx], y[idx], level[idx], pat)
        k = best_of(lambda: orb.ORBDescribe(ctx, rp, bp, *args), ctx)
        t = time.perf_counter()
        orb.ORBDescribe(ctx, rp, bp, *args)
        w = time.perf_counter() - t
        print(f"orb      n={n:6d}  kernels {k * 1e3:8.2f} us ({k * 1e6 / n:6.2f} ns/kp)  wall {w * 1e6:9.1f} us "
              f"(pyramids in HBM)", flush=True)
    k = best_of(lambda: orb.ORBDescribe(ctx, raw, blur, x, y, level, pat), ctx)
    t = time.perf_counter()
    orb.ORBDescribe(ctx, raw, blur, x, y, level, pat)
    w = time.perf_counter() - t
    print(f"orb      n=  1200  kernels {k * 1e3:8.2f} us  wall {w * 1e6:9.1f} us (host pyramids uploaded)", flush=True)
    c = cpu(lambda i: oc.orb_describe(o, raw, blur, x, y, level, pat), 20)
    print(f"orb      oracle {c * 1e3:8.2f} us/frame of 1200 keypoints (1 thread)", flush=True)


def main():
    ctx = Context(0)
    o = oc.load()
    if sys.argv[1:] == ["stereo"]:
        return stereo_bench(ctx, o)
    if sys.argv[1:] == ["orb"]:
        return orb_bench(ctx, o)
    m = ORBmatcher(ctx)
    rng = np.random.default_rng(11)
    pairs = [fr.synth_triang_pair(rng, n1=1200, n2=1200, forward=bool(i % 2)) for i in range(8)]
    for B in (1, 20, 256):
        P = [pairs[i % 8] for i in range(B)]
        k = best_of(lambda: m.SearchForTriangulationBatch([p[0] for p in P], [p[1] for p in P], [p[2] for p in P]), ctx)
        print(f"triang   B={B:4d}  kernel {k * 1e3 / B:8.2f} us/pair", flush=True)
    c = cpu(lambda i: oc.triangulation(o, *pairs[i % 8]), 64)
    print(f"triang   oracle {c * 1e3:8.2f} us/pair (1 thread)", flush=True)
    for nq in (3000, 9000):
        F = fr.synth_frame(rng, n=1200, stereo=False)
        Q = fr.synth_fuse_queries(rng, F, m=nq, match_frac=0.7)
        ids = np.arange(nq, dtype=np.int32)
        k = best_of(lambda: m.SearchByProjectionSim3(F, Q, ids, np.full(F.n, -1, np.int32), 8, 1.5), ctx)
        rounds = ctx.match_last_stats()["rounds"]
        c = cpu(lambda i: oc.sim3(o, F, Q, 8, 1.5, np.full(F.n, -1, np.int32)), 20)
        print(f"sim3     nq={nq:5d}  kernel {k * 1e3:8.2f} us  rounds {rounds}  oracle {c * 1e3:8.2f} us", flush=True)
    for n in (1000, 100000):
        lists = mp.synth_observations(rng, n_points=n, n_max=30)
        desc, start = mp.to_csr(lists)
        k = best_of(lambda: mp.ComputeDistinctiveDescriptors(ctx, desc=desc, start=start), ctx)
        c = cpu(lambda i: oc.distinctive(o, desc, start), 1 if n > 1000 else 10)
        print(f"distinct n={n:6d}  kernel {k * 1e3:9.2f} us ({k * 1e6 / n:7.1f} ns/point)  oracle {c * 1e3:10.1f} us",
              flush=True)
    init_bench(ctx, o)
    stereo_bench(ctx, o)
    orb_bench(ctx, o)


def init_bench(ctx, o):
    rng = np.random.default_rng(12)
    F1, F2, prev = fr.synth_init_pair(rng, n1=5000, n2=5000, level0=0.22)
    m = ORBmatcher(ctx, nnratio=0.9)
    k = best_of(lambda: m.SearchForInitialization(F1, F2, prev.copy(), 100), ctx)
    st = ctx.match_last_stats()
    c = cpu(lambda i: oc.initialization(o, F1, F2, prev, 100, 0.9, True), 10)
    print(f"init     5000x5000  kernel {k * 1e3:8.2f} us  rounds {st['rounds']}  oracle {c * 1e3:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
