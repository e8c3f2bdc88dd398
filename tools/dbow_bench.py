"""DBoW2 transform throughput: ORBvoc-shaped synthetic vocabulary (k = 10, L = 6), 1200 descriptors
per frame, B frames per launch; kernel device time.  python tools/dbow_bench.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_comments_ghr_amd import Context, vocabulary as vb  # noqa: E402


def main():
    ctx = Context(0)
    rng = np.random.default_rng(21)
    t = time.perf_counter()
    voc = vb.synth_vocabulary(rng, k=10, L=6, min_children=8, min_leaf_depth=6)
    print(f"vocabulary: {voc.n_nodes} nodes, {voc.n_words} words ({time.perf_counter() - t:.1f} s)", flush=True)
    gv = vb.ORBVocabulary(ctx, voc)
    pool = [vb.synth_features(rng, voc, n=1200) for _ in range(16)]
    for B in (1, 16, 256, 1024):
        sets = [pool[i % len(pool)] for i in range(B)]
        gv.transform_batch(sets, 4)
        ks = []
        t = time.perf_counter()
        for _ in range(3):
            gv.transform_batch(sets, 4)
            ks.append(ctx.last_kernel_ms())
        wall = (time.perf_counter() - t) / 3
        k = min(ks)
        print(f"B={B:5d}  kernel {k * 1e3 / B:9.2f} us/frame ({k:.3f} ms)   wall {wall * 1e6 / B:9.2f} us/frame", flush=True)


if __name__ == "__main__":
    main()
