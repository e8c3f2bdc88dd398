#!/usr/bin/env python3
"""Parity of each k_pose_opt wave-count variant (OSG_POSE_NW=1/2/4/8 and OSG_POSE_FUSE=0/1 pin it) against the
oracle on a small seeded batch.  Prints one JSON line per variant."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.init()
    from orb_slam3_comments_ghr_amd import Context, optimizer as op
    from tests import oracle_calls as oc
    ctx = Context(0)
    opt = op.Optimizer(ctx)
    oracle = oc.load()
    rng = np.random.default_rng(5)
    probs = [op.synth_pose_problem(rng, n_edges=int(rng.integers(30, 500))) for _ in range(8)]
    ref = oc.pose(oracle, probs)
    for v in sys.argv[1:] or ["1:0", "1:1", "2:0", "2:1", "4:0", "4:1", "8:0", "8:1"]:
        nw, fuse = v.split(":")
        os.environ["OSG_POSE_NW"] = nw
        os.environ["OSG_POSE_FUSE"] = fuse
        got = opt.PoseOptimization(probs)
        print(json.dumps(dict(nw=nw, fuse=fuse, it=[(g.lm_iterations, r.lm_iterations) for g, r in zip(got, ref)],
                              tr=[(g.lm_trials, r.lm_trials) for g, r in zip(got, ref)],
                              flags=[int(np.sum(g.outlier != r.outlier)) for g, r in zip(got, ref)],
                              dpose=[float(np.abs(g.pose - r.pose).max()) for g, r in zip(got, ref)])), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
