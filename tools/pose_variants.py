#!/usr/bin/env python3
"""Kernel time of every k_pose_opt variant (waves per frame, and the automatic choice) at 1 to
4096 frames per launch, for frames of 100 / 384 / 1000 edges.  Prints JSON lines."""
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
    ctx = Context(0)
    opt = op.Optimizer(ctx)
    for ne in [100, 384, 1000]:
        rng = np.random.default_rng(ne)
        p = op.synth_pose_problem(rng, n_edges=ne)
        for B in [1, 64, 1024, 4096]:
            row = {}
            for nw in ["1", "2", "4", "8", None]:
                if nw is None:
                    os.environ.pop("OSG_POSE_NW", None)
                else:
                    os.environ["OSG_POSE_NW"] = nw
                opt.PoseOptimization([p] * B)
                ks = []
                for _ in range(3):
                    g = opt.PoseOptimization([p] * B)
                    ks.append(ctx.last_kernel_ms())
                row[nw or "auto"] = round(min(ks) * 1e3, 1)
            print(json.dumps(dict(n_edges=ne, B=B, iters=g[0].lm_iterations, trials=g[0].lm_trials, kernel_us=row)), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
