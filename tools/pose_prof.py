#!/usr/bin/env python3
"""Phase breakdown of k_pose_opt from the in-kernel s_memtime counters (library built with
`make POSE_PROF=1`): cycles per frame in the buildSystem passes, the 6x6 solves, the exp-map
updates, the trial chi2 passes and the classifications, at 1 and 1024 frames per launch."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.init()
    from orb_slam3_comments_ghr_amd import Context, load_library, optimizer as op
    ctx = Context(0)
    lib = load_library()
    f = lib.osg_debug_pose_prof
    f.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros((64, 8), np.uint64)
    opt = op.Optimizer(ctx)
    rng = np.random.default_rng(5)
    probs = [op.synth_pose_problem(rng, n_edges=int(rng.integers(150, 500))) for _ in range(64)]
    for B in [1, 64, 1024]:
        pb = [probs[i % 64] for i in range(B)]
        opt.PoseOptimization(pb)
        f(buf.ctypes.data, 1)
        got = opt.PoseOptimization(pb)
        f(buf.ctypes.data, 1)
        m = min(B, 64)
        it = np.array([g.lm_iterations for g in got[:m]], float)
        tr = np.array([g.lm_trials for g in got[:m]], float)
        ne = np.array([len(p.kind) for p in pb[:m]], float)
        b = buf[:m].astype(float)
        d = dict(B=B, kernel_ms=ctx.last_kernel_ms(), n_edges=ne.mean(), iters=it.mean(), trials=tr.mean(),
                 cyc_total=b[:, 5].mean(), cyc_hpass=b[:, 0].mean(), cyc_hpass_per=(b[:, 0] / it).mean(),
                 cyc_solve_per=(b[:, 1] / tr).mean(), cyc_oplus_per=(b[:, 2] / tr).mean(),
                 cyc_chipass_per=(b[:, 3] / tr).mean(), cyc_class=b[:, 4].mean(),
                 cyc_per_edge_hpass=(b[:, 0] / it / ne).mean(), cyc_per_edge_chipass=(b[:, 3] / tr / ne).mean())
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in d.items()}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
