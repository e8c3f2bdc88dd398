#!/usr/bin/env python3
"""A/B of PoseOptimization's edge-order sums (OSG_POSE_ROWSUM=1 whole rows with the loads kept ahead,
=0 the per-chunk sums): single-call wall and kernel time of the drop-in's one-frame call (318-edge
pinhole frame, 600-edge KB8 two-camera frame) and the kernel time of a 256-frame batch, the variants
alternating.  One JSON line per (variant, repeat).  argv[1] names another 0/1 switch to alternate
instead (OSG_POSE_LANES: the solve and exp-map update spread over wave 0's lanes)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(f, n=60):
    for _ in range(5):
        f()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


def main():
    import torch
    torch.cuda.init()
    from orb_slam3_comments_ghr_amd import Context, optimizer as op, _abi
    ctx = Context(0)
    lib, h = ctx.lib, ctx.handle
    rng = np.random.default_rng(0x0B5EED03)
    singles = []
    for n_edges, cam, body in [(318, None, 0.0), (600, op.kb8_camera(), 0.4)]:
        P = op.synth_pose_problem(rng, n_edges=n_edges, **({} if cam is None else {"cam": cam, "body_frac": body}))
        ps = P.struct()
        r = _abi.OsgPoseResult()
        ob = np.zeros(P.n, np.uint8)
        r.outlier = ob.ctypes.data
        singles.append((n_edges, ps, r, ob, P))  # P keeps the arrays ps points at alive
    batch = [op.synth_pose_problem(rng, n_edges=int(rng.integers(200, 600))) for _ in range(256)]
    opt = op.Optimizer(ctx)
    sw = sys.argv[1] if len(sys.argv) > 1 else "OSG_POSE_ROWSUM"
    for rep in range(3 if len(sys.argv) > 1 else 2):
        for var in ["0", "1"]:
            os.environ[sw] = var
            d = {sw: var, "rep": rep}
            for n_edges, ps, r, *_ in singles:
                w = med(lambda: lib.osg_pose_optimization(h, C.byref(ps), C.byref(r)))
                ks = []
                for _ in range(20):
                    lib.osg_pose_optimization(h, C.byref(ps), C.byref(r))
                    ks.append(ctx.last_kernel_ms() * 1e3)
                d[f"single_{n_edges}"] = {"wall_us": round(w, 1), "kernel_us": round(float(np.median(ks)), 1),
                                          "pose": [float(x) for x in r.pose], "trials": r.lm_trials}
            opt.PoseOptimization(batch)
            ks = []
            for _ in range(10):
                opt.PoseOptimization(batch)
                ks.append(ctx.last_kernel_ms() * 1e3)
            d["batch256_kernel_us"] = round(float(np.median(ks)), 1)
            print(json.dumps(d), flush=True)
    os.environ.pop(sw, None)
    ctx.close()


if __name__ == "__main__":
    main()
