#!/usr/bin/env python3
"""Phase cycle counters of k_pose_opt (a `make POSE_PROF=1` build named by OSG_LIB_PATH) for the drop-in's
one-frame call (318-edge pinhole, 600-edge KB8 two-camera), alternating a 0/1 switch (argv[1], default
OSG_POSE_LANES).  One JSON line per (variant, frame, repeat): wave 0's cycles per phase."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KEYS = ["hpass", "solve", "oplus", "chipass", "class", "total", "pass_compute", "pass_sum"]


def main():
    import torch
    torch.cuda.init()
    from orb_slam3_comments_ghr_amd import Context, optimizer as op, _abi
    sw = sys.argv[1] if len(sys.argv) > 1 else "OSG_POSE_LANES"
    ctx = Context(0)
    lib, h = ctx.lib, ctx.handle
    f = lib.osg_debug_pose_prof
    f.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros((64, 8), np.uint64)
    rng = np.random.default_rng(0x0B5EED03)
    frames = []
    for n_edges, cam, body in [(318, None, 0.0), (600, op.kb8_camera(), 0.4)]:
        P = op.synth_pose_problem(rng, n_edges=n_edges, **({} if cam is None else {"cam": cam, "body_frac": body}))
        ps = P.struct()
        r = _abi.OsgPoseResult()
        ob = np.zeros(P.n, np.uint8)
        r.outlier = ob.ctypes.data
        frames.append((n_edges, ps, r, ob, P))  # P keeps the arrays ps points at alive
    for rep in range(2):
        for var in ["0", "1"]:
            os.environ[sw] = var
            for n_edges, ps, r, *_ in frames:
                for _ in range(3):
                    lib.osg_pose_optimization(h, C.byref(ps), C.byref(r))
                f(buf.ctypes.data, 1)
                lib.osg_pose_optimization(h, C.byref(ps), C.byref(r))
                f(buf.ctypes.data, 1)
                d = {sw: var, "rep": rep, "edges": n_edges, "trials": r.lm_trials, "iters": r.lm_iterations,
                     "kernel_us": round(ctx.last_kernel_ms() * 1e3, 1)}
                d.update({k: int(buf[0, i]) for i, k in enumerate(KEYS)})
                print(json.dumps(d), flush=True)
    os.environ.pop(sw, None)
    ctx.close()


if __name__ == "__main__":
    main()
