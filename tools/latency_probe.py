#!/usr/bin/env python3
"""Single-call latency breakdown of the drop-in entry points (one frame per call, as Tracking issues
them): wall time of the C-ABI call vs the device time of its kernel (ctx.last_kernel_ms), and with
OSG_MATCH_PROFILE=1 the matcher's in-kernel phase clocks.  With a `make POSE_PROF=1` library the
PoseOptimization phase counters are printed too."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(f, n=50):
    for _ in range(3):
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
    import orb_slam3_comments_ghr_amd as pkg
    if os.environ.get("OSG_PROBE_LIB"):  # a profiling build (make POSE_PROF=1 into another directory)
        pkg.LIB_PATH = os.environ["OSG_PROBE_LIB"]
    from orb_slam3_comments_ghr_amd import Context, frames as fr, optimizer as op, _abi
    ctx = Context(0)
    lib, h = ctx.lib, ctx.handle
    rng = np.random.default_rng(0x0B5EED10)
    F = fr.synth_frame_two_cam(rng, n_left=1000, n_right=1000, stereo_frac=0.5, width=512, height=512)
    L = fr.synth_last_queries_two_cam(rng, F, n_last=2000)
    Q = fr.synth_mp_queries_two_cam(rng, F, m=1500)
    S = fr.synth_slots(rng, F.n, frac_assigned=0.05)
    fs, ls, qs = F.struct(), L.struct(), Q.struct()
    sl, tk = S[0].copy(), np.ascontiguousarray(S[1], np.uint8)
    out = {}

    def mps():
        np.copyto(sl, S[0])
        lib.osg_search_by_projection_mps(h, C.byref(fs), C.byref(qs), 0.9, 3.0, 0, 20.0, sl.ctypes.data, tk.ctypes.data)

    def last():
        np.copyto(sl, S[0])
        lib.osg_search_by_projection_last(h, C.byref(fs), C.byref(ls), 7.0, 0, 1, sl.ctypes.data, tk.ctypes.data)

    rng3 = np.random.default_rng(0x0B5EED03)
    kf, f = fr.synth_bow_pair(rng3, n_kf=1200, n_f=1200, n_nodes=100)
    a, b = kf.struct(), f.struct()
    o = np.full(f.n, -1, np.int32)

    def bow():
        lib.osg_search_by_bow_kf_f(h, C.byref(a), C.byref(b), 0.7, 1, o.ctypes.data)

    # the bench's C5 latency problem (bench_c5: 32 frames, then their LastF and local-map queries)
    rngb = np.random.default_rng(0x0B5EED10)
    FP = [fr.synth_frame_two_cam(rngb, n_left=1000, n_right=1000, stereo_frac=0.5, width=512, height=512)
          for _ in range(32)]
    [fr.synth_last_queries_two_cam(rngb, f, n_last=2000) for f in FP]
    QP = [fr.synth_mp_queries_two_cam(rngb, f, m=1500) for f in FP]
    for x in QP:  # as bench_c5: the local map's MapPoints all have observations
        x.has_obs[:] = 1
    SP = [fr.synth_slots(rngb, f.n, frac_assigned=0.05) for f in FP]
    fsb, qsb = FP[0].struct(), QP[0].struct()
    slb, tkb = SP[0][0].copy(), np.ascontiguousarray(SP[0][1], np.uint8)

    def mps_bench():
        np.copyto(slb, SP[0][0])
        lib.osg_search_by_projection_mps(h, C.byref(fsb), C.byref(qsb), 0.9, 3.0, 0, 20.0, slb.ctypes.data,
                                         tkb.ctypes.data)

    for name, fn in [("mps", mps), ("mps_bench", mps_bench), ("last", last), ("bow", bow)]:
        w = med(fn)
        fn()
        out[name] = {"wall_us": round(w, 1), "kernel_us": round(ctx.last_kernel_ms() * 1e3, 1),
                     "stats": ctx.match_stats() if hasattr(ctx, "match_stats") else ctx.match_last_stats()}
        print(json.dumps({name: out[name]}), flush=True)
    for n_edges, cam, body in [(318, None, 0.0), (600, op.kb8_camera(), 0.4)]:
        P = op.synth_pose_problem(rng, n_edges=n_edges, **({} if cam is None else {"cam": cam, "body_frac": body}))
        ps = P.struct()
        r = _abi.OsgPoseResult()
        ob = np.zeros(P.n, np.uint8)
        r.outlier = ob.ctypes.data
        d = {}
        for var in ["4", "8", None]:  # 4 and 8 waves per frame, then the host's choice
            if var is None:
                os.environ.pop("OSG_POSE_NW", None)
            else:
                os.environ["OSG_POSE_NW"] = var
            w = med(lambda: lib.osg_pose_optimization(h, C.byref(ps), C.byref(r)))
            d[f"nw_{var or 'auto'}"] = {"wall_us": round(w, 1), "kernel_us": round(ctx.last_kernel_ms() * 1e3, 1),
                                         "iters": r.lm_iterations, "trials": r.lm_trials,
                                         "pose": [float(x) for x in r.pose], "n_inliers": r.n_inliers}
            if hasattr(lib, "osg_debug_pose_prof"):
                f_ = lib.osg_debug_pose_prof
                f_.argtypes = [C.c_void_p, C.c_int]
                buf = np.zeros((64, 8), np.uint64)
                f_(buf.ctypes.data, 1)
                lib.osg_pose_optimization(h, C.byref(ps), C.byref(r))
                f_(buf.ctypes.data, 1)
                d[f"nw_{var or 'auto'}"]["cycles"] = {k: int(buf[0, i]) for i, k in enumerate(
                    ["hpass", "solve", "oplus", "chipass", "class", "total", "pass_compute", "pass_sum"])}
        os.environ.pop("OSG_POSE_NW", None)
        print(json.dumps({f"pose_{n_edges}": d}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
