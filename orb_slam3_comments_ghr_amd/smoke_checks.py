"""Small end-to-end checks of every hot-path operator against the CPU oracle, used by
__graft_entry__.smoke() (the oracle is the checker only)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import frames as fr
from . import optimizer as op
from .matcher import ORBmatcher


def run(ctx, oracle):
    rng = np.random.default_rng(2024)
    m = ORBmatcher(ctx, 0.8, True)
    # SearchByProjection(Frame, vector<MapPoint*>)
    F = fr.synth_frame(rng, n=600)
    Q = fr.synth_mp_queries(rng, F, m=900)
    slots, taken = fr.synth_slots(rng, F.n)
    ref = slots.copy()
    rn = oracle.oracle_search_by_projection_mps(C.byref(F.struct()), C.byref(Q.struct()), 0.8, 3.0, 0, 50.0,
                                                ref.ctypes.data, np.ascontiguousarray(taken).ctypes.data)
    got = slots.copy()
    n = m.SearchByProjection(F, Q, 3.0, slot_mp=got, slot_taken=taken)
    if n != rn or not np.array_equal(got, ref):
        raise AssertionError("SearchByProjection(Frame, MapPoints) mismatch vs oracle")
    # SearchByBoW(KeyFrame, Frame)
    KF, Fb = fr.synth_bow_pair(rng, n_kf=500, n_f=500, n_nodes=40)
    ref = np.full(Fb.n, -1, np.int32)
    rn = oracle.oracle_search_by_bow_kf_f(C.byref(KF.struct()), C.byref(Fb.struct()), 0.7, 1, ref.ctypes.data)
    n, got = ORBmatcher(ctx, 0.7, True).SearchByBoW(KF, Fb)
    if n != rn or not np.array_equal(got, ref):
        raise AssertionError("SearchByBoW mismatch vs oracle")
    # PoseOptimization
    probs = [op.synth_pose_problem(rng, n_edges=200) for _ in range(4)]
    refp = op.oracle_pose(oracle, probs)
    gotp = op.Optimizer(ctx).PoseOptimization(probs)
    for g, r in zip(gotp, refp):
        if g.n_inliers != r.n_inliers or not np.array_equal(g.outlier, r.outlier) or \
                np.max(np.abs(g.pose - r.pose)) > 1e-6:
            raise AssertionError("PoseOptimization mismatch vs oracle")
    # LocalBundleAdjustment
    G = op.synth_lba_graph(rng, n_kf=6, n_points=400)
    refl = op.oracle_lba(oracle, G)
    gotl = op.Optimizer(ctx).LocalBundleAdjustment(G)
    if not np.array_equal(gotl.edge_bad, refl.edge_bad) or np.max(np.abs(gotl.point - refl.point)) > 1e-6 or \
            np.max(np.abs(gotl.pose - refl.pose)) > 1e-6:
        raise AssertionError("LocalBundleAdjustment mismatch vs oracle")
