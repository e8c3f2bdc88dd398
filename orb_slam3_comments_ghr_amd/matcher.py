"""Host mirror of the reference operator API ``ORB_SLAM3::ORBmatcher`` (ref:include/ORBmatcher.h:34-99)
on top of the C ABI.  Same names, argument meaning, defaults and in-place outputs; every search
runs on the GPU (there is no CPU fallback).

    m = ORBmatcher(ctx, nnratio=0.6, checkOri=True)
    n = m.SearchByProjection(F, mps, th=3, slot_mp=slots, slot_taken=taken)     # (Frame&, vector<MapPoint*>)
    n = m.SearchByProjection(CF, last, th, bMono, slot_mp=slots, slot_taken=t)  # (Frame&, const Frame&)
    n = m.SearchByProjection(CF, kfq, th, ORBdist, slot_mp=slots)               # (Frame&, KeyFrame*, set)
    n, vpMapPointMatches = m.SearchByBoW(KF, F)                                 # (KeyFrame*, Frame&)
    n, vpMatches12 = m.SearchByBoW(KF1, KF2, kf2=True)                          # (KeyFrame*, KeyFrame*)
    n, best_idx, best_dist = m.Fuse(KF, fq, th=3.0, bRight=False)               # Fuse(KeyFrame*, vector<MapPoint*>)
    n, best_idx, best_dist = m.Fuse(KF, fq, th, sim3=True)                      # Fuse(KeyFrame*, Sim3f, ...)
    n, vMatchedPairs = m.SearchForTriangulation(KF1, KF2, geom, bOnlyStereo, bCoarse)
    n = m.SearchByProjectionSim3(KF, fq, mp_id, vpMatched, th, ratioHamming[, vpPointsKFs, vpMatchedKF])
    n, vnMatches12 = m.SearchForInitialization(F1, F2, vbPrevMatched, windowSize)   # vbPrevMatched updated
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import Context, _abi, descriptor_distance
from .frames import BowSide, FrameSoA, FuseQueries, KFQueries, KFSide, LastQueries, MPQueries, TriangGeom


class ORBmatcher:
    TH_HIGH = _abi.TH_HIGH
    TH_LOW = _abi.TH_LOW
    HISTO_LENGTH = _abi.HISTO_LENGTH

    def __init__(self, ctx: Context, nnratio: float = 0.6, checkOri: bool = True):
        self.ctx = ctx
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)

    @staticmethod
    def DescriptorDistance(a, b) -> int:
        return descriptor_distance(a, b)

    def SearchByProjection(self, F: FrameSoA, q, *args, slot_mp=None, slot_taken=None, **kw) -> int:
        lib, h = self.ctx.lib, self.ctx.handle
        fs = F.struct()
        if slot_mp is None:
            slot_mp = np.full(F.n, -1, np.int32)
        assert slot_mp.dtype == np.int32 and slot_mp.flags["C_CONTIGUOUS"] and len(slot_mp) == F.n
        if isinstance(q, MPQueries):
            th = args[0] if len(args) > 0 else kw.get("th", 3.0)
            far = args[1] if len(args) > 1 else kw.get("bFarPoints", False)
            thfar = args[2] if len(args) > 2 else kw.get("thFarPoints", 50.0)
            taken = np.ascontiguousarray(slot_taken if slot_taken is not None else np.zeros(F.n), np.uint8)
            qs = q.struct()
            rc = lib.osg_search_by_projection_mps(h, C.byref(fs), C.byref(qs), self.mfNNratio, float(th),
                                                  int(bool(far)), float(thfar), slot_mp.ctypes.data,
                                                  taken.ctypes.data)
            return self.ctx.check(rc, "SearchByProjection(Frame, vector<MapPoint*>)")
        if isinstance(q, LastQueries):
            th = args[0] if len(args) > 0 else kw["th"]
            mono = args[1] if len(args) > 1 else kw["bMono"]
            taken = np.ascontiguousarray(slot_taken if slot_taken is not None else np.zeros(F.n), np.uint8)
            qs = q.struct()
            rc = lib.osg_search_by_projection_last(h, C.byref(fs), C.byref(qs), float(th), int(bool(mono)),
                                                   int(self.mbCheckOrientation), slot_mp.ctypes.data,
                                                   taken.ctypes.data)
            return self.ctx.check(rc, "SearchByProjection(Frame, Frame)")
        if isinstance(q, KFQueries):
            th = args[0] if len(args) > 0 else kw["th"]
            orb = args[1] if len(args) > 1 else kw["ORBdist"]
            qs = q.struct()
            rc = lib.osg_search_by_projection_kf(h, C.byref(fs), C.byref(qs), float(th), int(orb),
                                                 int(self.mbCheckOrientation), slot_mp.ctypes.data)
            return self.ctx.check(rc, "SearchByProjection(Frame, KeyFrame, set)")
        raise TypeError(f"no SearchByProjection overload for {type(q).__name__}")

    def SearchByBoW(self, KF: BowSide, other: BowSide, kf2: bool = False):
        lib, h = self.ctx.lib, self.ctx.handle
        a, b = KF.struct(), other.struct()
        if not kf2:
            out = np.full(other.n, -1, np.int32)
            rc = lib.osg_search_by_bow_kf_f(h, C.byref(a), C.byref(b), self.mfNNratio,
                                            int(self.mbCheckOrientation), out.ctypes.data)
            return self.ctx.check(rc, "SearchByBoW(KeyFrame, Frame)"), out
        out = np.full(KF.n, -1, np.int32)
        rc = lib.osg_search_by_bow_kf_kf(h, C.byref(a), C.byref(b), self.mfNNratio,
                                         int(self.mbCheckOrientation), out.ctypes.data)
        return self.ctx.check(rc, "SearchByBoW(KeyFrame, KeyFrame)"), out

    def Fuse(self, KF: FrameSoA, fq: FuseQueries, th: float = 3.0, bRight: bool = False, sim3: bool = False):
        """The search half of ``Fuse`` (ref:src/ORBmatcher.cc:1330-1541; ``sim3=True``: the Sim3
        overload :1553-1694, no reprojection gate).  Returns (nfused, best_idx, best_dist): per MapPoint
        the KeyFrame keypoint to fuse with (-1 = none).  The replace / add step is the caller's."""
        lib, h = self.ctx.lib, self.ctx.handle
        bi = np.full(fq.n, -1, np.int32)
        bd = np.full(fq.n, 256, np.int32)
        fs, qs = KF.struct(), fq.struct()
        rc = lib.osg_fuse_search(h, C.byref(fs), C.byref(qs), float(th), int(bool(bRight)), int(not sim3),
                                 bi.ctypes.data, bd.ctypes.data)
        return self.ctx.check(rc, "Fuse"), bi, bd

    def FuseBatch(self, KFs, fqs, th: float = 3.0, bRight: bool = False, sim3: bool = False):
        """B (KeyFrame, MapPoint list) Fuse searches in one launch; returns (nfused[B], [best_idx],
        [best_dist])."""
        lib, h = self.ctx.lib, self.ctx.handle
        B = len(KFs)
        assert len(fqs) == B
        fa = (_abi.OsgFrame * B)(*[F.struct() for F in KFs])
        qa = (_abi.OsgFuseQueries * B)(*[q.struct() for q in fqs])
        tot = sum(q.n for q in fqs)
        bi = np.full(tot, -1, np.int32)
        bd = np.full(tot, 256, np.int32)
        nf = np.zeros(B, np.int32)
        rc = lib.osg_fuse_search_batch(h, C.addressof(fa), C.addressof(qa), B, float(th), int(bool(bRight)),
                                       int(not sim3), bi.ctypes.data, bd.ctypes.data, nf.ctypes.data)
        self.ctx.check(rc, "Fuse batch")
        cuts = np.cumsum([0] + [q.n for q in fqs])
        return nf, [bi[a:b].copy() for a, b in zip(cuts[:-1], cuts[1:])], [bd[a:b].copy() for a, b in
                                                                           zip(cuts[:-1], cuts[1:])]

    def SearchBySim3(self, KF1: FrameSoA, KF2: FrameSoA, q12: FuseQueries, q21: FuseQueries, th: float):
        """``SearchBySim3(pKF1, pKF2, vpMatches12, S12, th)`` (ref:src/ORBmatcher.cc:1696-1939): q12 = KF1's
        MapPoints projected into KF2 (one per KF1 keypoint), q21 = KF2's into KF1.  Returns (nFound,
        match12): the KF2 keypoint matched to each KF1 keypoint (mutual best), -1 = none."""
        lib, h = self.ctx.lib, self.ctx.handle
        assert q12.n == KF1.n and q21.n == KF2.n, "one query per keypoint of each KeyFrame"
        a, b, qa, qb = KF1.struct(), KF2.struct(), q12.struct(), q21.struct()
        out = np.full(KF1.n, -1, np.int32)
        rc = lib.osg_search_by_sim3(h, C.byref(a), C.byref(b), C.byref(qa), C.byref(qb), float(th), out.ctypes.data)
        return self.ctx.check(rc, "SearchBySim3"), out

    def SearchByProjectionSim3(self, KF: FrameSoA, fq: FuseQueries, mp_id, vpMatched, th: int, ratioHamming: float,
                               vpPointsKFs=None, vpMatchedKF=None) -> int:
        """``SearchByProjection(KeyFrame*, Sim3f&, vpPoints, [vpPointsKFs,] vpMatched, [vpMatchedKF,] th,
        ratioHamming)`` (ref:src/ORBmatcher.cc:498-733).  ``fq`` holds the projected MapPoints (``valid`` =
        the caller's pre-search filters), ``mp_id[q]`` their ids; ``vpMatched`` (KF.n MapPoint ids, -1 =
        NULL) and ``vpMatchedKF`` are updated in place like the reference's output vectors."""
        lib, h = self.ctx.lib, self.ctx.handle
        vpMatched = np.asarray(vpMatched)
        sq = np.where(vpMatched >= 0, -2, -1).astype(np.int32)
        fs, qs = KF.struct(), fq.struct()
        rc = lib.osg_search_by_projection_sim3(h, C.byref(fs), C.byref(qs), float(th), float(ratioHamming),
                                               sq.ctypes.data)
        n = self.ctx.check(rc, "SearchByProjection(KeyFrame, Sim3)")
        new = np.nonzero(sq >= 0)[0]
        vpMatched[new] = np.asarray(mp_id)[sq[new]]
        if vpMatchedKF is not None:
            vpMatchedKF[new] = np.asarray(vpPointsKFs)[sq[new]]
        return n

    def SearchForInitialization(self, F1: FrameSoA, F2: FrameSoA, vbPrevMatched: np.ndarray, windowSize: int = 100):
        """``SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)``
        (ref:src/ORBmatcher.cc:735-878).  ``vbPrevMatched`` (F1.n x 2 float32) is updated in place;
        returns (nmatches, vnMatches12)."""
        lib, h = self.ctx.lib, self.ctx.handle
        assert vbPrevMatched.dtype == np.float32 and vbPrevMatched.flags["C_CONTIGUOUS"]
        assert vbPrevMatched.shape == (F1.n, 2)
        m12 = np.full(F1.n, -1, np.int32)
        a, b = F1.struct(), F2.struct()
        rc = lib.osg_search_for_initialization(h, C.byref(a), C.byref(b), vbPrevMatched.ctypes.data, int(windowSize),
                                               self.mfNNratio, int(self.mbCheckOrientation), m12.ctypes.data)
        return self.ctx.check(rc, "SearchForInitialization"), m12

    @staticmethod
    def _pairs(m12):
        i = np.nonzero(m12 >= 0)[0]
        return np.stack([i, m12[i]], axis=1).astype(np.int64)

    def SearchForTriangulation(self, KF1: KFSide, KF2: KFSide, geom: TriangGeom, bOnlyStereo: bool = False,
                               bCoarse: bool = False):
        """``SearchForTriangulation(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse)``
        (ref:src/ORBmatcher.cc:1045-1328).  Returns (nmatches, vMatchedPairs) with vMatchedPairs an
        (nmatches, 2) array of (KF1 index, KF2 index) in ascending KF1 index, as the reference fills it."""
        lib, h = self.ctx.lib, self.ctx.handle
        m12 = np.full(KF1.n, -1, np.int32)
        a, b, g = KF1.struct(), KF2.struct(), geom.struct()
        rc = lib.osg_search_for_triangulation(h, C.byref(a), C.byref(b), C.byref(g), int(bool(bOnlyStereo)),
                                              int(bool(bCoarse)), int(self.mbCheckOrientation), m12.ctypes.data)
        return self.ctx.check(rc, "SearchForTriangulation"), self._pairs(m12)

    def SearchForTriangulationBatch(self, KF1s, KF2s, geoms, bOnlyStereo: bool = False, bCoarse: bool = False):
        """B keyframe pairs in one launch (LocalMapping::CreateNewMapPoints' neighbour loop); returns
        (nmatches[B], [vMatchedPairs])."""
        lib, h = self.ctx.lib, self.ctx.handle
        B = len(KF1s)
        assert len(KF2s) == B and len(geoms) == B
        a = (_abi.OsgKfSide * B)(*[k.struct() for k in KF1s])
        b = (_abi.OsgKfSide * B)(*[k.struct() for k in KF2s])
        g = (_abi.OsgTriangGeom * B)(*[x.struct() for x in geoms])
        m12 = np.full(sum(k.n for k in KF1s), -1, np.int32)
        nm = np.zeros(B, np.int32)
        rc = lib.osg_search_for_triangulation_batch(h, C.addressof(a), C.addressof(b), C.addressof(g), B,
                                                    int(bool(bOnlyStereo)), int(bool(bCoarse)),
                                                    int(self.mbCheckOrientation), m12.ctypes.data, nm.ctypes.data)
        self.ctx.check(rc, "SearchForTriangulation batch")
        cuts = np.cumsum([0] + [k.n for k in KF1s])
        return nm, [self._pairs(m12[x:y]) for x, y in zip(cuts[:-1], cuts[1:])]

    # ---- batched forms (no reference counterpart: B independent problems in one launch) -------

    def SearchByProjectionBatch(self, Fs, qs, *args, slot_mps=None, slot_takens=None, **kw):
        """B independent SearchByProjection calls of one overload in one launch.  ``Fs`` / ``qs`` are
        sequences of FrameSoA and MPQueries / LastQueries / KFQueries; ``slot_mps`` (updated in place)
        and ``slot_takens`` per problem.  Returns the per-problem match counts."""
        lib, h = self.ctx.lib, self.ctx.handle
        B = len(Fs)
        assert len(qs) == B
        kind = type(qs[0])
        assert all(type(q) is kind for q in qs), "one overload per batch"
        fa = (_abi.OsgFrame * B)(*[F.struct() for F in Fs])
        sizes = [F.n for F in Fs]
        if slot_mps is None:
            slot_mps = [np.full(n, -1, np.int32) for n in sizes]
        for s, n in zip(slot_mps, sizes):
            assert s.dtype == np.int32 and len(s) == n
        slot = np.concatenate(slot_mps) if B else np.zeros(0, np.int32)
        nm = np.zeros(B, np.int32)
        if kind is MPQueries:
            th = args[0] if len(args) > 0 else kw.get("th", 3.0)
            far = args[1] if len(args) > 1 else kw.get("bFarPoints", False)
            thfar = args[2] if len(args) > 2 else kw.get("thFarPoints", 50.0)
            taken = np.concatenate([np.ascontiguousarray(t, np.uint8) for t in slot_takens]) if slot_takens \
                else np.zeros(len(slot), np.uint8)
            qa = (_abi.OsgMpQueries * B)(*[q.struct() for q in qs])
            rc = lib.osg_search_by_projection_mps_batch(h, C.addressof(fa), C.addressof(qa), B, self.mfNNratio,
                                                        float(th), int(bool(far)), float(thfar), slot.ctypes.data,
                                                        taken.ctypes.data, nm.ctypes.data)
        elif kind is LastQueries:
            th = args[0] if len(args) > 0 else kw["th"]
            mono = args[1] if len(args) > 1 else kw["bMono"]
            taken = np.concatenate([np.ascontiguousarray(t, np.uint8) for t in slot_takens]) if slot_takens \
                else np.zeros(len(slot), np.uint8)
            qa = (_abi.OsgLastQueries * B)(*[q.struct() for q in qs])
            rc = lib.osg_search_by_projection_last_batch(h, C.addressof(fa), C.addressof(qa), B, float(th),
                                                         int(bool(mono)), int(self.mbCheckOrientation),
                                                         slot.ctypes.data, taken.ctypes.data, nm.ctypes.data)
        elif kind is KFQueries:
            th = args[0] if len(args) > 0 else kw["th"]
            orb = args[1] if len(args) > 1 else kw["ORBdist"]
            qa = (_abi.OsgKfQueries * B)(*[q.struct() for q in qs])
            rc = lib.osg_search_by_projection_kf_batch(h, C.addressof(fa), C.addressof(qa), B, float(th), int(orb),
                                                       int(self.mbCheckOrientation), slot.ctypes.data,
                                                       nm.ctypes.data)
        else:
            raise TypeError(f"no SearchByProjection overload for {kind.__name__}")
        self.ctx.check(rc, "SearchByProjection batch")
        o = 0
        for s, n in zip(slot_mps, sizes):
            s[:] = slot[o:o + n]
            o += n
        return nm

    def SearchByBoWBatch(self, KFs, others, kf2: bool = False):
        """B independent SearchByBoW calls in one launch; returns (nmatches[B], list of outputs)."""
        lib, h = self.ctx.lib, self.ctx.handle
        B = len(KFs)
        assert len(others) == B
        a = (_abi.OsgBowSide * B)(*[k.struct() for k in KFs])
        b = (_abi.OsgBowSide * B)(*[o.struct() for o in others])
        sizes = [k.n for k in KFs] if kf2 else [o.n for o in others]
        out = np.full(sum(sizes), -1, np.int32)
        nm = np.zeros(B, np.int32)
        fn = lib.osg_search_by_bow_kf_kf_batch if kf2 else lib.osg_search_by_bow_kf_f_batch
        rc = fn(h, C.addressof(a), C.addressof(b), B, self.mfNNratio, int(self.mbCheckOrientation),
                out.ctypes.data, nm.ctypes.data)
        self.ctx.check(rc, "SearchByBoW batch")
        outs, o = [], 0
        for n in sizes:
            outs.append(out[o:o + n].copy())
            o += n
        return nm, outs
