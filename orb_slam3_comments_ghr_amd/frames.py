"""Structure-of-arrays views of the reference's Frame / KeyFrame / MapPoint fields.

These are what the ORB-SLAM3-side adapter gathers before calling the C ABI (see
INTEGRATION.md): plain numpy arrays with the reference's field meaning, plus ``.struct()``
builders for the ctypes mirrors in ``_abi``.  Also the seeded synthetic generators for the
matching configs.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _abi
from .synth import EUROC_BF, EUROC_FX, EUROC_H, EUROC_W


def _p(a):
    return None if a is None else int(a.ctypes.data)


def _c(a, dt):
    return None if a is None else np.ascontiguousarray(a, dtype=dt)


def pos_in_grid(x, y, min_x, min_y, inv_w, inv_h):
    """Frame::PosInGrid (ref:src/Frame.cc:973-989): round() of float products."""
    vx = ((np.float32(x) - np.float32(min_x)) * np.float32(inv_w)).astype(np.float32)
    vy = ((np.float32(y) - np.float32(min_y)) * np.float32(inv_h)).astype(np.float32)

    def cround(v):  # C round(): half away from zero, on the exact float value
        v = v.astype(np.float64)
        return np.where(v >= 0, np.floor(v + 0.5), np.ceil(v - 0.5)).astype(np.int64)

    return cround(vx), cround(vy)


def build_grid(kp_x, kp_y, min_x, min_y, inv_w, inv_h):
    """Frame::AssignFeaturesToGrid (ref:src/Frame.cc:469-507) as CSR, cell = ix*48 + iy."""
    px, py = pos_in_grid(kp_x, kp_y, min_x, min_y, inv_w, inv_h)
    ok = (px >= 0) & (px < _abi.GRID_COLS) & (py >= 0) & (py < _abi.GRID_ROWS)
    cell = np.where(ok, px * _abi.GRID_ROWS + py, -1)
    idx = np.nonzero(ok)[0]
    order = np.argsort(cell[idx], kind="stable")  # stable: ascending feature index inside a cell
    items = idx[order].astype(np.int32)
    counts = np.bincount(cell[idx], minlength=_abi.GRID_CELLS)
    start = np.zeros(_abi.GRID_CELLS + 1, np.int32)
    start[1:] = np.cumsum(counts)
    return start, items


def scale_factors(n_levels=8, factor=1.2):
    s = np.ones(n_levels, np.float32)
    for i in range(1, n_levels):
        s[i] = np.float32(s[i - 1] * np.float32(factor))
    return s


@dataclass
class FrameSoA:
    desc: np.ndarray          # n x 32 uint8
    kp_x: np.ndarray
    kp_y: np.ndarray
    kp_angle: np.ndarray
    kp_octave: np.ndarray
    u_right: np.ndarray | None = None
    min_x: float = 0.0
    max_x: float = float(EUROC_W)
    min_y: float = 0.0
    max_y: float = float(EUROC_H)
    scale: np.ndarray = field(default_factory=scale_factors)
    mb: float = EUROC_BF / EUROC_FX
    mbf: float = EUROC_BF
    nleft: int = -1
    grid_start: np.ndarray | None = None
    grid_idx: np.ndarray | None = None
    # two-camera rig (nleft != -1): keypoints [0, nleft) are mvKeys, [nleft, n) mvKeysRight
    grid_start_r: np.ndarray | None = None
    grid_idx_r: np.ndarray | None = None
    left_to_right: np.ndarray | None = None   # mvLeftToRightMatch[nleft], -1 = none
    right_to_left: np.ndarray | None = None   # mvRightToLeftMatch[n - nleft]

    def __post_init__(self):
        self.desc = _c(self.desc, np.uint8).reshape(-1, 32)
        self.kp_x = _c(self.kp_x, np.float32)
        self.kp_y = _c(self.kp_y, np.float32)
        self.kp_angle = _c(self.kp_angle, np.float32)
        self.kp_octave = _c(self.kp_octave, np.int32)
        self.u_right = _c(self.u_right, np.float32)
        self.scale = _c(self.scale, np.float32)
        self.inv_w = np.float32(np.float32(_abi.GRID_COLS) / np.float32(self.max_x - self.min_x))
        self.inv_h = np.float32(np.float32(_abi.GRID_ROWS) / np.float32(self.max_y - self.min_y))
        self.left_to_right = _c(self.left_to_right, np.int32)
        self.right_to_left = _c(self.right_to_left, np.int32)
        nl = self.n if self.nleft == -1 else self.nleft
        if self.grid_start is None:
            # AssignFeaturesToGrid (ref:src/Frame.cc:469-507): right keypoints go to mGridRight
            # with indices relative to Nleft
            self.grid_start, self.grid_idx = build_grid(self.kp_x[:nl], self.kp_y[:nl], self.min_x, self.min_y,
                                                        self.inv_w, self.inv_h)
        if self.nleft != -1 and self.grid_start_r is None:
            self.grid_start_r, self.grid_idx_r = build_grid(self.kp_x[nl:], self.kp_y[nl:], self.min_x,
                                                            self.min_y, self.inv_w, self.inv_h)

    @property
    def n(self):
        return self.desc.shape[0]

    def struct(self):
        s = _abi.OsgFrame()
        s.n = self.n
        s.nleft = self.nleft
        s.desc = _p(self.desc)
        s.kp_x = _p(self.kp_x)
        s.kp_y = _p(self.kp_y)
        s.kp_angle = _p(self.kp_angle)
        s.kp_octave = _p(self.kp_octave)
        s.u_right = _p(self.u_right)
        s.grid_start = _p(self.grid_start)
        s.grid_idx = _p(self.grid_idx)
        s.grid_start_r = _p(self.grid_start_r)
        s.grid_idx_r = _p(self.grid_idx_r)
        s.left_to_right = _p(self.left_to_right)
        s.right_to_left = _p(self.right_to_left)
        s.min_x, s.max_x, s.min_y, s.max_y = self.min_x, self.max_x, self.min_y, self.max_y
        s.grid_inv_w = float(self.inv_w)
        s.grid_inv_h = float(self.inv_h)
        s.scale_factors = _p(self.scale)
        s.n_levels = len(self.scale)
        s.mb = self.mb
        s.mbf = self.mbf
        return s


@dataclass
class MPQueries:
    """Local map points after Frame::isInFrustum (a5)."""
    mp_id: np.ndarray
    desc: np.ndarray
    usable: np.ndarray
    has_obs: np.ndarray
    in_view: np.ndarray
    proj_x: np.ndarray
    proj_y: np.ndarray
    proj_xr: np.ndarray
    view_cos: np.ndarray
    pred_level: np.ndarray
    track_depth: np.ndarray
    # right camera of a two-camera rig (Frame::isInFrustum with bRight, ref:src/Frame.cc:676-782)
    in_view_r: np.ndarray | None = None     # mbTrackInViewR
    proj_yr: np.ndarray | None = None       # mTrackProjYR (x is proj_xr)
    view_cos_r: np.ndarray | None = None    # mTrackViewCosR
    pred_level_r: np.ndarray | None = None  # mnTrackScaleLevelR, -1 = none

    _FIELDS = [("mp_id", np.int32), ("desc", np.uint8), ("usable", np.uint8), ("has_obs", np.uint8),
               ("in_view", np.uint8), ("proj_x", np.float32), ("proj_y", np.float32),
               ("proj_xr", np.float32), ("view_cos", np.float32), ("pred_level", np.int32),
               ("track_depth", np.float32), ("in_view_r", np.uint8), ("proj_yr", np.float32),
               ("view_cos_r", np.float32), ("pred_level_r", np.int32)]

    def __post_init__(self):
        for k, dt in self._FIELDS:
            setattr(self, k, _c(getattr(self, k), dt))

    def struct(self):
        s = _abi.OsgMpQueries()
        s.n = len(self.mp_id)
        for k, _ in self._FIELDS:
            setattr(s, k, _p(getattr(self, k)))
        return s


@dataclass
class LastQueries:
    """LastFrame map points projected into the current frame (a6)."""
    mp_id: np.ndarray
    desc: np.ndarray
    valid: np.ndarray
    has_obs: np.ndarray
    u: np.ndarray
    v: np.ndarray
    invz: np.ndarray
    octave: np.ndarray
    angle: np.ndarray
    tlc_z: float = 0.0
    u_r: np.ndarray | None = None   # mpCamera->project(Trl * x3Dc), two-camera rig only
    v_r: np.ndarray | None = None

    _FIELDS = [("mp_id", np.int32), ("desc", np.uint8), ("valid", np.uint8), ("has_obs", np.uint8),
               ("u", np.float32), ("v", np.float32), ("invz", np.float32), ("octave", np.int32),
               ("angle", np.float32), ("u_r", np.float32), ("v_r", np.float32)]

    def __post_init__(self):
        for k, dt in self._FIELDS:
            setattr(self, k, _c(getattr(self, k), dt))

    def struct(self):
        s = _abi.OsgLastQueries()
        s.n = len(self.mp_id)
        for k, _ in self._FIELDS:
            setattr(s, k, _p(getattr(self, k)))
        s.tlc_z = float(self.tlc_z)
        return s


@dataclass
class KFQueries:
    """KeyFrame map points projected into the current frame (a7, relocalisation)."""
    mp_id: np.ndarray
    desc: np.ndarray
    valid: np.ndarray
    u: np.ndarray
    v: np.ndarray
    pred_level: np.ndarray
    angle: np.ndarray

    def __post_init__(self):
        for k, dt in [("mp_id", np.int32), ("desc", np.uint8), ("valid", np.uint8), ("u", np.float32),
                      ("v", np.float32), ("pred_level", np.int32), ("angle", np.float32)]:
            setattr(self, k, _c(getattr(self, k), dt))

    def struct(self):
        s = _abi.OsgKfQueries()
        s.n = len(self.mp_id)
        for k in ["mp_id", "desc", "valid", "u", "v", "pred_level", "angle"]:
            setattr(s, k, _p(getattr(self, k)))
        return s


@dataclass
class FuseQueries:
    """MapPoints projected into a KeyFrame for ORBmatcher::Fuse (ref:src/ORBmatcher.cc:1366-1437):
    the caller's pre-search filters folded into ``valid``, the projection, ur = u - bf * invz,
    PredictScale, and the KeyFrame's mvInvLevelSigma2."""
    desc: np.ndarray
    valid: np.ndarray
    u: np.ndarray
    v: np.ndarray
    ur: np.ndarray | None
    pred_level: np.ndarray
    inv_level_sigma2: np.ndarray

    def __post_init__(self):
        for k, dt in [("desc", np.uint8), ("valid", np.uint8), ("u", np.float32), ("v", np.float32),
                      ("ur", np.float32), ("pred_level", np.int32), ("inv_level_sigma2", np.float32)]:
            setattr(self, k, _c(getattr(self, k), dt))

    @property
    def n(self):
        return len(self.valid)

    def struct(self):
        s = _abi.OsgFuseQueries()
        s.n = self.n
        for k in ["desc", "valid", "u", "v", "ur", "pred_level", "inv_level_sigma2"]:
            setattr(s, k, _p(getattr(self, k)))
        return s


def inv_level_sigma2(scale):
    """ORBextractor: mvLevelSigma2 = s * s, mvInvLevelSigma2 = 1.0f / mvLevelSigma2 (float)."""
    s = np.asarray(scale, np.float32)
    return (np.float32(1.0) / (s * s)).astype(np.float32)


@dataclass
class BowSide:
    """One side of SearchByBoW: descriptors, angles, map-point slots and the FeatureVector."""
    desc: np.ndarray
    angle: np.ndarray
    mp_id: np.ndarray
    mp_good: np.ndarray
    node_id: np.ndarray
    node_start: np.ndarray
    feat: np.ndarray
    nleft: int = -1

    def __post_init__(self):
        self.desc = _c(self.desc, np.uint8).reshape(-1, 32)
        self.angle = _c(self.angle, np.float32)
        self.mp_id = _c(self.mp_id, np.int32)
        self.mp_good = _c(self.mp_good, np.uint8)
        self.node_id = _c(self.node_id, np.uint32)
        self.node_start = _c(self.node_start, np.int32)
        self.feat = _c(self.feat, np.int32)

    @property
    def n(self):
        return self.desc.shape[0]

    def struct(self):
        s = _abi.OsgBowSide()
        s.n = self.n
        s.nleft = self.nleft
        s.desc = _p(self.desc)
        s.angle = _p(self.angle)
        s.mp_id = _p(self.mp_id)
        s.mp_good = _p(self.mp_good)
        s.fv.n_nodes = len(self.node_id)
        s.fv.node_id = _p(self.node_id)
        s.fv.node_start = _p(self.node_start)
        s.fv.feat = _p(self.feat)
        return s


# ------------------------------------------------------------------------------- generators

def _flip(rng, rows, p):
    bits = np.unpackbits(rows, axis=1)
    return np.packbits(bits ^ (rng.random(bits.shape) < p).astype(np.uint8), axis=1)


def synth_frame(rng, n=1200, stereo=True, n_levels=8, width=EUROC_W, height=EUROC_H):
    """Keypoints uniform in the image (EuRoC 752x480 by default), octave ~ geometric(1/1.2)
    truncated to 8 levels, angle U[0,360), 60 % with a stereo u_R (bf = 47.9)."""
    x = rng.uniform(0, width, n).astype(np.float32)
    y = rng.uniform(0, height, n).astype(np.float32)
    p = np.array([1.2 ** -i for i in range(n_levels)])
    oct_ = rng.choice(n_levels, size=n, p=p / p.sum()).astype(np.int32)
    ang = rng.uniform(0, 360, n).astype(np.float32)
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    ur = None
    if stereo:
        depth = rng.uniform(1, 10, n)
        ur = np.where(rng.random(n) < 0.6, x - EUROC_BF / depth, -1.0).astype(np.float32)
    return FrameSoA(desc=desc, kp_x=x, kp_y=y, kp_angle=ang, kp_octave=oct_, u_right=ur,
                    scale=scale_factors(n_levels), max_x=float(width), max_y=float(height))


def synth_mp_queries(rng, F: FrameSoA, m=3000, noise_px=3.0, match_frac=0.6):
    """Local map points whose projections land near frame keypoints (a5)."""
    n = F.n
    tgt = rng.integers(0, n, m)
    is_match = rng.random(m) < match_frac
    px = np.where(is_match, F.kp_x[tgt] + rng.normal(0, noise_px, m), rng.uniform(0, F.max_x, m))
    py = np.where(is_match, F.kp_y[tgt] + rng.normal(0, noise_px, m), rng.uniform(0, F.max_y, m))
    desc = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    desc[is_match] = _flip(rng, F.desc[tgt[is_match]], 0.06)
    lvl = np.clip(F.kp_octave[tgt] + rng.integers(-1, 2, m), 0, len(F.scale) - 1)
    depth = rng.uniform(0.5, 60.0, m)
    pxr = (px - EUROC_BF / depth).astype(np.float32)
    if F.u_right is not None:
        pxr = np.where(is_match & (F.u_right[tgt] > 0), F.u_right[tgt] + rng.normal(0, 1.0, m), pxr)
    return MPQueries(
        mp_id=np.arange(1000, 1000 + m), desc=desc, usable=rng.random(m) < 0.98,
        has_obs=rng.random(m) < 0.93, in_view=rng.random(m) < 0.85, proj_x=px, proj_y=py,
        proj_xr=pxr, view_cos=rng.uniform(0.99, 1.0, m), pred_level=lvl, track_depth=depth)


def synth_slots(rng, n, frac_assigned=0.1, frac_taken=0.7, id_base=500000):
    slot_mp = np.where(rng.random(n) < frac_assigned, id_base + np.arange(n), -1).astype(np.int32)
    slot_taken = ((slot_mp >= 0) & (rng.random(n) < frac_taken)).astype(np.uint8)
    return slot_mp, slot_taken


def synth_last_queries(rng, F: FrameSoA, n_last=1000, noise_px=2.0, match_frac=0.7, tlc_z=0.0):
    n = F.n
    tgt = rng.integers(0, n, n_last)
    is_match = rng.random(n_last) < match_frac
    u = np.where(is_match, F.kp_x[tgt] + rng.normal(0, noise_px, n_last), rng.uniform(-20, F.max_x + 20, n_last))
    v = np.where(is_match, F.kp_y[tgt] + rng.normal(0, noise_px, n_last), rng.uniform(-20, F.max_y + 20, n_last))
    desc = rng.integers(0, 256, (n_last, 32), dtype=np.uint8)
    desc[is_match] = _flip(rng, F.desc[tgt[is_match]], 0.06)
    depth = rng.uniform(1, 20, n_last)
    invz = (1.0 / depth * np.where(rng.random(n_last) < 0.02, -1, 1)).astype(np.float32)
    if F.u_right is not None:
        # make the stereo check pass for most true matches: u_R(target) ~ u - mbf*invz
        pass
    octv = np.where(is_match, F.kp_octave[tgt], rng.integers(0, len(F.scale), n_last)).astype(np.int32)
    ang = np.where(is_match, F.kp_angle[tgt] + 7.0 + rng.normal(0, 3, n_last), rng.uniform(0, 360, n_last))
    ang = np.mod(ang, 360).astype(np.float32)
    mp_id = np.where(rng.random(n_last) < 0.9, 2000 + np.arange(n_last), -1)
    valid = (mp_id >= 0) & (rng.random(n_last) < 0.9)
    return LastQueries(mp_id=mp_id, desc=desc, valid=valid, has_obs=rng.random(n_last) < 0.9, u=u, v=v,
                       invz=invz, octave=octv, angle=ang, tlc_z=tlc_z)


def synth_kf_queries(rng, F: FrameSoA, n_kf=1000, noise_px=2.0, match_frac=0.6):
    n = F.n
    tgt = rng.integers(0, n, n_kf)
    is_match = rng.random(n_kf) < match_frac
    u = np.where(is_match, F.kp_x[tgt] + rng.normal(0, noise_px, n_kf), rng.uniform(0, EUROC_W, n_kf))
    v = np.where(is_match, F.kp_y[tgt] + rng.normal(0, noise_px, n_kf), rng.uniform(0, EUROC_H, n_kf))
    desc = rng.integers(0, 256, (n_kf, 32), dtype=np.uint8)
    desc[is_match] = _flip(rng, F.desc[tgt[is_match]], 0.06)
    lvl = np.clip(F.kp_octave[tgt] + rng.integers(-1, 2, n_kf), 0, len(F.scale) - 1)
    ang = np.where(is_match, F.kp_angle[tgt] + 7.0 + rng.normal(0, 3, n_kf), rng.uniform(0, 360, n_kf))
    return KFQueries(mp_id=3000 + np.arange(n_kf), desc=desc, valid=rng.random(n_kf) < 0.7, u=u, v=v,
                     pred_level=lvl, angle=np.mod(ang, 360))


def synth_fuse_queries(rng, F: FrameSoA, m=1000, noise_px=1.0, match_frac=0.6, valid_frac=0.85, right=False):
    """MapPoints of a neighbouring keyframe projected into keyframe F (LocalMapping::SearchInNeighbors):
    match_frac of them land near a keypoint of F (pixel noise, the keypoint's octave or one above as
    the predicted level, a noisy copy of its descriptor, ur near its u_R), the rest anywhere."""
    lo, hi = (F.nleft, F.n) if right else (0, F.n if F.nleft < 0 else F.nleft)
    tgt = rng.integers(lo, max(hi, lo + 1), m)
    is_match = (rng.random(m) < match_frac) & (hi > lo)
    tgt = np.minimum(tgt, max(F.n - 1, 0))
    u = np.where(is_match, F.kp_x[tgt] + rng.normal(0, noise_px, m), rng.uniform(F.min_x, F.max_x, m))
    v = np.where(is_match, F.kp_y[tgt] + rng.normal(0, noise_px, m), rng.uniform(F.min_y, F.max_y, m))
    nl = len(F.scale)
    lvl = np.where(is_match, np.clip(F.kp_octave[tgt] + rng.integers(0, 2, m), 0, nl - 1), rng.integers(0, nl, m))
    desc = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    desc[is_match] = _flip(rng, F.desc[tgt[is_match]], 0.05)
    ur = u - EUROC_BF / rng.uniform(1, 10, m)
    if F.u_right is not None:
        loc = tgt - (F.nleft if right else 0)
        kr = F.u_right[np.clip(loc, 0, F.n - 1)]
        ur = np.where(is_match & (kr >= 0), kr + rng.normal(0, noise_px, m), ur)
    return FuseQueries(desc=desc, valid=rng.random(m) < valid_frac, u=u, v=v, ur=ur, pred_level=lvl,
                       inv_level_sigma2=inv_level_sigma2(F.scale))


def synth_sim3_pair(rng, n1=1000, n2=1000, shared=0.5, noise_px=1.0, valid_frac=0.9, cross_frac=0.1):
    """SearchBySim3's inputs (ref:src/ORBmatcher.cc:1696-1939): two keyframes and, per keypoint of each,
    its MapPoint projected into the other (FuseQueries, one per slot).  `shared` of KF1's slots see a
    point KF2 also sees: q12 lands near that KF2 keypoint with a noisy copy of its descriptor and q21
    back near the KF1 keypoint (mutual); `cross_frac` of those are redirected so the two directions
    disagree; the rest project anywhere with random descriptors."""
    F1 = synth_frame(rng, n=n1, stereo=False)
    F2 = synth_frame(rng, n=n2, stereo=False)
    nl = len(F1.scale)

    def q_for(F, m):
        return dict(u=rng.uniform(F.min_x, F.max_x, m).astype(np.float32),
                    v=rng.uniform(F.min_y, F.max_y, m).astype(np.float32),
                    lvl=rng.integers(0, nl, m).astype(np.int32),
                    desc=rng.integers(0, 256, (m, 32), dtype=np.uint8))
    a, b = q_for(F2, n1), q_for(F1, n2)
    k = int(shared * min(n1, n2))
    i1 = rng.choice(n1, k, replace=False)
    i2 = rng.choice(n2, k, replace=False)

    def aim(q, F, src, dst):
        q["u"][src] = F.kp_x[dst] + rng.normal(0, noise_px, len(src))
        q["v"][src] = F.kp_y[dst] + rng.normal(0, noise_px, len(src))
        q["lvl"][src] = np.clip(F.kp_octave[dst] + rng.integers(0, 2, len(src)), 0, nl - 1)
        q["desc"][src] = _flip(rng, F.desc[dst], 0.05)
    aim(a, F2, i1, i2)
    back = i1.copy()
    cross = rng.random(k) < cross_frac
    back[cross] = rng.integers(0, n1, int(cross.sum()))
    aim(b, F1, i2, back)

    def fq(q, F, m):
        return FuseQueries(desc=q["desc"], valid=rng.random(m) < valid_frac, u=q["u"], v=q["v"], ur=None,
                           pred_level=q["lvl"], inv_level_sigma2=inv_level_sigma2(F.scale))
    return F1, F2, fq(a, F2, n1), fq(b, F1, n2)


def _featvec(rng, n, n_nodes, zipf=1.1, node_base=0):
    w = 1.0 / np.arange(1, n_nodes + 1) ** zipf
    node_of = rng.choice(n_nodes, size=n, p=w / w.sum())
    ids = np.sort(rng.choice(np.arange(node_base, node_base + 10 * n_nodes), size=n_nodes, replace=False))
    used = np.unique(node_of)
    node_id = ids[used].astype(np.uint32)
    node_start = np.zeros(len(used) + 1, np.int32)
    feat = []
    for k, nd in enumerate(used):
        f = np.nonzero(node_of == nd)[0]
        feat.append(f)
        node_start[k + 1] = node_start[k] + len(f)
    return node_id, node_start, np.concatenate(feat).astype(np.int32), node_of, ids


def synth_bow_pair(rng, n_kf=1200, n_f=1200, n_nodes=100, mp_frac=0.7, copy_frac=0.6, flip=0.06,
                   f_is_kf=False, nleft_kf=-1, nleft_f=-1):
    """KF and F (or KF2) sharing a vocabulary: 60 % of the second side's descriptors are noisy copies
    of KF features (same node), angle offset +7 deg +- 3.  ``nleft_*`` != -1 makes
    that side a two-camera rig: indices >= nleft are right-camera keypoints, and its FeatureVector
    holds both (ComputeBoW runs on the vconcat'ed descriptors)."""
    kf_desc = rng.integers(0, 256, (n_kf, 32), dtype=np.uint8)
    kf_ang = rng.uniform(0, 360, n_kf).astype(np.float32)
    w = 1.0 / np.arange(1, n_nodes + 1) ** 1.1
    node_ids = np.sort(rng.choice(np.arange(0, 10 * n_nodes), size=n_nodes, replace=False)).astype(np.uint32)
    kf_node = rng.choice(n_nodes, size=n_kf, p=w / w.sum())
    f_desc = rng.integers(0, 256, (n_f, 32), dtype=np.uint8)
    f_ang = rng.uniform(0, 360, n_f).astype(np.float32)
    f_node = rng.choice(n_nodes, size=n_f, p=w / w.sum())
    src = rng.integers(0, n_kf, n_f)
    cp = rng.random(n_f) < copy_frac
    f_desc[cp] = _flip(rng, kf_desc[src[cp]], flip)
    f_node[cp] = kf_node[src[cp]]
    f_ang[cp] = np.mod(kf_ang[src[cp]] - 7.0 - rng.normal(0, 3, cp.sum()), 360).astype(np.float32)

    def fv(node_of):
        used = np.unique(node_of)
        start = np.zeros(len(used) + 1, np.int32)
        feats = []
        for k, nd in enumerate(used):
            f = np.nonzero(node_of == nd)[0]
            feats.append(f)
            start[k + 1] = start[k] + len(f)
        return node_ids[used], start, np.concatenate(feats).astype(np.int32)

    a = fv(kf_node)
    b = fv(f_node)
    kf_mp = np.where(rng.random(n_kf) < mp_frac, 10000 + np.arange(n_kf), -1).astype(np.int32)
    kf_good = ((kf_mp >= 0) & (rng.random(n_kf) < 0.98)).astype(np.uint8)
    KF = BowSide(kf_desc, kf_ang, kf_mp, kf_good, *a, nleft=nleft_kf)
    if f_is_kf:
        f_mp = np.where(rng.random(n_f) < mp_frac, 20000 + np.arange(n_f), -1).astype(np.int32)
        f_good = ((f_mp >= 0) & (rng.random(n_f) < 0.98)).astype(np.uint8)
    else:
        f_mp = np.full(n_f, -1, np.int32)
        f_good = np.zeros(n_f, np.uint8)
    Fb = BowSide(f_desc, f_ang, f_mp, f_good, *b, nleft=nleft_f)
    return KF, Fb


# ---------------------------------------------------------------- two-camera rig generators

def synth_frame_two_cam(rng, n_left=600, n_right=600, stereo_frac=0.5, n_levels=8, width=EUROC_W, height=EUROC_H):
    """A two-camera Frame (ref:src/Frame.cc:1485-1536): Nleft = n_left, N = n_left + n_right,
    descriptors vconcat(left, right).  ``stereo_frac`` of the right keypoints are stereo partners
    of a left keypoint (ComputeStereoFishEyeMatches): shifted by a disparity, same octave, a
    noisy copy of the left descriptor; mvLeftToRightMatch / mvRightToLeftMatch record the pairs."""
    L = synth_frame(rng, n=n_left, stereo=False, n_levels=n_levels, width=width, height=height)
    xr = rng.uniform(0, width, n_right).astype(np.float32)
    yr = rng.uniform(0, height, n_right).astype(np.float32)
    p = np.array([1.2 ** -i for i in range(n_levels)])
    octr = rng.choice(n_levels, size=n_right, p=p / p.sum()).astype(np.int32)
    angr = rng.uniform(0, 360, n_right).astype(np.float32)
    descr = rng.integers(0, 256, (n_right, 32), dtype=np.uint8)
    n_pair = int(stereo_frac * min(n_left, n_right))
    li = rng.choice(n_left, size=n_pair, replace=False)
    ri = rng.choice(n_right, size=n_pair, replace=False)
    disp = rng.uniform(2, 60, n_pair)
    xr[ri] = np.clip(L.kp_x[li] - disp, 0, width - 1)
    yr[ri] = np.clip(L.kp_y[li] + rng.normal(0, 0.5, n_pair), 0, height - 1)
    octr[ri] = L.kp_octave[li]
    angr[ri] = np.mod(L.kp_angle[li] + rng.normal(0, 2, n_pair), 360)
    descr[ri] = _flip(rng, L.desc[li], 0.03)
    l2r = np.full(n_left, -1, np.int32)
    r2l = np.full(n_right, -1, np.int32)
    l2r[li] = ri
    r2l[ri] = li
    return FrameSoA(desc=np.concatenate([L.desc, descr]), kp_x=np.concatenate([L.kp_x, xr]),
                    kp_y=np.concatenate([L.kp_y, yr]), kp_angle=np.concatenate([L.kp_angle, angr]),
                    kp_octave=np.concatenate([L.kp_octave, octr]), u_right=None, nleft=n_left,
                    left_to_right=l2r, right_to_left=r2l, scale=scale_factors(n_levels),
                    max_x=float(width), max_y=float(height))


def synth_mp_queries_two_cam(rng, F: FrameSoA, m=1500, noise_px=2.5, match_frac=0.7, right_only_frac=0.2):
    """a5 queries for a two-camera Frame: the left-camera fields as synth_mp_queries, plus the
    right projection (mbTrackInViewR, mTrackProjXR/YR, mTrackViewCosR, mnTrackScaleLevelR).
    Matched queries copy a left keypoint (projected near its stereo partner on the right when it
    has one) or, for ``right_only_frac`` of them, a right keypoint."""
    nl, nr = F.nleft, F.n - F.nleft
    nlev = len(F.scale)
    is_match = rng.random(m) < match_frac
    right_only = is_match & (rng.random(m) < right_only_frac)
    tl = rng.integers(0, nl, m)
    tr = np.where(right_only, rng.integers(0, nr, m), F.left_to_right[tl])
    has_r = tr >= 0
    trc = np.maximum(tr, 0)
    px = np.where(is_match & ~right_only, F.kp_x[tl] + rng.normal(0, noise_px, m), rng.uniform(0, F.max_x, m))
    py = np.where(is_match & ~right_only, F.kp_y[tl] + rng.normal(0, noise_px, m), rng.uniform(0, F.max_y, m))
    pxr = np.where(is_match & has_r, F.kp_x[nl + trc] + rng.normal(0, noise_px, m), rng.uniform(0, F.max_x, m))
    pyr = np.where(is_match & has_r, F.kp_y[nl + trc] + rng.normal(0, noise_px, m), rng.uniform(0, F.max_y, m))
    desc = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    lm = is_match & ~right_only
    desc[lm] = _flip(rng, F.desc[tl[lm]], 0.06)
    desc[right_only] = _flip(rng, F.desc[nl + trc[right_only]], 0.06)
    lvl = np.clip(F.kp_octave[tl] + rng.integers(-1, 2, m), 0, nlev - 1)
    lvl_r = np.clip(F.kp_octave[nl + trc] + rng.integers(-1, 2, m), 0, nlev - 1)
    lvl_r = np.where(rng.random(m) < 0.1, -1, lvl_r)
    depth = rng.uniform(0.5, 60.0, m)
    return MPQueries(
        mp_id=np.arange(1000, 1000 + m), desc=desc, usable=rng.random(m) < 0.98,
        has_obs=rng.random(m) < 0.93, in_view=rng.random(m) < 0.8, proj_x=px, proj_y=py,
        proj_xr=pxr, view_cos=rng.uniform(0.99, 1.0, m), pred_level=lvl, track_depth=depth,
        in_view_r=rng.random(m) < 0.75, proj_yr=pyr, view_cos_r=rng.uniform(0.99, 1.0, m),
        pred_level_r=lvl_r)


def synth_last_queries_two_cam(rng, F: FrameSoA, n_last=800, noise_px=2.0, match_frac=0.7, tlc_z=0.0):
    """a6 queries for a two-camera current Frame: left projection as synth_last_queries, plus the
    right-camera projection (u_r, v_r) near the left target's stereo partner when it has one."""
    nl = F.nleft
    L = synth_last_queries(rng, FrameSoA(desc=F.desc[:nl], kp_x=F.kp_x[:nl], kp_y=F.kp_y[:nl],
                                         kp_angle=F.kp_angle[:nl], kp_octave=F.kp_octave[:nl],
                                         scale=F.scale, max_x=F.max_x, max_y=F.max_y),
                           n_last=n_last, noise_px=noise_px, match_frac=match_frac, tlc_z=tlc_z)
    # nearest left keypoint of each projection stands in for the target
    tl = np.argmin(np.abs(L.u[:, None] - F.kp_x[None, :nl]) + np.abs(L.v[:, None] - F.kp_y[None, :nl]), axis=1)
    tr = F.left_to_right[tl]
    ok = tr >= 0
    trc = np.maximum(tr, 0)
    L.u_r = np.where(ok, F.kp_x[nl + trc] + rng.normal(0, noise_px, n_last),
                     rng.uniform(-20, F.max_x + 20, n_last)).astype(np.float32)
    L.v_r = np.where(ok, F.kp_y[nl + trc] + rng.normal(0, noise_px, n_last),
                     rng.uniform(-20, F.max_y + 20, n_last)).astype(np.float32)
    return L


# ------------------------------------------------------------- b3 SearchForTriangulation

@dataclass
class KFSide:
    """One keyframe of SearchForTriangulation (osg_kf_side): keypoints as the reference indexes them
    (mvKeysUn, or mvKeys / mvKeysRight on a two-camera rig), mvuRight, MapPoint presence, the level
    tables and mFeatVec as CSR."""
    desc: np.ndarray
    kp_x: np.ndarray
    kp_y: np.ndarray
    kp_angle: np.ndarray
    kp_octave: np.ndarray
    u_right: np.ndarray | None
    has_mp: np.ndarray
    node_id: np.ndarray
    node_start: np.ndarray
    feat: np.ndarray
    nleft: int = -1
    two_cam: int = 0
    scale: np.ndarray = field(default_factory=scale_factors)

    def __post_init__(self):
        self.desc = _c(self.desc, np.uint8).reshape(-1, 32)
        self.kp_x = _c(self.kp_x, np.float32)
        self.kp_y = _c(self.kp_y, np.float32)
        self.kp_angle = _c(self.kp_angle, np.float32)
        self.kp_octave = _c(self.kp_octave, np.int32)
        self.u_right = _c(self.u_right, np.float32)
        self.has_mp = _c(self.has_mp, np.uint8)
        self.node_id = _c(self.node_id, np.uint32)
        self.node_start = _c(self.node_start, np.int32)
        self.feat = _c(self.feat, np.int32)
        self.scale = _c(self.scale, np.float32)
        self.level_sigma2 = (self.scale * self.scale).astype(np.float32)  # ORBextractor: s * s in float

    @property
    def n(self):
        return self.desc.shape[0]

    def struct(self):
        s = _abi.OsgKfSide()
        s.n, s.nleft, s.two_cam = self.n, self.nleft, int(self.two_cam)
        s.desc = _p(self.desc)
        s.kp_x, s.kp_y = _p(self.kp_x), _p(self.kp_y)
        s.kp_angle, s.kp_octave = _p(self.kp_angle), _p(self.kp_octave)
        s.u_right = _p(self.u_right)
        s.has_mp = _p(self.has_mp)
        s.level_sigma2 = _p(self.level_sigma2)
        s.scale_factors = _p(self.scale)
        s.n_levels = len(self.scale)
        s.fv.n_nodes = len(self.node_id)
        s.fv.node_id = _p(self.node_id)
        s.fv.node_start = _p(self.node_start)
        s.fv.feat = _p(self.feat)
        return s


@dataclass
class TriangGeom:
    """The epipole and the fundamental matrices the reference builds before its loop
    (ref:src/ORBmatcher.cc:1052-1083; Pinhole.cpp:194-197): F12[k] for k = 2 * bRight1 + bRight2."""
    ep: tuple
    F12: np.ndarray            # (4, 3, 3) float32; [0] only without a rig
    pinhole: bool = True
    R12: np.ndarray | None = None   # KannalaBrandt8: (4, 3, 3) float32 per camera pair
    t12: np.ndarray | None = None   # (4, 3)
    kb: np.ndarray | None = None    # (4, 8): KF1 mpCamera, mpCamera2, KF2 mpCamera, mpCamera2

    def struct(self):
        s = _abi.OsgTriangGeom()
        s.ep_x, s.ep_y = float(self.ep[0]), float(self.ep[1])
        F = np.zeros((4, 3, 3), np.float32)
        F[:len(self.F12)] = self.F12
        for i, v in enumerate(F.reshape(-1)):
            s.F12[i] = float(v)
        s.pinhole = int(bool(self.pinhole))
        for name, shape in (("R12", (4, 3, 3)), ("t12", (4, 3)), ("kb", (4, 8))):
            a = getattr(self, name)
            if a is None:
                continue
            z = np.zeros(shape, np.float32)
            z[:len(a)] = a
            dst = getattr(s, name)
            for i, v in enumerate(z.reshape(-1)):
                dst[i] = float(v)
        return s


KB8_TRIANG = np.array([458.654, 457.296, 367.215, 248.375, 3.48e-3, 7.15e-4, -2.05e-3, 2.03e-4], np.float32)


def kb8_project(p, X):
    """KannalaBrandt8::project in float64 (test geometry; the operators take float keypoints)."""
    X = np.asarray(X, np.float64)
    r2 = np.hypot(X[..., 0], X[..., 1])
    theta = np.arctan2(r2, X[..., 2])
    psi = np.arctan2(X[..., 1], X[..., 0])
    r = theta + p[4] * theta ** 3 + p[5] * theta ** 5 + p[6] * theta ** 7 + p[7] * theta ** 9
    return np.stack([p[0] * r * np.cos(psi) + p[2], p[1] * r * np.sin(psi) + p[3]], -1)


def _rot(rng, deg):
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    th = np.deg2rad(deg)
    Kx = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def fundamental(K1, K2, R12, t12):
    """Pinhole::epipolarConstrain's F12 = K1^-T [t12]x R12 K2^-1 (float64 here, stored as float)."""
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    return (np.linalg.inv(K1).T @ tx @ R12 @ np.linalg.inv(K2)).astype(np.float32)


def synth_triang_pair(rng, n1=1000, n2=1000, n_nodes=100, common=0.6, mp_frac=0.5, stereo=True, forward=False,
                      two_cam=False, noise=0.7, flip=0.05, n_levels=8, distract=0.15, kb8=False):
    """Two keyframes seeing one scene (EuRoC pinhole, 752x480): KF2 is KF1 moved 0.25 m sideways
    (``forward``: 0.4 m along the optical axis, so the epipole lies in the image) and turned 2 deg.
    ``common`` of the keypoints are projections of shared points (noise ``noise`` px x 1.2^octave,
    noisy descriptor copies, same vocabulary node, angle offset -7 +- 3 deg); the rest are random.
    ``mp_frac`` of each side already carry a MapPoint; ``stereo`` gives half of them a mvuRight.
    ``two_cam``: each keyframe is a two-camera rig (Nleft = n/2; right camera 0.11 m to the right),
    keypoints [0, Nleft) in the left camera, the rest in the right one.  ``kb8``: KannalaBrandt8 cameras
    (EuRoC focal, TUM-VI-like distortion): shared keypoints are KB8 projections of points 2-8 m in front
    and the geometry carries R12 / t12 / camera parameters for the triangulating epipolarConstrain.
    Returns (KF1, KF2, geom)."""
    from .synth import EUROC_CX, EUROC_CY, EUROC_FY
    K = np.array([[EUROC_FX, 0, EUROC_CX], [0, EUROC_FY, EUROC_CY], [0, 0, 1.0]])
    R2 = _rot(rng, 2.0)
    C2 = np.array([0.05, 0.01, 0.4]) if forward else np.array([0.25, 0.02, 0.03])
    Tcw = {(1, 0): (np.eye(3), np.zeros(3)), (2, 0): (R2, -R2 @ C2)}
    b = np.array([-0.11, 0.0, 0.0])  # right camera: x_r = x_l + b
    if two_cam:
        for k in (1, 2):
            R, t = Tcw[(k, 0)]
            Tcw[(k, 1)] = (R, t + b)
    ns = (n1, n2)
    nleft = [n // 2 if two_cam else -1 for n in ns]
    cams = [np.where(np.arange(n) < nl, 0, 1) if two_cam else np.zeros(n, int) for n, nl in zip(ns, nleft)]
    p = np.array([1.2 ** -i for i in range(n_levels)])
    octs = [rng.choice(n_levels, size=n, p=p / p.sum()).astype(np.int32) for n in ns]
    xs = [rng.uniform(0, EUROC_W, n) for n in ns]
    ys = [rng.uniform(0, EUROC_H, n) for n in ns]
    angs = [rng.uniform(0, 360, n) for n in ns]
    descs = [rng.integers(0, 256, (n, 32), dtype=np.uint8) for n in ns]
    w = 1.0 / np.arange(1, n_nodes + 1) ** 1.1
    nodes = [rng.choice(n_nodes, size=n, p=w / w.sum()) for n in ns]
    depth = [rng.uniform(1, 10, n) for n in ns]
    # shared points: pick KF1 keypoints, back-project to a depth, reproject into KF2's camera
    m = int(common * min(n1, n2))
    i1 = rng.choice(n1, size=m, replace=False)
    i2 = rng.choice(n2, size=m, replace=False)
    Kinv = np.linalg.inv(K)
    keep = np.zeros(m, bool)
    for j in range(m):
        a, c = i1[j], i2[j]
        R1, t1 = Tcw[(1, cams[0][a])]
        if kb8:
            Xc = np.array([rng.uniform(-4, 4), rng.uniform(-3, 3), rng.uniform(2, 8)])
            u1 = kb8_project(KB8_TRIANG, Xc)
            if not (0 <= u1[0] < EUROC_W and 0 <= u1[1] < EUROC_H):
                continue
            xs[0][a], ys[0][a] = u1
        else:
            Xc = Kinv @ np.array([xs[0][a], ys[0][a], 1.0]) * rng.uniform(2, 8)
        Xw = R1.T @ (Xc - t1)
        R, t = Tcw[(2, cams[1][c])]
        X2 = R @ Xw + t
        if X2[2] <= 0.1:
            continue
        u = kb8_project(KB8_TRIANG, X2) if kb8 else K @ (X2 / X2[2])
        if not (0 <= u[0] < EUROC_W and 0 <= u[1] < EUROC_H):
            continue
        keep[j] = True
        s = 1.2 ** octs[0][a]
        octs[1][c] = octs[0][a]
        xs[1][c] = u[0] + rng.normal(0, noise * s)
        ys[1][c] = u[1] + rng.normal(0, noise * s)
        xs[0][a] += rng.normal(0, noise * s)
        ys[0][a] += rng.normal(0, noise * s)
        descs[1][c] = _flip(rng, descs[0][a][None], flip)[0]
        nodes[1][c] = nodes[0][a]
        angs[1][c] = np.mod(angs[0][a] - 7.0 - rng.normal(0, 3), 360)
        depth[1][c] = X2[2]
    # distractors: KF2 keypoints outside the shared set that copy a shared KF1 descriptor (a third
    # exactly: ties in node order) in the same node, at a random position (or, ``forward``, beside
    # the epipole), so the epipolar / epipole tests and the '<=' tie rule decide the best match
    rest = np.setdiff1d(np.arange(n2), i2[keep])
    src = i1[keep]
    n_dis = min(len(rest), int(distract * n2)) if len(src) else 0
    dis = rng.choice(rest, size=n_dis, replace=False)
    for j, c in enumerate(dis):
        a = src[rng.integers(len(src))]
        descs[1][c] = descs[0][a] if j % 3 == 0 else _flip(rng, descs[0][a][None], 0.04)[0]
        nodes[1][c] = nodes[0][a]
        octs[1][c] = octs[0][a]
    node_ids = np.sort(rng.choice(np.arange(0, 10 * n_nodes), size=n_nodes, replace=False)).astype(np.uint32)
    sides = []
    for k in range(2):
        n = ns[k]
        used = np.unique(nodes[k])
        start = np.zeros(len(used) + 1, np.int32)
        feats = []
        for q, nd in enumerate(used):
            f = np.nonzero(nodes[k] == nd)[0]
            feats.append(f)
            start[q + 1] = start[q] + len(f)
        x = np.clip(xs[k], 0, EUROC_W - 1e-3).astype(np.float32)
        ur = None
        if stereo and not two_cam:
            ur = np.where(rng.random(n) < 0.5, x - EUROC_BF / depth[k], -1.0).astype(np.float32)
        sides.append(KFSide(desc=descs[k], kp_x=x, kp_y=np.clip(ys[k], 0, EUROC_H - 1e-3), kp_angle=angs[k],
                            kp_octave=octs[k], u_right=ur, has_mp=rng.random(n) < mp_frac,
                            node_id=node_ids[used], node_start=start, feat=np.concatenate(feats),
                            nleft=nleft[k], two_cam=int(two_cam), scale=scale_factors(n_levels)))
    F, R12s, t12s = [], [], []
    for c1 in (0, 1) if two_cam else (0,):
        for c2 in (0, 1) if two_cam else (0,):
            R1, t1 = Tcw[(1, c1)]
            R2_, t2 = Tcw[(2, c2)]
            R12 = R1 @ R2_.T                 # T12 = T1w * T2w^-1
            t12 = t1 - R12 @ t2
            F.append(fundamental(K, K, R12, t12))
            R12s.append(R12.astype(np.float32))
            t12s.append(t12.astype(np.float32))
    Rl2, tl2 = Tcw[(2, 0)]
    e = Rl2 @ np.zeros(3) + tl2             # T2w * Cw (KF1 centre = world origin)
    if kb8:
        epk = kb8_project(KB8_TRIANG, e)
        ep = (np.float32(epk[0]), np.float32(epk[1]))
    else:
        ep = (np.float32(EUROC_FX * e[0] / e[2] + EUROC_CX), np.float32(EUROC_FY * e[1] / e[2] + EUROC_CY))
    if forward and n_dis:                   # a third of the distractors within ~20 px of the epipole
        near = dis[: n_dis // 3]
        sides[1].kp_x[near] = np.float32(ep[0]) + rng.uniform(-20, 20, len(near)).astype(np.float32)
        sides[1].kp_y[near] = np.float32(ep[1]) + rng.uniform(-20, 20, len(near)).astype(np.float32)
    if kb8:
        return sides[0], sides[1], TriangGeom(ep=ep, F12=np.stack(F), pinhole=False, R12=np.stack(R12s),
                                              t12=np.stack(t12s), kb=np.tile(KB8_TRIANG, (4, 1)))
    return sides[0], sides[1], TriangGeom(ep=ep, F12=np.stack(F))


# ------------------------------------------------------------- b6 SearchForInitialization

def synth_init_pair(rng, n1=2000, n2=2000, match=0.7, level0=0.5, shift=(12.0, -4.0), noise=1.5, steal=0.15,
                    n_levels=8):
    """Monocular initialisation (Tracking::MonocularInitialization, 2x features): F2 sees F1's scene
    moved by ``shift`` px (+ noise); ``match`` of F1's keypoints have a noisy descriptor copy in F2 (same
    octave; ``level0`` of all keypoints at octave 0, the only level the matcher reads).  ``steal`` of
    the matched F2 keypoints get a second, LATER F1 keypoint nearby with a closer descriptor copy, so
    vnMatches21 steals and vMatchedDistance skips happen.  Returns (F1, F2, vbPrevMatched = F1's
    keypoint positions)."""
    def frame(n):
        x = rng.uniform(0, EUROC_W, n).astype(np.float32)
        y = rng.uniform(0, EUROC_H, n).astype(np.float32)
        oct_ = np.where(rng.random(n) < level0, 0, rng.integers(1, n_levels, n)).astype(np.int32)
        return x, y, oct_, rng.uniform(0, 360, n).astype(np.float32), rng.integers(0, 256, (n, 32), dtype=np.uint8)
    x1, y1, o1, a1, d1 = frame(n1)
    x2, y2, o2, a2, d2 = frame(n2)
    m = int(match * min(n1, n2))
    i1 = rng.choice(n1 // 2, size=min(m, n1 // 2), replace=False)   # steal partners come from the upper half
    i2 = rng.choice(n2, size=len(i1), replace=False)
    x2[i2] = np.clip(x1[i1] + shift[0] + rng.normal(0, noise, len(i1)), 0, EUROC_W - 1e-3)
    y2[i2] = np.clip(y1[i1] + shift[1] + rng.normal(0, noise, len(i1)), 0, EUROC_H - 1e-3)
    o2[i2] = o1[i1]
    a2[i2] = np.mod(a1[i1] - 7 - rng.normal(0, 3, len(i1)), 360)
    d2[i2] = _flip(rng, d1[i1], 0.08)
    ns = int(steal * len(i1))
    later = rng.choice(np.arange(n1 // 2, n1), size=ns, replace=False)
    src = rng.choice(len(i1), size=ns, replace=False)
    x1[later] = x1[i1[src]] + rng.normal(0, 2.0, ns)
    y1[later] = y1[i1[src]] + rng.normal(0, 2.0, ns)
    o1[later] = o1[i1[src]]
    a1[later] = a1[i1[src]]
    d1[later] = _flip(rng, d2[i2[src]], 0.03)
    F1 = FrameSoA(desc=d1, kp_x=np.clip(x1, 0, EUROC_W - 1e-3), kp_y=np.clip(y1, 0, EUROC_H - 1e-3), kp_angle=a1,
                  kp_octave=o1, scale=scale_factors(n_levels))
    F2 = FrameSoA(desc=d2, kp_x=x2, kp_y=y2, kp_angle=a2, kp_octave=o2, scale=scale_factors(n_levels))
    prev = np.stack([F1.kp_x, F1.kp_y], axis=1).astype(np.float32)
    return F1, F2, prev
