"""Host mirror of ``ORB_SLAM3::Optimizer::PoseOptimization`` / ``LocalBundleAdjustment``
(ref:include/Optimizer.h:55,77) on the C ABI in include/osg_ba.h, plus the seeded synthetic
problems of SURVEY.md §8d (C3 PoseOptimization, C4 LocalBA 50 KF x 10k points).

The graph gathering that the reference does from Frame / KeyFrame / MapPoint (window selection,
vertex ids, edge insertion order, float->double casts) is the adapter's job; here a problem is
given directly as those arrays.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field, replace

import numpy as np

from . import Context, _abi
from .synth import EUROC_BF, EUROC_CX, EUROC_CY, EUROC_FX, EUROC_FY, EUROC_H, EUROC_W


def _p(a):
    return None if a is None else int(a.ctypes.data)


def pinhole_camera(fx=EUROC_FX, fy=EUROC_FY, cx=EUROC_CX, cy=EUROC_CY, bf=EUROC_BF, trl=None):
    c = _abi.OsgCamera()
    c.type = _abi.CAM_PINHOLE
    for i, v in enumerate([fx, fy, cx, cy, 0, 0, 0, 0]):
        c.p[i] = v
    c.fx, c.fy, c.cx, c.cy, c.bf = fx, fy, cx, cy, bf
    t = trl if trl is not None else [0, 0, 0, 1, 0, 0, 0]
    for i in range(7):
        c.trl[i] = t[i]
    return c


def kb8_camera(fx=190.98, fy=190.97, cx=254.93, cy=256.90, k=(3.48e-3, 7.15e-4, -2.05e-3, 2.03e-4), trl=None):
    c = _abi.OsgCamera()
    c.type = _abi.CAM_KB8
    for i, v in enumerate([fx, fy, cx, cy, *k]):
        c.p[i] = v
    c.fx, c.fy, c.cx, c.cy, c.bf = fx, fy, cx, cy, 0.0
    t = trl if trl is not None else [0, 0, 0, 1, 0, 0, 0]
    for i in range(7):
        c.trl[i] = t[i]
    return c


# ----------------------------------------------------------------------------- geometry helpers
def rot_to_quat(m):
    """Eigen Quaternion(Matrix3) (trace method), coeffs (x, y, z, w)."""
    q = np.zeros(4)
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0:
        s = np.sqrt(t + 1.0)
        q[3] = 0.5 * s
        s = 0.5 / s
        q[0] = (m[2, 1] - m[1, 2]) * s
        q[1] = (m[0, 2] - m[2, 0]) * s
        q[2] = (m[1, 0] - m[0, 1]) * s
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        s = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q[i] = 0.5 * s
        s = 0.5 / s
        q[3] = (m[k, j] - m[j, k]) * s
        q[j] = (m[j, i] + m[i, j]) * s
        q[k] = (m[k, i] + m[i, k]) * s
    if q[3] < 0:
        q = -q
    return q / np.linalg.norm(q)


def quat_to_rot(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def look_at(center, target, up=(0, -1, 0)):
    """Tcw (world->camera) for a camera at `center` looking at `target` (z forward, y down)."""
    z = np.asarray(target, float) - np.asarray(center, float)
    z /= np.linalg.norm(z)
    x = np.cross(np.asarray(up, float), z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    Rcw = np.stack([x, y, z])
    tcw = -Rcw @ np.asarray(center, float)
    return Rcw, tcw


def small_rotation(rng, deg):
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    a = np.deg2rad(deg) * rng.normal()
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(a) * K + (1 - np.cos(a)) * K @ K


def pose7(R, t):
    """Sophus SE3f -> g2o SE3Quat as the reference does: float quaternion / translation cast to
    double (ref:src/Optimizer.cc:97)."""
    q = rot_to_quat(R).astype(np.float32).astype(np.float64)
    return np.concatenate([q, np.asarray(t, np.float32).astype(np.float64)])


def inv_level_sigma2(n_levels=8, factor=1.2):
    s = np.ones(n_levels, np.float32)
    for i in range(1, n_levels):
        s[i] = np.float32(s[i - 1] * np.float32(factor))
    return (np.float32(1.0) / (s * s)).astype(np.float32)


# ----------------------------------------------------------------------------- problem containers
@dataclass
class PoseProblem:
    pose: np.ndarray          # 7 doubles (q xyzw, t)
    kind: np.ndarray          # int8 per edge
    xw: np.ndarray            # n x 3 double
    obs: np.ndarray           # n x 3 double
    inv_sigma2: np.ndarray    # float32 per edge
    cam: object = field(default_factory=pinhole_camera)
    cam2: object = field(default_factory=pinhole_camera)

    def __post_init__(self):
        self.pose = np.ascontiguousarray(self.pose, np.float64)
        self.kind = np.ascontiguousarray(self.kind, np.int8)
        self.xw = np.ascontiguousarray(self.xw, np.float64).reshape(-1, 3)
        self.obs = np.ascontiguousarray(self.obs, np.float64).reshape(-1, 3)
        self.inv_sigma2 = np.ascontiguousarray(self.inv_sigma2, np.float32)

    @property
    def n(self):
        return len(self.kind)

    def struct(self):
        s = _abi.OsgPoseProblem()
        for i in range(7):
            s.pose[i] = float(self.pose[i])
        s.n_edges = self.n
        s.kind, s.xw, s.obs, s.inv_sigma2 = _p(self.kind), _p(self.xw), _p(self.obs), _p(self.inv_sigma2)
        s.cam = self.cam
        s.cam2 = self.cam2
        return s


@dataclass
class PoseResult:
    pose: np.ndarray
    outlier: np.ndarray
    n_inliers: int
    lm_iterations: int
    lm_trials: int


@dataclass
class BAGraph:
    pose: np.ndarray          # np x 7
    pose_fixed: np.ndarray    # np uint8
    point: np.ndarray         # npt x 3
    e_point: np.ndarray
    e_pose: np.ndarray
    e_kind: np.ndarray
    e_cam: np.ndarray
    e_obs: np.ndarray         # ne x 3
    e_inv_sigma2: np.ndarray
    cams: list
    iterations: int = 10
    user_lambda_init: float = 0.0
    e_robust: np.ndarray | None = None   # BundleAdjustment: per-edge Huber flag (None: every edge)
    huber_mono: float = 0.0              # deltas as the reference's floats (0: LocalBundleAdjustment's)
    huber_stereo: float = 0.0

    def __post_init__(self):
        self.pose = np.ascontiguousarray(self.pose, np.float64).reshape(-1, 7)
        self.pose_fixed = np.ascontiguousarray(self.pose_fixed, np.uint8)
        self.point = np.ascontiguousarray(self.point, np.float64).reshape(-1, 3)
        self.e_point = np.ascontiguousarray(self.e_point, np.int32)
        self.e_pose = np.ascontiguousarray(self.e_pose, np.int32)
        self.e_kind = np.ascontiguousarray(self.e_kind, np.int8)
        self.e_cam = np.ascontiguousarray(self.e_cam, np.int32)
        self.e_obs = np.ascontiguousarray(self.e_obs, np.float64).reshape(-1, 3)
        self.e_inv_sigma2 = np.ascontiguousarray(self.e_inv_sigma2, np.float32)
        if self.e_robust is not None:
            self.e_robust = np.ascontiguousarray(self.e_robust, np.uint8)
        self._cams = (_abi.OsgCamera * max(1, len(self.cams)))(*self.cams)

    def struct(self):
        s = _abi.OsgBaGraph()
        s.n_poses = len(self.pose)
        s.pose, s.pose_fixed = _p(self.pose), _p(self.pose_fixed)
        s.n_points = len(self.point)
        s.point = _p(self.point)
        s.n_edges = len(self.e_point)
        s.e_point, s.e_pose, s.e_kind = _p(self.e_point), _p(self.e_pose), _p(self.e_kind)
        s.e_cam, s.e_obs, s.e_inv_sigma2 = _p(self.e_cam), _p(self.e_obs), _p(self.e_inv_sigma2)
        s.n_cams = len(self.cams)
        s.cams = C.addressof(self._cams)
        s.iterations = self.iterations
        s.user_lambda_init = self.user_lambda_init
        s.e_robust = _p(self.e_robust)
        s.huber_mono, s.huber_stereo = self.huber_mono, self.huber_stereo
        return s


@dataclass
class BAResult:
    pose: np.ndarray
    point: np.ndarray
    edge_bad: np.ndarray
    iterations: int
    trials: int
    chi2_initial: float
    chi2_final: float
    aborted: int
    edge_chi2: np.ndarray | None = None   # e->chi2() of each edge's last computed error


def run_pose(fn, problems, handle=None):
    """Call a PoseOptimization entry point on problems: the batch API (handle given) or a
    per-problem function fn(problem_structs, result_structs)."""
    res_structs = (_abi.OsgPoseResult * len(problems))()
    outl = [np.zeros(p.n, np.uint8) for p in problems]
    for r, o in zip(res_structs, outl):
        r.outlier = _p(o)
    probs = (_abi.OsgPoseProblem * len(problems))(*[p.struct() for p in problems])
    rc = fn(probs, res_structs) if handle is None else fn(handle, probs, len(problems), res_structs)
    out = [PoseResult(np.array(list(r.pose)), o, r.n_inliers, r.lm_iterations, r.lm_trials)
           for r, o in zip(res_structs, outl)]
    return rc, out


def make_ba_result(G: BAGraph, chi2: bool = True):
    """(osg_ba_result, its output arrays): pose, point, edge_bad, edge_chi2 (None unless `chi2`: the
    per-edge chi2 is read only by the map-merge BA's level-1 marking; LocalMapping's LBA needs the
    classification alone, and each requested array is another device-to-host copy)."""
    R = _abi.OsgBaResult()
    out = (np.zeros_like(G.pose), np.zeros_like(G.point), np.zeros(len(G.e_point), np.uint8),
           np.zeros(len(G.e_point), np.float64) if chi2 else None)
    R.pose, R.point, R.edge_bad, R.edge_chi2 = (_p(a) for a in out)
    return R, out


def finish_ba_result(R, out) -> "BAResult":
    pose, point, bad, chi2 = out
    return BAResult(pose, point, bad, R.iterations, R.trials, R.chi2_initial, R.chi2_final, R.aborted, chi2)


class Optimizer:
    """``Optimizer::PoseOptimization`` / ``LocalBundleAdjustment`` on the GPU."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def PoseOptimization(self, problems):
        """Batch form: one launch for all frames.  Returns the per-frame results (the reference's
        return value is ``n_inliers``)."""
        single = isinstance(problems, PoseProblem)
        probs = [problems] if single else list(problems)
        lib, h = self.ctx.lib, self.ctx.handle
        rc, out = run_pose(lib.osg_pose_optimization_batch, probs, handle=h)
        self.ctx.check(rc, "PoseOptimization")
        return out[0] if single else out

    def LocalBundleAdjustment(self, G: BAGraph, stop_flag: np.ndarray | None = None) -> BAResult:
        lib, h = self.ctx.lib, self.ctx.handle
        R, out = make_ba_result(G, chi2=False)
        gs = G.struct()
        if stop_flag is not None:
            assert stop_flag.dtype == np.uint8, "stop flag is one byte (bool *pbStopFlag)"
        sf = None if stop_flag is None else _p(stop_flag)
        rc = lib.osg_local_bundle_adjustment(h, C.byref(gs), C.byref(R), sf)
        self.ctx.check(rc, "LocalBundleAdjustment")
        return finish_ba_result(R, out)

    def BundleAdjustment(self, G: BAGraph, stop_flag: np.ndarray | None = None) -> BAResult:
        """The g2o part of ``Optimizer::BundleAdjustment`` (global BA, ref:src/Optimizer.cc:2850-3237):
        ``G`` built as the reference builds it (``synth_gba_graph`` / the adapter), optimize(G.iterations).
        The reference reads no outlier flags after a global BA; ``edge_bad`` is informational."""
        lib, h = self.ctx.lib, self.ctx.handle
        R, out = make_ba_result(G)
        gs = G.struct()
        if stop_flag is not None:
            assert stop_flag.dtype == np.uint8, "stop flag is one byte (bool *pbStopFlag)"
        sf = None if stop_flag is None else _p(stop_flag)
        self.ctx.check(lib.osg_bundle_adjustment(h, C.byref(gs), C.byref(R), sf), "BundleAdjustment")
        return finish_ba_result(R, out)

    GlobalBundleAdjustemnt = BundleAdjustment  # the reference's spelling (ref:include/Optimizer.h)

    def LocalBundleAdjustmentMerge(self, G: BAGraph, stop_flag: np.ndarray | None = None, mp_bad=None):
        """``LocalBundleAdjustment(pMainKF, vpAdjustKF, vpFixedKF, pbStopFlag)`` — the map-merge window BA
        (ref:src/Optimizer.cc:5211-5672): two g2o passes on the GPU, see merge_local_bundle_adjustment."""
        return merge_local_bundle_adjustment(G, lambda g, s: self.BundleAdjustment(g, stop_flag=s), stop_flag, mp_bad)

    def LocalBundleAdjustmentBatch(self, graphs, stop_flag: np.ndarray | None = None) -> list:
        """B independent windows in lockstep, one launch per kernel per LM trial for all of them
        (no reference counterpart; each graph follows the single-graph LM exactly)."""
        lib, h = self.ctx.lib, self.ctx.handle
        B = len(graphs)
        made = [make_ba_result(G, chi2=False) for G in graphs]
        gs = (_abi.OsgBaGraph * B)(*[G.struct() for G in graphs])
        rs = (_abi.OsgBaResult * B)(*[m[0] for m in made])
        if stop_flag is not None:
            assert stop_flag.dtype == np.uint8, "stop flag is one byte (bool *pbStopFlag)"
        sf = None if stop_flag is None else _p(stop_flag)
        rc = lib.osg_local_bundle_adjustment_batch(h, C.addressof(gs), B, C.addressof(rs), sf)
        self.ctx.check(rc, "LocalBundleAdjustment batch")
        return [finish_ba_result(R, m[1]) for m, R in zip(made, rs)]


LBA_KERNELS = ["errors", "linearize", "pose_red", "lambda_init", "schur_point", "schur_rows", "schur_pairs",
               "chol", "chol_back", "update", "step_reduce", "classify"]


def lba_kernel_times(ctx, enable: bool) -> dict:
    """osg_lba_kernel_times: per-kernel device time (HIP events) of the LBA engine since the last
    enable, as {kernel: (ms, launch groups)}; enable=True (re)starts the timing, False stops it."""
    ms = np.zeros(len(LBA_KERNELS), np.float64)
    n = np.zeros(len(LBA_KERNELS), np.int64)
    ctx.check(ctx.lib.osg_lba_kernel_times(ctx.handle, int(enable), _p(ms), _p(n)), "lba_kernel_times")
    return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(LBA_KERNELS)}


def lba_structure_counts(G: "BAGraph") -> dict:
    """Sizes of the BlockSolver structure of a graph (ba.hip build_structure): free poses with an
    edge, landmarks, (landmark, free pose) blocks, and Schur contributions sum_l k_l (k_l + 1) / 2
    (k_l = free poses observing landmark l)."""
    fixed = np.asarray(G.pose_fixed).astype(bool)
    ep, et = np.asarray(G.e_pose), np.asarray(G.e_point)
    free = ~fixed[ep]
    blocks = np.unique(et[free].astype(np.int64) * (len(G.pose) + 1) + ep[free])
    k = np.bincount((blocks // (len(G.pose) + 1)).astype(np.int64), minlength=len(G.point))
    return {"free_poses": int(len(np.unique(ep[free]))), "landmarks": int(len(np.unique(et))),
            "blocks": int(len(blocks)), "contributions": int((k * (k + 1) // 2).sum())}


# ----------------------------------------------------------------------------- generators
def kb8_project(cam, Xc):
    """KannalaBrandt8::project (ref:src/CameraModels/KannalaBrandt8.cpp:76-99) in float64."""
    k = [float(cam.p[i]) for i in range(8)]
    th = np.arctan2(np.hypot(Xc[:, 0], Xc[:, 1]), Xc[:, 2])
    ps = np.arctan2(Xc[:, 1], Xc[:, 0])
    r = th + k[4] * th ** 3 + k[5] * th ** 5 + k[6] * th ** 7 + k[7] * th ** 9
    return k[0] * r * np.cos(ps) + k[2], k[1] * r * np.sin(ps) + k[3]


# TUM-VI-like right-from-left extrinsic of the fisheye pair: 10.1 cm baseline, ~0.5 deg rotation
TUMVI_TRL = [0.0021, -0.0023, 0.0011, 0.99999, -0.101, 0.0005, -0.0004]


def synth_pose_problem(rng, n_edges=400, stereo_frac=0.6, outlier_frac=0.1, n_levels=8, cam=None, body_frac=0.0):
    """C3 PoseOptimization: Xw depth U[1,10] m in front of the camera, pose perturbed by
    1 cm / 0.5 deg, pixel noise 1 px * 1.2^octave, 10 % outliers (+20..50 px), stereo u_R for
    60 % of the edges (bf = 47.9).  With a KB8 camera and ``body_frac`` > 0 (C5, two-camera rig),
    that fraction of the edges are right-camera observations (EdgeSE3ProjectXYZOnlyPoseToBody, the
    second camera ``kb8_camera(trl=TUMVI_TRL)``)."""
    cam = cam or pinhole_camera()
    Rcw = small_rotation(rng, 20.0)
    tcw = rng.normal(0, 1.0, 3)
    if cam.type == _abi.CAM_KB8:
        # fisheye (TUM-VI-like 512 x 512): directions up to 70 deg off-axis, projected by KB8
        th = rng.uniform(0.05, 1.2, n_edges)
        ps = rng.uniform(-np.pi, np.pi, n_edges)
        d = rng.uniform(1.0, 10.0, n_edges)
        Xc = np.stack([d * np.sin(th) * np.cos(ps), d * np.sin(th) * np.sin(ps), d * np.cos(th)], 1)
        k = [float(cam.p[i]) for i in range(8)]
        r = th + k[4] * th ** 3 + k[5] * th ** 5 + k[6] * th ** 7 + k[7] * th ** 9
        u = k[0] * r * np.cos(ps) + k[2]
        v = k[1] * r * np.sin(ps) + k[3]
        z = Xc[:, 2]
        stereo_frac = 0.0  # no rectified stereo on a fisheye rig
    else:
        u = rng.uniform(20, EUROC_W - 20, n_edges)
        v = rng.uniform(20, EUROC_H - 20, n_edges)
        z = rng.uniform(1.0, 10.0, n_edges)
        Xc = np.stack([(u - EUROC_CX) / EUROC_FX * z, (v - EUROC_CY) / EUROC_FY * z, z], 1)
    Xw = (Xc - tcw) @ Rcw  # Rcw^T (Xc - t)
    Xw = Xw.astype(np.float32).astype(np.float64)
    octv = rng.choice(n_levels, n_edges, p=np.array([1.2 ** -i for i in range(n_levels)]) / sum(1.2 ** -i for i in range(n_levels)))
    sig = 1.2 ** octv
    obs = np.zeros((n_edges, 3))
    obs[:, 0] = u + rng.normal(0, 1, n_edges) * sig
    obs[:, 1] = v + rng.normal(0, 1, n_edges) * sig
    out = rng.random(n_edges) < outlier_frac
    obs[out, 0] += rng.uniform(20, 50, out.sum()) * rng.choice([-1, 1], out.sum())
    obs[out, 1] += rng.uniform(20, 50, out.sum()) * rng.choice([-1, 1], out.sum())
    stereo = rng.random(n_edges) < stereo_frac
    obs[:, 2] = np.where(stereo, obs[:, 0] - EUROC_BF / z + rng.normal(0, 0.5, n_edges), 0.0)
    obs = obs.astype(np.float32).astype(np.float64)  # keypoints are float
    kind = np.where(stereo, _abi.EDGE_STEREO, _abi.EDGE_MONO).astype(np.int8)
    # perturbed initial pose
    R0 = small_rotation(rng, 0.5) @ Rcw
    t0 = tcw + rng.normal(0, 0.01, 3)
    isig = inv_level_sigma2(n_levels)[octv]
    cam2 = cam
    if cam.type == _abi.CAM_KB8 and body_frac > 0:
        cam2 = kb8_camera(trl=TUMVI_TRL)
        q = np.array(TUMVI_TRL[:4]) / np.linalg.norm(TUMVI_TRL[:4])
        from scipy.spatial.transform import Rotation
        Rrl = Rotation.from_quat(q).as_matrix()
        Xr = Xc @ Rrl.T + np.array(TUMVI_TRL[4:])
        body = (rng.random(n_edges) < body_frac) & (Xr[:, 2] > 0.1)
        ur, vr = kb8_project(cam2, Xr[body])
        sb = sig[body]
        obs[body, 0] = ur + rng.normal(0, 1, body.sum()) * sb
        obs[body, 1] = vr + rng.normal(0, 1, body.sum()) * sb
        obs[body, 2] = 0.0
        ob = body & out
        obs[ob, 0] += rng.uniform(20, 50, ob.sum()) * rng.choice([-1, 1], ob.sum())
        obs = obs.astype(np.float32).astype(np.float64)
        kind = np.where(body, _abi.EDGE_BODY, kind).astype(np.int8)
    return PoseProblem(pose7(R0, t0), kind, Xw, obs, isig, cam=cam, cam2=cam2)


def synth_lba_graph(rng, n_kf=50, n_points=10000, k_range=(2, 8), n_fixed=2, stereo_frac=0.0,
                    outlier_frac=0.01, n_levels=8, radius=6.0, arc_deg=50.0):
    """C4 LocalBundleAdjustment: n_kf keyframes on an arc (radius 6 m, ~5 m long) looking at a
    4 x 4 x 2 m box of points; each point observed by k ~ U{2..8} keyframes that see it; pixel
    noise 1 px * 1.2^octave; pose noise 1 cm / 0.3 deg; point noise 2 cm; 1 % gross outliers.
    KeyFrames 0..n_fixed-1 are fixed (init KF + fixed observers)."""
    cam = pinhole_camera()
    ang = np.deg2rad(np.linspace(-arc_deg / 2, arc_deg / 2, n_kf))
    centers = np.stack([radius * np.sin(ang), 0.3 * np.sin(3 * ang), -radius * np.cos(ang)], 1)
    Rs, ts = [], []
    for c in centers:
        R, t = look_at(c, [0, 0, 0])
        Rs.append(R)
        ts.append(t)
    P = np.stack([rng.uniform(-2, 2, n_points), rng.uniform(-2, 2, n_points), rng.uniform(-1, 1, n_points)], 1)
    isig_tab = inv_level_sigma2(n_levels)
    e_point, e_pose, e_obs, e_isig, e_kind = [], [], [], [], []
    for p in range(n_points):
        # keyframes that see the point inside the image
        Xc = np.einsum("kij,j->ki", np.array(Rs), P[p]) + np.array(ts)
        u = EUROC_FX * Xc[:, 0] / Xc[:, 2] + EUROC_CX
        v = EUROC_FY * Xc[:, 1] / Xc[:, 2] + EUROC_CY
        vis = np.nonzero((Xc[:, 2] > 0.5) & (u > 0) & (u < EUROC_W) & (v > 0) & (v < EUROC_H))[0]
        if len(vis) < 2:
            continue
        k = min(len(vis), int(rng.integers(k_range[0], k_range[1] + 1)))
        obs_kf = np.sort(rng.choice(vis, k, replace=False))
        for kf in obs_kf:
            octv = int(rng.choice(n_levels, p=np.array([1.2 ** -i for i in range(n_levels)]) / sum(1.2 ** -i for i in range(n_levels))))
            s = 1.2 ** octv
            uu = u[kf] + rng.normal() * s
            vv = v[kf] + rng.normal() * s
            if rng.random() < outlier_frac:
                uu += rng.uniform(20, 50) * rng.choice([-1, 1])
                vv += rng.uniform(20, 50) * rng.choice([-1, 1])
            st = rng.random() < stereo_frac
            ur = uu - EUROC_BF / Xc[kf, 2] + rng.normal() * 0.5 if st else 0.0
            e_point.append(p)
            e_pose.append(kf)
            e_obs.append([uu, vv, ur])
            e_isig.append(isig_tab[octv])
            e_kind.append(_abi.EDGE_STEREO if st else _abi.EDGE_MONO)
    e_point = np.array(e_point)
    used = np.unique(e_point)
    remap = -np.ones(n_points, int)
    remap[used] = np.arange(len(used))
    e_point = remap[e_point]
    P = P[used]
    poses = []
    for i, (R, t) in enumerate(zip(Rs, ts)):
        if i >= n_fixed:
            R = small_rotation(rng, 0.3) @ R
            t = t + rng.normal(0, 0.01, 3)
        poses.append(pose7(R, t))
    Pn = (P + rng.normal(0, 0.02, P.shape)).astype(np.float32).astype(np.float64)
    fixed = np.zeros(n_kf, np.uint8)
    fixed[:n_fixed] = 1
    obs = np.array(e_obs, np.float32).astype(np.float64)
    return BAGraph(np.array(poses), fixed, Pn, e_point, np.array(e_pose), np.array(e_kind, np.int8),
                   np.zeros(len(e_point), np.int32), obs, np.array(e_isig, np.float32), [cam])


def gba_robust_settings(G: BAGraph, bRobust: bool = True) -> BAGraph:
    """Give an LBA-shaped graph BundleAdjustment's kernels (ref:src/Optimizer.cc:2933-2934,
    3000-3007, 3041-3047, 3083-3085): deltas float(sqrt(5.99)) / float(sqrt(7.815)); mono and stereo
    edges carry them only when bRobust, body edges always."""
    G.huber_mono = float(np.float32(np.sqrt(5.99)))
    G.huber_stereo = float(np.float32(np.sqrt(7.815)))
    G.e_robust = np.where(G.e_kind == _abi.EDGE_BODY, 1, int(bool(bRobust))).astype(np.uint8)
    return G


def synth_gba_graph(rng, n_kf=120, n_points=20000, bRobust=False, iterations=10, stereo_frac=0.0, **kw):
    """A whole-map BA: keyframes on a longer arc, only the map's init KeyFrame fixed, every point with
    its observations.  Defaults: LoopClosing's GlobalBundleAdjustemnt(map, 10, &mbStopGBA, nLoopKF,
    false) (ref:src/LoopClosing.cc:3084); the monocular initialisation runs (map, 20) with bRobust
    true (ref:src/Tracking.cc:3076)."""
    G = synth_lba_graph(rng, n_kf=n_kf, n_points=n_points, n_fixed=1, stereo_frac=stereo_frac,
                        arc_deg=kw.pop("arc_deg", 120.0), **kw)
    G.iterations = iterations
    return gba_robust_settings(G, bRobust)


def synth_map_graph(rng, n_kf=1500, n_points=150000, spacing=0.3, k_range=(2, 6), bRobust=False, iterations=10,
                    stereo_frac=0.0, n_levels=8, loop=False, vectorized=False):
    """A map-scale whole-map BA (GlobalBundleAdjustemnt on a long sequence): n_kf keyframes 'spacing'
    m apart along a 0.45 km path, looking sideways at points 4 .. 6 m away spread along it, so a
    keyframe shares points only with its neighbours (~27 on each side) and the reduced camera
    system is a band, as in an open trajectory without loop closures.  Each point is observed by
    k ~ U{k_range} of the keyframes that see it; pixel noise 1 px * 1.2^octave, pose noise 1 cm /
    0.3 deg, point noise 2 cm; the first keyframe is fixed (the map's init KeyFrame).

    loop=True: the same path closed into a circle (radius n_kf spacing / 2 pi, cameras looking
    outwards at a ring of points), so the last keyframes share points with the first ones — the map
    LoopClosing hands to GlobalBundleAdjustemnt after closing a loop (ref:src/LoopClosing.cc:2436):
    the reduced camera system is the band plus the two corner blocks that join its ends.

    vectorized=True draws each point's observing keyframes and levels array-wise (another random stream
    than the per-point loop, the same distribution): the maps of many thousand keyframes build in
    seconds."""
    cam = pinhole_camera()
    L = spacing * (n_kf - 1)
    cx = np.arange(n_kf) * spacing
    cy = 0.1 * np.sin(np.arange(n_kf) * 0.05)
    yaw = np.deg2rad(rng.normal(0, 2.0, n_kf))
    Rs = np.stack([np.array([[np.cos(a), 0, -np.sin(a)], [0, 1, 0], [np.sin(a), 0, np.cos(a)]]) for a in yaw])
    if loop:
        Rc = spacing * n_kf / (2 * np.pi)
        th = 2 * np.pi * np.arange(n_kf) / n_kf
        # camera axes in world coordinates: x along the tangent, y down (world y), z outwards
        R0 = np.stack([np.array([[np.sin(a), 0, -np.cos(a)], [0, 1, 0], [np.cos(a), 0, np.sin(a)]]) for a in th])
        Rs = np.einsum("kij,kjl->kil", Rs, R0)
        C = np.stack([Rc * np.cos(th), cy, Rc * np.sin(th)], 1)
    else:
        C = np.stack([cx, cy, np.zeros(n_kf)], 1)
    ts = -np.einsum("kij,kj->ki", Rs, C)
    P = np.stack([rng.uniform(-1.0, L + 1.0, n_points), rng.uniform(-1.5, 1.5, n_points),
                  rng.uniform(4.0, 6.0, n_points)], 1)
    if loop:  # the same draws as angle (path position) and distance off the path, on the ring
        phi = 2 * np.pi * P[:, 0] / (spacing * n_kf)
        rho = Rc + P[:, 2]
        P = np.stack([rho * np.cos(phi), P[:, 1], rho * np.sin(phi)], 1)
        pos = phi / (2 * np.pi) * n_kf   # path position in keyframes
    else:
        pos = P[:, 0] / spacing
    isig_tab = inv_level_sigma2(n_levels)
    lev_p = np.array([1.2 ** -i for i in range(n_levels)])
    lev_p /= lev_p.sum()
    W = int(np.ceil(6.0 * 0.85 / spacing)) + 2  # keyframes within reach of a point
    e_point, e_pose, e_obs, e_kind, e_lev = [], [], [], [], []
    for p0 in range(0, n_points, 20000):
        Pc = P[p0:p0 + 20000]
        if loop:
            base = np.round(pos[p0:p0 + 20000]).astype(int) - W
            cand = (base[:, None] + np.arange(2 * W + 1)[None, :]) % n_kf  # (m, 2W+1)
        else:
            base = np.clip(np.round(pos[p0:p0 + 20000]).astype(int) - W, 0, None)
            cand = np.clip(base[:, None] + np.arange(2 * W + 1)[None, :], 0, n_kf - 1)  # (m, 2W+1)
        Xc = np.einsum("mkij,mj->mki", Rs[cand], Pc) + ts[cand]
        u = EUROC_FX * Xc[..., 0] / Xc[..., 2] + EUROC_CX
        v = EUROC_FY * Xc[..., 1] / Xc[..., 2] + EUROC_CY
        vis = (Xc[..., 2] > 0.5) & (u > 0) & (u < EUROC_W) & (v > 0) & (v < EUROC_H)
        vis[:, 1:] &= cand[:, 1:] != cand[:, :-1]  # clipped duplicates
        if vectorized:
            nvis = vis.sum(1)
            kk = np.minimum(nvis, rng.integers(k_range[0], k_range[1] + 1, len(Pc)))
            kk[nvis < 2] = 0
            key = np.where(vis, rng.random(vis.shape), 2.0)   # k uniformly chosen visible candidates
            order = np.argsort(key, 1)
            take = np.arange(vis.shape[1])[None, :] < kk[:, None]
            mi, ji = np.nonzero(take)
            jsel = order[mi, ji]
            srt = np.lexsort((jsel, mi))                       # per point in candidate order, as np.sort
            mi, jsel = mi[srt], jsel[srt]
            e_point.extend((p0 + mi).tolist())
            e_pose.extend(cand[mi, jsel].tolist())
            e_obs.extend(np.stack([u[mi, jsel], v[mi, jsel], Xc[mi, jsel, 2]], 1).tolist())
            e_lev.extend(rng.choice(n_levels, len(mi), p=lev_p).tolist())
            continue
        for m in range(len(Pc)):
            idx = np.nonzero(vis[m])[0]
            if len(idx) < 2:
                continue
            k = min(len(idx), int(rng.integers(k_range[0], k_range[1] + 1)))
            sel = np.sort(rng.choice(idx, k, replace=False))
            for j in sel:
                e_point.append(p0 + m)
                e_pose.append(cand[m, j])
                e_obs.append((u[m, j], v[m, j], Xc[m, j, 2]))
                e_lev.append(int(rng.choice(n_levels, p=lev_p)))
    e_point = np.array(e_point)
    e_pose = np.array(e_pose)
    e_obs = np.array(e_obs)
    e_lev = np.array(e_lev)
    ne = len(e_point)
    s = 1.2 ** e_lev
    obs = np.zeros((ne, 3))
    obs[:, 0] = e_obs[:, 0] + rng.normal(0, 1, ne) * s
    obs[:, 1] = e_obs[:, 1] + rng.normal(0, 1, ne) * s
    st = rng.random(ne) < stereo_frac
    obs[:, 2] = np.where(st, obs[:, 0] - EUROC_BF / e_obs[:, 2] + rng.normal(0, 0.5, ne), 0.0)
    used = np.unique(e_point)
    remap = -np.ones(n_points, int)
    remap[used] = np.arange(len(used))
    e_point = remap[e_point]
    P = P[used]
    poses = []
    for i in range(n_kf):
        R, t = Rs[i], ts[i]
        if i >= 1:  # about the keyframe's own centre: 0.3 deg and 1 cm
            R = small_rotation(rng, 0.3) @ R
            t = -R @ (C[i] + rng.normal(0, 0.01, 3))
        poses.append(pose7(R, t))
    Pn = (P + rng.normal(0, 0.02, P.shape)).astype(np.float32).astype(np.float64)
    fixed = np.zeros(n_kf, np.uint8)
    fixed[0] = 1
    G = BAGraph(np.array(poses), fixed, Pn, e_point, e_pose, np.where(st, _abi.EDGE_STEREO, _abi.EDGE_MONO).astype(np.int8),
                np.zeros(ne, np.int32), obs.astype(np.float32).astype(np.float64),
                isig_tab[e_lev].astype(np.float32), [cam])
    G.iterations = iterations
    return gba_robust_settings(G, bRobust)


def depth_positive(G: BAGraph, pose, point, edges):
    """isDepthPositive of the given edges: z of SE3Quat::map(X) = q X q* + t (Eigen's quaternion-vector
    product), > 0."""
    q = np.asarray(pose, np.float64).reshape(-1, 7)[G.e_pose[edges]]
    X = np.asarray(point, np.float64).reshape(-1, 3)[G.e_point[edges]]
    u, w = q[:, :3], q[:, 3:4]
    uv = 2.0 * np.cross(u, X)
    return (X + w * uv + np.cross(u, uv) + q[:, 4:7])[:, 2] > 0


def merge_local_bundle_adjustment(G: BAGraph, run, stop_flag=None, mp_bad=None):
    """The g2o part of Optimizer::LocalBundleAdjustment(pMainKF, vpAdjustKF, vpFixedKF, pbStopFlag)
    (ref:src/Optimizer.cc:5211-5672) on a graph gathered as it builds it: mono / stereo edges (no
    right-camera edges), BundleAdjustment's Huber deltas, vpFixedKF fixed.  ``run(graph, stop_flag)`` is
    one g2o optimize through the C ABI (Optimizer.BundleAdjustment; the oracle in tests):
      1. optimize(5) with Huber on every edge (:5448-5449);
      2. unless stopped: edges with chi2 > 5.991 / 7.815 or behind the camera go to level 1, every kernel
         is dropped (edges of bad MapPoints are skipped by both steps), and a fresh LM optimize(10) runs on
         the level-0 edges (:5451-5498);
      3. the final classification (:5506-5546): level-0 edges by their second-pass errors, level-1 edges by
         their first-pass chi2 (never recomputed) and the final depth.
    Returns (pose, point, erase flag per edge, stopped before the first pass)."""
    ne = len(G.e_point)
    mp_bad = np.zeros(len(G.point), bool) if mp_bad is None else np.asarray(mp_bad, bool)
    if stop_flag is not None and stop_flag[0]:  # :5444-5446: return before optimising
        return G.pose.copy(), G.point.copy(), np.zeros(ne, np.uint8), True
    G1 = gba_robust_settings(replace(G, iterations=5), True)
    r1 = run(G1, stop_flag)
    skip = mp_bad[G.e_point]
    if stop_flag is not None and stop_flag[0]:  # bDoMore = false: the first pass's classification
        return r1.pose, r1.point, (r1.edge_bad.astype(bool) & ~skip).astype(np.uint8), False
    level1 = r1.edge_bad.astype(bool) & ~skip
    keep = np.nonzero(~level1)[0]
    G2 = BAGraph(r1.pose, G.pose_fixed, r1.point, G.e_point[keep], G.e_pose[keep], G.e_kind[keep], G.e_cam[keep],
                 G.e_obs[keep], G.e_inv_sigma2[keep], G.cams, iterations=10, e_robust=skip[keep].astype(np.uint8),
                 huber_mono=G1.huber_mono, huber_stereo=G1.huber_stereo)
    r2 = run(G2, stop_flag)
    bad = np.zeros(ne, bool)
    bad[keep] = r2.edge_bad.astype(bool)
    l1 = np.nonzero(level1)[0]
    th = np.where(G.e_kind[l1] == _abi.EDGE_STEREO, 7.815, 5.991)
    bad[l1] = (r1.edge_chi2[l1] > th) | ~depth_positive(G, r2.pose, r2.point, l1)
    return r2.pose, r2.point, (bad & ~skip).astype(np.uint8), False
