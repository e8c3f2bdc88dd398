"""Second, independent restatement of PoseOptimization / LocalBundleAdjustment in numpy (float64,
with the reference's float casts).  Test infrastructure only: pins the C oracle
(tests/test_oracle_ba.py); never used by the product.

Deliberately built differently from oracle/oracle_ba.c so a shared mistake is unlikely:
rotations as matrices (scipy Rotation for matrix <-> quaternion) instead of quaternion algebra,
vectorised edge errors / Jacobians, the normal equations assembled as one dense matrix and solved
whole (no Schur complement; g2o's Schur + LDL^T solves the same system).  The Jacobians are checked
against central differences in the tests.  LM control follows
ref:Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-194 and the ORB-SLAM3 call
sites ref:src/Optimizer.cc:71-420 (PoseOptimization) and :1877-2203 (LocalBundleAdjustment).
"""
import math

import numpy as np
from scipy.spatial.transform import Rotation

MONO, STEREO, BODY = 0, 1, 2
f32 = np.float32


def skew(w):
    return np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])


def quat_of(R):
    q = Rotation.from_matrix(R).as_quat()  # x y z w
    return -q if q[3] < 0 else q


def mat_of(q):
    return Rotation.from_quat(np.asarray(q, float)).as_matrix()


def se3_exp(xi):
    """g2o SE3Quat::exp (ref:Thirdparty/g2o/g2o/types/se3quat.h:223-257): xi = [omega, upsilon]."""
    w, u = xi[:3], xi[3:]
    th = math.sqrt(w @ w)
    W = skew(w)
    W2 = W @ W
    if th < 1e-5:
        R = np.eye(3) + W + W2
        V = R
    else:
        R = np.eye(3) + math.sin(th) / th * W + (1 - math.cos(th)) / th ** 2 * W2
        V = np.eye(3) + (1 - math.cos(th)) / th ** 2 * W + (th - math.sin(th)) / th ** 3 * W2
    return mat_of(quat_of(R)), V @ u


class Pose:
    """Tcw as (R, t); quaternion form normalised with w >= 0 like SE3Quat."""

    def __init__(self, p7):
        self.R = mat_of(p7[:4])
        self.t = np.array(p7[4:], float)

    def copy(self):
        c = Pose.__new__(Pose)
        c.R, c.t = self.R.copy(), self.t.copy()
        return c

    def oplus(self, xi):  # exp(xi) * T
        Re, te = se3_exp(xi)
        self.R = mat_of(quat_of(Re @ self.R))
        self.t = Re @ self.t + te

    def p7(self):
        return np.concatenate([quat_of(self.R), self.t])


def project(cam, X, exact=False):
    """ref:src/CameraModels/Pinhole.cpp:50-71 / KannalaBrandt8.cpp:62-104 (double overloads; KB8
    takes atan2f / sqrtf of float casts, dropped with exact=True)."""
    p = [float(cam.p[i]) for i in range(8)]
    x, y, z = X[:, 0], X[:, 1], X[:, 2]
    if cam.type == 1 and exact:
        theta = np.arctan2(np.sqrt(x * x + y * y), z)
        psi = np.arctan2(y, x)
        r = theta + p[4] * theta ** 3 + p[5] * theta ** 5 + p[6] * theta ** 7 + p[7] * theta ** 9
        return np.stack([p[0] * r * np.cos(psi) + p[2], p[1] * r * np.sin(psi) + p[3]], 1)
    if cam.type == 1:
        theta = np.arctan2(np.sqrt((x * x + y * y).astype(f32)), z.astype(f32)).astype(f32).astype(float)
        psi = np.arctan2(y.astype(f32), x.astype(f32)).astype(f32).astype(float)
        r = theta + p[4] * theta ** 3 + p[5] * theta ** 5 + p[6] * theta ** 7 + p[7] * theta ** 9
        return np.stack([p[0] * r * np.cos(psi) + p[2], p[1] * r * np.sin(psi) + p[3]], 1)
    return np.stack([p[0] * x / z + p[2], p[1] * y / z + p[3]], 1)


def project_jac(cam, X):
    """d(project)/dX, ref:src/CameraModels/Pinhole.cpp:122-133 / KannalaBrandt8.cpp:229-260."""
    p = [float(cam.p[i]) for i in range(8)]
    x, y, z = X[:, 0], X[:, 1], X[:, 2]
    J = np.zeros((len(X), 2, 3))
    if cam.type == 1:
        r2 = x * x + y * y
        r = np.sqrt(r2)
        th = np.arctan2(r, z)
        f = th + p[4] * th ** 3 + p[5] * th ** 5 + p[6] * th ** 7 + p[7] * th ** 9
        fd = 1 + 3 * p[4] * th ** 2 + 5 * p[5] * th ** 4 + 7 * p[6] * th ** 6 + 9 * p[7] * th ** 8
        den = r2 * (r2 + z * z)
        J[:, 0, 0] = p[0] * (fd * z * x * x / den + f * y * y / r ** 3)
        J[:, 1, 0] = p[1] * (fd * z * y * x / den - f * y * x / r ** 3)
        J[:, 0, 1] = p[0] * (fd * z * y * x / den - f * y * x / r ** 3)
        J[:, 1, 1] = p[1] * (fd * z * y * y / den + f * x * x / r ** 3)
        J[:, 0, 2] = -p[0] * fd * x / (r2 + z * z)
        J[:, 1, 2] = -p[1] * fd * y / (r2 + z * z)
    else:
        J[:, 0, 0] = p[0] / z
        J[:, 0, 2] = -p[0] * x / (z * z)
        J[:, 1, 1] = p[1] / z
        J[:, 1, 2] = -p[1] * y / (z * z)
    return J


def dpose_dxc(Xc):
    """d(Xc)/d(xi) for the left-multiplied update: [-[Xc]x | I] (g2o's SE3deriv rows)."""
    n = len(Xc)
    D = np.zeros((n, 3, 6))
    D[:, :, :3] = -np.stack([skew(v) for v in Xc])
    D[:, :, 3:] = np.eye(3)
    return D


class Edges:
    """Edges of one problem.  kind, pose index, point index (-1: fixed xw), obs (n x 3), w, camera."""

    def __init__(self, kind, pose, point, xw, obs, w, cams, cam_idx, unary):
        self.kind = np.asarray(kind, int)
        self.pose = np.asarray(pose, int)
        self.point = np.asarray(point, int)
        self.xw = xw
        self.obs = np.asarray(obs, float)
        self.w = np.asarray(w, f32).astype(float)
        self.cams = cams
        self.cam_idx = np.asarray(cam_idx, int)
        self.unary = unary
        n = len(self.kind)
        self.dim = np.where(self.kind == STEREO, 3, 2)
        self.delta = np.where(self.kind == STEREO, float(f32(math.sqrt(7.815))), float(f32(math.sqrt(5.991))))
        self.dsqr = (self.delta * self.delta).astype(f32).astype(float)
        self.robust = np.ones(n, bool)
        self.err = np.zeros((n, 3))

    def points_of(self, points, sel):
        if self.unary:
            return self.xw[sel]
        return points[self.point[sel]]

    def camera_frame(self, poses, points, sel):
        """Xc per edge (left camera; BODY edges: right camera) and the left-camera point."""
        X = self.points_of(points, sel)
        Xl = np.stack([poses[k].R @ X[i] + poses[k].t for i, k in enumerate(self.pose[sel])]) if len(X) else X
        Xc = Xl.copy()
        for i, e in enumerate(np.nonzero(sel)[0]):
            if self.kind[e] == BODY:
                c = self.cams[self.cam_idx[e]]
                Rrl = mat_of([c.trl[j] for j in range(4)])
                Xc[i] = Rrl @ Xl[i] + np.array([c.trl[4], c.trl[5], c.trl[6]])
        return X, Xl, Xc

    def compute_error(self, poses, points, sel, exact=False):
        """exact=True drops the reference's float casts (for finite-difference checks only)."""
        if not sel.any():
            return
        X, Xl, Xc = self.camera_frame(poses, points, sel)
        idx = np.nonzero(sel)[0]
        for i, e in enumerate(idx):
            c = self.cams[self.cam_idx[e]]
            if self.kind[e] == STEREO:
                # const float invz = 1.0f / trans_xyz[2]: double division, rounded to float
                invz = 1.0 / Xc[i, 2] if exact else f32(1.0 / Xc[i, 2])
                u = Xc[i, 0] * float(invz) * c.fx + c.cx
                v = Xc[i, 1] * float(invz) * c.fy + c.cy
                if self.unary or exact:  # EdgeStereoSE3ProjectXYZOnlyPose: double member bf
                    ur = u - float(c.bf) * float(invz)
                else:           # EdgeStereoSE3ProjectXYZ::cam_project(.., const float& bf)
                    ur = u - float(f32(c.bf) * invz)
                self.err[e] = self.obs[e] - np.array([u, v, ur])
            else:
                uv = project(c, Xc[i:i + 1], exact)[0]
                self.err[e, :2] = self.obs[e, :2] - uv
                self.err[e, 2] = 0.0

    def chi2(self):
        return (self.err * self.err).sum(1) * self.w

    def rho(self, chi2):
        """Huber rho(e2) and rho'(e2) (ref:robust_kernel_impl.cpp:78-91); plain chi2 without kernel."""
        big = (chi2 > self.dsqr) & self.robust
        s = np.sqrt(np.where(big, chi2, 1.0))
        r0 = np.where(big, 2 * s * self.delta - self.dsqr, chi2)
        r1 = np.where(big, self.delta / s, 1.0)
        return r0, r1

    def jacobians(self, poses, points, sel):
        """e = obs - pi(.): returns (J_pose n x 3 x 6, J_point n x 3 x 3), rows past dim zero."""
        X, Xl, Xc = self.camera_frame(poses, points, sel)
        idx = np.nonzero(sel)[0]
        Jp = np.zeros((len(idx), 3, 6))
        Jx = np.zeros((len(idx), 3, 3))
        D = dpose_dxc(Xl)
        for i, e in enumerate(idx):
            c = self.cams[self.cam_idx[e]]
            R = poses[self.pose[e]].R
            if self.kind[e] == STEREO:
                x, y, z = Xc[i]
                A = np.array([[c.fx / z, 0, -c.fx * x / z ** 2], [0, c.fy / z, -c.fy * y / z ** 2],
                              [c.fx / z, 0, -c.fx * x / z ** 2 + c.bf / z ** 2]])
                M = np.eye(3)
            elif self.kind[e] == BODY:
                A = np.zeros((3, 3))
                A[:2] = project_jac(c, Xc[i:i + 1])[0]
                M = mat_of([c.trl[j] for j in range(4)])
            else:
                A = np.zeros((3, 3))
                A[:2] = project_jac(c, Xc[i:i + 1])[0]
                M = np.eye(3)
            Jp[i] = -(A @ M @ D[i])
            Jx[i] = -(A @ M @ R)
        return Jp, Jx


class LM:
    """g2o OptimizationAlgorithmLevenberg over a dense normal-equation system."""

    def __init__(self, E, poses, points, pose_fixed, user_lambda=0.0, require_positive=False):
        self.E, self.poses, self.points = E, poses, points
        self.pose_fixed = pose_fixed
        self.user_lambda = user_lambda
        self.require_positive = require_positive
        self.trials = 0

    def initialize(self, active):
        E = self.E
        self.active = active.copy()
        used_pose = np.zeros(len(self.poses), bool)
        used_pose[E.pose[active]] = True
        self.free = [i for i in range(len(self.poses)) if used_pose[i] and not self.pose_fixed[i]]
        if E.unary:
            self.lm_pts = []
        else:
            used_pt = np.zeros(len(self.points), bool)
            used_pt[E.point[active]] = True
            self.lm_pts = list(np.nonzero(used_pt)[0])
        self.pidx = {p: 6 * k for k, p in enumerate(self.free)}
        base = 6 * len(self.free)
        self.lidx = {p: base + 3 * k for k, p in enumerate(self.lm_pts)}
        self.dim = base + 3 * len(self.lm_pts)

    def robust_chi2(self):
        """activeRobustChi2 (ref:Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:104-120)."""
        r0, _ = self.E.rho(self.E.chi2())
        return float(r0[self.active].sum())

    def build(self):
        E, a = self.E, self.active
        H = np.zeros((self.dim, self.dim))
        b = np.zeros(self.dim)
        sel = np.zeros(len(E.kind), bool)
        sel[a] = True
        Jp, Jx = E.jacobians(self.poses, self.points, sel)
        _, r1 = E.rho(E.chi2())
        for i, e in enumerate(np.nonzero(sel)[0]):
            d = E.dim[e]
            ww = r1[e] * E.w[e]
            err = E.err[e, :d]
            blocks = []
            if E.pose[e] in self.pidx:
                blocks.append((self.pidx[E.pose[e]], Jp[i, :d]))
            if not E.unary and E.point[e] in self.lidx:
                blocks.append((self.lidx[E.point[e]], Jx[i, :d]))
            for (oi, Ji) in blocks:
                b[oi:oi + Ji.shape[1]] -= r1[e] * Ji.T @ (E.w[e] * err)
                for (oj, Jj) in blocks:
                    H[oi:oi + Ji.shape[1], oj:oj + Jj.shape[1]] += Ji.T @ (ww * Jj)
        self.H, self.b = H, b

    def solve_linear(self, lam):
        A = self.H + lam * np.eye(self.dim)
        if self.require_positive:
            try:
                np.linalg.cholesky(A)
            except np.linalg.LinAlgError:
                return None
        try:
            return np.linalg.solve(A, self.b)
        except np.linalg.LinAlgError:
            return None

    def apply(self, x):
        for p, o in self.pidx.items():
            self.poses[p].oplus(x[o:o + 6])
        for p, o in self.lidx.items():
            self.points[p] = self.points[p] + x[o:o + 3]

    def errors(self):
        sel = np.zeros(len(self.E.kind), bool)
        sel[self.active] = True
        self.E.compute_error(self.poses, self.points, sel)

    def solve(self, iteration, stop=None):
        """One OptimizationAlgorithmLevenberg::solve; returns False to terminate."""
        self.errors()
        current = self.robust_chi2()
        ini = current
        self.build()
        if iteration == 0:
            if self.user_lambda > 0:
                self.lam = self.user_lambda
            else:
                self.lam = 1e-5 * float(np.abs(np.diag(self.H)).max()) if self.dim else 0.0
            self.ni = 2.0
            self.nbad = 0
        q = 0
        while True:
            bk = ([p.copy() for p in self.poses], self.points.copy())
            x = self.solve_linear(self.lam)
            self.trials += 1
            ok = x is not None
            if not ok:
                x = np.zeros(self.dim)
            self.apply(x)
            self.errors()
            temp = self.robust_chi2() if ok else np.finfo(float).max
            rho = (current - temp) / (float(x @ (self.lam * x + self.b)) + 1e-3)
            if rho > 0 and np.isfinite(temp):
                alpha = min(1.0 - (2 * rho - 1) ** 3, 2.0 / 3.0)
                self.lam *= max(1.0 / 3.0, alpha)
                self.ni = 2.0
                current = temp
            else:
                self.lam *= self.ni
                self.ni *= 2
                self.poses[:], self.points = bk[0], bk[1]
            q += 1
            if not (rho < 0 and q < 10 and not (stop is not None and stop)):
                break
        self.current = current
        if q == 10 or rho == 0:
            return False
        self.nbad = self.nbad + 1 if (ini - current) * 1e3 < ini else 0
        return self.nbad < 3

    def optimize(self, iterations, stop=None):
        if self.dim == 0:
            return 0
        n = 0
        for i in range(iterations):
            if stop is not None and stop:
                break
            n += 1
            if not self.solve(i, stop):
                break
        return n


def pose_optimization(P):
    """ref:src/Optimizer.cc:71-420 on an osg_pose_problem-like object (pose, kind, xw, obs,
    inv_sigma2, cam, cam2).  Returns (pose7, outlier flags, n_inliers, lm_iterations)."""
    n = len(P.kind)
    if n < 3:
        return np.array(P.pose, float), np.zeros(n, np.uint8), 0, 0
    cams = [P.cam, P.cam2]
    E = Edges(P.kind, np.zeros(n, int), -np.ones(n, int), np.asarray(P.xw, float).reshape(-1, 3),
              np.asarray(P.obs, float).reshape(-1, 3), P.inv_sigma2, cams,
              np.where(np.asarray(P.kind) == BODY, 1, 0), unary=True)
    level = np.zeros(n, int)
    outlier = np.zeros(n, bool)
    iters = 0
    nbad = 0
    pose = None
    for it in range(4):
        poses = [Pose(np.asarray(P.pose, float))]
        lm = LM(E, poses, np.zeros((0, 3)), [False], require_positive=True)
        lm.initialize(np.nonzero(level == 0)[0])
        iters += lm.optimize(10)
        pose = poses[0]
        nbad = 0
        for e in range(n):
            if outlier[e]:
                sel = np.zeros(n, bool)
                sel[e] = True
                E.compute_error(poses, None, sel)
            c2 = float(f32(E.chi2()[e]))
            th = float(f32(7.815)) if E.kind[e] == STEREO else float(f32(5.991))
            if c2 > th:
                outlier[e] = True
                level[e] = 1
                nbad += 1
            else:
                outlier[e] = False
                level[e] = 0
            if it == 2:
                E.robust[e] = False
        if n < 10:
            break
    return pose.p7(), outlier.astype(np.uint8), n - nbad, iters


def local_bundle_adjustment(G):
    """g2o part of ref:src/Optimizer.cc:1877-2203 on a BAGraph.  Returns (pose (np x 7),
    point (npt x 3), edge_bad, iterations, chi2_initial, chi2_final)."""
    return local_bundle_adjustment_chi2(G)[:6]


def local_bundle_adjustment_chi2(G):
    """local_bundle_adjustment plus each edge's chi2 of its last computed error (e->chi2())."""
    poses = [Pose(p) for p in np.asarray(G.pose, float).reshape(-1, 7)]
    points = np.asarray(G.point, float).reshape(-1, 3).copy()
    ne = len(G.e_pose)
    E = Edges(G.e_kind, G.e_pose, G.e_point, None, np.asarray(G.e_obs, float).reshape(-1, 3), G.e_inv_sigma2,
              G.cams, G.e_cam, unary=False)
    # BundleAdjustment's kernels (ref:src/Optimizer.cc:2933-2934, 3000-3007): its own deltas, and no
    # kernel at all on the edges the graph marks
    if G.huber_mono > 0 or G.huber_stereo > 0:
        E.delta = np.where(E.kind == STEREO, float(f32(G.huber_stereo)), float(f32(G.huber_mono)))
        E.dsqr = (E.delta * E.delta).astype(f32).astype(float)
    if G.e_robust is not None:
        E.robust = np.asarray(G.e_robust, bool).copy()
    lm = LM(E, poses, points, np.asarray(G.pose_fixed, bool), user_lambda=G.user_lambda_init)
    lm.initialize(np.arange(ne))
    lm.errors()
    chi_ini = lm.robust_chi2()
    iters = lm.optimize(G.iterations)
    stale = E.err.copy()
    lm.points = lm.points  # accepted state
    lm.errors()
    chi_fin = lm.robust_chi2()
    E.err = stale  # classification reads each edge's last computed error
    sel = np.ones(ne, bool)
    _, Xl, Xc = E.camera_frame(lm.poses, lm.points, sel)
    depth_ok = Xc[:, 2] > 0
    th = np.where(E.kind == STEREO, 7.815, 5.991)
    bad = ((E.chi2() > th) | ~depth_ok).astype(np.uint8)
    return np.stack([p.p7() for p in lm.poses]), lm.points, bad, iters, chi_ini, chi_fin, E.chi2()
