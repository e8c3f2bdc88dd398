// ba_common.h — FP64 device math shared by PoseOptimization (pose.hip) and LocalBundleAdjustment
// (ba.hip): g2o SE3Quat, the camera models, the ORB-SLAM3 / g2o reprojection edges and Huber.
//
//   SE3Quat exp / * / map / normalizeRotation   ref:Thirdparty/g2o/g2o/types/se3quat.h:104-284
//   VertexSE3Expmap::oplusImpl (exp(d) * T)     ref:Thirdparty/g2o/g2o/types/types_six_dof_expmap.h:73-76
//   Pinhole project / projectJac                ref:src/CameraModels/Pinhole.cpp:50-133
//   KannalaBrandt8 project / projectJac         ref:src/CameraModels/KannalaBrandt8.cpp:62-104,229-260
//   EdgeSE3ProjectXYZ[OnlyPose][ToBody]         ref:src/OptimizableTypes.cpp:58-265, ref:include/OptimizableTypes.h:32-158
//   EdgeStereoSE3ProjectXYZ[OnlyPose]           ref:Thirdparty/g2o/g2o/types/types_six_dof_expmap.cpp:190-404
//   RobustKernelHuber::robustify (float dsqr)   ref:Thirdparty/g2o/g2o/core/robust_kernel_impl.cpp:64-91
#pragma once
#include <hip/hip_runtime.h>

#include "exact_math.h"
#include "glibc_math.h"
#include "osg_internal.h"

namespace osgba {

struct SE3 {
    double q[4];  // x y z w
    double t[3];
};

__host__ __device__ inline void quat_normalize_rot(double *q)
{
    if (q[3] < 0) {
        q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3];
    }
    const double n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    if (n2 > 0) {
        const double n = sqrt(n2);
        q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
    }
}
__host__ __device__ inline void quat_mul(const double *a, const double *b, double *o)
{
    double r[4];
    r[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    r[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    r[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    r[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    o[0] = r[0]; o[1] = r[1]; o[2] = r[2]; o[3] = r[3];
}
__host__ __device__ inline void quat_rotate(const double *q, const double *v, double *o)
{
    double uv0 = q[1] * v[2] - q[2] * v[1], uv1 = q[2] * v[0] - q[0] * v[2], uv2 = q[0] * v[1] - q[1] * v[0];
    uv0 += uv0; uv1 += uv1; uv2 += uv2;
    const double c0 = q[1] * uv2 - q[2] * uv1, c1 = q[2] * uv0 - q[0] * uv2, c2 = q[0] * uv1 - q[1] * uv0;
    o[0] = v[0] + q[3] * uv0 + c0;
    o[1] = v[1] + q[3] * uv1 + c1;
    o[2] = v[2] + q[3] * uv2 + c2;
}
__host__ __device__ inline void quat_to_R(const double *q, double R[3][3])
{
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz; R[0][2] = txz + twy;
    R[1][0] = txy + twz; R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
    R[2][0] = txz - twy; R[2][1] = tyz + twx; R[2][2] = 1 - (txx + tyy);
}
// Eigen quaternionbase_assign_impl<Matrix3>; the largest-diagonal branch is spelled out per
// index (constant subscripts keep the matrix in registers)
__host__ __device__ inline void quat_from_R_branch(const double m[3][3], int i, double *q)
{
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double mii, mjj, mkk, mkj, mjk, mji, mij, mki, mik;
    if (i == 0) {
        mii = m[0][0]; mjj = m[1][1]; mkk = m[2][2]; mkj = m[2][1]; mjk = m[1][2];
        mji = m[1][0]; mij = m[0][1]; mki = m[2][0]; mik = m[0][2];
    } else if (i == 1) {
        mii = m[1][1]; mjj = m[2][2]; mkk = m[0][0]; mkj = m[0][2]; mjk = m[2][0];
        mji = m[2][1]; mij = m[1][2]; mki = m[0][1]; mik = m[1][0];
    } else {
        mii = m[2][2]; mjj = m[0][0]; mkk = m[1][1]; mkj = m[1][0]; mjk = m[0][1];
        mji = m[0][2]; mij = m[2][0]; mki = m[1][2]; mik = m[2][1];
    }
    double s = sqrt(mii - mjj - mkk + 1.0);
    const double qi = 0.5 * s;
    s = 0.5 / s;
    const double qw = (mkj - mjk) * s;
    const double qj = (mji + mij) * s;
    const double qk = (mki + mik) * s;
    q[3] = qw;
    q[0] = i == 0 ? qi : (j == 0 ? qj : qk);
    q[1] = i == 1 ? qi : (j == 1 ? qj : qk);
    q[2] = i == 2 ? qi : (j == 2 ? qj : qk);
    (void)k;
}
__host__ __device__ inline void R_to_quat(const double m[3][3], double *q)
{
    const double t = m[0][0] + m[1][1] + m[2][2];
    if (t > 0) {
        double s = sqrt(t + 1.0);
        q[3] = 0.5 * s;
        s = 0.5 / s;
        q[0] = (m[2][1] - m[1][2]) * s;
        q[1] = (m[0][2] - m[2][0]) * s;
        q[2] = (m[1][0] - m[0][1]) * s;
    } else {
        int i = 0;
        if (m[1][1] > m[0][0]) i = 1;
        if (m[2][2] > (i == 0 ? m[0][0] : m[1][1])) i = 2;
        quat_from_R_branch(m, i, q);
    }
}
__host__ __device__ inline SE3 se3_from7(const double *p)
{
    SE3 T;
    for (int i = 0; i < 4; i++) T.q[i] = p[i];
    for (int i = 0; i < 3; i++) T.t[i] = p[4 + i];
    quat_normalize_rot(T.q);
    return T;
}
__host__ __device__ inline void se3_to7(const SE3 &T, double *p)
{
    for (int i = 0; i < 4; i++) p[i] = T.q[i];
    for (int i = 0; i < 3; i++) p[4 + i] = T.t[i];
}
__host__ __device__ inline void se3_map(const SE3 &T, const double *x, double *o)
{
    double r[3];
    quat_rotate(T.q, x, r);
    o[0] = r[0] + T.t[0];
    o[1] = r[1] + T.t[1];
    o[2] = r[2] + T.t[2];
}
__host__ __device__ inline SE3 se3_mul(const SE3 &A, const SE3 &B)
{
    SE3 r = A;
    double rt[3];
    quat_rotate(A.q, B.t, rt);
    r.t[0] += rt[0]; r.t[1] += rt[1]; r.t[2] += rt[2];
    quat_mul(A.q, B.q, r.q);
    quat_normalize_rot(r.q);
    return r;
}
// UNI: every lane holds the same update (PoseOptimization), see osgx::sincos_rn_small
template <bool UNI = false>
__host__ __device__ inline SE3 se3_exp(const double *upd)
{
    const double w0 = upd[0], w1 = upd[1], w2 = upd[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double Om[3][3] = {{0, -w2, w1}, {w2, 0, -w0}, {-w1, w0, 0}};
    double Om2[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Om2[i][j] = Om[i][0] * Om[0][j] + Om[i][1] * Om[1][j] + Om[i][2] * Om[2][j];
    double R[3][3], V[3][3];
    if (theta < 0.00001) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = (i == j ? 1.0 : 0.0) + Om[i][j] + Om2[i][j];
                V[i][j] = R[i][j];
            }
    } else {
        // sin / cos / pow(theta, 3) of the reference, correctly rounded (exact_math.h)
        double st, ct;
        osgx::sincos_ref<UNI>(theta, st, ct);
        const double a = st / theta;
        const double b = (1 - ct) / (theta * theta);
        const double c = (theta - st) / osgx::cube_rn(theta);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = (i == j ? 1.0 : 0.0) + a * Om[i][j] + b * Om2[i][j];
                V[i][j] = (i == j ? 1.0 : 0.0) + b * Om[i][j] + c * Om2[i][j];
            }
    }
    SE3 O;
    R_to_quat(R, O.q);
    for (int i = 0; i < 3; i++) O.t[i] = V[i][0] * upd[3] + V[i][1] * upd[4] + V[i][2] * upd[5];
    quat_normalize_rot(O.q);
    return O;
}
template <bool UNI = false>
__host__ __device__ inline void se3_oplus(SE3 &T, const double *upd)
{
    const SE3 E = se3_exp<UNI>(upd);
    T = se3_mul(E, T);
}

// ------------------------------------------------------------------------------ cameras
__device__ inline void cam_project(const osg_camera &c, const double *v, double *uv)
{
    if (c.type == OSG_CAM_KB8) {
        const double x2_plus_y2 = v[0] * v[0] + v[1] * v[1];
        // the host libm's atan2f, restated bit for bit (glibc_math.h)
        const double theta = osgm::atan2f_fd(sqrtf((float)x2_plus_y2), (float)v[2]);
        const double psi = osgm::atan2f_fd((float)v[1], (float)v[0]);
        const double theta2 = theta * theta;
        const double theta3 = theta * theta2;
        const double theta5 = theta3 * theta2;
        const double theta7 = theta5 * theta2;
        const double theta9 = theta7 * theta2;
        const double r = theta + c.p[4] * theta3 + c.p[5] * theta5 + c.p[6] * theta7 + c.p[7] * theta9;
        double sp, cp;
        osgx::sincos_psi(psi, sp, cp);  // correctly rounded, as the oracle (exact_math.h)
        uv[0] = c.p[0] * r * cp + c.p[2];
        uv[1] = c.p[1] * r * sp + c.p[3];
    } else {
        uv[0] = c.p[0] * v[0] / v[2] + c.p[2];
        uv[1] = c.p[1] * v[1] / v[2] + c.p[3];
    }
}
__device__ inline void cam_project_jac(const osg_camera &c, const double *v, double J[2][3])
{
    if (c.type == OSG_CAM_KB8) {
        const double x2 = v[0] * v[0], y2 = v[1] * v[1], z2 = v[2] * v[2];
        const double r2 = x2 + y2;
        const double r = sqrt(r2);
        const double r3 = r2 * r;
        const double theta = osgx::atan2_rn(r, v[2]);  // correctly rounded, as the oracle
        const double theta2 = theta * theta, theta3 = theta2 * theta;
        const double theta4 = theta2 * theta2, theta5 = theta4 * theta;
        const double theta6 = theta2 * theta4, theta7 = theta6 * theta;
        const double theta8 = theta4 * theta4, theta9 = theta8 * theta;
        const double f = theta + theta3 * c.p[4] + theta5 * c.p[5] + theta7 * c.p[6] + theta9 * c.p[7];
        const double fd = 1 + 3 * c.p[4] * theta2 + 5 * c.p[5] * theta4 + 7 * c.p[6] * theta6 + 9 * c.p[7] * theta8;
        J[0][0] = c.p[0] * (fd * v[2] * x2 / (r2 * (r2 + z2)) + f * y2 / r3);
        J[1][0] = c.p[1] * (fd * v[2] * v[1] * v[0] / (r2 * (r2 + z2)) - f * v[1] * v[0] / r3);
        J[0][1] = c.p[0] * (fd * v[2] * v[1] * v[0] / (r2 * (r2 + z2)) - f * v[1] * v[0] / r3);
        J[1][1] = c.p[1] * (fd * v[2] * y2 / (r2 * (r2 + z2)) + f * x2 / r3);
        J[0][2] = -c.p[0] * fd * v[0] / (r2 + z2);
        J[1][2] = -c.p[1] * fd * v[1] / (r2 + z2);
    } else {
        J[0][0] = c.p[0] / v[2];
        J[0][1] = 0.0;
        J[0][2] = -c.p[0] * v[0] / (v[2] * v[2]);
        J[1][0] = 0.0;
        J[1][1] = c.p[1] / v[2];
        J[1][2] = -c.p[1] * v[1] / (v[2] * v[2]);
    }
}

// ------------------------------------------------------------------------------ edges
// binary = the point is a vertex (LBA: EdgeSE3ProjectXYZ*, g2o EdgeStereoSE3ProjectXYZ);
// unary  = the point is a constant Xw (PoseOptimization: *OnlyPose*).
__device__ inline void edge_error(int kind, bool binary, const osg_camera &cam, const SE3 &T, const double *X,
                                  const double *obs, double *err)
{
    double Xc[3];
    if (kind == OSG_EDGE_BODY) {
        const SE3 Trl = se3_from7(cam.trl);
        const SE3 Trw = se3_mul(Trl, T);
        se3_map(Trw, X, Xc);
        double uv[2];
        cam_project(cam, Xc, uv);
        err[0] = obs[0] - uv[0];
        err[1] = obs[1] - uv[1];
        err[2] = 0.0;
    } else if (kind == OSG_EDGE_STEREO) {
        se3_map(T, X, Xc);
        const double fx = cam.fx, fy = cam.fy, cx = cam.cx, cy = cam.cy;
        const float invz = (float)(1.0f / Xc[2]);
        const double r0 = Xc[0] * invz * fx + cx;
        const double r1 = Xc[1] * invz * fy + cy;
        double r2;
        if (binary) {
            const float bff = (float)(double)cam.bf;  // const float& bf parameter
            const float prod = bff * invz;
            r2 = r0 - prod;
        } else {
            const double bfd = cam.bf;                 // double member bf
            r2 = r0 - bfd * invz;
        }
        err[0] = obs[0] - r0;
        err[1] = obs[1] - r1;
        err[2] = obs[2] - r2;
    } else {
        se3_map(T, X, Xc);
        double uv[2];
        cam_project(cam, Xc, uv);
        err[0] = obs[0] - uv[0];
        err[1] = obs[1] - uv[1];
        err[2] = 0.0;
    }
}

__device__ inline bool edge_depth_positive(int kind, const osg_camera &cam, const SE3 &T, const double *X)
{
    double Xc[3];
    if (kind == OSG_EDGE_BODY) {
        const SE3 Trw = se3_mul(se3_from7(cam.trl), T);
        se3_map(Trw, X, Xc);
    } else {
        se3_map(T, X, Xc);
    }
    return Xc[2] > 0.0;
}

__device__ inline void se3deriv(const double *p, double S[3][6])
{
    const double x = p[0], y = p[1], z = p[2];
    S[0][0] = 0; S[0][1] = z; S[0][2] = -y; S[0][3] = 1; S[0][4] = 0; S[0][5] = 0;
    S[1][0] = -z; S[1][1] = 0; S[1][2] = x; S[1][3] = 0; S[1][4] = 1; S[1][5] = 0;
    S[2][0] = y; S[2][1] = -x; S[2][2] = 0; S[2][3] = 0; S[2][4] = 0; S[2][5] = 1;
}

// Jp: d(error)/d(pose) (dim x 6); Jx: d(error)/d(point) (dim x 3, binary edges only)
__device__ inline void edge_jacobians(int kind, bool binary, const osg_camera &cam, const SE3 &T, const double *X,
                                      double Jp[3][6], double Jx[3][3])
{
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 6; j++) Jp[i][j] = 0.0;
        for (int j = 0; j < 3; j++) Jx[i][j] = 0.0;
    }
    if (kind == OSG_EDGE_MONO) {
        double Xc[3], PJ[2][3], S[3][6];
        se3_map(T, X, Xc);
        cam_project_jac(cam, Xc, PJ);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++) PJ[i][j] = -PJ[i][j];
        se3deriv(Xc, S);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 6; j++) Jp[i][j] = PJ[i][0] * S[0][j] + PJ[i][1] * S[1][j] + PJ[i][2] * S[2][j];
        if (binary) {
            double R[3][3];
            quat_to_R(T.q, R);
            for (int i = 0; i < 2; i++)
                for (int j = 0; j < 3; j++) Jx[i][j] = PJ[i][0] * R[0][j] + PJ[i][1] * R[1][j] + PJ[i][2] * R[2][j];
        }
    } else if (kind == OSG_EDGE_BODY) {
        const SE3 Trl = se3_from7(cam.trl);
        double Xl[3], Xr[3], PJ[2][3], Rrl[3][3], S[3][6], A[2][3];
        se3_map(T, X, Xl);
        se3_map(Trl, Xl, Xr);
        cam_project_jac(cam, Xr, PJ);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++) PJ[i][j] = -PJ[i][j];
        quat_to_R(Trl.q, Rrl);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++) A[i][j] = PJ[i][0] * Rrl[0][j] + PJ[i][1] * Rrl[1][j] + PJ[i][2] * Rrl[2][j];
        se3deriv(Xl, S);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 6; j++) Jp[i][j] = A[i][0] * S[0][j] + A[i][1] * S[1][j] + A[i][2] * S[2][j];
        if (binary) {
            const SE3 Trw = se3_mul(Trl, T);
            double Rrw[3][3];
            quat_to_R(Trw.q, Rrw);
            for (int i = 0; i < 2; i++)
                for (int j = 0; j < 3; j++)
                    Jx[i][j] = PJ[i][0] * Rrw[0][j] + PJ[i][1] * Rrw[1][j] + PJ[i][2] * Rrw[2][j];
        }
    } else {  // STEREO, explicit g2o formulas
        double Xc[3];
        se3_map(T, X, Xc);
        const double fx = cam.fx, fy = cam.fy, bf = cam.bf;
        const double x = Xc[0], y = Xc[1], z = Xc[2];
        if (binary) {
            double R[3][3];
            quat_to_R(T.q, R);
            const double z_2 = z * z;
            for (int j = 0; j < 3; j++) {
                Jx[0][j] = -fx * R[0][j] / z + fx * x * R[2][j] / z_2;
                Jx[1][j] = -fy * R[1][j] / z + fy * y * R[2][j] / z_2;
                Jx[2][j] = Jx[0][j] - bf * R[2][j] / z_2;
            }
            Jp[0][0] = x * y / z_2 * fx;
            Jp[0][1] = -(1 + (x * x / z_2)) * fx;
            Jp[0][2] = y / z * fx;
            Jp[0][3] = -1. / z * fx;
            Jp[0][5] = x / z_2 * fx;
            Jp[1][0] = (1 + y * y / z_2) * fy;
            Jp[1][1] = -x * y / z_2 * fy;
            Jp[1][2] = -x / z * fy;
            Jp[1][4] = -1. / z * fy;
            Jp[1][5] = y / z_2 * fy;
            Jp[2][0] = Jp[0][0] - bf * y / z_2;
            Jp[2][1] = Jp[0][1] + bf * x / z_2;
            Jp[2][2] = Jp[0][2];
            Jp[2][3] = Jp[0][3];
            Jp[2][5] = Jp[0][5] - bf / z_2;
        } else {
            const double invz = 1.0 / z;
            const double invz_2 = invz * invz;
            Jp[0][0] = x * y * invz_2 * fx;
            Jp[0][1] = -(1 + (x * x * invz_2)) * fx;
            Jp[0][2] = y * invz * fx;
            Jp[0][3] = -invz * fx;
            Jp[0][5] = x * invz_2 * fx;
            Jp[1][0] = (1 + y * y * invz_2) * fy;
            Jp[1][1] = -x * y * invz_2 * fy;
            Jp[1][2] = -x * invz * fy;
            Jp[1][4] = -invz * fy;
            Jp[1][5] = y * invz_2 * fy;
            Jp[2][0] = Jp[0][0] - bf * y * invz_2;
            Jp[2][1] = Jp[0][1] + bf * x * invz_2;
            Jp[2][2] = Jp[0][2];
            Jp[2][3] = Jp[0][3];
            Jp[2][5] = Jp[0][5] - bf * invz_2;
        }
    }
}

__device__ inline double chi2_of(const double *err, int dim, double w)
{
    // dim is 2 or 3; spelled out so err stays in registers (a dynamic index sends it to scratch)
    double s = 0;
    s += err[0] * (w * err[0]);
    s += err[1] * (w * err[1]);
    if (dim > 2) s += err[2] * (w * err[2]);
    return s;
}

// Huber: rho = (rho0, rho1); dsqr is a float member in the reference
__device__ inline void huber(double e, double delta, float dsqr_f, double &rho0, double &rho1)
{
    const double dsqr = dsqr_f;
    if (e <= dsqr) {
        rho0 = e;
        rho1 = 1.;
    } else {
        const double sqrte = sqrt(e);
        rho0 = 2 * sqrte * delta - dsqr;
        rho1 = delta / sqrte;
    }
}

// wave64 sum of a double
__device__ inline double wave_sum(double v)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

}  // namespace osgba
