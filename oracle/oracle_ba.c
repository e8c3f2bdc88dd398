/*
 * oracle_ba.c — CPU restatement of ORB-SLAM3's PoseOptimization / LocalBundleAdjustment and the
 * g2o Levenberg–Marquardt + BlockSolver<6,3> inner loop they run.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg as the checker / CPU baseline; never linked into the product library.
 *
 * Followed (ref: = the reference tree):
 *   PoseOptimization            ref:src/Optimizer.cc:71-420
 *   LocalBundleAdjustment       ref:src/Optimizer.cc:1877-2203 (graph given already gathered)
 *   LM solve / lambda / scale   ref:Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:43-194
 *   optimize / active set       ref:Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:61-120,181-301,405-493
 *   BlockSolver build / Schur   ref:Thirdparty/g2o/g2o/core/block_solver.hpp:143-295,354-604
 *   quadratic forms             ref:Thirdparty/g2o/g2o/core/base_binary_edge.hpp:55-120, base_unary_edge.hpp:43-70
 *   Huber                       ref:Thirdparty/g2o/g2o/core/robust_kernel_impl.cpp:64-91 (dsqr stored as float)
 *   edges                       ref:src/OptimizableTypes.cpp:58-265, ref:include/OptimizableTypes.h:32-158,
 *                               ref:Thirdparty/g2o/g2o/types/types_six_dof_expmap.cpp:190-404
 *   SE3Quat exp / oplus / map   ref:Thirdparty/g2o/g2o/types/se3quat.h:104-284, types_six_dof_expmap.h:73-76
 *   cameras                     ref:src/CameraModels/Pinhole.cpp:50-133, KannalaBrandt8.cpp:62-260
 *
 * Third-party arithmetic restated from Eigen's published algorithms (Eigen is unpinned and absent):
 * Quaternion(Matrix3) (trace method), quaternion product / vector rotation (Eigen 3.3
 * _transformVector), 3x3 inverse by cofactors.  Linear solves: the reference uses Eigen::LDLT
 * (PoseOptimization) and Eigen::SimplicialLDLT with AMD ordering (LBA); the restatement factorises
 * the same matrix with a dense unpivoted LDL^T.  Results therefore agree to rounding (~1e-12
 * relative), not bitwise — the BA parity tolerance in DESIGN.md accounts for this.
 */
#include <float.h>
#include <math.h>
#include <quadmath.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ---------------------------------------------------------------- libm calls of the reference
 * SE3Quat::exp's sin(theta), cos(theta), pow(theta, 3) and the LM rule's pow(2 rho - 1, 3) are
 * evaluated CORRECTLY ROUNDED here: the mathematical value carried in double-double (~106 bits)
 * and rounded once.  The reference takes them from whatever libm it links; glibc 2.35 misrounds
 * 0.06-0.09 % of these arguments, so the reference's last bit is platform-dependent, and the
 * correctly rounded value is the one canonical reading of the expression.  This restatement sums
 * the Taylor terms by their recurrence (term_k = -term_{k-1} x^2 / ((2k+o-1)(2k+o))), unlike the
 * device's Horner over tabulated coefficients (csrc/exact_math.h); tests/test_exact_math.py checks
 * both against mpmath and against each other.  sin / cos take the series on [0, 0.8] (LM update
 * magnitudes) and libm beyond, like the device. */
typedef struct {
    double hi, lo;
} ddouble;
static ddouble dd_norm(double a, double b)
{ /* fast two-sum, |a| >= |b| */
    ddouble r;
    r.hi = a + b;
    r.lo = b - (r.hi - a);
    return r;
}
static ddouble dd_sum(ddouble a, ddouble b)
{
    const double s = a.hi + b.hi, v = s - a.hi;
    const double e = (a.hi - (s - v)) + (b.hi - v);
    return dd_norm(s, e + a.lo + b.lo);
}
static ddouble dd_prod(ddouble a, ddouble b)
{
    const double p = a.hi * b.hi;
    const double e = fma(a.hi, b.hi, -p);
    return dd_norm(p, e + (a.hi * b.lo + a.lo * b.hi));
}
static ddouble dd_div_int(ddouble a, double d)
{ /* a / d for an exactly representable integer d */
    const double q1 = a.hi / d;
    const double r = fma(-q1, d, a.hi) + a.lo; /* remainder, exact first term */
    return dd_norm(q1, r / d);
}
/* Parity runs evaluate the reference's libm calls correctly rounded (above).  The bench's
 * cpu_baseline legs time the reference's own arithmetic instead: oracle_set_libm(1) routes
 * sin / cos / pow(., 3) and the KB8 projection's cos / sin / atan2 through the host libm, whose cost
 * is what the reference pays (results then differ from the GPU's by the libm's last bit). */
static int g_libm = 0;
void oracle_set_libm(int on) { g_libm = on; }

double oracle_ref_pow3(double t)
{
    if (g_libm) return pow(t, 3);
    const double p = t * t, q = p * t;
    if (!(fabs(q) < 1e300) || !(fabs(p) < 1e300) || q == 0.0) return q;
    ddouble T = {t, 0.0};
    ddouble c = dd_prod(dd_prod(T, T), T);
    return c.hi + c.lo;
}
static double ref_series(double x, int odd)
{
    ddouble X = {x, 0.0};
    const ddouble x2 = dd_prod(X, X);
    ddouble term = odd ? X : (ddouble){1.0, 0.0}, sum = term;
    for (int k = 1; k < 30; k++) {
        term = dd_div_int(dd_prod(term, x2), (double)((2 * k - 1 + odd) * (2 * k + odd)));
        term.hi = -term.hi;
        term.lo = -term.lo;
        sum = dd_sum(sum, term);
        if (fabs(term.hi) < 1e-40 * fabs(sum.hi)) break;
    }
    return sum.hi + sum.lo;
}
double oracle_ref_sin(double x)
{
    if (g_libm) return sin(x);
    return (x >= 0.0 && x <= 0.8) ? ref_series(x, 1) : sin(x);
}
double oracle_ref_cos(double x)
{
    if (g_libm) return cos(x);
    return (x >= 0.0 && x <= 0.8) ? ref_series(x, 0) : cos(x);
}

/* ---------------------------------------------------------------- SE3Quat (x y z w | t) */
typedef struct {
    double q[4]; /* x y z w (Eigen coeffs order) */
    double t[3];
} se3;

static void quat_normalize_rot(double *q)
{ /* SE3Quat::normalizeRotation, ref:Thirdparty/g2o/g2o/types/se3quat.h:280-284 */
    if (q[3] < 0) {
        q[0] = -q[0];
        q[1] = -q[1];
        q[2] = -q[2];
        q[3] = -q[3];
    }
    const double n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    if (n2 > 0) {
        const double n = sqrt(n2);
        q[0] /= n;
        q[1] /= n;
        q[2] /= n;
        q[3] /= n;
    }
}
static void quat_mul(const double *a, const double *b, double *o)
{
    double r[4];
    r[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    r[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    r[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    r[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    memcpy(o, r, sizeof r);
}
static void quat_rotate(const double *q, const double *v, double *o)
{ /* Eigen 3.3 QuaternionBase::_transformVector */
    double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
    uv[0] += uv[0];
    uv[1] += uv[1];
    uv[2] += uv[2];
    const double c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2],
                         q[0] * uv[1] - q[1] * uv[0]};
    o[0] = v[0] + q[3] * uv[0] + c[0];
    o[1] = v[1] + q[3] * uv[1] + c[1];
    o[2] = v[2] + q[3] * uv[2] + c[2];
}
static void quat_to_R(const double *q, double R[3][3])
{ /* Eigen QuaternionBase::toRotationMatrix */
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0][0] = 1 - (tyy + tzz);
    R[0][1] = txy - twz;
    R[0][2] = txz + twy;
    R[1][0] = txy + twz;
    R[1][1] = 1 - (txx + tzz);
    R[1][2] = tyz - twx;
    R[2][0] = txz - twy;
    R[2][1] = tyz + twx;
    R[2][2] = 1 - (txx + tyy);
}
static void R_to_quat(double m[3][3], double *q)
{ /* Eigen quaternionbase_assign_impl<Matrix3> */
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
        if (m[2][2] > m[i][i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
        q[i] = 0.5 * s;
        s = 0.5 / s;
        q[3] = (m[k][j] - m[j][k]) * s;
        q[j] = (m[j][i] + m[i][j]) * s;
        q[k] = (m[k][i] + m[i][k]) * s;
    }
}
static void se3_set(se3 *T, const double *p7)
{ /* SE3Quat(Quaterniond, Vector3d) — normalizeRotation in the ctor */
    memcpy(T->q, p7, 4 * sizeof(double));
    memcpy(T->t, p7 + 4, 3 * sizeof(double));
    quat_normalize_rot(T->q);
}
static void se3_get(const se3 *T, double *p7)
{
    memcpy(p7, T->q, 4 * sizeof(double));
    memcpy(p7 + 4, T->t, 3 * sizeof(double));
}
static void se3_map(const se3 *T, const double *x, double *o)
{
    double r[3];
    quat_rotate(T->q, x, r);
    o[0] = r[0] + T->t[0];
    o[1] = r[1] + T->t[1];
    o[2] = r[2] + T->t[2];
}
static void se3_mul(const se3 *A, const se3 *B, se3 *O)
{ /* SE3Quat::operator*, ref:se3quat.h:104-110 */
    se3 r = *A;
    double rt[3];
    quat_rotate(A->q, B->t, rt);
    r.t[0] += rt[0];
    r.t[1] += rt[1];
    r.t[2] += rt[2];
    quat_mul(A->q, B->q, r.q);
    quat_normalize_rot(r.q);
    *O = r;
}
static void se3_exp(const double *upd, se3 *O)
{ /* SE3Quat::exp, ref:se3quat.h:223-257 */
    const double w[3] = {upd[0], upd[1], upd[2]};
    const double u[3] = {upd[3], upd[4], upd[5]};
    const double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double Om[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    double Om2[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Om2[i][j] = Om[i][0] * Om[0][j] + Om[i][1] * Om[1][j] + Om[i][2] * Om[2][j];
    double R[3][3], V[3][3];
    if (theta < 0.00001) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[i][j] = (i == j ? 1.0 : 0.0) + Om[i][j] + Om2[i][j];
        memcpy(V, R, sizeof R);
    } else {
        const double a = oracle_ref_sin(theta) / theta;
        const double b = (1 - oracle_ref_cos(theta)) / (theta * theta);
        const double c = (theta - oracle_ref_sin(theta)) / (oracle_ref_pow3(theta));
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = (i == j ? 1.0 : 0.0) + a * Om[i][j] + b * Om2[i][j];
                V[i][j] = (i == j ? 1.0 : 0.0) + b * Om[i][j] + c * Om2[i][j];
            }
    }
    R_to_quat(R, O->q);
    for (int i = 0; i < 3; i++) O->t[i] = V[i][0] * u[0] + V[i][1] * u[1] + V[i][2] * u[2];
    quat_normalize_rot(O->q);
}
static void se3_oplus(se3 *T, const double *upd)
{ /* VertexSE3Expmap::oplusImpl: exp(update) * estimate */
    se3 E;
    se3_exp(upd, &E);
    se3_mul(&E, T, T);
}

/* ---------------------------------------------------------------- cameras (double overloads) */
static void cam_project(const osg_camera *c, const double *v, double *uv)
{
    if (c->type == OSG_CAM_KB8) {
        const double x2_plus_y2 = v[0] * v[0] + v[1] * v[1];
        const double theta = atan2f(sqrtf((float)x2_plus_y2), (float)v[2]);
        const double psi = atan2f((float)v[1], (float)v[0]);
        const double theta2 = theta * theta;
        const double theta3 = theta * theta2;
        const double theta5 = theta3 * theta2;
        const double theta7 = theta5 * theta2;
        const double theta9 = theta7 * theta2;
        const double r = theta + c->p[4] * theta3 + c->p[5] * theta5 + c->p[6] * theta7 + c->p[7] * theta9;
        /* cos / sin correctly rounded (libm's last bit is host-dependent; csrc/exact_math.h sincos_psi) */
        uv[0] = c->p[0] * r * (g_libm ? cos(psi) : (double)cosq((__float128)psi)) + c->p[2];
        uv[1] = c->p[1] * r * (g_libm ? sin(psi) : (double)sinq((__float128)psi)) + c->p[3];
    } else {
        uv[0] = c->p[0] * v[0] / v[2] + c->p[2];
        uv[1] = c->p[1] * v[1] / v[2] + c->p[3];
    }
}
static void cam_project_jac(const osg_camera *c, const double *v, double J[2][3])
{
    if (c->type == OSG_CAM_KB8) {
        const double x2 = v[0] * v[0], y2 = v[1] * v[1], z2 = v[2] * v[2];
        const double r2 = x2 + y2;
        const double r = sqrt(r2);
        const double r3 = r2 * r;
        const double theta = g_libm ? atan2(r, v[2]) : (double)atan2q((__float128)r, (__float128)v[2]); /* CR: atan2_rn */
        const double theta2 = theta * theta, theta3 = theta2 * theta;
        const double theta4 = theta2 * theta2, theta5 = theta4 * theta;
        const double theta6 = theta2 * theta4, theta7 = theta6 * theta;
        const double theta8 = theta4 * theta4, theta9 = theta8 * theta;
        const double f = theta + theta3 * c->p[4] + theta5 * c->p[5] + theta7 * c->p[6] + theta9 * c->p[7];
        const double fd = 1 + 3 * c->p[4] * theta2 + 5 * c->p[5] * theta4 + 7 * c->p[6] * theta6 +
                          9 * c->p[7] * theta8;
        J[0][0] = c->p[0] * (fd * v[2] * x2 / (r2 * (r2 + z2)) + f * y2 / r3);
        J[1][0] = c->p[1] * (fd * v[2] * v[1] * v[0] / (r2 * (r2 + z2)) - f * v[1] * v[0] / r3);
        J[0][1] = c->p[0] * (fd * v[2] * v[1] * v[0] / (r2 * (r2 + z2)) - f * v[1] * v[0] / r3);
        J[1][1] = c->p[1] * (fd * v[2] * y2 / (r2 * (r2 + z2)) + f * x2 / r3);
        J[0][2] = -c->p[0] * fd * v[0] / (r2 + z2);
        J[1][2] = -c->p[1] * fd * v[1] / (r2 + z2);
    } else {
        J[0][0] = c->p[0] / v[2];
        J[0][1] = 0.f;
        J[0][2] = -c->p[0] * v[0] / (v[2] * v[2]);
        J[1][0] = 0.f;
        J[1][1] = c->p[1] / v[2];
        J[1][2] = -c->p[1] * v[1] / (v[2] * v[2]);
    }
}

/* ---------------------------------------------------------------- edges */
typedef struct {
    int pose;        /* pose vertex index */
    int point;       /* point vertex index, -1: unary edge with constant xw */
    int kind;
    int dim;         /* 2 or 3 */
    const osg_camera *cam;
    double xw[3];
    double obs[3];
    double w;        /* information diagonal = (double)invSigma2 */
    int robust;      /* Huber attached */
    double delta;    /* _delta */
    float dsqr;      /* dsqr (float member in the reference) */
    int level;       /* 0 active, 1 outlier (PoseOptimization) */
    double err[3];   /* _error as last computed */
} edge_t;

static void edge_point(const edge_t *e, const double *points, double *X)
{
    if (e->point < 0) memcpy(X, e->xw, sizeof e->xw);
    else memcpy(X, points + 3 * e->point, 3 * sizeof(double));
}

static void edge_compute_error(edge_t *e, const se3 *poses, const double *points)
{
    const se3 *T = &poses[e->pose];
    double X[3], Xc[3];
    edge_point(e, points, X);
    if (e->kind == OSG_EDGE_BODY) {
        se3 Trl, Trw;
        se3_set(&Trl, e->cam->trl);
        se3_mul(&Trl, T, &Trw);
        se3_map(&Trw, X, Xc);
        double uv[2];
        cam_project(e->cam, Xc, uv);
        e->err[0] = e->obs[0] - uv[0];
        e->err[1] = e->obs[1] - uv[1];
    } else if (e->kind == OSG_EDGE_STEREO) {
        se3_map(T, X, Xc);
        const double fx = e->cam->fx, fy = e->cam->fy, cx = e->cam->cx, cy = e->cam->cy;
        const float invz = 1.0f / Xc[2];
        double r0 = Xc[0] * invz * fx + cx;
        double r1 = Xc[1] * invz * fy + cy;
        double r2;
        if (e->point >= 0) {
            /* EdgeStereoSE3ProjectXYZ::cam_project(xyz, const float& bf): bf*invz in float */
            const float bff = (float)(double)e->cam->bf;
            const float prod = bff * invz;
            r2 = r0 - prod;
        } else {
            /* EdgeStereoSE3ProjectXYZOnlyPose::cam_project: double member bf */
            const double bfd = e->cam->bf;
            r2 = r0 - bfd * invz;
        }
        e->err[0] = e->obs[0] - r0;
        e->err[1] = e->obs[1] - r1;
        e->err[2] = e->obs[2] - r2;
    } else {
        se3_map(T, X, Xc);
        double uv[2];
        cam_project(e->cam, Xc, uv);
        e->err[0] = e->obs[0] - uv[0];
        e->err[1] = e->obs[1] - uv[1];
    }
}

static double edge_chi2(const edge_t *e)
{ /* BaseEdge::chi2 = e' * Omega * e with Omega = w * I */
    double s = 0;
    for (int i = 0; i < e->dim; i++) s += e->err[i] * (e->w * e->err[i]);
    return s;
}

static void huber(const edge_t *e, double x, double rho[3])
{ /* RobustKernelHuber::robustify, ref:robust_kernel_impl.cpp:78-91 */
    const double dsqr = e->dsqr;
    if (x <= dsqr) {
        rho[0] = x;
        rho[1] = 1.;
        rho[2] = 0.;
    } else {
        const double sqrte = sqrt(x);
        rho[0] = 2 * sqrte * e->delta - dsqr;
        rho[1] = e->delta / sqrte;
        rho[2] = -0.5 * rho[1] / x;
    }
}

static int edge_depth_positive(const edge_t *e, const se3 *poses, const double *points)
{
    const se3 *T = &poses[e->pose];
    double X[3], Xc[3];
    edge_point(e, points, X);
    if (e->kind == OSG_EDGE_BODY) {
        se3 Trl, Trw;
        se3_set(&Trl, e->cam->trl);
        se3_mul(&Trl, T, &Trw);
        se3_map(&Trw, X, Xc);
    } else {
        se3_map(T, X, Xc);
    }
    return Xc[2] > 0.0;
}

static void se3deriv(const double *p, double S[3][6])
{
    const double x = p[0], y = p[1], z = p[2];
    const double s[3][6] = {{0.f, z, -y, 1.f, 0.f, 0.f}, {-z, 0.f, x, 0.f, 1.f, 0.f}, {y, -x, 0.f, 0.f, 0.f, 1.f}};
    memcpy(S, s, sizeof s);
}

/* Jacobians: Jp (dim x 6) w.r.t. the pose, Jx (dim x 3) w.r.t. the point (binary edges). */
static void edge_linearize(const edge_t *e, const se3 *poses, const double *points, double Jp[3][6],
                           double Jx[3][3])
{
    const se3 *T = &poses[e->pose];
    double X[3];
    edge_point(e, points, X);
    memset(Jp, 0, sizeof(double) * 18);
    memset(Jx, 0, sizeof(double) * 9);
    if (e->kind == OSG_EDGE_MONO) {
        double Xc[3], PJ[2][3], R[3][3], S[3][6];
        se3_map(T, X, Xc);
        cam_project_jac(e->cam, Xc, PJ);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++) PJ[i][j] = -PJ[i][j];
        se3deriv(Xc, S);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 6; j++) Jp[i][j] = PJ[i][0] * S[0][j] + PJ[i][1] * S[1][j] + PJ[i][2] * S[2][j];
        if (e->point >= 0) {
            quat_to_R(T->q, R);
            for (int i = 0; i < 2; i++)
                for (int j = 0; j < 3; j++) Jx[i][j] = PJ[i][0] * R[0][j] + PJ[i][1] * R[1][j] + PJ[i][2] * R[2][j];
        }
    } else if (e->kind == OSG_EDGE_BODY) {
        se3 Trl, Trw;
        se3_set(&Trl, e->cam->trl);
        double Xl[3], Xr[3], PJ[2][3], Rrl[3][3], S[3][6], A[2][3];
        se3_map(T, X, Xl);
        se3_map(&Trl, Xl, Xr);
        cam_project_jac(e->cam, Xr, PJ);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++) PJ[i][j] = -PJ[i][j];
        quat_to_R(Trl.q, Rrl);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++) A[i][j] = PJ[i][0] * Rrl[0][j] + PJ[i][1] * Rrl[1][j] + PJ[i][2] * Rrl[2][j];
        se3deriv(Xl, S);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 6; j++) Jp[i][j] = A[i][0] * S[0][j] + A[i][1] * S[1][j] + A[i][2] * S[2][j];
        if (e->point >= 0) {
            double Rrw[3][3];
            se3_mul(&Trl, T, &Trw);
            quat_to_R(Trw.q, Rrw);
            for (int i = 0; i < 2; i++)
                for (int j = 0; j < 3; j++)
                    Jx[i][j] = PJ[i][0] * Rrw[0][j] + PJ[i][1] * Rrw[1][j] + PJ[i][2] * Rrw[2][j];
        }
    } else { /* STEREO: explicit g2o formulas */
        double Xc[3];
        se3_map(T, X, Xc);
        const double fx = e->cam->fx, fy = e->cam->fy, bf = e->cam->bf;
        const double x = Xc[0], y = Xc[1], z = Xc[2];
        if (e->point >= 0) {
            double R[3][3];
            quat_to_R(T->q, R);
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
            Jp[0][4] = 0;
            Jp[0][5] = x / z_2 * fx;
            Jp[1][0] = (1 + y * y / z_2) * fy;
            Jp[1][1] = -x * y / z_2 * fy;
            Jp[1][2] = -x / z * fy;
            Jp[1][3] = 0;
            Jp[1][4] = -1. / z * fy;
            Jp[1][5] = y / z_2 * fy;
            Jp[2][0] = Jp[0][0] - bf * y / z_2;
            Jp[2][1] = Jp[0][1] + bf * x / z_2;
            Jp[2][2] = Jp[0][2];
            Jp[2][3] = Jp[0][3];
            Jp[2][4] = 0;
            Jp[2][5] = Jp[0][5] - bf / z_2;
        } else {
            const double invz = 1.0 / z;
            const double invz_2 = invz * invz;
            Jp[0][0] = x * y * invz_2 * fx;
            Jp[0][1] = -(1 + (x * x * invz_2)) * fx;
            Jp[0][2] = y * invz * fx;
            Jp[0][3] = -invz * fx;
            Jp[0][4] = 0;
            Jp[0][5] = x * invz_2 * fx;
            Jp[1][0] = (1 + y * y * invz_2) * fy;
            Jp[1][1] = -x * y * invz_2 * fy;
            Jp[1][2] = -x * invz * fy;
            Jp[1][3] = 0;
            Jp[1][4] = -invz * fy;
            Jp[1][5] = y * invz_2 * fy;
            Jp[2][0] = Jp[0][0] - bf * y * invz_2;
            Jp[2][1] = Jp[0][1] + bf * x * invz_2;
            Jp[2][2] = Jp[0][2];
            Jp[2][3] = Jp[0][3];
            Jp[2][4] = 0;
            Jp[2][5] = Jp[0][5] - bf * invz_2;
        }
    }
}

/* ---------------------------------------------------------------- optimizer */
typedef struct {
    int n_poses, n_points, n_edges;
    se3 *poses;
    double *points;
    const uint8_t *pose_fixed;
    edge_t *edges;
    /* active structure (rebuilt by initialize) */
    int *active;       /* active edge list (ids ascending) */
    int n_active;
    int *pose_h;       /* hessian block index per pose, -1 fixed/inactive */
    int *point_h;      /* landmark block index per point, -1 inactive */
    int nhp, nhl;      /* free active poses / points */
    int *hp_pose;      /* hessian pose block -> pose index */
    int *hl_point;
    /* Hpl blocks: per active edge, the block it writes into */
    int *edge_blk;     /* -1 for unary / fixed pose */
    int n_blk;
    int *blk_pose_h, *blk_point_h;
    int *lm_blk_start, *lm_blk;  /* per landmark: its blocks sorted by pose hessian index */
    /* system */
    double *Hpp;       /* nhp x 36 (diagonal blocks; no pose-pose edges on this path) */
    double *Hll;       /* nhl x 9 */
    double *Hpl;       /* n_blk x 18 (6x3, row-major) */
    double *b, *x;     /* 6 nhp + 3 nhl */
    double *Hs;        /* dense Schur (6nhp)^2 */
    double *Dinv;      /* nhl x 9 */
    double *coef;
    /* push/pop backup */
    se3 *bk_poses;
    double *bk_points;
    /* LM state */
    double lambda, ni;
    int nBad;
    double user_lambda;
    int trials;
    const volatile uint8_t *stop;
} graph_t;

static int cmp_int(const void *a, const void *b)
{
    return (*(const int *)a) - (*(const int *)b);
}

/* SparseOptimizer::initializeOptimization(level 0) + BlockSolver::buildStructure */
static void g_initialize(graph_t *g)
{
    g->n_active = 0;
    int *pose_cnt = (int *)calloc(g->n_poses + 1, sizeof(int));
    int *point_cnt = (int *)calloc(g->n_points + 1, sizeof(int));
    for (int k = 0; k < g->n_edges; k++) {
        edge_t *e = &g->edges[k];
        if (e->level != 0) continue;
        const int pose_free = !g->pose_fixed[e->pose];
        const int all_fixed = !pose_free && e->point < 0; /* points are never fixed on this path */
        if (all_fixed) continue;
        g->active[g->n_active++] = k;
        pose_cnt[e->pose]++;
        if (e->point >= 0) point_cnt[e->point]++;
    }
    g->nhp = 0;
    for (int i = 0; i < g->n_poses; i++) {
        if (!g->pose_fixed[i] && pose_cnt[i] > 0) {
            g->pose_h[i] = g->nhp;
            g->hp_pose[g->nhp++] = i;
        } else g->pose_h[i] = -1;
    }
    g->nhl = 0;
    for (int i = 0; i < g->n_points; i++) {
        if (point_cnt[i] > 0) {
            g->point_h[i] = g->nhl;
            g->hl_point[g->nhl++] = i;
        } else g->point_h[i] = -1;
    }
    /* Hpl blocks: one per (free pose, point) pair, shared by parallel edges */
    g->n_blk = 0;
    int *lm_cnt = (int *)calloc(g->nhl + 1, sizeof(int));
    for (int a = 0; a < g->n_active; a++) {
        edge_t *e = &g->edges[g->active[a]];
        g->edge_blk[g->active[a]] = -1;
        if (e->point < 0) continue;
        const int ph = g->pose_h[e->pose];
        if (ph < 0) continue;
        lm_cnt[g->point_h[e->point]]++;
    }
    /* build per-landmark block lists, dedup by pose */
    g->lm_blk_start[0] = 0;
    for (int l = 0; l < g->nhl; l++) g->lm_blk_start[l + 1] = g->lm_blk_start[l] + lm_cnt[l];
    int *fill = (int *)calloc(g->nhl + 1, sizeof(int));
    int *tmp_pose = (int *)malloc(sizeof(int) * (g->lm_blk_start[g->nhl] + 1));
    for (int a = 0; a < g->n_active; a++) {
        edge_t *e = &g->edges[g->active[a]];
        if (e->point < 0) continue;
        const int ph = g->pose_h[e->pose];
        if (ph < 0) continue;
        const int lh = g->point_h[e->point];
        tmp_pose[g->lm_blk_start[lh] + fill[lh]++] = ph;
    }
    /* dedup + sort per landmark, assign block ids */
    int nb = 0;
    int *new_start = (int *)malloc(sizeof(int) * (g->nhl + 1));
    new_start[0] = 0;
    for (int l = 0; l < g->nhl; l++) {
        int *p = tmp_pose + g->lm_blk_start[l];
        const int c = fill[l];
        qsort(p, c, sizeof(int), cmp_int);
        int u = 0;
        for (int i = 0; i < c; i++)
            if (u == 0 || p[u - 1] != p[i]) p[u++] = p[i];
        for (int i = 0; i < u; i++) {
            g->blk_pose_h[nb] = p[i];
            g->blk_point_h[nb] = l;
            g->lm_blk[nb] = nb;
            nb++;
        }
        new_start[l + 1] = nb;
    }
    memcpy(g->lm_blk_start, new_start, sizeof(int) * (g->nhl + 1));
    g->n_blk = nb;
    /* map each active binary edge to its block */
    for (int a = 0; a < g->n_active; a++) {
        const int k = g->active[a];
        edge_t *e = &g->edges[k];
        if (e->point < 0) continue;
        const int ph = g->pose_h[e->pose];
        if (ph < 0) continue;
        const int lh = g->point_h[e->point];
        for (int bb = g->lm_blk_start[lh]; bb < g->lm_blk_start[lh + 1]; bb++)
            if (g->blk_pose_h[bb] == ph) {
                g->edge_blk[k] = bb;
                break;
            }
    }
    free(new_start);
    free(tmp_pose);
    free(fill);
    free(lm_cnt);
    free(pose_cnt);
    free(point_cnt);
}

static void g_compute_active_errors(graph_t *g)
{
    for (int a = 0; a < g->n_active; a++) edge_compute_error(&g->edges[g->active[a]], g->poses, g->points);
}

static double g_active_robust_chi2(graph_t *g)
{
    double chi = 0.0;
    for (int a = 0; a < g->n_active; a++) {
        const edge_t *e = &g->edges[g->active[a]];
        if (e->robust) {
            double rho[3];
            huber(e, edge_chi2(e), rho);
            chi += rho[0];
        } else chi += edge_chi2(e);
    }
    return chi;
}

/* BlockSolver::buildSystem: per active edge linearizeOplus + constructQuadraticForm */
static void g_build_system(graph_t *g)
{
    const int sp = 6 * g->nhp;
    memset(g->Hpp, 0, sizeof(double) * 36 * g->nhp);
    memset(g->Hll, 0, sizeof(double) * 9 * g->nhl);
    memset(g->Hpl, 0, sizeof(double) * 18 * g->n_blk);
    memset(g->b, 0, sizeof(double) * (sp + 3 * g->nhl));
    for (int a = 0; a < g->n_active; a++) {
        const int k = g->active[a];
        edge_t *e = &g->edges[k];
        double Jp[3][6], Jx[3][3];
        edge_linearize(e, g->poses, g->points, Jp, Jx);
        const int D = e->dim;
        const int ph = g->pose_h[e->pose];
        double rho1 = 1.0;
        if (e->robust) {
            double rho[3];
            huber(e, edge_chi2(e), rho);
            rho1 = rho[1];
        }
        const double ww = rho1 * e->w; /* weightedOmega diagonal */
        if (e->point < 0) {
            /* BaseUnaryEdge::constructQuadraticForm */
            if (ph < 0) continue;
            double *H = g->Hpp + 36 * ph;
            double *bp = g->b + 6 * ph;
            for (int i = 0; i < 6; i++) {
                double s = 0;
                for (int d = 0; d < D; d++) s += rho1 * Jp[d][i] * (e->w * e->err[d]);
                bp[i] -= s;
                for (int j = 0; j < 6; j++) {
                    double h = 0;
                    for (int d = 0; d < D; d++) h += Jp[d][i] * ww * Jp[d][j];
                    H[i * 6 + j] += h;
                }
            }
        } else {
            /* BaseBinaryEdge::constructQuadraticForm: from = point (A = Jx), to = pose (B = Jp) */
            const int lh = g->point_h[e->point];
            double omega_r[3];
            for (int d = 0; d < D; d++) omega_r[d] = -(e->w * e->err[d]) * rho1;
            double *bl = g->b + sp + 3 * lh;
            double *Hl = g->Hll + 9 * lh;
            for (int i = 0; i < 3; i++) {
                double s = 0;
                for (int d = 0; d < D; d++) s += Jx[d][i] * omega_r[d];
                bl[i] += s;
                for (int j = 0; j < 3; j++) {
                    double h = 0;
                    for (int d = 0; d < D; d++) h += Jx[d][i] * ww * Jx[d][j];
                    Hl[i * 3 + j] += h;
                }
            }
            if (ph >= 0) {
                double *Hb = g->Hpl + 18 * g->edge_blk[k];
                for (int i = 0; i < 6; i++)
                    for (int j = 0; j < 3; j++) {
                        double h = 0;
                        for (int d = 0; d < D; d++) h += Jp[d][i] * ww * Jx[d][j];
                        Hb[i * 3 + j] += h;
                    }
                double *bp = g->b + 6 * ph;
                double *H = g->Hpp + 36 * ph;
                for (int i = 0; i < 6; i++) {
                    double s = 0;
                    for (int d = 0; d < D; d++) s += Jp[d][i] * omega_r[d];
                    bp[i] += s;
                    for (int j = 0; j < 6; j++) {
                        double h = 0;
                        for (int d = 0; d < D; d++) h += Jp[d][i] * ww * Jp[d][j];
                        H[i * 6 + j] += h;
                    }
                }
            }
        }
    }
}

static double g_lambda_init(graph_t *g)
{ /* computeLambdaInit, ref:optimization_algorithm_levenberg.cpp:171-185 */
    if (g->user_lambda > 0) return g->user_lambda;
    double maxDiagonal = 0.;
    for (int i = 0; i < g->nhp; i++)
        for (int j = 0; j < 6; j++) maxDiagonal = fmax(fabs(g->Hpp[36 * i + 7 * j]), maxDiagonal);
    for (int i = 0; i < g->nhl; i++)
        for (int j = 0; j < 3; j++) maxDiagonal = fmax(fabs(g->Hll[9 * i + 4 * j]), maxDiagonal);
    return 1e-5 * maxDiagonal;
}

static void inv3(const double *m, double *o)
{ /* Eigen compute_inverse<Matrix3>: cofactors, det along column 0 */
#define M(i, j) m[(i)*3 + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    const double c00 = COF(0, 0), c10 = COF(1, 0), c20 = COF(2, 0);
    const double det = c00 * M(0, 0) + c10 * M(1, 0) + c20 * M(2, 0);
    const double invdet = 1.0 / det;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) o[i * 3 + j] = COF(j, i) * invdet;
#undef COF
#undef M
}

/* LDL^T without pivoting (returns 0 on a zero / non-positive pivot).  The dense algorithm restricted
 * to the matrix's envelope: row i's entries left of its first nonzero f[i] are zero in A and stay
 * zero in L (fill-in never leaves a row's profile), so every sum runs from max(f[i], f[j]) instead of
 * 0 — the same nonzero terms in the same order.  A map-scale BundleAdjustment's reduced camera
 * system is banded (keyframes share points with their neighbours only), which keeps the map-scale
 * parity test in seconds (ref: Eigen's SimplicialLDLT, which g2o's LinearSolverEigen uses, likewise
 * works on the sparsity only). */
static int ldlt_solve(double *A, int n, const double *bvec, double *x, int require_positive)
{
    /* A is row-major n x n symmetric; factor in place: A = L D L^T */
    int *f = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        int k = 0;
        while (k < i && A[(size_t)i * n + k] == 0.0) k++;
        f[i] = k;
    }
    for (int j = 0; j < n; j++) {
        const double *Aj = A + (size_t)j * n;
        double d = Aj[j];
        for (int k = f[j]; k < j; k++) d -= Aj[k] * Aj[k] * A[(size_t)k * n + k];
        if (d == 0.0 || (require_positive && !(d > 0.0))) {
            free(f);
            return 0;
        }
        A[(size_t)j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            if (f[i] > j) continue;  /* outside row i's profile: stays 0 */
            double *Ai = A + (size_t)i * n;
            double s = Ai[j];
            for (int k = f[i] > f[j] ? f[i] : f[j]; k < j; k++) s -= Ai[k] * Aj[k] * A[(size_t)k * n + k];
            Ai[j] = s / d;
        }
    }
    free(f);
    for (int i = 0; i < n; i++) {
        double s = bvec[i];
        for (int k = 0; k < i; k++) s -= A[i * n + k] * x[k];
        x[i] = s;
    }
    for (int i = 0; i < n; i++) x[i] /= A[i * n + i];
    for (int i = n - 1; i >= 0; i--) {
        double s = x[i];
        for (int k = i + 1; k < n; k++) s -= A[k * n + i] * x[k];
        x[i] = s;
    }
    return 1;
}

/* BlockSolver::setLambda + solve (Schur) + restoreDiagonal folded: the diagonal backup is
 * implicit because lambda is added on the fly to copies. */
static int g_solve(graph_t *g, double lambda, int require_positive)
{
    const int nhp = g->nhp, nhl = g->nhl, sp = 6 * nhp;
    /* Hschur = Hpp (+lambda) */
    memset(g->Hs, 0, sizeof(double) * sp * sp);
    for (int i = 0; i < nhp; i++)
        for (int r = 0; r < 6; r++)
            for (int c = 0; c < 6; c++)
                g->Hs[(6 * i + r) * sp + 6 * i + c] = g->Hpp[36 * i + 6 * r + c] + (r == c ? lambda : 0.0);
    memset(g->coef, 0, sizeof(double) * sp);
    for (int l = 0; l < nhl; l++) {
        double D[9];
        memcpy(D, g->Hll + 9 * l, sizeof D);
        D[0] += lambda;
        D[4] += lambda;
        D[8] += lambda;
        double *Di = g->Dinv + 9 * l;
        inv3(D, Di);
        const double *bl = g->b + sp + 3 * l;
        double db[3];
        for (int r = 0; r < 3; r++) db[r] = Di[3 * r] * bl[0] + Di[3 * r + 1] * bl[1] + Di[3 * r + 2] * bl[2];
        for (int o = g->lm_blk_start[l]; o < g->lm_blk_start[l + 1]; o++) {
            const int i1 = g->blk_pose_h[o];
            const double *Bi = g->Hpl + 18 * o;
            double BDinv[18];
            for (int r = 0; r < 6; r++)
                for (int c = 0; c < 3; c++)
                    BDinv[3 * r + c] = Bi[3 * r] * Di[c] + Bi[3 * r + 1] * Di[3 + c] + Bi[3 * r + 2] * Di[6 + c];
            for (int r = 0; r < 6; r++) g->coef[6 * i1 + r] += Bi[3 * r] * db[0] + Bi[3 * r + 1] * db[1] + Bi[3 * r + 2] * db[2];
            for (int in = o; in < g->lm_blk_start[l + 1]; in++) {
                const int i2 = g->blk_pose_h[in];
                const double *Bj = g->Hpl + 18 * in;
                for (int r = 0; r < 6; r++)
                    for (int c = 0; c < 6; c++) {
                        const double v = BDinv[3 * r] * Bj[3 * c] + BDinv[3 * r + 1] * Bj[3 * c + 1] +
                                         BDinv[3 * r + 2] * Bj[3 * c + 2];
                        g->Hs[(6 * i1 + r) * sp + 6 * i2 + c] -= v;
                    }
            }
        }
    }
    /* mirror the upper triangle (the linear solvers read the upper part only) */
    for (int r = 0; r < sp; r++)
        for (int c = 0; c < r; c++) g->Hs[r * sp + c] = g->Hs[c * sp + r];
    double *bs = (double *)malloc(sizeof(double) * (sp + 1));
    for (int i = 0; i < sp; i++) bs[i] = g->b[i] - g->coef[i];
    const int ok = ldlt_solve(g->Hs, sp, bs, g->x, require_positive);
    free(bs);
    if (!ok) return 0;
    /* landmarks: xl = Dinv (bl - Hpl^T xp) */
    for (int l = 0; l < nhl; l++) {
        double cl[3];
        memcpy(cl, g->b + sp + 3 * l, sizeof cl);
        for (int o = g->lm_blk_start[l]; o < g->lm_blk_start[l + 1]; o++) {
            const int i1 = g->blk_pose_h[o];
            const double *Bi = g->Hpl + 18 * o;
            for (int c = 0; c < 3; c++) {
                double s = 0;
                for (int r = 0; r < 6; r++) s += Bi[3 * r + c] * (-g->x[6 * i1 + r]);
                cl[c] += s;
            }
        }
        const double *Di = g->Dinv + 9 * l;
        for (int r = 0; r < 3; r++)
            g->x[sp + 3 * l + r] = Di[3 * r] * cl[0] + Di[3 * r + 1] * cl[1] + Di[3 * r + 2] * cl[2];
    }
    return 1;
}

static void g_update(graph_t *g)
{
    for (int i = 0; i < g->nhp; i++) se3_oplus(&g->poses[g->hp_pose[i]], g->x + 6 * i);
    const int sp = 6 * g->nhp;
    for (int l = 0; l < g->nhl; l++) {
        double *p = g->points + 3 * g->hl_point[l];
        p[0] += g->x[sp + 3 * l];
        p[1] += g->x[sp + 3 * l + 1];
        p[2] += g->x[sp + 3 * l + 2];
    }
}

enum { SOLVE_OK = 0, SOLVE_TERMINATE = 1 };

/* OptimizationAlgorithmLevenberg::solve, ref:optimization_algorithm_levenberg.cpp:61-169 */
static int g_lm_solve(graph_t *g, int iteration, int require_positive)
{
    g_compute_active_errors(g);
    double currentChi = g_active_robust_chi2(g);
    double tempChi = currentChi;
    const double iniChi = currentChi;
    g_build_system(g);
    if (iteration == 0) {
        g->lambda = g_lambda_init(g);
        g->ni = 2;
        g->nBad = 0;
    }
    double rho = 0;
    int qmax = 0;
    const int vec = 6 * g->nhp + 3 * g->nhl;
    do {
        /* push */
        memcpy(g->bk_poses, g->poses, sizeof(se3) * g->n_poses);
        memcpy(g->bk_points, g->points, sizeof(double) * 3 * g->n_points);
        const int ok2 = g_solve(g, g->lambda, require_positive);
        g->trials++;
        g_update(g);
        g_compute_active_errors(g);
        tempChi = g_active_robust_chi2(g);
        if (!ok2) tempChi = DBL_MAX;
        rho = (currentChi - tempChi);
        double scale = 0.;
        for (int j = 0; j < vec; j++) scale += g->x[j] * (g->lambda * g->x[j] + g->b[j]);
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && isfinite(tempChi)) {
            double alpha = 1. - oracle_ref_pow3(2 * rho - 1);
            alpha = fmin(alpha, 2. / 3.);
            const double scaleFactor = fmax(1. / 3., alpha);
            g->lambda *= scaleFactor;
            g->ni = 2;
            currentChi = tempChi;
        } else {
            g->lambda *= g->ni;
            g->ni *= 2;
            memcpy(g->poses, g->bk_poses, sizeof(se3) * g->n_poses);
            memcpy(g->points, g->bk_points, sizeof(double) * 3 * g->n_points);
        }
        qmax++;
    } while (rho < 0 && qmax < 10 && !(g->stop && *g->stop));
    if (qmax == 10 || rho == 0) return SOLVE_TERMINATE;
    if ((iniChi - currentChi) * 1e3 < iniChi) g->nBad++;
    else g->nBad = 0;
    if (g->nBad >= 3) return SOLVE_TERMINATE;
    return SOLVE_OK;
}

/* SparseOptimizer::optimize(iterations); returns the number of solve() calls */
static int g_optimize(graph_t *g, int iterations, int require_positive)
{
    if (g->nhp + g->nhl == 0) return -1; /* "0 vertices to optimize" */
    int cj = 0;
    int ok = 1;
    for (int i = 0; i < iterations && !(g->stop && *g->stop) && ok; i++) {
        const int res = g_lm_solve(g, i, require_positive);
        ok = (res == SOLVE_OK);
        cj++;
    }
    return cj;
}

static void g_alloc(graph_t *g)
{
    const int np = g->n_poses, npt = g->n_points, ne = g->n_edges;
    g->active = (int *)malloc(sizeof(int) * (ne + 1));
    g->pose_h = (int *)malloc(sizeof(int) * (np + 1));
    g->point_h = (int *)malloc(sizeof(int) * (npt + 1));
    g->hp_pose = (int *)malloc(sizeof(int) * (np + 1));
    g->hl_point = (int *)malloc(sizeof(int) * (npt + 1));
    g->edge_blk = (int *)malloc(sizeof(int) * (ne + 1));
    g->blk_pose_h = (int *)malloc(sizeof(int) * (ne + 1));
    g->blk_point_h = (int *)malloc(sizeof(int) * (ne + 1));
    g->lm_blk_start = (int *)malloc(sizeof(int) * (npt + 2));
    g->lm_blk = (int *)malloc(sizeof(int) * (ne + 1));
    g->Hpp = (double *)malloc(sizeof(double) * 36 * (np + 1));
    g->Hll = (double *)malloc(sizeof(double) * 9 * (npt + 1));
    g->Hpl = (double *)malloc(sizeof(double) * 18 * (ne + 1));
    g->b = (double *)malloc(sizeof(double) * (6 * np + 3 * npt + 1));
    g->x = (double *)malloc(sizeof(double) * (6 * np + 3 * npt + 1));
    g->Hs = (double *)malloc(sizeof(double) * (size_t)(6 * np) * (6 * np) + 8);
    g->Dinv = (double *)malloc(sizeof(double) * 9 * (npt + 1));
    g->coef = (double *)malloc(sizeof(double) * (6 * np + 1));
    g->bk_poses = (se3 *)malloc(sizeof(se3) * (np + 1));
    g->bk_points = (double *)malloc(sizeof(double) * 3 * (npt + 1));
    g->trials = 0;
}
static void g_free(graph_t *g)
{
    free(g->active);
    free(g->pose_h);
    free(g->point_h);
    free(g->hp_pose);
    free(g->hl_point);
    free(g->edge_blk);
    free(g->blk_pose_h);
    free(g->blk_point_h);
    free(g->lm_blk_start);
    free(g->lm_blk);
    free(g->Hpp);
    free(g->Hll);
    free(g->Hpl);
    free(g->b);
    free(g->x);
    free(g->Hs);
    free(g->Dinv);
    free(g->coef);
    free(g->bk_poses);
    free(g->bk_points);
}

/* ---------------------------------------------------------------- PoseOptimization */
/* ref:src/Optimizer.cc:71-420 */
int oracle_pose_optimization(const osg_pose_problem *P, osg_pose_result *R)
{
    const int N = P->n_edges;
    const float deltaMono = sqrt(5.991);
    const float deltaStereo = sqrt(7.815);
    memcpy(R->pose, P->pose, sizeof R->pose);
    R->lm_iterations = 0;
    R->lm_trials = 0;
    for (int i = 0; i < N; i++) R->outlier[i] = 0;
    const int nInitialCorrespondences = N;
    if (nInitialCorrespondences < 3) {
        R->n_inliers = 0;
        return 0;
    }
    graph_t g;
    memset(&g, 0, sizeof g);
    g.n_poses = 1;
    g.n_points = 0;
    g.n_edges = N;
    uint8_t fixed0 = 0;
    g.pose_fixed = &fixed0;
    se3 pose0;
    g.poses = &pose0;
    double dummy_pt[3] = {0, 0, 0};
    g.points = dummy_pt;
    g.edges = (edge_t *)calloc(N, sizeof(edge_t));
    for (int i = 0; i < N; i++) {
        edge_t *e = &g.edges[i];
        e->pose = 0;
        e->point = -1;
        e->kind = P->kind[i];
        e->dim = (e->kind == OSG_EDGE_STEREO) ? 3 : 2;
        e->cam = (e->kind == OSG_EDGE_BODY) ? &P->cam2 : &P->cam;
        memcpy(e->xw, P->xw + 3 * i, 3 * sizeof(double));
        memcpy(e->obs, P->obs + 3 * i, 3 * sizeof(double));
        e->w = (double)P->inv_sigma2[i];
        e->robust = 1;
        e->delta = (e->kind == OSG_EDGE_STEREO) ? (double)deltaStereo : (double)deltaMono;
        e->dsqr = (float)(e->delta * e->delta);
        e->level = 0;
    }
    g_alloc(&g);
    const float chi2Mono[4] = {5.991, 5.991, 5.991, 5.991};
    const float chi2Stereo[4] = {7.815, 7.815, 7.815, 7.815};
    const int its[4] = {10, 10, 10, 10};
    int nBad = 0;
    for (int it = 0; it < 4; it++) {
        se3_set(&pose0, P->pose);
        g_initialize(&g);
        const int n = g_optimize(&g, its[it], 1);
        if (n > 0) R->lm_iterations += n;
        nBad = 0;
        for (int i = 0; i < N; i++) {
            edge_t *e = &g.edges[i];
            if (R->outlier[i]) edge_compute_error(e, g.poses, g.points);
            const float chi2 = (float)edge_chi2(e);
            const float th = (e->kind == OSG_EDGE_STEREO) ? chi2Stereo[it] : chi2Mono[it];
            if (chi2 > th) {
                R->outlier[i] = 1;
                e->level = 1;
                nBad++;
            } else {
                R->outlier[i] = 0;
                e->level = 0;
            }
            if (it == 2) e->robust = 0;
        }
        if (N < 10) break;
    }
    se3_get(&pose0, R->pose);
    R->lm_trials = g.trials;
    R->n_inliers = nInitialCorrespondences - nBad;
    g_free(&g);
    free(g.edges);
    return R->n_inliers;
}

/* ---------------------------------------------------------------- LocalBundleAdjustment */
/* ref:src/Optimizer.cc:1877-2203 (the part after the graph is gathered) */
int oracle_local_bundle_adjustment(const osg_ba_graph *G, osg_ba_result *R, const volatile uint8_t *stop)
{
    /* LocalBundleAdjustment's deltas (ref:src/Optimizer.cc:1951-1952) unless the graph carries
     * BundleAdjustment's (thHuber2D = sqrt(5.99), thHuber3D, ref:src/Optimizer.cc:2933-2934) */
    const float thHuberMono = G->huber_mono > 0.f ? G->huber_mono : (float)sqrt(5.991);
    const float thHuberStereo = G->huber_stereo > 0.f ? G->huber_stereo : (float)sqrt(7.815);
    graph_t g;
    memset(&g, 0, sizeof g);
    g.n_poses = G->n_poses;
    g.n_points = G->n_points;
    g.n_edges = G->n_edges;
    g.pose_fixed = G->pose_fixed;
    g.poses = (se3 *)malloc(sizeof(se3) * (G->n_poses + 1));
    for (int i = 0; i < G->n_poses; i++) se3_set(&g.poses[i], G->pose + 7 * i);
    g.points = (double *)malloc(sizeof(double) * 3 * (G->n_points + 1));
    memcpy(g.points, G->point, sizeof(double) * 3 * G->n_points);
    g.edges = (edge_t *)calloc(G->n_edges + 1, sizeof(edge_t));
    for (int i = 0; i < G->n_edges; i++) {
        edge_t *e = &g.edges[i];
        e->pose = G->e_pose[i];
        e->point = G->e_point[i];
        e->kind = G->e_kind[i];
        e->dim = (e->kind == OSG_EDGE_STEREO) ? 3 : 2;
        e->cam = &G->cams[G->e_cam[i]];
        memcpy(e->obs, G->e_obs + 3 * i, 3 * sizeof(double));
        e->w = (double)G->e_inv_sigma2[i];
        /* no kernel attached (BundleAdjustment, bRobust = false): the plain chi2 / quadratic form */
        e->robust = G->e_robust ? (G->e_robust[i] != 0) : 1;
        e->delta = (e->kind == OSG_EDGE_STEREO) ? (double)thHuberStereo : (double)thHuberMono;
        e->dsqr = (float)(e->delta * e->delta);
        e->level = 0;
    }
    g_alloc(&g);
    g.user_lambda = G->user_lambda_init;
    g.stop = stop;
    R->aborted = 0;
    R->iterations = 0;
    R->chi2_initial = R->chi2_final = 0.0;
    if (stop && *stop) {
        /* ref:src/Optimizer.cc:2112-2114: return before optimising, nothing written back */
        R->aborted = 1;
        R->trials = 0;
        for (int i = 0; i < G->n_edges; i++) R->edge_bad[i] = 0;
        if (R->edge_chi2)
            for (int i = 0; i < G->n_edges; i++) R->edge_chi2[i] = 0.0;
        memcpy(R->pose, G->pose, sizeof(double) * 7 * G->n_poses);
        memcpy(R->point, G->point, sizeof(double) * 3 * G->n_points);
        g_free(&g);
        free(g.poses);
        free(g.points);
        free(g.edges);
        return 0;
    } else {
        g_initialize(&g);
        g_compute_active_errors(&g);
        R->chi2_initial = g_active_robust_chi2(&g);
        const int n = g_optimize(&g, G->iterations, 0);
        R->iterations = n > 0 ? n : 0;
        R->aborted = (stop && *stop) ? 1 : 0;
        /* chi2 of the accepted state */
        edge_t *tmp = (edge_t *)malloc(sizeof(edge_t) * (g.n_edges + 1));
        memcpy(tmp, g.edges, sizeof(edge_t) * g.n_edges);
        g_compute_active_errors(&g);
        R->chi2_final = g_active_robust_chi2(&g);
        memcpy(g.edges, tmp, sizeof(edge_t) * g.n_edges); /* keep the stale _error for classification */
        free(tmp);
    }
    R->trials = g.trials;
    /* classification with the edges' last computed errors (ref:src/Optimizer.cc:2125-2168) */
    for (int i = 0; i < G->n_edges; i++) {
        const edge_t *e = &g.edges[i];
        const double th = (e->kind == OSG_EDGE_STEREO) ? 7.815 : 5.991;
        R->edge_bad[i] = (edge_chi2(e) > th || !edge_depth_positive(e, g.poses, g.points)) ? 1 : 0;
        if (R->edge_chi2) R->edge_chi2[i] = edge_chi2(e);
    }
    for (int i = 0; i < G->n_poses; i++) se3_get(&g.poses[i], R->pose + 7 * i);
    memcpy(R->point, g.points, sizeof(double) * 3 * G->n_points);
    g_free(&g);
    free(g.poses);
    free(g.points);
    free(g.edges);
    return R->iterations;
}
