// kb8_epipolar.h — KannalaBrandt8::epipolarConstrain for SearchForTriangulation with bCoarse = false
// (ref:src/ORBmatcher.cc:1246 -> ref:src/CameraModels/KannalaBrandt8.cpp:321-326, TriangulateMatches
// :438-489, unproject :180-222, project :83-104, Triangulate :552-565).
//
// One lane evaluates the whole test: unproject both keypoints (Newton on theta, float), the parallax
// cosine, the two-view DLT triangulation, depth in both cameras, the reprojection errors in both.
// The reference's float expressions are kept in their order (translation unit built with
// -ffp-contract=off).  Its libm atan2f / tanf / cos / sin are evaluated as fixed double-precision
// kernels rounded once to float (fdlibm's published sin / cos / atan coefficients, Cody-Waite pi/2
// reduction), and Eigen's JacobiSVD null vector of the 4x4 DLT matrix as the smallest-eigenvalue
// eigenvector of A^T A by cyclic Jacobi rotations in double: deterministic, and the same operations
// in the same order as the oracle's restatement (oracle/oracle_triang.c), so the match decisions are
// bit-identical to it; against the reference binary they are unpinned at libm / Eigen's last ulp.
#pragma once

namespace kb8 {

__device__ inline double sin_k(double x, double y)
{
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double z = x * x, v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

__device__ inline double cos_k(double x, double y)
{
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}

// |x| <= 4: psi in [-pi, pi], theta in [0, pi / 2]
__device__ inline void sincos_d(double x, double &sn, double &cs)
{
    const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
    const double n = rint(x * 6.36619772367581382433e-01);
    const double r = x - n * pio2_1;
    const double w = n * pio2_1t;
    const double y0 = r - w;
    const double y1 = (r - y0) - w;
    const double s0 = sin_k(y0, y1), c0 = cos_k(y0, y1);
    switch (((int)n) & 3) {
    case 0: sn = s0; cs = c0; break;
    case 1: sn = c0; cs = -s0; break;
    case 2: sn = -s0; cs = -c0; break;
    default: sn = -c0; cs = s0; break;
    }
}

__device__ inline double atan_pos(double x)
{
    const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                              1.57079632679489655800e+00};
    const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                              6.12323399573676603587e-17};
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    int id;
    if (x > 1.0e16) return atanhi[3] + atanlo[3];
    if (x < 0.4375) {
        id = -1;
    } else if (x < 1.1875) {
        if (x < 0.6875) {
            id = 0;
            x = (2.0 * x - 1.0) / (2.0 + x);
        } else {
            id = 1;
            x = (x - 1.0) / (x + 1.0);
        }
    } else if (x < 2.4375) {
        id = 2;
        x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {
        id = 3;
        x = -1.0 / x;
    }
    const double z = x * x, w = z * z;
    const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    return atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
}

__device__ inline double atan2_d(double y, double x)
{
    const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    if (y == 0.0) return (x >= 0.0 && !signbit(x)) ? y : (signbit(y) ? -pi : pi);
    if (x == 0.0) return y > 0 ? 1.57079632679489655800e+00 : -1.57079632679489655800e+00;
    const double z = atan_pos(fabs(y / x));
    if (x > 0) return y > 0 ? z : -z;
    return y > 0 ? pi - (z - pi_lo) : (z - pi_lo) - pi;
}

__device__ inline float atan2f_(float y, float x) { return (float)atan2_d((double)y, (double)x); }
__device__ inline float tanf_(float t)
{
    double s, c;
    sincos_d((double)t, s, c);
    return (float)(s / c);
}

// KannalaBrandt8::unproject; p = {fx, fy, cx, cy, k0, k1, k2, k3}, precision 1e-6
__device__ inline void unproject(const float *p, float u, float v, float r[3])
{
    const float pwx = (u - p[2]) / p[0], pwy = (v - p[3]) / p[1];
    float scale = 1.f;
    float theta_d = sqrtf(pwx * pwx + pwy * pwy);
    theta_d = fminf(fmaxf(-(float)(3.14159265358979323846 / 2.f), theta_d), (float)(3.14159265358979323846 / 2.f));
    if (theta_d > 1e-8) {
        float theta = theta_d;
        for (int j = 0; j < 10; j++) {
            const float theta2 = theta * theta, theta4 = theta2 * theta2, theta6 = theta4 * theta2,
                        theta8 = theta4 * theta4;
            const float k0_theta2 = p[4] * theta2, k1_theta4 = p[5] * theta4;
            const float k2_theta6 = p[6] * theta6, k3_theta8 = p[7] * theta8;
            const float theta_fix = (theta * (1 + k0_theta2 + k1_theta4 + k2_theta6 + k3_theta8) - theta_d) /
                                    (1 + 3 * k0_theta2 + 5 * k1_theta4 + 7 * k2_theta6 + 9 * k3_theta8);
            theta = theta - theta_fix;
            if (fabsf(theta_fix) < 1e-6f) break;
        }
        scale = tanf_(theta) / theta_d;
    }
    r[0] = pwx * scale;
    r[1] = pwy * scale;
    r[2] = 1.f;
}

// KannalaBrandt8::project(Eigen::Vector3f)
__device__ inline void project(const float *p, const float X[3], float uv[2])
{
    const float x2_plus_y2 = X[0] * X[0] + X[1] * X[1];
    const float theta = atan2f_(sqrtf(x2_plus_y2), X[2]);
    const float psi = atan2f_(X[1], X[0]);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r = theta + p[4] * theta3 + p[5] * theta5 + p[6] * theta7 + p[7] * theta9;
    double sp, cp;
    sincos_d((double)psi, sp, cp);
    uv[0] = p[0] * r * (float)cp + p[2];
    uv[1] = p[1] * r * (float)sp + p[3];
}

// JacobiSVD V.col(3) of the 4x4 DLT matrix: smallest-eigenvalue eigenvector of A^T A, cyclic Jacobi
// (p < q in row order, 12 sweeps, a rotation skipped when |M_pq| == 0)
__device__ inline void null4(const float A[4][4], double v[4])
{
    double M[4][4], V[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 4; k++) s += (double)A[k][i] * (double)A[k][j];
            M[i][j] = s;
            V[i][j] = i == j ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 12; sweep++)
#pragma unroll
        for (int pp = 0; pp < 3; pp++)
#pragma unroll
            for (int q = pp + 1; q < 4; q++) {
                const double apq = M[pp][q];
                if (apq == 0.0) continue;
                const double tau = (M[q][q] - M[pp][pp]) / (2.0 * apq);
                const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
                const double c = 1.0 / sqrt(1.0 + t * t), sn = t * c;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double mkp = M[k][pp], mkq = M[k][q];
                    M[k][pp] = c * mkp - sn * mkq;
                    M[k][q] = sn * mkp + c * mkq;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double mpk = M[pp][k], mqk = M[q][k];
                    M[pp][k] = c * mpk - sn * mqk;
                    M[q][k] = sn * mpk + c * mqk;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double vkp = V[k][pp], vkq = V[k][q];
                    V[k][pp] = c * vkp - sn * vkq;
                    V[k][q] = sn * vkp + c * vkq;
                }
            }
    // the first least diagonal entry, and its column of V, with static indices only (a dynamic index
    // would put M and V in scratch memory)
    int m = 0;
    double best = M[0][0];
#pragma unroll
    for (int i = 1; i < 4; i++)
        if (M[i][i] < best) {
            best = M[i][i];
            m = i;
        }
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = m == 0 ? V[k][0] : m == 1 ? V[k][1] : m == 2 ? V[k][2] : V[k][3];
}

// TriangulateMatches with this = cam1 (pCamera1), pCamera2 = cam2: z1 with p3D = x3D, or the reference's
// negative codes -1..-5 (p3D untouched)
// the part after the two unprojections (r1 = cam1.unproject(kp1), r2 = cam2.unproject(kp2))
__device__ inline float triangulate_rays(const float *cam1, const float *cam2, const float *r1, const float *r2,
                                         float x1, float y1, float x2, float y2, const float *R12, const float *t12,
                                         float sigmaLevel, float unc, float *p3D)
{
    float r21[3];
#pragma unroll
    for (int i = 0; i < 3; i++) r21[i] = R12[3 * i] * r2[0] + R12[3 * i + 1] * r2[1] + R12[3 * i + 2] * r2[2];
    const float dot = r1[0] * r21[0] + r1[1] * r21[1] + r1[2] * r21[2];
    const float n1 = sqrtf(r1[0] * r1[0] + r1[1] * r1[1] + r1[2] * r1[2]);
    const float n21 = sqrtf(r21[0] * r21[0] + r21[1] * r21[1] + r21[2] * r21[2]);
    const float cosParallaxRays = dot / (n1 * n21);
    if (cosParallaxRays > 0.9998) return -1;
    float R21[9], t2[3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) R21[3 * i + j] = R12[3 * j + i];
#pragma unroll
    for (int i = 0; i < 3; i++) t2[i] = -(R21[3 * i] * t12[0] + R21[3 * i + 1] * t12[1] + R21[3 * i + 2] * t12[2]);
    const float T1[3][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}};
    const float T2[3][4] = {{R21[0], R21[1], R21[2], t2[0]}, {R21[3], R21[4], R21[5], t2[1]},
                            {R21[6], R21[7], R21[8], t2[2]}};
    float A[4][4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        A[0][j] = r1[0] * T1[2][j] - T1[0][j];
        A[1][j] = r1[1] * T1[2][j] - T1[1][j];
        A[2][j] = r2[0] * T2[2][j] - T2[0][j];
        A[3][j] = r2[1] * T2[2][j] - T2[1][j];
    }
    double h[4];
    null4(A, h);
    const float hf[4] = {(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    const float x3D[3] = {hf[0] / hf[3], hf[1] / hf[3], hf[2] / hf[3]};
    const float z1 = x3D[2];
    if (z1 <= 0) return -2;
    const float z2 = (R21[6] * x3D[0] + R21[7] * x3D[1] + R21[8] * x3D[2]) + t2[2];
    if (z2 <= 0) return -3;
    float uv1[2];
    project(cam1, x3D, uv1);
    const float errX1 = uv1[0] - x1, errY1 = uv1[1] - y1;
    if ((errX1 * errX1 + errY1 * errY1) > 5.991 * sigmaLevel) return -4;
    float x3D2[3], uv2[2];
#pragma unroll
    for (int i = 0; i < 3; i++)
        x3D2[i] = (R21[3 * i] * x3D[0] + R21[3 * i + 1] * x3D[1] + R21[3 * i + 2] * x3D[2]) + t2[i];
    project(cam2, x3D2, uv2);
    const float errX2 = uv2[0] - x2, errY2 = uv2[1] - y2;
    if ((errX2 * errX2 + errY2 * errY2) > 5.991 * unc) return -5;
    p3D[0] = x3D[0];
    p3D[1] = x3D[1];
    p3D[2] = x3D[2];
    return z1;
}

__device__ inline float triangulate_matches(const float *cam1, const float *cam2, float x1, float y1, float x2,
                                            float y2, const float *R12, const float *t12, float sigmaLevel,
                                            float unc, float *p3D)
{
    float r1[3], r2[3];
    unproject(cam1, x1, y1, r1);
    unproject(cam2, x2, y2, r2);
    return triangulate_rays(cam1, cam2, r1, r2, x1, y1, x2, y2, R12, t12, sigmaLevel, unc, p3D);
}

// epipolarConstrain: TriangulateMatches(...) > 0.0001f (ref:src/CameraModels/KannalaBrandt8.cpp:321-326)
__device__ inline bool epipolar_constrain(const float *cam1, const float *cam2, float x1, float y1, float x2,
                                          float y2, const float *R12, const float *t12, float sigmaLevel, float unc)
{
    float p3D[3];
    return triangulate_matches(cam1, cam2, x1, y1, x2, y2, R12, t12, sigmaLevel, unc, p3D) > 0.0001f;
}

}  // namespace kb8
