/* oracle_triang.c — CPU restatement of ORBmatcher::SearchForTriangulation.
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, never linked into the product.
 *
 *   ref:src/ORBmatcher.cc:1045-1328   the FeatureVector merge-walk, the per-pair tests, the
 *                                     rotation histogram and vMatchedPairs
 *   ref:src/CameraModels/Pinhole.cpp:189-219   epipolarConstrain
 *   ref:src/CameraModels/KannalaBrandt8.cpp:62-104,180-222,321-326,438-489,552-565
 *                                     KannalaBrandt8 epipolarConstrain = TriangulateMatches > 1e-4
 *                                     (unproject, project, the DLT triangulation)
 * The epipole and the F12 matrices are the caller's (osg_triang_geom, ref:src/ORBmatcher.cc:1052-1083).
 * Literal loop structure: std::map lower_bound jumps, `bestDist = TH_LOW`, `dist > TH_LOW ||
 * dist > bestDist` (so equal distances move the best to the later keypoint), no vbMatched2 claim
 * (commented out in this fork, :1262).  Output: vMatches12 per KF1 keypoint after the histogram. */
#include <math.h>
#include <stdlib.h>

#include "oracle.h"

static int lower_bound_u32(const uint32_t *a, int lo, int hi, uint32_t key)
{
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* Pinhole::epipolarConstrain, F(r, c) = F[3r + c] */
static int epipolar_constrain(const float *F, float x1, float y1, float x2, float y2, float unc)
{
    const float a = x1 * F[0] + y1 * F[3] + F[6];
    const float b = x1 * F[1] + y1 * F[4] + F[7];
    const float c = x1 * F[2] + y1 * F[5] + F[8];
    const float num = a * x2 + b * y2 + c;
    const float den = a * a + b * b;
    if (den == 0) return 0;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * unc;
}

/* ---- KannalaBrandt8::epipolarConstrain --------------------------------------------------------
 * The reference runs float arithmetic with libm's atan2f / tanf / cos / sin and Eigen's JacobiSVD.
 * Here: the same float expressions in the same order; the transcendental functions as fixed
 * double-precision kernels (fdlibm's published coefficients: Cody-Waite pi/2 reduction + the sin /
 * cos / atan minimax polynomials) rounded once to float, and the SVD's null vector as the
 * smallest-eigenvalue eigenvector of A^T A by cyclic Jacobi in double.  So parity with the
 * reference's binary is unpinned at the last ulp (libm and Eigen rounding), while the GPU
 * restatement (csrc/kb8_epipolar.h) evaluates the same operations in the same order. */
static double kb_sin_k(double x, double y)
{
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double z = x * x, v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
static double kb_cos_k(double x, double y)
{
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}
/* |x| <= 4 (every argument here: psi in [-pi, pi], theta in [0, pi/2]) */
static void kb_sincos_d(double x, double *sn, double *cs)
{
    const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
    const double n = rint(x * 6.36619772367581382433e-01);
    const double r = x - n * pio2_1;
    const double w = n * pio2_1t;
    const double y0 = r - w;
    const double y1 = (r - y0) - w;
    const double s0 = kb_sin_k(y0, y1), c0 = kb_cos_k(y0, y1);
    switch (((int)n) & 3) {
    case 0: *sn = s0; *cs = c0; break;
    case 1: *sn = c0; *cs = -s0; break;
    case 2: *sn = -s0; *cs = -c0; break;
    default: *sn = -c0; *cs = s0; break;
    }
}
/* fdlibm atan for x >= 0 */
static double kb_atan_pos(double x)
{
    static const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                      9.82793723247329054082e-01, 1.57079632679489655800e+00};
    static const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                      1.39033110312309984516e-17, 6.12323399573676603587e-17};
    static const double aT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                                  -1.11111104054623557880e-01, 9.09088713343650656196e-02, -7.69187620504482999495e-02,
                                  6.66107313738753120669e-02, -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                                  -3.65315727442169155270e-02, 1.62858201153657823623e-02};
    int id;
    if (x > 1.0e16) return atanhi[3] + atanlo[3];
    if (x < 0.4375) {
        id = -1;
    } else if (x < 1.1875) {
        if (x < 0.6875) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
        else { id = 1; x = (x - 1.0) / (x + 1.0); }
    } else if (x < 2.4375) {
        id = 2; x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {
        id = 3; x = -1.0 / x;
    }
    const double z = x * x, w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    return atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
}
/* atan2(y, x) in double for finite arguments (fdlibm's quadrant rules) */
static double kb_atan2_d(double y, double x)
{
    const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    if (y == 0.0) return (x >= 0.0 && !signbit(x)) ? y : (signbit(y) ? -pi : pi);
    if (x == 0.0) return y > 0 ? 1.57079632679489655800e+00 : -1.57079632679489655800e+00;
    const double z = kb_atan_pos(fabs(y / x));
    if (x > 0) return y > 0 ? z : -z;
    return y > 0 ? pi - (z - pi_lo) : (z - pi_lo) - pi;
}
static float kb_atan2f(float y, float x) { return (float)kb_atan2_d((double)y, (double)x); }
static float kb_tanf(float t)
{
    double s, c;
    kb_sincos_d((double)t, &s, &c);
    return (float)(s / c);
}
static float kb_cosf(float t)
{
    double s, c;
    kb_sincos_d((double)t, &s, &c);
    return (float)c;
}
static float kb_sinf(float t)
{
    double s, c;
    kb_sincos_d((double)t, &s, &c);
    return (float)s;
}

/* KannalaBrandt8::unproject (KannalaBrandt8.cpp:180-222); p = {fx, fy, cx, cy, k0..k3}, precision 1e-6 */
static void kb_unproject(const float *p, float u, float v, float r[3])
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
        scale = kb_tanf(theta) / theta_d;
    }
    r[0] = pwx * scale;
    r[1] = pwy * scale;
    r[2] = 1.f;
}

/* KannalaBrandt8::project(Eigen::Vector3f) (KannalaBrandt8.cpp:83-104) */
static void kb_project(const float *p, const float X[3], float uv[2])
{
    const float x2_plus_y2 = X[0] * X[0] + X[1] * X[1];
    const float theta = kb_atan2f(sqrtf(x2_plus_y2), X[2]);
    const float psi = kb_atan2f(X[1], X[0]);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r = theta + p[4] * theta3 + p[5] * theta5 + p[6] * theta7 + p[7] * theta9;
    uv[0] = p[0] * r * kb_cosf(psi) + p[2];
    uv[1] = p[1] * r * kb_sinf(psi) + p[3];
}

/* the null vector of the 4x4 DLT matrix A (JacobiSVD V.col(3)): smallest-eigenvalue eigenvector of
 * M = A^T A by cyclic Jacobi rotations (p < q in row order, 12 sweeps, skipped when |M_pq| == 0) */
static void kb_null4(const float A[4][4], double v[4])
{
    double M[4][4], V[4][4];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0.0;
            for (int k = 0; k < 4; k++) s += (double)A[k][i] * (double)A[k][j];
            M[i][j] = s;
            V[i][j] = i == j ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 12; sweep++)
        for (int pp = 0; pp < 3; pp++)
            for (int q = pp + 1; q < 4; q++) {
                const double apq = M[pp][q];
                if (apq == 0.0) continue;
                const double tau = (M[q][q] - M[pp][pp]) / (2.0 * apq);
                const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
                const double c = 1.0 / sqrt(1.0 + t * t), sn = t * c;
                for (int k = 0; k < 4; k++) {
                    const double mkp = M[k][pp], mkq = M[k][q];
                    M[k][pp] = c * mkp - sn * mkq;
                    M[k][q] = sn * mkp + c * mkq;
                }
                for (int k = 0; k < 4; k++) {
                    const double mpk = M[pp][k], mqk = M[q][k];
                    M[pp][k] = c * mpk - sn * mqk;
                    M[q][k] = sn * mpk + c * mqk;
                }
                for (int k = 0; k < 4; k++) {
                    const double vkp = V[k][pp], vkq = V[k][q];
                    V[k][pp] = c * vkp - sn * vkq;
                    V[k][q] = sn * vkp + c * vkq;
                }
            }
    int m = 0;
    for (int i = 1; i < 4; i++)
        if (M[i][i] < M[m][m]) m = i;
    for (int k = 0; k < 4; k++) v[k] = V[k][m];
}

/* KannalaBrandt8::TriangulateMatches (KannalaBrandt8.cpp:438-520): this = cam1; z1 with p3D = x3D, or the
 * reference's negative codes (p3D untouched) */
static float kb_triangulate_matches(const float *cam1, const float *cam2, float x1, float y1, float x2, float y2,
                                    const float *R12, const float *t12, float sigmaLevel, float unc, float *p3D)
{
    float r1[3], r2[3], r21[3];
    kb_unproject(cam1, x1, y1, r1);
    kb_unproject(cam2, x2, y2, r2);
    for (int i = 0; i < 3; i++) r21[i] = R12[3 * i] * r2[0] + R12[3 * i + 1] * r2[1] + R12[3 * i + 2] * r2[2];
    const float dot = r1[0] * r21[0] + r1[1] * r21[1] + r1[2] * r21[2];
    const float n1 = sqrtf(r1[0] * r1[0] + r1[1] * r1[1] + r1[2] * r1[2]);
    const float n21 = sqrtf(r21[0] * r21[0] + r21[1] * r21[1] + r21[2] * r21[2]);
    const float cosParallaxRays = dot / (n1 * n21);
    if (cosParallaxRays > 0.9998) return -1;
    /* Tcw1 = [I | 0], Tcw2 = [R21 | -R21 t12], R21 = R12^T */
    float R21[9], t2[3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R21[3 * i + j] = R12[3 * j + i];
    for (int i = 0; i < 3; i++) t2[i] = -(R21[3 * i] * t12[0] + R21[3 * i + 1] * t12[1] + R21[3 * i + 2] * t12[2]);
    const float T1[3][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}};
    const float T2[3][4] = {{R21[0], R21[1], R21[2], t2[0]}, {R21[3], R21[4], R21[5], t2[1]},
                            {R21[6], R21[7], R21[8], t2[2]}};
    float A[4][4];                                                              /* Triangulate, :552-565 */
    for (int j = 0; j < 4; j++) {
        A[0][j] = r1[0] * T1[2][j] - T1[0][j];
        A[1][j] = r1[1] * T1[2][j] - T1[1][j];
        A[2][j] = r2[0] * T2[2][j] - T2[0][j];
        A[3][j] = r2[1] * T2[2][j] - T2[1][j];
    }
    double h[4];
    kb_null4(A, h);
    const float hf[4] = {(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    const float x3D[3] = {hf[0] / hf[3], hf[1] / hf[3], hf[2] / hf[3]};
    const float z1 = x3D[2];
    if (z1 <= 0) return -2;
    const float z2 = (R21[6] * x3D[0] + R21[7] * x3D[1] + R21[8] * x3D[2]) + t2[2];
    if (z2 <= 0) return -3;
    float uv1[2];
    kb_project(cam1, x3D, uv1);
    const float errX1 = uv1[0] - x1, errY1 = uv1[1] - y1;
    if ((errX1 * errX1 + errY1 * errY1) > 5.991 * sigmaLevel) return -4;
    float x3D2[3], uv2[2];
    for (int i = 0; i < 3; i++) x3D2[i] = (R21[3 * i] * x3D[0] + R21[3 * i + 1] * x3D[1] + R21[3 * i + 2] * x3D[2]) + t2[i];
    kb_project(cam2, x3D2, uv2);
    const float errX2 = uv2[0] - x2, errY2 = uv2[1] - y2;
    if ((errX2 * errX2 + errY2 * errY2) > 5.991 * unc) return -5;
    p3D[0] = x3D[0];
    p3D[1] = x3D[1];
    p3D[2] = x3D[2];
    return z1;
}

/* epipolarConstrain = TriangulateMatches(...) > 0.0001f (KannalaBrandt8.cpp:321-326) */
static int kb_epipolar_constrain(const float *cam1, const float *cam2, float x1, float y1, float x2, float y2,
                                 const float *R12, const float *t12, float sigmaLevel, float unc)
{
    float p3D[3];
    return kb_triangulate_matches(cam1, cam2, x1, y1, x2, y2, R12, t12, sigmaLevel, unc, p3D) > 0.0001f;
}

/* exported for tests/test_oracle_triang.py: one KannalaBrandt8::epipolarConstrain evaluation */
int oracle_kb8_epipolar_constrain(const float *cam1, const float *cam2, float x1, float y1, float x2, float y2,
                                  const float *R12, const float *t12, float sigmaLevel, float unc)
{
    return kb_epipolar_constrain(cam1, cam2, x1, y1, x2, y2, R12, t12, sigmaLevel, unc);
}

/* Frame::ComputeStereoFishEyeMatches (ref:src/Frame.cc:1546-1603), serial: BFMatcher(NORM_HAMMING)
 * (ref:src/Frame.cc:47).knnMatch(k = 2) per left stereo row in query order (OpenCV's K-nearest insertion:
 * a distance equal to the first neighbour's becomes the second), Lowe's ratio (float * 0.7 in double),
 * TriangulateMatches(cam2, kpL, kpR, mRlr, mtlr, sigma2[octL], sigma2[octR]) > 0.0001f; later queries
 * overwrite mvRightToLeftMatch.  Unmatched mvStereo3Dpoints rows are 0 here (uninitialised in the reference). */
int oracle_stereo_fisheye_matches(int32_t n_left, int32_t mono_left, const uint8_t *dl, const float *kl,
                                  const int32_t *ol, int32_t n_right, int32_t mono_right, const uint8_t *dr,
                                  const float *kr, const int32_t *orr, const float *sig2, const float *caml,
                                  const float *camr, const float *Rlr, const float *tlr, int32_t *l2r, int32_t *r2l,
                                  float *depth, float *p3d)
{
    for (int i = 0; i < n_left; i++) {
        l2r[i] = -1;
        depth[i] = -1.0f;
        p3d[3 * i] = p3d[3 * i + 1] = p3d[3 * i + 2] = 0.f;
    }
    for (int j = 0; j < n_right; j++) r2l[j] = -1;
    int nMatches = 0;
    if (n_right - mono_right < 2) return 0; /* knnMatch returns < 2 neighbours: (*it).size() >= 2 fails */
    for (int i = mono_left; i < n_left; i++) {
        int b1 = 0x7fffffff, b2 = 0x7fffffff, j1 = -1;
        for (int j = mono_right; j < n_right; j++) {
            int d = 0;
            for (int k = 0; k < 32; k++) d += __builtin_popcount((unsigned)(dl[32 * i + k] ^ dr[32 * j + k]));
            if (d < b1) {
                b2 = b1;
                b1 = d;
                j1 = j;
            } else if (d < b2) {
                b2 = d;
            }
        }
        if (!((double)(float)b1 < (double)(float)b2 * 0.7)) continue;
        float x3[3];
        const float z = kb_triangulate_matches(caml, camr, kl[2 * i], kl[2 * i + 1], kr[2 * j1], kr[2 * j1 + 1], Rlr,
                                               tlr, sig2[ol[i]], sig2[orr[j1]], x3);
        if (z > 0.0001f) {
            l2r[i] = j1;
            r2l[j1] = i;
            for (int k = 0; k < 3; k++) p3d[3 * i + k] = x3[k];
            depth[i] = z;
            nMatches++;
        }
    }
    return nMatches;
}

void oracle_kb8_unproject(const float *cam, float u, float v, float *r) { kb_unproject(cam, u, v, r); }
void oracle_kb8_project(const float *cam, const float *X, float *uv) { kb_project(cam, X, uv); }

int oracle_search_for_triangulation(const osg_kf_side *K1, const osg_kf_side *K2, const osg_triang_geom *G,
                                    int bOnlyStereo, int bCoarse, int checkOri, int32_t *vMatches12)
{
    const osg_featvec *f1 = &K1->fv, *f2 = &K2->fv;
    int nmatches = 0;
    for (int i = 0; i < K1->n; i++) vMatches12[i] = -1;
    /* rotHist[bin] = list of idx1 (vector<int> rotHist[HISTO_LENGTH]) */
    int *hist = (int *)malloc(sizeof(int) * OSG_HISTO_LENGTH * (size_t)(K1->n > 0 ? K1->n : 1));
    int hn[OSG_HISTO_LENGTH] = {0};
    int a = 0, b = 0;
    while (a < f1->n_nodes && b < f2->n_nodes) {
        if (f1->node_id[a] == f2->node_id[b]) {
            for (int i1 = f1->node_start[a]; i1 < f1->node_start[a + 1]; i1++) {
                const int idx1 = f1->feat[i1];
                if (K1->has_mp[idx1]) continue;                                              /* :1129-1132 */
                const int bStereo1 = !K1->two_cam && K1->u_right && K1->u_right[idx1] >= 0;  /* :1135 */
                if (bOnlyStereo && !bStereo1) continue;
                const float kp1x = K1->kp_x[idx1], kp1y = K1->kp_y[idx1];
                const int bRight1 = !(K1->nleft == -1 || idx1 < K1->nleft);                  /* :1146-1147 */
                const uint8_t *d1 = K1->desc + 32 * (size_t)idx1;
                int bestDist = OSG_TH_LOW;
                int bestIdx2 = -1;
                for (int i2 = f2->node_start[b]; i2 < f2->node_start[b + 1]; i2++) {
                    const int idx2 = f2->feat[i2];
                    if (K2->has_mp[idx2]) continue;                                          /* :1165 */
                    const int bStereo2 = !K2->two_cam && K2->u_right && K2->u_right[idx2] >= 0;
                    if (bOnlyStereo && !bStereo2) continue;
                    const int dist = oracle_descriptor_distance(d1, K2->desc + 32 * (size_t)idx2);
                    if (dist > OSG_TH_LOW || dist > bestDist) continue;                      /* :1180 */
                    const float kp2x = K2->kp_x[idx2], kp2y = K2->kp_y[idx2];
                    const int oct2 = K2->kp_octave[idx2];
                    const int bRight2 = !(K2->nleft == -1 || idx2 < K2->nleft);
                    if (!bStereo1 && !bStereo2 && !K1->two_cam) {                            /* :1189-1203 */
                        const float distex = G->ep_x - kp2x;
                        const float distey = G->ep_y - kp2y;
                        if (distex * distex + distey * distey < 100 * K2->scale_factors[oct2]) continue;
                    }
                    int k = 0;                                                               /* :1205-1244 */
                    if (K1->two_cam && K2->two_cam) {
                        if (bRight1 && bRight2) k = 3;
                        else if (bRight1 && !bRight2) k = 2;
                        else if (!bRight1 && bRight2) k = 1;
                        else k = 0;
                    }
                    int ok = bCoarse;                                                        /* :1246 */
                    if (!ok && G->pinhole) ok = epipolar_constrain(G->F12[k], kp1x, kp1y, kp2x, kp2y, K2->level_sigma2[oct2]);
                    else if (!ok)  /* pCamera1 = bRight1 ? mpCamera2 : mpCamera of KF1, pCamera2 likewise of KF2 */
                        ok = kb_epipolar_constrain(G->kb[bRight1 ? 1 : 0], G->kb[bRight2 ? 3 : 2], kp1x, kp1y, kp2x,
                                                   kp2y, G->R12[k], G->t12[k], K1->level_sigma2[K1->kp_octave[idx1]],
                                                   K2->level_sigma2[oct2]);
                    if (ok) {
                        bestIdx2 = idx2;
                        bestDist = dist;
                    }
                }
                if (bestIdx2 >= 0) {                                                         /* :1252-1280 */
                    vMatches12[idx1] = bestIdx2;
                    nmatches++;
                    if (checkOri) {
                        const int bin = oracle_rot_bin(K1->kp_angle[idx1], K2->kp_angle[bestIdx2]);
                        hist[bin * (size_t)K1->n + hn[bin]++] = idx1;
                    }
                }
            }
            a++;
            b++;
        } else if (f1->node_id[a] < f2->node_id[b]) {
            a = lower_bound_u32(f1->node_id, a, f1->n_nodes, f2->node_id[b]);
        } else {
            b = lower_bound_u32(f2->node_id, b, f2->n_nodes, f1->node_id[a]);
        }
    }
    if (checkOri) {                                                                          /* :1297-1316 */
        int ind1 = -1, ind2 = -1, ind3 = -1;
        oracle_compute_three_maxima(hn, OSG_HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int i = 0; i < OSG_HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j = 0; j < hn[i]; j++) {
                vMatches12[hist[i * (size_t)K1->n + j]] = -1;
                nmatches--;
            }
        }
    }
    free(hist);
    return nmatches;
}
