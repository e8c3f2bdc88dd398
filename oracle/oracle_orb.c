/* oracle_orb.c — CPU restatement of ORBextractor's per-keypoint stages.
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, never linked into the product.
 *  * IC_Angle (ref:src/ORBextractor.cc:89-136): the intensity centroid over the circular patch of
 *    radius HALF_PATCH_SIZE = 15 bounded per row by umax, centred at (cvRound(pt.x), cvRound(pt.y)),
 *    m_10 / m_01 summed in the reference's loop order, then fastAtan2((float)m_01, (float)m_10).
 *  * computeOrbDescriptor (ref:src/ORBextractor.cc:148-208): angle * factorPI, a = cos, b = sin as
 *    std::cos(float) / std::sin(float) (libm cosf / sinf), the 32 x 8 pattern pairs at
 *    (cvRound(x a - y b), cvRound(x b + y a)) around the rounded centre, bit j of byte i =
 *    I(p[16 i + 2 j]) < I(p[16 i + 2 j + 1]).
 * cvRound is round-half-even (rintf).  fastAtan2 is OpenCV's cv::fastAtan2, which the reference
 * tree does not hold: its published polynomial (degrees, 4 odd terms, DBL_EPSILON guard) is
 * restated below; parity with OpenCV itself is unpinned.  The descriptor reads the blurred level as
 * the reference's continuous clone (workingMat, :1628): center[dy * step + dx] with step = cols, so a
 * point left of column 0 reads the previous row's end.  A read outside the whole blurred buffer
 * (the reference reads whatever heap lies there) is defined as 0 and counted per keypoint, as the GPU
 * path does; an orientation box leaving the level returns -(k + 1) for the first such keypoint k
 * (the GPU path's OSG_E_INVALID). */
#include <float.h>
#include <math.h>

#include "oracle.h"

#define HALF_PATCH_SIZE 15

float oracle_fast_atan2(float y, float x)
{
    const float r2d = (float)(180 / 3.1415926535897932384626433832795);
    const float p1 = 0.9997878412794807f * r2d, p3 = -0.3258083974640975f * r2d;
    const float p5 = 0.1555786518463281f * r2d, p7 = -0.04432655554792128f * r2d;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

static int inside(const osg_image_pyramid *P, int l, int x, int y)
{
    return x >= 0 && y >= 0 && x < P->cols[l] && y < P->rows[l];
}

int oracle_orb_describe(const osg_image_pyramid *raw, const osg_image_pyramid *blurred, const osg_orb_keypoints *K,
                        const int32_t *pattern, const int32_t *umax, int compute_angle, float *angle, uint8_t *desc)
{
    const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);   /* :139 */
    int n_outside = 0;
    for (int k = 0; k < K->n; k++) {
        const int l = K->level[k];
        const int cx = (int)rintf(K->x[k]), cy = (int)rintf(K->y[k]);
        if (compute_angle) {                                                      /* :89-136 */
            if (!inside(raw, l, cx - HALF_PATCH_SIZE, cy - HALF_PATCH_SIZE) ||
                !inside(raw, l, cx + HALF_PATCH_SIZE, cy + HALF_PATCH_SIZE))
                return -(k + 1);
            const uint8_t *center = raw->data[l] + (size_t)cy * raw->step[l] + cx;
            const int step = raw->step[l];
            int m_01 = 0, m_10 = 0;
            for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
            for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
                int v_sum = 0;
                const int d = umax[v];
                for (int u = -d; u <= d; ++u) {
                    const int val_plus = center[u + v * step], val_minus = center[u - v * step];
                    v_sum += (val_plus - val_minus);
                    m_10 += u * (val_plus + val_minus);
                }
                m_01 += v * v_sum;
            }
            angle[k] = oracle_fast_atan2((float)m_01, (float)m_10);
        }
        const float ang = angle[k] * factorPI;                                    /* :153-154 */
        const float a = cosf(ang), b = sinf(ang);
        const uint8_t *img = blurred->data[l];
        const int step = blurred->step[l], rows = blurred->rows[l], cols = blurred->cols[l];
        int outside = 0;
        for (int i = 0; i < 32; ++i) {                                            /* :166-205 */
            const int32_t *p = pattern + 32 * i;  /* 16 points of (x, y) */
            int val = 0;
            for (int j = 0; j < 8; ++j) {
                int t[2];
                for (int s = 0; s < 2; s++) {
                    const float px = (float)p[4 * j + 2 * s], py = (float)p[4 * j + 2 * s + 1];
                    const int dy = (int)rintf(px * b + py * a);
                    const int dx = (int)rintf(px * a - py * b);
                    /* workingMat is a continuous clone: the linear offset, wrapping across rows */
                    const long long off = (long long)(cy + dy) * cols + (cx + dx);
                    if (off < 0 || off >= (long long)rows * cols) {
                        outside = 1;
                        t[s] = 0;
                    } else {
                        t[s] = img[(size_t)(off / cols) * step + (size_t)(off % cols)];
                    }
                }
                val |= (t[0] < t[1]) << j;
            }
            desc[32 * k + i] = (uint8_t)val;
        }
        n_outside += outside;
    }
    return n_outside;
}
