/* oracle_stereo.c — CPU restatement of Frame::ComputeStereoMatches (ref:src/Frame.cc:1117-1373).
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, never linked into the product.
 * Literal: vRowIndices built by pushing every right keypoint onto rows floor(y - r) .. ceil(y + r)
 * (r = 2 mvScaleFactors[octave]); per left keypoint the candidates of row (size_t)vL in that
 * order, the octave +-1 and [minU, maxU] tests, the first minimum DescriptorDistance below TH_HIGH,
 * accepted below thOrbDist; the 11 x 11 SAD for incR = -5..5 (cv::norm NORM_L1, an integer held in
 * a float), the parabola fit, the disparity range test and the 0.01 clamp; then vDistIdx sorted as
 * pair<int,int>, the median vDistIdx[size / 2].first and the removal walk from the back.
 * Where the reference has undefined behaviour or throws, this restatement (and the GPU path)
 * defines it: rows outside [0, nRows) are not indexed (no push / no candidates), a SAD patch that
 * would leave the level image gives no match (cv::Mat::rowRange/colRange assert), and an empty
 * vDistIdx removes nothing.  Image levels are read through data[l] + row * step[l] (host memory). */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
    int dist, idx;
} dist_idx;

static int cmp_pair(const void *a, const void *b)  /* std::pair<int,int> operator< */
{
    const dist_idx *x = (const dist_idx *)a, *y = (const dist_idx *)b;
    if (x->dist != y->dist) return x->dist < y->dist ? -1 : 1;
    return (x->idx > y->idx) - (x->idx < y->idx);
}

static int sad_11x11(const osg_image_pyramid *PL, const osg_image_pyramid *PR, int level, int vL, int uL, int uR)
{
    const uint8_t *L = PL->data[level], *R = PR->data[level];
    const int sl = PL->step[level], sr = PR->step[level];
    int s = 0;
    for (int r = -5; r <= 5; r++)
        for (int c = -5; c <= 5; c++)
            s += abs((int)L[(size_t)(vL + r) * sl + (uL + c)] - (int)R[(size_t)(vL + r) * sr + (uR + c)]);
    return s;
}

int oracle_compute_stereo_matches(const osg_stereo_frame *F, float *mvuRight, float *mvDepth)
{
    const int N = F->n, Nr = F->n_right;
    for (int i = 0; i < N; i++) mvuRight[i] = mvDepth[i] = -1.0f;                /* :1134-1135 */
    if (N == 0) return 0;
    const int thOrbDist = (OSG_TH_HIGH + OSG_TH_LOW) / 2;                          /* :1138 */
    const int nRows = F->left.rows[0];                                             /* :1141 */
    /* vRowIndices (:1147-1170) as per-row counts + a second fill pass, push order = iR order */
    int *cnt = (int *)calloc((size_t)nRows + 1, sizeof(int));
    for (int iR = 0; iR < Nr; iR++) {
        const float kpY = F->yr[iR];
        const float r = 2.0f * F->scale_factors[F->octave_r[iR]];
        const int maxr = (int)ceil(kpY + r);
        const int minr = (int)floor(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) cnt[yi + 1]++;
    }
    for (int yi = 0; yi < nRows; yi++) cnt[yi + 1] += cnt[yi];
    int *rows = (int *)malloc(sizeof(int) * (size_t)(cnt[nRows] > 0 ? cnt[nRows] : 1));
    int *fill = (int *)malloc(sizeof(int) * (size_t)(nRows > 0 ? nRows : 1));
    memcpy(fill, cnt, sizeof(int) * (size_t)nRows);
    for (int iR = 0; iR < Nr; iR++) {
        const float kpY = F->yr[iR];
        const float r = 2.0f * F->scale_factors[F->octave_r[iR]];
        const int maxr = (int)ceil(kpY + r);
        const int minr = (int)floor(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) rows[fill[yi]++] = iR;
    }
    const float minZ = F->mb;                                                      /* :1178-1180 */
    const float minD = 0;
    const float maxD = F->mbf / minZ;
    dist_idx *vDistIdx = (dist_idx *)malloc(sizeof(dist_idx) * (size_t)N);
    int nDist = 0;
    for (int iL = 0; iL < N; iL++) {                                               /* :1188 */
        const int levelL = F->octave[iL];
        const float vL = F->y[iL];
        const float uL = F->x[iL];
        if (!(vL >= 0) || (int)vL >= nRows) continue;                              /* vRowIndices[vL] */
        const int row = (int)vL;
        const int c0 = cnt[row], c1 = cnt[row + 1];
        if (c1 == c0) continue;                                                    /* :1198-1199 */
        const float minU = uL - maxD;
        const float maxU = uL - minD;
        if (maxU < 0) continue;                                                    /* :1206-1207 */
        int bestDist = OSG_TH_HIGH;
        int bestIdxR = 0;
        const uint8_t *dL = F->desc + 32 * (size_t)iL;
        for (int iC = c0; iC < c1; iC++) {                                         /* :1217-1243 */
            const int iR = rows[iC];
            if (F->octave_r[iR] < levelL - 1 || F->octave_r[iR] > levelL + 1) continue;
            const float uR = F->xr[iR];
            if (uR >= minU && uR <= maxU) {
                const int dist = oracle_descriptor_distance(dL, F->desc_r + 32 * (size_t)iR);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = iR;
                }
            }
        }
        if (bestDist < thOrbDist) {                                                /* :1248 */
            const float uR0 = F->xr[bestIdxR];
            const float scaleFactor = F->inv_scale_factors[levelL];
            const float scaleduL = roundf(uL * scaleFactor);
            const float scaledvL = roundf(vL * scaleFactor);
            const float scaleduR0 = roundf(uR0 * scaleFactor);
            const int w = 5, L = 5;
            const float iniu = scaleduR0 + L - w;                                  /* :1280-1284 */
            const float endu = scaleduR0 + L + w + 1;
            if (iniu < 0 || endu >= F->right.cols[levelL]) continue;
            /* the patches of :1264 and :1290 must lie inside the level images */
            const int pu = (int)scaleduL, pv = (int)scaledvL, pr = (int)scaleduR0;
            if (pv - w < 0 || pv + w >= F->left.rows[levelL] || pv + w >= F->right.rows[levelL] || pu - w < 0 ||
                pu + w >= F->left.cols[levelL] || pr - L - w < 0 || pr + L + w >= F->right.cols[levelL])
                continue;
            int bestDistS = INT32_MAX;                                             /* :1267 (shadows) */
            int bestincR = 0;
            float vDists[11];
            for (int incR = -L; incR <= +L; incR++) {                              /* :1287-1303 */
                const float dist = (float)sad_11x11(&F->left, &F->right, levelL, pv, pu, pr + incR);
                if (dist < bestDistS) {
                    bestDistS = (int)dist;
                    bestincR = incR;
                }
                vDists[L + incR] = dist;
            }
            if (bestincR == -L || bestincR == L) continue;                         /* :1306-1307 */
            const float dist1 = vDists[L + bestincR - 1];                          /* :1320-1324 */
            const float dist2 = vDists[L + bestincR];
            const float dist3 = vDists[L + bestincR + 1];
            const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
            if (deltaR < -1 || deltaR > 1) continue;                               /* :1327-1328 */
            float bestuR = F->scale_factors[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
            float disparity = (uL - bestuR);
            if (disparity >= minD && disparity < maxD) {                           /* :1336-1351 */
                if (disparity <= 0) {
                    disparity = 0.01;
                    bestuR = uL - 0.01;
                }
                mvDepth[iL] = F->mbf / disparity;
                mvuRight[iL] = bestuR;
                vDistIdx[nDist].dist = bestDistS;
                vDistIdx[nDist].idx = iL;
                nDist++;
            }
        }
    }
    int nmatches = nDist;
    if (nDist > 0) {                                                               /* :1358-1372 */
        qsort(vDistIdx, (size_t)nDist, sizeof(dist_idx), cmp_pair);
        const float median = vDistIdx[nDist / 2].dist;
        const float thDist = 1.5f * 1.4f * median;
        for (int i = nDist - 1; i >= 0; i--) {
            if (vDistIdx[i].dist < thDist) break;
            mvuRight[vDistIdx[i].idx] = -1;
            mvDepth[vDistIdx[i].idx] = -1;
            nmatches--;
        }
    }
    free(cnt);
    free(rows);
    free(fill);
    free(vDistIdx);
    return nmatches;
}
