/* oracle_triang.c — CPU restatement of ORBmatcher::SearchForTriangulation.
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, never linked into the product.
 *
 *   ref:src/ORBmatcher.cc:1045-1328   the FeatureVector merge-walk, the per-pair tests, the
 *                                     rotation histogram and vMatchedPairs
 *   ref:src/CameraModels/Pinhole.cpp:189-219   epipolarConstrain
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
                    if (bCoarse || epipolar_constrain(G->F12[k], kp1x, kp1y, kp2x, kp2y,
                                                      K2->level_sigma2[oct2])) {             /* :1246 */
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
