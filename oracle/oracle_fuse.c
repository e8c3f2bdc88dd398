/* oracle_fuse.c — CPU restatement of the search half of ORBmatcher::Fuse (both overloads).
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, never linked into the product.
 *
 *   gated = 1  Fuse(KeyFrame*, vector<MapPoint*>, th, bRight)   ref:src/ORBmatcher.cc:1330-1541
 *   gated = 0  Fuse(KeyFrame*, Sim3f, vector<MapPoint*>, th, …)  ref:src/ORBmatcher.cc:1553-1694
 *   area       KeyFrame::GetFeaturesInArea                        ref:src/KeyFrame.cc:859-907
 *              (= Frame::GetFeaturesInArea without the level test)
 * The pre-search filters and the projection are the caller's (osg.h); the replace / add step is
 * the caller's too. */
#include <stdlib.h>

#include "oracle.h"

int oracle_fuse_search(const osg_frame *KF, const osg_fuse_queries *Q, float th, int right, int gated,
                       int32_t *best_idx, int32_t *best_dist)
{
    int nfused = 0;
    int32_t *vIndices = (int32_t *)malloc(sizeof(int32_t) * (size_t)(KF->n > 0 ? KF->n : 1));
    const int off = (right && KF->nleft != -1) ? KF->nleft : 0;
    for (int i = 0; i < Q->n; i++) {
        best_idx[i] = -1;
        best_dist[i] = 256;
        if (!Q->valid[i]) continue;
        const int nPredictedLevel = Q->pred_level[i];
        const float radius = th * KF->scale_factors[nPredictedLevel];                      /* :1437, :1626 */
        const float u = Q->u[i], v = Q->v[i];
        const int nc = oracle_frame_features_in_area(KF, u, v, radius, -1, -1, right, vIndices); /* :1439, :1629 */
        if (nc == 0) continue;
        const uint8_t *dMP = Q->desc + 32 * (size_t)i;
        int bestDist = gated ? 256 : 0x7FFFFFFF; /* :1451 / :1638 */
        int bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            int idx = vIndices[c];
            const int k = idx + off;                       /* mvKeysUn / mvKeys / mvKeysRight[idx] */
            const int kpLevel = KF->kp_octave[k];
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue; /* :1462, :1645 */
            if (gated) {
                const float kpx = KF->kp_x[k], kpy = KF->kp_y[k];
                if (KF->u_right && KF->u_right[idx] >= 0) { /* :1466, mvuRight[idx] before the NLeft offset */
                    const float kpr = KF->u_right[idx];
                    const float ex = u - kpx;
                    const float ey = v - kpy;
                    const float er = Q->ur[i] - kpr;
                    const float e2 = ex * ex + ey * ey + er * er;
                    if ((double)(e2 * Q->inv_level_sigma2[kpLevel]) > 7.8) continue; /* :1480 */
                } else {
                    const float ex = u - kpx;
                    const float ey = v - kpy;
                    const float e2 = ex * ex + ey * ey;
                    if ((double)(e2 * Q->inv_level_sigma2[kpLevel]) > 5.99) continue; /* :1493 */
                }
            }
            idx = k;                                       /* :1498 idx += NLeft */
            const int dist = oracle_descriptor_distance(dMP, KF->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        best_dist[i] = bestDist < 256 ? bestDist : 256;
        if (bestDist <= OSG_TH_LOW) { /* :1514, :1661 */
            best_idx[i] = bestIdx;
            nfused++;
        }
    }
    free(vIndices);
    return nfused;
}
