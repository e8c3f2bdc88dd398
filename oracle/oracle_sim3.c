/* oracle_sim3.c — CPU restatement of the Sim3 projection matchers of LoopClosing.
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, never linked into the product.
 *
 *   SearchByProjection(KeyFrame*, Sim3f&, vpPoints, vpMatched, th, ratioHamming)   ref:src/ORBmatcher.cc:498-621
 *   SearchByProjection(KeyFrame*, Sim3f&, vpPoints, vpPointsKFs, ...)              ref:src/ORBmatcher.cc:623-733
 * The caller's pre-search part (bad / already found / depth / image / distance / angle, the
 * projection and PredictScale) arrives folded into the queries (osg.h).  The loop body from
 * GetFeaturesInArea on is literal: vpMatched is written as soon as a MapPoint is accepted. */
#include <stdlib.h>

#include "oracle.h"

int oracle_search_by_projection_sim3(const osg_frame *KF, const osg_fuse_queries *Q, float th, float ratioHamming,
                                     int32_t *slot_query)
{
    int nmatches = 0;
    int32_t *vIndices = (int32_t *)malloc(sizeof(int32_t) * (size_t)(KF->n > 0 ? KF->n : 1));
    for (int iMP = 0; iMP < Q->n; iMP++) {
        if (!Q->valid[iMP]) continue;
        const int nPredictedLevel = Q->pred_level[iMP];
        const float radius = th * KF->scale_factors[nPredictedLevel];                            /* :574 */
        const int nc = oracle_frame_features_in_area(KF, Q->u[iMP], Q->v[iMP], radius, -1, -1, 0, vIndices);
        if (nc == 0) continue;
        const uint8_t *dMP = Q->desc + 32 * (size_t)iMP;
        int bestDist = 256, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int idx = vIndices[c];
            if (slot_query[idx] != -1) continue;                                                  /* vpMatched[idx] */
            const int kpLevel = KF->kp_octave[idx];
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            const int dist = oracle_descriptor_distance(dMP, KF->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        if (bestDist <= OSG_TH_LOW * ratioHamming) {                                             /* :612 */
            slot_query[bestIdx] = iMP;
            nmatches++;
        }
    }
    free(vIndices);
    return nmatches;
}
