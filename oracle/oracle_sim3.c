/* oracle_sim3.c — CPU restatement of the Sim3 projection matchers of LoopClosing.
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, never linked into the product.
 *
 *   SearchByProjection(KeyFrame*, Sim3f&, vpPoints, vpMatched, th, ratioHamming)   ref:src/ORBmatcher.cc:498-621
 *   SearchByProjection(KeyFrame*, Sim3f&, vpPoints, vpPointsKFs, ...)              ref:src/ORBmatcher.cc:623-733
 * The caller's pre-search part (bad / already found / depth / image / distance / angle, the
 * projection and PredictScale) arrives folded into the queries (osg.h).  The loop body from
 * GetFeaturesInArea on is literal: vpMatched is written as soon as a MapPoint is accepted.
 *   SearchBySim3(KeyFrame*, KeyFrame*, vpMatches12, S12, th)                      ref:src/ORBmatcher.cc:1696-1939 */
#include <limits.h>
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

/* ORBmatcher::SearchBySim3 (ref:src/ORBmatcher.cc:1696-1939) with the projections and pre-search
 * filters of both directions folded into q12 / q21 by the caller (one query per keypoint of KF1 /
 * KF2, see include/osg.h): for each query in order, KeyFrame::GetFeaturesInArea on the other
 * KeyFrame, levels [pred - 1, pred], strict '<' minimum from INT_MAX (:1781-1800), accepted iff
 * bestDist <= TH_HIGH (:1802-1805); then the mutual check in KF1 order (:1920-1936). */
static void sim3_direction(const osg_frame *KF, const osg_fuse_queries *Q, float th, int32_t *vnMatch)
{
    int32_t *vIndices = (int32_t *)malloc(sizeof(int32_t) * (size_t)(KF->n > 0 ? KF->n : 1));
    for (int i = 0; i < Q->n; i++) {
        vnMatch[i] = -1;
        if (!Q->valid[i]) continue;
        const int nPredictedLevel = Q->pred_level[i];
        const float radius = th * KF->scale_factors[nPredictedLevel];                 /* :1777 / :1857 */
        const int nc = oracle_frame_features_in_area(KF, Q->u[i], Q->v[i], radius, -1, -1, 0, vIndices);
        if (nc == 0) continue;
        const uint8_t *dMP = Q->desc + 32 * (size_t)i;
        int bestDist = INT_MAX, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int idx = vIndices[c];
            const int kpLevel = KF->kp_octave[idx];
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            const int dist = oracle_descriptor_distance(dMP, KF->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        if (bestDist <= OSG_TH_HIGH) vnMatch[i] = bestIdx;
    }
    free(vIndices);
}

int oracle_search_by_sim3(const osg_frame *KF1, const osg_frame *KF2, const osg_fuse_queries *Q12,
                          const osg_fuse_queries *Q21, float th, int32_t *match12)
{
    int32_t *vnMatch1 = (int32_t *)malloc(sizeof(int32_t) * (size_t)(Q12->n > 0 ? Q12->n : 1));
    int32_t *vnMatch2 = (int32_t *)malloc(sizeof(int32_t) * (size_t)(Q21->n > 0 ? Q21->n : 1));
    sim3_direction(KF2, Q12, th, vnMatch1);
    sim3_direction(KF1, Q21, th, vnMatch2);
    int nFound = 0;
    for (int i1 = 0; i1 < Q12->n; i1++) {
        const int idx2 = vnMatch1[i1];
        match12[i1] = -1;
        if (idx2 >= 0 && vnMatch2[idx2] == i1) {
            match12[i1] = idx2;
            nFound++;
        }
    }
    free(vnMatch1);
    free(vnMatch2);
    return nFound;
}
