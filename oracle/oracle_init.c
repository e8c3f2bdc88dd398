/* oracle_init.c — CPU restatement of ORBmatcher::SearchForInitialization (ref:src/ORBmatcher.cc:735-878).
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, never linked into the product.
 * Literal: F1 keypoints in order, level 0 only, Frame::GetFeaturesInArea(prev, windowSize, 0, 0),
 * the vMatchedDistance skip, top-2 with INT_MAX sentinels, the ratio test against
 * (float)bestDist2 * nnratio, the vnMatches21 steal, rotHist lists holding every accepted event,
 * ComputeThreeMaxima and the final vbPrevMatched update. */
#include <limits.h>
#include <stdlib.h>

#include "oracle.h"

int oracle_search_for_initialization(const osg_frame *F1, const osg_frame *F2, float *prev_xy, int windowSize,
                                     float mfNNratio, int checkOri, int32_t *vnMatches12)
{
    int nmatches = 0;
    const int n1 = F1->n, n2 = F2->n;
    int *vMatchedDistance = (int *)malloc(sizeof(int) * (size_t)(n2 > 0 ? n2 : 1));
    int *vnMatches21 = (int *)malloc(sizeof(int) * (size_t)(n2 > 0 ? n2 : 1));
    int32_t *vIndices2 = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n2 > 0 ? n2 : 1));
    int *hist = (int *)malloc(sizeof(int) * OSG_HISTO_LENGTH * (size_t)(n1 > 0 ? n1 : 1));
    int hn[OSG_HISTO_LENGTH] = {0};
    for (int i = 0; i < n1; i++) vnMatches12[i] = -1;
    for (int i = 0; i < n2; i++) {
        vMatchedDistance[i] = INT_MAX;
        vnMatches21[i] = -1;
    }
    for (int i1 = 0; i1 < n1; i1++) {
        const int level1 = F1->kp_octave[i1];
        if (level1 > 0) continue;                                                          /* :760-762 */
        const int nc = oracle_frame_features_in_area(F2, prev_xy[2 * i1], prev_xy[2 * i1 + 1], (float)windowSize,
                                                     level1, level1, 0, vIndices2);       /* :764 */
        if (nc == 0) continue;
        const uint8_t *d1 = F1->desc + 32 * (size_t)i1;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = vIndices2[c];
            const int dist = oracle_descriptor_distance(d1, F2->desc + 32 * (size_t)i2);
            if (vMatchedDistance[i2] <= dist) continue;                                    /* :781-782 */
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= OSG_TH_LOW) {                                                      /* :794 */
            if (bestDist < (float)bestDist2 * mfNNratio) {
                if (vnMatches21[bestIdx2] >= 0) {                                          /* :798-802 */
                    vnMatches12[vnMatches21[bestIdx2]] = -1;
                    nmatches--;
                }
                vnMatches12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (checkOri) {
                    const int bin = oracle_rot_bin(F1->kp_angle[i1], F2->kp_angle[bestIdx2]);
                    hist[bin * (size_t)n1 + hn[bin]++] = i1;
                }
            }
        }
    }
    if (checkOri) {                                                                        /* :843-866 */
        int ind1 = -1, ind2 = -1, ind3 = -1;
        oracle_compute_three_maxima(hn, OSG_HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int i = 0; i < OSG_HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j = 0; j < hn[i]; j++) {
                const int idx1 = hist[i * (size_t)n1 + j];
                if (vnMatches12[idx1] >= 0) {
                    vnMatches12[idx1] = -1;
                    nmatches--;
                }
            }
        }
    }
    for (int i1 = 0; i1 < n1; i1++)                                                        /* :869-871 */
        if (vnMatches12[i1] >= 0) {
            prev_xy[2 * i1] = F2->kp_x[vnMatches12[i1]];
            prev_xy[2 * i1 + 1] = F2->kp_y[vnMatches12[i1]];
        }
    free(vMatchedDistance);
    free(vnMatches21);
    free(vIndices2);
    free(hist);
    return nmatches;
}
