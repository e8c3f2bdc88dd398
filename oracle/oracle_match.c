/*
 * oracle_match.c — CPU restatement of ORB-SLAM3's matching hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library, and only as the checker / the timed CPU baseline.  The product path
 * (liborbslam3_amd.so) never links or calls it.
 *
 * Each function is a line-by-line restatement of the cited reference loop, sequential and
 * single-threaded like the reference (ORBmatcher is serial).  Float expressions are evaluated
 * exactly as written in the reference with no FMA contraction (built with -ffp-contract=off).
 *
 * Parity pinning: the reference ships no tests or golden vectors for this path
 *  and cannot be built here (Eigen/OpenCV/Sophus absent).  The restatement
 * is pinned by hand-derived known-answer tests and an independent numpy implementation
 * (tests/test_oracle_*.py); committed fixtures under tests/golden/ are generated from it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/osg.h"
#include "oracle.h"

/* ref:src/ORBmatcher.cc:2388-2408 — SWAR popcount over 8 x int32. */
int oracle_descriptor_distance(const uint8_t *a, const uint8_t *b)
{
    const int32_t *pa = (const int32_t *)a;
    const int32_t *pb = (const int32_t *)b;
    int dist = 0;
    for (int i = 0; i < 8; i++, pa++, pb++) {
        unsigned int v = (unsigned int)(*pa ^ *pb);
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

/* Brute-force top-2 with the candidate-loop semantics of ref:src/ORBmatcher.cc:316-355. */
void oracle_hamming_top2(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *best_idx,
                         int32_t *best_dist, int32_t *second_dist)
{
    for (int i = 0; i < nq; i++) {
        int bestDist1 = 256, bestIdx = -1, bestDist2 = 256;
        const uint8_t *dq = q + (size_t)i * 32;
        for (int j = 0; j < nt; j++) {
            const int dist = oracle_descriptor_distance(dq, t + (size_t)j * 32);
            if (dist < bestDist1) {
                bestDist2 = bestDist1;
                bestDist1 = dist;
                bestIdx = j;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        best_idx[i] = bestIdx;
        best_dist[i] = bestDist1;
        second_dist[i] = bestDist2;
    }
}

/* Multi-threaded driver for the CPU baseline timing only: one contiguous query slice per
 * thread, each slice computed by the serial loop above (no change to per-query semantics). */
#include <pthread.h>
typedef struct {
    const uint8_t *q, *t;
    int q0, q1, nt;
    int32_t *bi, *bd, *sd;
} top2_job;
static void *top2_worker(void *p)
{
    top2_job *j = (top2_job *)p;
    oracle_hamming_top2(j->q + (size_t)j->q0 * 32, j->q1 - j->q0, j->t, j->nt, j->bi + j->q0,
                        j->bd + j->q0, j->sd + j->q0);
    return NULL;
}
void oracle_hamming_top2_mt(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *best_idx,
                            int32_t *best_dist, int32_t *second_dist, int nthreads)
{
    if (nthreads <= 1) {
        oracle_hamming_top2(q, nq, t, nt, best_idx, best_dist, second_dist);
        return;
    }
    pthread_t th[256];
    top2_job jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int k = 0; k < nthreads; k++) {
        jobs[k].q = q;
        jobs[k].t = t;
        jobs[k].nt = nt;
        jobs[k].q0 = (int)((long long)nq * k / nthreads);
        jobs[k].q1 = (int)((long long)nq * (k + 1) / nthreads);
        jobs[k].bi = best_idx;
        jobs[k].bd = best_dist;
        jobs[k].sd = second_dist;
        pthread_create(&th[k], NULL, top2_worker, &jobs[k]);
    }
    for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
}

/* ---- candidate generation -------------------------------------------------------------- */

/* ref:src/Frame.cc:868-962 (Frame::GetFeaturesInArea).  Writes candidate indices (relative to
 * the chosen camera) into out (capacity >= n); returns the count.  Enumeration order is the
 * reference's: ix outer, iy inner, cell insertion order. */
int oracle_frame_features_in_area(const osg_frame *F, float x, float y, float r, int minLevel,
                                  int maxLevel, int bRight, int32_t *out)
{
    int cnt = 0;
    const float factorX = r;
    const float factorY = r;
    int minCX = (int)floorf((x - F->min_x - factorX) * F->grid_inv_w);
    if (minCX < 0) minCX = 0;
    if (minCX >= OSG_GRID_COLS) return 0;
    int maxCX = (int)ceilf((x - F->min_x + factorX) * F->grid_inv_w);
    if (maxCX > OSG_GRID_COLS - 1) maxCX = OSG_GRID_COLS - 1;
    if (maxCX < 0) return 0;
    int minCY = (int)floorf((y - F->min_y - factorY) * F->grid_inv_h);
    if (minCY < 0) minCY = 0;
    if (minCY >= OSG_GRID_ROWS) return 0;
    int maxCY = (int)ceilf((y - F->min_y + factorY) * F->grid_inv_h);
    if (maxCY > OSG_GRID_ROWS - 1) maxCY = OSG_GRID_ROWS - 1;
    if (maxCY < 0) return 0;

    /* ref:src/Frame.cc:919 — quirk kept: (minLevel>0) || (maxLevel>=0) */
    const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    const int32_t *gs = bRight ? F->grid_start_r : F->grid_start;
    const int32_t *gi = bRight ? F->grid_idx_r : F->grid_idx;
    const int off = (bRight && F->nleft != -1) ? F->nleft : 0;

    for (int ix = minCX; ix <= maxCX; ix++) {
        for (int iy = minCY; iy <= maxCY; iy++) {
            const int cell = ix * OSG_GRID_ROWS + iy;
            for (int j = gs[cell]; j < gs[cell + 1]; j++) {
                const int idx = gi[j];
                const int k = idx + off;
                if (bCheckLevels) {
                    if (F->kp_octave[k] < minLevel) continue;
                    if (maxLevel >= 0)
                        if (F->kp_octave[k] > maxLevel) continue;
                }
                const float distx = F->kp_x[k] - x;
                const float disty = F->kp_y[k] - y;
                if (fabsf(distx) < factorX && fabsf(disty) < factorY) out[cnt++] = idx;
            }
        }
    }
    return cnt;
}

/* ref:src/ORBmatcher.cc:2341-2383 */
void oracle_compute_three_maxima(const int *histo_size, int L, int *ind1, int *ind2, int *ind3)
{
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = histo_size[i];
        if (s > max1) {
            max3 = max2;
            max2 = max1;
            max1 = s;
            *ind3 = *ind2;
            *ind2 = *ind1;
            *ind1 = i;
        } else if (s > max2) {
            max3 = max2;
            max2 = s;
            *ind3 = *ind2;
            *ind2 = i;
        } else if (s > max3) {
            max3 = s;
            *ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        *ind2 = -1;
        *ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        *ind3 = -1;
    }
}

/* rotation histogram: 30 growable int lists (vector<int> rotHist[HISTO_LENGTH]) */
typedef struct {
    int *v[OSG_HISTO_LENGTH];
    int n[OSG_HISTO_LENGTH];
    int cap[OSG_HISTO_LENGTH];
} rot_hist;

static void hist_init(rot_hist *h)
{
    for (int i = 0; i < OSG_HISTO_LENGTH; i++) {
        h->cap[i] = 64;
        h->n[i] = 0;
        h->v[i] = (int *)malloc(sizeof(int) * 64);
    }
}
static void hist_free(rot_hist *h)
{
    for (int i = 0; i < OSG_HISTO_LENGTH; i++) free(h->v[i]);
}
static void hist_push(rot_hist *h, int bin, int val)
{
    if (h->n[bin] == h->cap[bin]) {
        h->cap[bin] *= 2;
        h->v[bin] = (int *)realloc(h->v[bin], sizeof(int) * h->cap[bin]);
    }
    h->v[bin][h->n[bin]++] = val;
}
/* ref:src/ORBmatcher.cc:411-418 — factor = 1.0f/HISTO_LENGTH (the upstream bug, kept). */
int oracle_rot_bin(float angle_a, float angle_b)
{
    const float factor = 1.0f / OSG_HISTO_LENGTH;
    float rot = angle_a - angle_b;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == OSG_HISTO_LENGTH) bin = 0;
    return bin;
}
/* apply rotation consistency: null out slots in non-top-3 bins, return the number removed */
static int hist_apply(rot_hist *h, int32_t *slots)
{
    int ind1 = -1, ind2 = -1, ind3 = -1;
    oracle_compute_three_maxima(h->n, OSG_HISTO_LENGTH, &ind1, &ind2, &ind3);
    int removed = 0;
    for (int i = 0; i < OSG_HISTO_LENGTH; i++) {
        if (i == ind1 || i == ind2 || i == ind3) continue;
        for (int j = 0; j < h->n[i]; j++) {
            slots[h->v[i][j]] = -1;
            removed++;
        }
    }
    return removed;
}

/* slot "blocks matching" test: mvpMapPoints[i] && Observations() > 0 */
typedef struct {
    int32_t *slot_mp;
    uint8_t *taken; /* current taken state per slot */
} slot_state;

static float radius_by_viewing_cos(float viewCos)
{
    /* ref:src/ORBmatcher.cc:245-252 */
    if (viewCos > 0.998) return 2.5f;
    return 4.0f;
}

/* ---- a5: SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFar) ----- */
/* ref:src/ORBmatcher.cc:44-242 */
int oracle_search_by_projection_mps(const osg_frame *F, const osg_mp_queries *Q, float nnratio,
                                    float th, int bFarPoints, float thFarPoints, int32_t *slot_mp,
                                    const uint8_t *slot_taken_in)
{
    int nmatches = 0;
    const int bFactor = th != 1.0f;
    uint8_t *taken = (uint8_t *)malloc(F->n > 0 ? F->n : 1);
    memcpy(taken, slot_taken_in, F->n);
    int32_t *vIndices = (int32_t *)malloc(sizeof(int32_t) * (F->n > 0 ? F->n : 1));

    for (int iMP = 0; iMP < Q->n; iMP++) {
        const int inR = Q->in_view_r ? Q->in_view_r[iMP] : 0;
        if (!Q->in_view[iMP] && !inR) continue;
        if (bFarPoints && Q->track_depth[iMP] > thFarPoints) continue;
        if (!Q->usable[iMP]) continue;
        const uint8_t *MPdescriptor = Q->desc + (size_t)iMP * 32;
        const int mp = Q->mp_id[iMP];
        const uint8_t hobs = Q->has_obs[iMP];

        if (Q->in_view[iMP]) {
            const int nPredictedLevel = Q->pred_level[iMP];
            float r = radius_by_viewing_cos(Q->view_cos[iMP]);
            if (bFactor) r *= th;
            const int nc = oracle_frame_features_in_area(F, Q->proj_x[iMP], Q->proj_y[iMP],
                                                         r * F->scale_factors[nPredictedLevel],
                                                         nPredictedLevel - 1, nPredictedLevel, 0,
                                                         vIndices);
            if (nc > 0) {
                int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                for (int c = 0; c < nc; c++) {
                    const int idx = vIndices[c];
                    if (slot_mp[idx] >= 0 && taken[idx]) continue;
                    if (F->nleft == -1 && F->u_right && F->u_right[idx] > 0) {
                        const float er = fabsf(Q->proj_xr[iMP] - F->u_right[idx]);
                        if (er > r * F->scale_factors[nPredictedLevel]) continue;
                    }
                    const int dist = oracle_descriptor_distance(MPdescriptor, F->desc + (size_t)idx * 32);
                    if (dist < bestDist) {
                        bestDist2 = bestDist;
                        bestDist = dist;
                        bestLevel2 = bestLevel;
                        bestLevel = F->kp_octave[idx];
                        bestIdx = idx;
                    } else if (dist < bestDist2) {
                        bestLevel2 = F->kp_octave[idx];
                        bestDist2 = dist;
                    }
                }
                if (bestDist <= OSG_TH_HIGH) {
                    if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2)
                        continue; /* NB: skips the right-camera pass of this MapPoint too */
                    if (bestLevel != bestLevel2 || (float)bestDist <= nnratio * (float)bestDist2) {
                        slot_mp[bestIdx] = mp;
                        taken[bestIdx] = hobs;
                        if (F->nleft != -1 && F->left_to_right && F->left_to_right[bestIdx] != -1) {
                            const int s2 = F->left_to_right[bestIdx] + F->nleft;
                            slot_mp[s2] = mp;
                            taken[s2] = hobs;
                            nmatches++;
                        }
                        nmatches++;
                    }
                }
            }
        }

        if (F->nleft != -1 && inR) {
            const int nPredictedLevel = Q->pred_level_r[iMP];
            if (nPredictedLevel != -1) {
                float r = radius_by_viewing_cos(Q->view_cos_r[iMP]);
                const int nc = oracle_frame_features_in_area(F, Q->proj_xr[iMP], Q->proj_yr[iMP],
                                                             r * F->scale_factors[nPredictedLevel],
                                                             nPredictedLevel - 1, nPredictedLevel,
                                                             1, vIndices);
                if (nc == 0) continue;
                int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                for (int c = 0; c < nc; c++) {
                    const int idx = vIndices[c];
                    const int s = idx + F->nleft;
                    if (slot_mp[s] >= 0 && taken[s]) continue;
                    const int dist = oracle_descriptor_distance(MPdescriptor, F->desc + (size_t)s * 32);
                    if (dist < bestDist) {
                        bestDist2 = bestDist;
                        bestDist = dist;
                        bestLevel2 = bestLevel;
                        bestLevel = F->kp_octave[s];
                        bestIdx = idx;
                    } else if (dist < bestDist2) {
                        bestLevel2 = F->kp_octave[s];
                        bestDist2 = dist;
                    }
                }
                if (bestDist <= OSG_TH_HIGH) {
                    if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2)
                        continue;
                    if (F->right_to_left && F->right_to_left[bestIdx] != -1) {
                        const int s2 = F->right_to_left[bestIdx];
                        slot_mp[s2] = mp;
                        taken[s2] = hobs;
                        nmatches++;
                    }
                    slot_mp[bestIdx + F->nleft] = mp;
                    taken[bestIdx + F->nleft] = hobs;
                    nmatches++;
                }
            }
        }
    }
    free(vIndices);
    free(taken);
    return nmatches;
}

/* ---- a6: SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono) ------ */
/* ref:src/ORBmatcher.cc:1957-2191 */
int oracle_search_by_projection_last(const osg_frame *CF, const osg_last_queries *L, float th,
                                     int bMono, int checkOri, int32_t *slot_mp,
                                     const uint8_t *slot_taken_in)
{
    int nmatches = 0;
    rot_hist H;
    hist_init(&H);
    uint8_t *taken = (uint8_t *)malloc(CF->n > 0 ? CF->n : 1);
    memcpy(taken, slot_taken_in, CF->n);
    int32_t *vIndices2 = (int32_t *)malloc(sizeof(int32_t) * (CF->n > 0 ? CF->n : 1));

    const int bForward = L->tlc_z > CF->mb && !bMono;
    const int bBackward = -L->tlc_z > CF->mb && !bMono;

    for (int i = 0; i < L->n; i++) {
        if (!L->valid[i]) continue;
        const float invzc = L->invz[i];
        if (invzc < 0) continue;
        const float u = L->u[i], v = L->v[i];
        if (u < CF->min_x || u > CF->max_x) continue;
        if (v < CF->min_y || v > CF->max_y) continue;
        const int nLastOctave = L->octave[i];
        const float radius = th * CF->scale_factors[nLastOctave];
        int nc;
        if (bForward)
            nc = oracle_frame_features_in_area(CF, u, v, radius, nLastOctave, -1, 0, vIndices2);
        else if (bBackward)
            nc = oracle_frame_features_in_area(CF, u, v, radius, 0, nLastOctave, 0, vIndices2);
        else
            nc = oracle_frame_features_in_area(CF, u, v, radius, nLastOctave - 1, nLastOctave + 1, 0,
                                               vIndices2);
        if (nc == 0) continue;
        const uint8_t *dMP = L->desc + (size_t)i * 32;
        const int mp = L->mp_id[i];
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = vIndices2[c];
            if (slot_mp[i2] >= 0 && taken[i2]) continue;
            if (CF->nleft == -1 && CF->u_right && CF->u_right[i2] > 0) {
                const float ur = u - CF->mbf * invzc;
                const float er = fabsf(ur - CF->u_right[i2]);
                if (er > radius) continue;
            }
            const int dist = oracle_descriptor_distance(dMP, CF->desc + (size_t)i2 * 32);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= OSG_TH_HIGH) {
            slot_mp[bestIdx2] = mp;
            taken[bestIdx2] = L->has_obs[i];
            nmatches++;
            if (checkOri) hist_push(&H, oracle_rot_bin(L->angle[i], CF->kp_angle[bestIdx2]), bestIdx2);
        }
        if (CF->nleft != -1) {
            const float ur_ = L->u_r[i], vr_ = L->v_r[i];
            int ncr;
            if (bForward)
                ncr = oracle_frame_features_in_area(CF, ur_, vr_, radius, nLastOctave, -1, 1, vIndices2);
            else if (bBackward)
                ncr = oracle_frame_features_in_area(CF, ur_, vr_, radius, 0, nLastOctave, 1, vIndices2);
            else
                ncr = oracle_frame_features_in_area(CF, ur_, vr_, radius, nLastOctave - 1,
                                                    nLastOctave + 1, 1, vIndices2);
            int bestDistR = 256, bestIdxR = -1;
            for (int c = 0; c < ncr; c++) {
                const int i2 = vIndices2[c];
                const int s = i2 + CF->nleft;
                if (slot_mp[s] >= 0 && taken[s]) continue;
                const int dist = oracle_descriptor_distance(dMP, CF->desc + (size_t)s * 32);
                if (dist < bestDistR) {
                    bestDistR = dist;
                    bestIdxR = i2;
                }
            }
            if (bestDistR <= OSG_TH_HIGH) {
                const int s = bestIdxR + CF->nleft;
                slot_mp[s] = mp;
                taken[s] = L->has_obs[i];
                nmatches++;
                if (checkOri) hist_push(&H, oracle_rot_bin(L->angle[i], CF->kp_angle[s]), s);
            }
        }
    }
    if (checkOri) nmatches -= hist_apply(&H, slot_mp);
    hist_free(&H);
    free(vIndices2);
    free(taken);
    return nmatches;
}

/* ---- a7: SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist) ------- */
/* ref:src/ORBmatcher.cc:2203-2330 */
int oracle_search_by_projection_kf(const osg_frame *CF, const osg_kf_queries *K, float th,
                                   int ORBdist, int checkOri, int32_t *slot_mp)
{
    int nmatches = 0;
    rot_hist H;
    hist_init(&H);
    int32_t *vIndices2 = (int32_t *)malloc(sizeof(int32_t) * (CF->n > 0 ? CF->n : 1));
    for (int i = 0; i < K->n; i++) {
        if (!K->valid[i]) continue;
        const int lvl = K->pred_level[i];
        const float radius = th * CF->scale_factors[lvl];
        const int nc = oracle_frame_features_in_area(CF, K->u[i], K->v[i], radius, lvl - 1, lvl + 1, 0,
                                                     vIndices2);
        if (nc == 0) continue;
        const uint8_t *dMP = K->desc + (size_t)i * 32;
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = vIndices2[c];
            if (slot_mp[i2] >= 0) continue;
            const int dist = oracle_descriptor_distance(dMP, CF->desc + (size_t)i2 * 32);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= ORBdist) {
            slot_mp[bestIdx2] = K->mp_id[i];
            nmatches++;
            if (checkOri) hist_push(&H, oracle_rot_bin(K->angle[i], CF->kp_angle[bestIdx2]), bestIdx2);
        }
    }
    if (checkOri) nmatches -= hist_apply(&H, slot_mp);
    hist_free(&H);
    free(vIndices2);
    return nmatches;
}

/* lower_bound over the ascending node ids of a FeatureVector */
static int fv_lower_bound(const osg_featvec *fv, int from, uint32_t key)
{
    int lo = from, hi = fv->n_nodes;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (fv->node_id[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/* ---- a3: SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) ----------------------------- */
/* ref:src/ORBmatcher.cc:262-496 */
int oracle_search_by_bow_kf_f(const osg_bow_side *KF, const osg_bow_side *F, float nnratio,
                              int checkOri, int32_t *out_mp)
{
    for (int i = 0; i < F->n; i++) out_mp[i] = -1;
    int nmatches = 0;
    rot_hist H;
    hist_init(&H);
    int KFit = 0, Fit = 0;
    const int KFend = KF->fv.n_nodes, Fend = F->fv.n_nodes;
    while (KFit != KFend && Fit != Fend) {
        if (KF->fv.node_id[KFit] == F->fv.node_id[Fit]) {
            for (int a = KF->fv.node_start[KFit]; a < KF->fv.node_start[KFit + 1]; a++) {
                const int realIdxKF = KF->fv.feat[a];
                if (!KF->mp_good[realIdxKF]) continue;
                const int mp = KF->mp_id[realIdxKF];
                const uint8_t *dKF = KF->desc + (size_t)realIdxKF * 32;
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                int bestDist1R = 256, bestIdxFR = -1, bestDist2R = 256;
                for (int b = F->fv.node_start[Fit]; b < F->fv.node_start[Fit + 1]; b++) {
                    const int realIdxF = F->fv.feat[b];
                    if (out_mp[realIdxF] >= 0) continue;
                    const int dist = oracle_descriptor_distance(dKF, F->desc + (size_t)realIdxF * 32);
                    if (F->nleft == -1) {
                        if (dist < bestDist1) {
                            bestDist2 = bestDist1;
                            bestDist1 = dist;
                            bestIdxF = realIdxF;
                        } else if (dist < bestDist2) {
                            bestDist2 = dist;
                        }
                    } else {
                        if (realIdxF < F->nleft && dist < bestDist1) {
                            bestDist2 = bestDist1;
                            bestDist1 = dist;
                            bestIdxF = realIdxF;
                        } else if (realIdxF < F->nleft && dist < bestDist2) {
                            bestDist2 = dist;
                        }
                        if (realIdxF >= F->nleft && dist < bestDist1R) {
                            bestDist2R = bestDist1R;
                            bestDist1R = dist;
                            bestIdxFR = realIdxF;
                        } else if (realIdxF >= F->nleft && dist < bestDist2R) {
                            bestDist2R = dist;
                        }
                    }
                }
                if (bestDist1 <= OSG_TH_LOW) {
                    if ((float)bestDist1 < nnratio * (float)bestDist2) {
                        out_mp[bestIdxF] = mp;
                        if (checkOri)
                            hist_push(&H, oracle_rot_bin(KF->angle[realIdxKF], F->angle[bestIdxF]), bestIdxF);
                        nmatches++;
                    }
                    if (bestDist1R <= OSG_TH_LOW) {
                        /* ratio disabled by '|| true' (ref:src/ORBmatcher.cc:425) */
                        out_mp[bestIdxFR] = mp;
                        if (checkOri)
                            hist_push(&H, oracle_rot_bin(KF->angle[realIdxKF], F->angle[bestIdxFR]), bestIdxFR);
                        nmatches++;
                    }
                }
            }
            KFit++;
            Fit++;
        } else if (KF->fv.node_id[KFit] < F->fv.node_id[Fit]) {
            KFit = fv_lower_bound(&KF->fv, KFit, F->fv.node_id[Fit]);
        } else {
            Fit = fv_lower_bound(&F->fv, Fit, KF->fv.node_id[KFit]);
        }
    }
    if (checkOri) nmatches -= hist_apply(&H, out_mp);
    hist_free(&H);
    return nmatches;
}

/* ---- a4: SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&) -------------------------- */
/* ref:src/ORBmatcher.cc:890-1043.  Two-camera keyframes skip idx >= mvKeysUn.size()
 * (ref:src/ORBmatcher.cc:934-936,953-955).  For a two-camera rig mvKeysUn = mvKeys holds the left
 * keypoints only (ref:src/Frame.cc:1022,1485), so mvKeysUn.size() == NLeft; the FeatureVector
 * (built on the vconcat'ed descriptors) can hold indices up to N. */
int oracle_search_by_bow_kf_kf(const osg_bow_side *K1, const osg_bow_side *K2, float nnratio,
                               int checkOri, int32_t *out_mp12)
{
    for (int i = 0; i < K1->n; i++) out_mp12[i] = -1;
    uint8_t *vbMatched2 = (uint8_t *)calloc(K2->n > 0 ? K2->n : 1, 1);
    int nmatches = 0;
    rot_hist H;
    hist_init(&H);
    int f1 = 0, f2 = 0;
    const int f1end = K1->fv.n_nodes, f2end = K2->fv.n_nodes;
    while (f1 != f1end && f2 != f2end) {
        if (K1->fv.node_id[f1] == K2->fv.node_id[f2]) {
            for (int a = K1->fv.node_start[f1]; a < K1->fv.node_start[f1 + 1]; a++) {
                const int idx1 = K1->fv.feat[a];
                if (K1->nleft != -1 && idx1 >= K1->nleft) continue;
                if (!K1->mp_good[idx1]) continue;
                const uint8_t *d1 = K1->desc + (size_t)idx1 * 32;
                int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
                for (int b = K2->fv.node_start[f2]; b < K2->fv.node_start[f2 + 1]; b++) {
                    const int idx2 = K2->fv.feat[b];
                    if (K2->nleft != -1 && idx2 >= K2->nleft) continue;
                    if (vbMatched2[idx2] || K2->mp_id[idx2] < 0) continue;
                    if (!K2->mp_good[idx2]) continue;
                    const int dist = oracle_descriptor_distance(d1, K2->desc + (size_t)idx2 * 32);
                    if (dist < bestDist1) {
                        bestDist2 = bestDist1;
                        bestDist1 = dist;
                        bestIdx2 = idx2;
                    } else if (dist < bestDist2) {
                        bestDist2 = dist;
                    }
                }
                if (bestDist1 < OSG_TH_LOW) {
                    if ((float)bestDist1 < nnratio * (float)bestDist2) {
                        out_mp12[idx1] = K2->mp_id[bestIdx2];
                        vbMatched2[bestIdx2] = 1;
                        if (checkOri)
                            hist_push(&H, oracle_rot_bin(K1->angle[idx1], K2->angle[bestIdx2]), idx1);
                        nmatches++;
                    }
                }
            }
            f1++;
            f2++;
        } else if (K1->fv.node_id[f1] < K2->fv.node_id[f2]) {
            f1 = fv_lower_bound(&K1->fv, f1, K2->fv.node_id[f2]);
        } else {
            f2 = fv_lower_bound(&K2->fv, f2, K1->fv.node_id[f1]);
        }
    }
    if (checkOri) nmatches -= hist_apply(&H, out_mp12);
    hist_free(&H);
    free(vbMatched2);
    return nmatches;
}
