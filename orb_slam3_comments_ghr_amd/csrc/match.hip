// match.hip — the ORBmatcher search operators on gfx950.
//
//   osg_search_by_projection_mps   ← ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th, far, thFar)   ref:src/ORBmatcher.cc:44-242
//   osg_search_by_projection_last  ← ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)             ref:src/ORBmatcher.cc:1957-2191
//   osg_search_by_projection_kf    ← ORBmatcher::SearchByProjection(Frame&, KeyFrame*, set<MapPoint*>, th, dist)  ref:src/ORBmatcher.cc:2203-2330
//   osg_search_by_bow_kf_f         ← ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)             ref:src/ORBmatcher.cc:262-496
//   osg_search_by_bow_kf_kf        ← ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)          ref:src/ORBmatcher.cc:890-1043
//
// Every one of these is "for each query (map point / keyframe feature) in order: candidates from a
// grid window or a vocabulary node, skip slots already taken, top-2 by DescriptorDistance, accept
// by threshold (+ratio), take the slot", followed by the rotation-histogram filter.  The take is
// an order-dependent greedy: an accepted query removes its slot from every LATER query's
// candidate set.  One workgroup (1024 threads) per problem runs:
//
//   1. count   — each thread enumerates the windows of a contiguous run of queries exactly as
//                Frame::GetFeaturesInArea does (ix outer, iy inner, cell order; same float
//                arithmetic, no FMA contraction) and counts candidates that pass the static
//                filters (levels, window, stereo u_R check);
//   2. scan    — block prefix sum → candidate CSR offsets;
//   3. fill    — second enumeration writes {slot | dist << 16 | octave << 25} per candidate;
//                the 256-bit distance is 8 x (v_xor + v_bcnt) on the query held in VGPRs;
//   4. resolve — Jacobi fixed point of the greedy:  r_q = f_q({slots taken by accepted p < q}).
//                Round k recomputes every r_q from the claims (LDS atomicMin of the query index
//                per slot) of round k-1.  After round k queries 0..k-1 are final, and a round with
//                no change is the unique fixed point = the sequential result (proof by induction
//                on q), so the answer is bit-exact while all queries are evaluated in parallel;
//   5. finish  — last assignment per slot, rotation histogram with the reference's 1/30 factor,
//                ComputeThreeMaxima, removal, nmatches.
#include <algorithm>

#include "match_common.h"

namespace {

enum { MODE_MPS = 0, MODE_LAST = 1, MODE_KF = 2, MODE_BOW_KF_F = 3, MODE_BOW_KF_KF = 4 };

constexpr int MT = 1024;               // threads per problem
constexpr int MAX_SLOTS = 8192;        // LDS claim arrays
constexpr int INT_BIG = 0x7FFFFFFF;

struct MatchArgs {
    int nq, n_slots;
    int nleft;                // slot side: Frame::Nleft (-1: one camera / rectified stereo)
    // slot side (Frame F / KeyFrame 2)
    const uint32_t *fdesc;
    const float *kp_x, *kp_y, *slot_angle;
    const int32_t *kp_octave;
    const float *u_right;     // NULL for a two-camera rig (the u_R check needs Nleft == -1)
    const int32_t *grid_start, *grid_idx;
    const int32_t *grid_start_r, *grid_idx_r;   // mGridRight, indices relative to nleft
    const int32_t *l2r, *r2l;                    // mvLeftToRightMatch / mvRightToLeftMatch
    float min_x, max_x, min_y, max_y, inv_w, inv_h;
    const float *scale;
    float mb, mbf;
    // queries
    const uint32_t *qdesc;
    const int32_t *q_mp;
    const uint8_t *q_has_obs;
    const float *q_angle;
    const float *q_x, *q_y, *q_f0, *q_f1, *q_f2;
    const int32_t *q_lvl;
    const uint8_t *q_m0, *q_m1;
    // right-camera query fields (two-camera rig)
    const float *q_xr, *q_yr, *q_f0r;
    const int32_t *q_lvl_r;
    const uint8_t *q_m0r;
    const int32_t *q_cb, *q_ce, *cand_list;
    const uint8_t *slot_ok;
    const int32_t *slot_mp2;  // KF-KF: KF2 MapPoint ids
    // parameters
    float nnratio, th, th_far, tlc_z;
    int far_points, orb_dist, check_ori, mono;
    // state / outputs
    int32_t *slot_mp;         // in/out (out_mp for KF-F)
    const uint8_t *slot_taken;
    int32_t *out_q;           // KF-KF: per query result
    // scratch
    int32_t *q_off;           // nq + 1: candidate CSR
    int32_t *q_mid;           // nq: first right-camera candidate of each query
    uint32_t *cands;
    int32_t *q_res;           // 2 nq: {left slot, right slot}, -1 = no match
    uint8_t *q_bin;           // 2 nq
    int32_t *status;          // [0] candidates, [1] nmatches, [2] rounds, [3] overflow, [4] serial
    int cap;
};

struct Win {
    float x, y, r;
    int minL, maxL;
    float sx, sr;
    bool valid, stereo;
};

// result of one query: the slot matched by the left (or only) camera pass and by the right pass
struct QRes {
    int l, r;
};

__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

__device__ __forceinline__ uint32_t dist256(const uint32_t (&a)[8], const uint32_t *__restrict__ b)
{
    const uint4 b0 = *(const uint4 *)b, b1 = *(const uint4 *)(b + 4);
    uint32_t d = __popc(a[0] ^ b0.x);
    d = bcnt_acc(a[1] ^ b0.y, d);
    d = bcnt_acc(a[2] ^ b0.z, d);
    d = bcnt_acc(a[3] ^ b0.w, d);
    d = bcnt_acc(a[4] ^ b1.x, d);
    d = bcnt_acc(a[5] ^ b1.y, d);
    d = bcnt_acc(a[6] ^ b1.z, d);
    d = bcnt_acc(a[7] ^ b1.w, d);
    return d;
}

// ref:src/ORBmatcher.cc:245-252 (float viewCos compared with the double literal 0.998)
__device__ __forceinline__ float radius_by_viewing_cos(float viewCos)
{
    return ((double)viewCos > 0.998) ? 2.5f : 4.0f;
}

// Search window of the left (or only) camera pass.
template <int MODE>
__device__ Win query_window(const MatchArgs &A, int q)
{
    Win w;
    w.valid = false;
    w.stereo = false;
    w.sx = 0.f;
    w.sr = 0.f;
    if (MODE == MODE_MPS) {
        // ref:src/ORBmatcher.cc:55-80
        if (!A.q_m0[q]) return w;                                     // mbTrackInView
        if (A.far_points && A.q_f2[q] > A.th_far) return w;          // mTrackDepth > thFarPoints
        if (!A.q_m1[q]) return w;                                     // isBad()
        const int lvl = A.q_lvl[q];
        float r = radius_by_viewing_cos(A.q_f0[q]);
        if (A.th != 1.0f) r *= A.th;
        w.r = r * A.scale[lvl];
        w.x = A.q_x[q];
        w.y = A.q_y[q];
        w.minL = lvl - 1;
        w.maxL = lvl;
        w.stereo = true;
        w.sx = A.q_f1[q];   // mTrackProjXR
        w.sr = w.r;         // r * mvScaleFactors[nPredictedLevel]
        w.valid = true;
    } else if (MODE == MODE_LAST) {
        // ref:src/ORBmatcher.cc:1984-2030
        if (!A.q_m0[q]) return w;
        const float invzc = A.q_f0[q];
        if (invzc < 0) return w;
        const float u = A.q_x[q], v = A.q_y[q];
        if (u < A.min_x || u > A.max_x) return w;
        if (v < A.min_y || v > A.max_y) return w;
        const int oct = A.q_lvl[q];
        const float radius = A.th * A.scale[oct];
        const bool bForward = A.tlc_z > A.mb && !A.mono;
        const bool bBackward = -A.tlc_z > A.mb && !A.mono;
        if (bForward) {
            w.minL = oct;
            w.maxL = -1;
        } else if (bBackward) {
            w.minL = 0;
            w.maxL = oct;
        } else {
            w.minL = oct - 1;
            w.maxL = oct + 1;
        }
        w.x = u;
        w.y = v;
        w.r = radius;
        w.stereo = true;
        const float prod = A.mbf * invzc;
        w.sx = u - prod;   // ur = uv(0) - mbf * invzc
        w.sr = radius;
        w.valid = true;
    } else if (MODE == MODE_KF) {
        // ref:src/ORBmatcher.cc:2262-2265
        if (!A.q_m0[q]) return w;
        const int lvl = A.q_lvl[q];
        w.r = A.th * A.scale[lvl];
        w.x = A.q_x[q];
        w.y = A.q_y[q];
        w.minL = lvl - 1;
        w.maxL = lvl + 1;
        w.valid = true;
    }
    return w;
}

// Search window of the right-camera pass of a two-camera rig.  wl / cl: the left window and its
// candidate count (GetFeaturesInArea size).
template <int MODE>
__device__ Win query_window_r(const MatchArgs &A, int q, const Win &wl, int cl)
{
    Win w;
    w.valid = false;
    w.stereo = false;
    w.sx = 0.f;
    w.sr = 0.f;
    if (A.nleft < 0) return w;
    if (MODE == MODE_MPS) {
        // ref:src/ORBmatcher.cc:185-196: mbTrackInViewR, mnTrackScaleLevelR != -1, radius from
        // mTrackViewCosR (no th factor), levels (lvl-1, lvl), right grid at mTrackProjXR/YR
        if (!A.q_m0r[q]) return w;
        if (A.far_points && A.q_f2[q] > A.th_far) return w;
        if (!A.q_m1[q]) return w;
        const int lvl = A.q_lvl_r[q];
        if (lvl == -1) return w;
        w.r = radius_by_viewing_cos(A.q_f0r[q]) * A.scale[lvl];
        w.x = A.q_xr[q];
        w.y = A.q_yr[q];
        w.minL = lvl - 1;
        w.maxL = lvl;
        w.valid = true;
    } else if (MODE == MODE_LAST) {
        // ref:src/ORBmatcher.cc:2096-2110: same radius and levels at the right-camera projection;
        // an empty left window has already 'continue'd (:2040-2041)
        if (!wl.valid || cl == 0) return w;
        w = wl;
        w.x = A.q_xr[q];
        w.y = A.q_yr[q];
        w.stereo = false;
    }
    return w;
}

// Frame::GetFeaturesInArea (ref:src/Frame.cc:868-962) + the caller's static per-candidate skips.
// RIGHT walks mGridRight; candidates are written as slot indices (right keypoints at nleft + i).
template <bool FILL, bool RIGHT>
__device__ int enum_grid(const MatchArgs &A, const Win &w, const uint32_t (&qd)[8], uint32_t *out)
{
    const float factorX = w.r, factorY = w.r;
    int minCX = (int)floorf((w.x - A.min_x - factorX) * A.inv_w);
    if (minCX < 0) minCX = 0;
    if (minCX >= OSG_GRID_COLS) return 0;
    int maxCX = (int)ceilf((w.x - A.min_x + factorX) * A.inv_w);
    if (maxCX > OSG_GRID_COLS - 1) maxCX = OSG_GRID_COLS - 1;
    if (maxCX < 0) return 0;
    int minCY = (int)floorf((w.y - A.min_y - factorY) * A.inv_h);
    if (minCY < 0) minCY = 0;
    if (minCY >= OSG_GRID_ROWS) return 0;
    int maxCY = (int)ceilf((w.y - A.min_y + factorY) * A.inv_h);
    if (maxCY > OSG_GRID_ROWS - 1) maxCY = OSG_GRID_ROWS - 1;
    if (maxCY < 0) return 0;
    const bool bCheckLevels = (w.minL > 0) || (w.maxL >= 0);  // ref:src/Frame.cc:919 quirk
    const int32_t *gs = RIGHT ? A.grid_start_r : A.grid_start;
    const int32_t *gi = RIGHT ? A.grid_idx_r : A.grid_idx;
    const int off = RIGHT ? A.nleft : 0;
    int cnt = 0;
    for (int ix = minCX; ix <= maxCX; ix++) {
        for (int iy = minCY; iy <= maxCY; iy++) {
            const int cell = ix * OSG_GRID_ROWS + iy;
            const int j1 = gs[cell + 1];
            for (int j = gs[cell]; j < j1; j++) {
                const int k = gi[j] + off;
                const int oct = A.kp_octave[k];
                if (bCheckLevels) {
                    if (oct < w.minL) continue;
                    if (w.maxL >= 0 && oct > w.maxL) continue;
                }
                const float distx = A.kp_x[k] - w.x;
                const float disty = A.kp_y[k] - w.y;
                if (!(fabsf(distx) < factorX && fabsf(disty) < factorY)) continue;
                if (!RIGHT && w.stereo && A.u_right) {
                    const float ur = A.u_right[k];
                    if (ur > 0) {
                        const float er = fabsf(w.sx - ur);
                        if (er > w.sr) continue;
                    }
                }
                if (FILL) {
                    const uint32_t d = dist256(qd, A.fdesc + (size_t)k * 8);
                    out[cnt] = (uint32_t)k | (d << 16) | ((uint32_t)(oct & 0x7F) << 25);
                }
                cnt++;
            }
        }
    }
    return cnt;
}

// Candidates of query q: left-camera ones first, then right-camera ones; cl = left count.
template <int MODE, bool FILL>
__device__ int enum_query(const MatchArgs &A, int q, uint32_t *out, int &cl)
{
    uint32_t qd[8];
    if (FILL) {
        const uint4 a = *(const uint4 *)(A.qdesc + (size_t)q * 8);
        const uint4 b = *(const uint4 *)(A.qdesc + (size_t)q * 8 + 4);
        qd[0] = a.x; qd[1] = a.y; qd[2] = a.z; qd[3] = a.w;
        qd[4] = b.x; qd[5] = b.y; qd[6] = b.z; qd[7] = b.w;
    }
    if (MODE == MODE_BOW_KF_F || MODE == MODE_BOW_KF_KF) {
        int cnt = 0;
        const int e = A.q_ce[q];
        for (int j = A.q_cb[q]; j < e; j++) {
            const int idx = A.cand_list[j];
            if (MODE == MODE_BOW_KF_KF && !A.slot_ok[idx]) continue;  // !pMP2 || isBad || right camera
            if (FILL) {
                const uint32_t d = dist256(qd, A.fdesc + (size_t)idx * 8);
                out[cnt] = (uint32_t)idx | (d << 16);
            }
            cnt++;
        }
        cl = cnt;
        return cnt;
    } else {
        const Win w = query_window<MODE>(A, q);
        const int c0 = w.valid ? enum_grid<FILL, false>(A, w, qd, out) : 0;
        cl = c0;
        int c1 = 0;
        if (MODE == MODE_MPS || MODE == MODE_LAST) {
            const Win wr = query_window_r<MODE>(A, q, w, c0);
            if (wr.valid) c1 = enum_grid<FILL, true>(A, wr, qd, FILL ? out + c0 : nullptr);
        }
        return c0 + c1;
    }
}

// bestDist / bestLevel / bestDist2 / bestLevel2 / bestIdx of the reference loops
struct Top2 {
    int best = 256, bl = -1, second = 256, sl = -1, bslot = -1;
    __device__ __forceinline__ void push(int d, int l, int s)
    {
        if (d < best) {
            second = best;
            sl = bl;
            best = d;
            bl = l;
            bslot = s;
        } else if (d < second) {
            second = d;
            sl = l;
        }
    }
};

// One query in reference order.  blocked(s): is slot s unavailable to q given the assignments of
// the queries before q (Jacobi: claims of the previous round; serial: the live slot state).
template <int MODE, typename Blocked>
__device__ __forceinline__ QRes eval_query(const MatchArgs &A, int q, Blocked blocked)
{
    QRes res{-1, -1};
    const int e0 = A.q_off[q], em = A.q_mid[q], e1 = A.q_off[q + 1];
    Top2 L, R;
    if (MODE == MODE_BOW_KF_F) {
        // ref:src/ORBmatcher.cc:316-441: one loop, separate top-2 for left / right keypoints
        for (int e = e0; e < e1; e++) {
            const uint32_t c = A.cands[e];
            const int s = (int)(c & 0xFFFFu);
            if (blocked(s)) continue;
            const int d = (int)((c >> 16) & 0x1FFu);
            if (A.nleft < 0 || s < A.nleft) L.push(d, 0, s);
            else R.push(d, 0, s);
        }
        if (L.best <= OSG_TH_LOW) {
            if ((float)L.best < A.nnratio * (float)L.second) res.l = L.bslot;
            if (R.best <= OSG_TH_LOW) res.r = R.bslot;  // ratio disabled by '|| true' (:425)
        }
        return res;
    }
    for (int e = e0; e < em; e++) {
        const uint32_t c = A.cands[e];
        const int s = (int)(c & 0xFFFFu);
        if (blocked(s)) continue;
        L.push((int)((c >> 16) & 0x1FFu), (int)(c >> 25), s);
    }
    bool acc, skip_r = false;
    if (MODE == MODE_MPS) {  // ref:src/ORBmatcher.cc:147-167 (a ratio failure 'continue's past the right pass)
        acc = L.best <= OSG_TH_HIGH && !(L.bl == L.sl && (float)L.best > A.nnratio * (float)L.second);
        skip_r = L.best <= OSG_TH_HIGH && !acc;
    } else if (MODE == MODE_LAST) {  // ref:src/ORBmatcher.cc:2070
        acc = L.best <= OSG_TH_HIGH;
    } else if (MODE == MODE_KF) {  // ref:src/ORBmatcher.cc:2287
        acc = L.best <= A.orb_dist;
    } else {  // MODE_BOW_KF_KF, ref:src/ORBmatcher.cc:985-987
        acc = L.best < OSG_TH_LOW && (float)L.best < A.nnratio * (float)L.second;
    }
    res.l = acc ? L.bslot : -1;
    if ((MODE == MODE_MPS || MODE == MODE_LAST) && em < e1 && !skip_r) {
        // the left pass of q itself may have written the stereo partner slot; its state is then
        // q's own Observations() > 0
        int own = -1;
        bool own_blocked = false;
        if (MODE == MODE_MPS && res.l >= 0 && A.l2r) {
            const int t = A.l2r[res.l];
            if (t != -1) {
                own = t + A.nleft;
                own_blocked = A.q_has_obs[q] != 0;
            }
        }
        for (int e = em; e < e1; e++) {
            const uint32_t c = A.cands[e];
            const int s = (int)(c & 0xFFFFu);
            if (s == own ? own_blocked : blocked(s)) continue;
            R.push((int)((c >> 16) & 0x1FFu), (int)(c >> 25), s);
        }
        bool accr;
        if (MODE == MODE_MPS)  // ref:src/ORBmatcher.cc:222-238
            accr = R.best <= OSG_TH_HIGH && !(R.bl == R.sl && (float)R.best > A.nnratio * (float)R.second);
        else  // ref:src/ORBmatcher.cc:2133
            accr = R.best <= OSG_TH_HIGH;
        res.r = accr ? R.bslot : -1;
    }
    return res;
}

// Every slot q writes: the direct matches and, for a5 on a two-camera rig, each one's stereo
// partner (ref:src/ORBmatcher.cc:154-163, 226-236).  Returns the count (<= 4).
template <int MODE>
__device__ __forceinline__ int assigned_slots(const MatchArgs &A, QRes r, int (&out)[4])
{
    int n = 0;
    if (r.l >= 0) {
        out[n++] = r.l;
        if (MODE == MODE_MPS && A.l2r) {
            const int t = A.l2r[r.l];
            if (t != -1) out[n++] = t + A.nleft;
        }
    }
    if (r.r >= 0) {
        if (MODE == MODE_MPS && A.r2l) {
            const int t = A.r2l[r.r - A.nleft];
            if (t != -1) out[n++] = t;
        }
        out[n++] = r.r;
    }
    return n;
}

__device__ __forceinline__ QRes load_res(const MatchArgs &A, int q)
{
    return QRes{A.q_res[2 * q], A.q_res[2 * q + 1]};
}
__device__ __forceinline__ void store_res(const MatchArgs &A, int q, QRes r)
{
    A.q_res[2 * q] = r.l;
    A.q_res[2 * q + 1] = r.r;
}

__device__ __forceinline__ int rot_bin(float a, float b)
{  // ref:src/ORBmatcher.cc:411-418, factor = 1.0f/HISTO_LENGTH (kept upstream bug)
    const float factor = 1.0f / OSG_HISTO_LENGTH;
    float rot = a - b;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == OSG_HISTO_LENGTH) bin = 0;
    return bin;
}

template <int MODE>
__global__ __launch_bounds__(MT) void k_match(MatchArgs A)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int NS = A.n_slots;
    int *claimA = (int *)smem;
    int *claimB = claimA + NS;
    int *lastS = claimB + NS;
    uint8_t *taken0 = (uint8_t *)(lastS + NS);
    uint8_t *removedS = taken0 + ((NS + 15) & ~15);
    __shared__ int s_scan[MT];
    __shared__ int s_hist[OSG_HISTO_LENGTH];
    __shared__ int s_keep[3];
    __shared__ int s_red[2];

    const int tid = threadIdx.x;
    const int nq = A.nq;
    const int per = (nq + MT - 1) / MT;
    const int q0 = min(nq, tid * per), q1 = min(nq, q0 + per);

    // ---- 1. count
    int my = 0;
    for (int q = q0; q < q1; q++) {
        int cl;
        const int c = enum_query<MODE, false>(A, q, nullptr, cl);
        A.q_off[q] = c;  // temporarily the count
        my += c;
    }
    // ---- 2. block scan (inclusive, Hillis-Steele)
    s_scan[tid] = my;
    __syncthreads();
    for (int o = 1; o < MT; o <<= 1) {
        const int v = tid >= o ? s_scan[tid - o] : 0;
        __syncthreads();
        s_scan[tid] += v;
        __syncthreads();
    }
    const int total = s_scan[MT - 1];
    if (total > A.cap) {
        if (tid == 0) {
            A.status[0] = total;
            A.status[3] = 1;
        }
        return;
    }
    // ---- 3. fill
    {
        int off = s_scan[tid] - my;
        for (int q = q0; q < q1; q++) {
            const int c = A.q_off[q];
            int cl;
            A.q_off[q] = off;
            enum_query<MODE, true>(A, q, A.cands + off, cl);
            A.q_mid[q] = off + cl;
            off += c;
        }
        if (tid == MT - 1) A.q_off[nq] = total;
    }
    // ---- 4. resolve: init slot state
    for (int s = tid; s < NS; s += MT) {
        claimA[s] = INT_BIG;
        claimB[s] = INT_BIG;
        lastS[s] = -1;
        removedS[s] = 0;
        uint8_t t0 = 0;
        if (MODE == MODE_MPS || MODE == MODE_LAST) t0 = (A.slot_mp[s] >= 0 && A.slot_taken[s]) ? 1 : 0;
        else if (MODE == MODE_KF) t0 = (A.slot_mp[s] >= 0) ? 1 : 0;
        taken0[s] = t0;
    }
    if (tid < OSG_HISTO_LENGTH) s_hist[tid] = 0;
    __syncthreads();
    for (int q = q0; q < q1; q++)
        store_res(A, q, eval_query<MODE>(A, q, [&](int s) { return taken0[s] || claimA[s] < q; }));
    __syncthreads();
    // Jacobi rounds.  A slot is blocked for q when it was blocked initially or a query p < q
    // whose MapPoint has observations wrote it (SearchByBoW / a7: any earlier write).
    int rounds = 0;
    int *cur = claimB, *other = claimA;
    for (;;) {
        rounds++;
        for (int q = q0; q < q1; q++) {
            const bool claims = (MODE == MODE_MPS || MODE == MODE_LAST) ? (A.q_has_obs[q] != 0) : true;
            if (!claims) continue;
            int sl[4];
            const int n = assigned_slots<MODE>(A, load_res(A, q), sl);
            for (int i = 0; i < n; i++) atomicMin(&cur[sl[i]], q);
        }
        __syncthreads();
        int changed = 0;
        for (int q = q0; q < q1; q++) {
            const QRes r2 = eval_query<MODE>(A, q, [&](int s) { return taken0[s] || cur[s] < q; });
            const QRes r1 = load_res(A, q);
            if (r2.l != r1.l || r2.r != r1.r) {
                changed = 1;
                store_res(A, q, r2);
            }
        }
        for (int s = tid; s < NS; s += MT) other[s] = INT_BIG;
        const int any = __syncthreads_or(changed);
        int *t = cur;
        cur = other;
        other = t;
        if (!any || rounds > nq + 1) break;
    }
    // 'other' now holds the claims of the converged results.  The monotone rule above is exact
    // unless a stereo-partner write of a5 by a MapPoint WITHOUT observations lands on a slot that
    // was blocked: that write unblocks it (the slot's state is its last writer's).  Such a run is
    // redone serially in query order on the live slot state.
    int serial = 0;
    if (MODE == MODE_MPS && A.nleft >= 0) {
        int need = 0;
        for (int q = q0; q < q1; q++) {
            if (A.q_has_obs[q]) continue;
            const QRes r = load_res(A, q);
            if (r.l >= 0 && A.l2r && A.l2r[r.l] != -1) {
                const int s = A.l2r[r.l] + A.nleft;
                need |= (taken0[s] || other[s] < q) ? 1 : 0;
            }
            if (r.r >= 0 && A.r2l && A.r2l[r.r - A.nleft] != -1) {
                const int s = A.r2l[r.r - A.nleft];
                need |= (taken0[s] || other[s] < q) ? 1 : 0;
            }
        }
        serial = __syncthreads_or(need);
        if (serial) {
            if (tid == 0) {
                for (int q = 0; q < nq; q++) {
                    const QRes r = eval_query<MODE>(A, q, [&](int s) { return taken0[s] != 0; });
                    store_res(A, q, r);
                    int sl[4];
                    const int n = assigned_slots<MODE>(A, r, sl);
                    for (int i = 0; i < n; i++) taken0[sl[i]] = A.q_has_obs[q];
                }
            }
            __syncthreads();
        }
    }
    // ---- 5. finish: last assignment, rotation histogram, removal, counts
    int nacc = 0;
    const bool ori = A.check_ori && MODE != MODE_MPS;
    for (int q = q0; q < q1; q++) {
        const QRes r = load_res(A, q);
        int sl[4];
        const int n = assigned_slots<MODE>(A, r, sl);
        nacc += n;
        if (MODE != MODE_BOW_KF_KF)
            for (int i = 0; i < n; i++) atomicMax(&lastS[sl[i]], q);
        if (ori) {
            if (r.l >= 0) {
                const int bin = rot_bin(A.q_angle[q], A.slot_angle[r.l]);
                A.q_bin[2 * q] = (uint8_t)bin;
                atomicAdd(&s_hist[bin], 1);
            }
            if (r.r >= 0) {
                const int bin = rot_bin(A.q_angle[q], A.slot_angle[r.r]);
                A.q_bin[2 * q + 1] = (uint8_t)bin;
                atomicAdd(&s_hist[bin], 1);
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        // ComputeThreeMaxima, ref:src/ORBmatcher.cc:2341-2383
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < OSG_HISTO_LENGTH; i++) {
            const int sz = s_hist[i];
            if (sz > max1) {
                max3 = max2; max2 = max1; max1 = sz;
                ind3 = ind2; ind2 = ind1; ind1 = i;
            } else if (sz > max2) {
                max3 = max2; max2 = sz;
                ind3 = ind2; ind2 = i;
            } else if (sz > max3) {
                max3 = sz;
                ind3 = i;
            }
        }
        if (max2 < 0.1f * (float)max1) {
            ind2 = -1;
            ind3 = -1;
        } else if (max3 < 0.1f * (float)max1) {
            ind3 = -1;
        }
        s_keep[0] = ind1;
        s_keep[1] = ind2;
        s_keep[2] = ind3;
        s_red[0] = 0;
    }
    __syncthreads();
    int nrem = 0;
    for (int q = q0; q < q1; q++) {
        const QRes r = load_res(A, q);
        bool removed_l = false;
        if (ori) {
            if (r.l >= 0) {
                const int bin = A.q_bin[2 * q];
                removed_l = !(bin == s_keep[0] || bin == s_keep[1] || bin == s_keep[2]);
                if (removed_l) {
                    nrem++;
                    if (MODE != MODE_BOW_KF_KF) removedS[r.l] = 1;
                }
            }
            if (r.r >= 0) {
                const int bin = A.q_bin[2 * q + 1];
                if (!(bin == s_keep[0] || bin == s_keep[1] || bin == s_keep[2])) {
                    nrem++;
                    removedS[r.r] = 1;
                }
            }
        }
        if (MODE == MODE_BOW_KF_KF) A.out_q[q] = (r.l >= 0 && !removed_l) ? A.slot_mp2[r.l] : -1;
    }
    atomicAdd(&s_red[0], nacc - nrem);
    __syncthreads();
    if (MODE != MODE_BOW_KF_KF) {
        for (int s = tid; s < NS; s += MT) {
            if (removedS[s]) A.slot_mp[s] = -1;
            else if (lastS[s] >= 0) A.slot_mp[s] = A.q_mp[lastS[s]];
        }
    }
    if (tid == 0) {
        A.status[1] = s_red[0];
        A.status[2] = rounds;
        A.status[0] = total;
        A.status[3] = 0;
        A.status[4] = serial;
    }
}

size_t match_lds_bytes(int ns)
{
    return (size_t)ns * 3 * sizeof(int) + 2 * (((size_t)ns + 15) & ~size_t(15));
}

// Upload the packed inputs + the in/out slot array, launch (growing the candidate buffer when the
// count pass reports more than the capacity), download slot array / out_q + status.
template <int MODE>
int run_match(osg_ctx *ctx, MatchArgs A, const osg_packer &pk, int32_t *host_slot, int n_slot_io,
              int32_t *host_out_q, int32_t *out_nmatches, void **dev_base_out)
{
    (void)dev_base_out;
    const int nq = A.nq, NS = A.n_slots;
    OSG_REQUIRE(ctx, NS <= MAX_SLOTS, "%d slots exceed the %d supported per problem", NS, MAX_SLOTS);
    // layout of the device io block: [status 16 ints][slot 'n_slot_io' ints][out_q nq ints]
    const size_t io_bytes = 64 + sizeof(int32_t) * ((size_t)n_slot_io + (size_t)nq) + 64;
    char *pin = (char *)osg_pinned(ctx, pk.total + io_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));  // pinned block may still be in use
    pk.fill(pin);
    char *dev_in = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, pk.total + 256);
    char *dev_io = nullptr;
    OSG_ALLOC(ctx, dev_io, SLOT_TMP1, io_bytes);
    char *pin_io = pin + ((pk.total + 255) & ~size_t(255));
    std::memset(pin_io, 0, 64);
    if (n_slot_io > 0) std::memcpy(pin_io + 64, host_slot, sizeof(int32_t) * n_slot_io);
    if (pk.total) OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_in, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_io, pin_io, 64 + sizeof(int32_t) * n_slot_io, hipMemcpyHostToDevice,
                                      ctx->stream));
    A.status = (int32_t *)dev_io;
    A.slot_mp = (int32_t *)(dev_io + 64);
    A.out_q = (int32_t *)(dev_io + 64 + sizeof(int32_t) * n_slot_io);
    int cap = std::max(nq * 64, 1 << 16);
    size_t lds = match_lds_bytes(NS);
    for (int attempt = 0; attempt < 2; attempt++) {
        OSG_ALLOC(ctx, A.q_off, SLOT_TMP2, sizeof(int32_t) * ((size_t)nq + 1));
        OSG_ALLOC(ctx, A.q_res, SLOT_TMP3, sizeof(int32_t) * 2 * ((size_t)nq + 1));
        OSG_ALLOC(ctx, A.q_bin, SLOT_TMP4, 2 * (size_t)nq + 16);
        OSG_ALLOC(ctx, A.q_mid, SLOT_TMP6, sizeof(int32_t) * ((size_t)nq + 1));
        OSG_ALLOC(ctx, A.cands, SLOT_TMP5, sizeof(uint32_t) * (size_t)cap);
        A.cap = cap;
        hipLaunchKernelGGL(k_match<MODE>, dim3(1), dim3(MT), lds, ctx->stream, A);
        OSG_HIP_CHECK(ctx, hipGetLastError());
        int32_t st[5];
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(st, dev_io, sizeof st, hipMemcpyDeviceToHost, ctx->stream));
        OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
        if (st[3] == 0) {
            *out_nmatches = st[1];
            ctx->match_stats[0] = st[0];
            ctx->match_stats[1] = st[2];
            ctx->match_stats[2] = st[4];
            ctx->match_stats[3] = st[1];
            break;
        }
        cap = st[0] + 1024;
        if (attempt == 1) return osg_set_error(ctx, OSG_E_HIP, "candidate buffer overflow after resize");
    }
    const size_t back = sizeof(int32_t) * ((size_t)n_slot_io + (host_out_q ? (size_t)nq : 0));
    if (back) {
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(pin_io + 64, dev_io + 64, back, hipMemcpyDeviceToHost, ctx->stream));
        OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
        if (n_slot_io > 0) std::memcpy(host_slot, pin_io + 64, sizeof(int32_t) * n_slot_io);
        if (host_out_q) std::memcpy(host_out_q, pin_io + 64 + sizeof(int32_t) * n_slot_io, sizeof(int32_t) * nq);
    }
    return OSG_OK;
}

// Pointer fields of MatchArgs are first filled with packer offsets (+1 so that offset 0 is not
// confused with "absent"), then relocated against the device block.
template <typename T>
void set_off(T *&field, size_t off)
{
    field = (off == SIZE_MAX) ? nullptr : (T *)(uintptr_t)(off + 1);
}
template <typename T>
void relocate(T *&field, char *base)
{
    if (field) field = (T *)(base + ((uintptr_t)field - 1));
}

#define OSG_RELOCATE_ALL(A, base)                                                                            \
    do {                                                                                                     \
        relocate(A.fdesc, base); relocate(A.kp_x, base); relocate(A.kp_y, base); relocate(A.slot_angle, base); \
        relocate(A.kp_octave, base); relocate(A.u_right, base); relocate(A.grid_start, base);                \
        relocate(A.grid_idx, base); relocate(A.scale, base); relocate(A.qdesc, base); relocate(A.q_mp, base); \
        relocate(A.q_has_obs, base); relocate(A.q_angle, base); relocate(A.q_x, base); relocate(A.q_y, base); \
        relocate(A.q_f0, base); relocate(A.q_f1, base); relocate(A.q_f2, base); relocate(A.q_lvl, base);     \
        relocate(A.q_m0, base); relocate(A.q_m1, base); relocate(A.q_cb, base); relocate(A.q_ce, base);     \
        relocate(A.cand_list, base); relocate(A.slot_ok, base); relocate(A.slot_mp2, base);                  \
        relocate(A.slot_taken, base); relocate(A.grid_start_r, base); relocate(A.grid_idx_r, base);          \
        relocate(A.l2r, base); relocate(A.r2l, base); relocate(A.q_xr, base); relocate(A.q_yr, base);       \
        relocate(A.q_f0r, base); relocate(A.q_lvl_r, base); relocate(A.q_m0r, base);                         \
    } while (0)

template <int MODE>
int launch_packed(osg_ctx *ctx, MatchArgs &A, osg_packer &pk, int32_t *host_slot, int n_slot_io,
                  int32_t *host_out_q)
{
    char *dev_in = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, pk.total + 256);
    OSG_RELOCATE_ALL(A, dev_in);
    int nm = 0;
    const int rc = run_match<MODE>(ctx, A, pk, host_slot, n_slot_io, host_out_q, &nm, nullptr);
    if (rc < 0) return rc;
    return nm;
}

void frame_into_args(MatchArgs &A, osg_packer &pk, const osg_frame *F)
{
    A.n_slots = F->n;
    A.nleft = F->nleft;
    set_off(A.fdesc, pk.add(F->desc, (size_t)F->n * 32));
    set_off(A.kp_x, pk.add(F->kp_x, sizeof(float) * F->n));
    set_off(A.kp_y, pk.add(F->kp_y, sizeof(float) * F->n));
    set_off(A.slot_angle, pk.add(F->kp_angle, sizeof(float) * F->n));
    set_off(A.kp_octave, pk.add(F->kp_octave, sizeof(int32_t) * F->n));
    // the u_R check runs only for Nleft == -1 (ref:src/ORBmatcher.cc:97, :2055)
    set_off(A.u_right, F->nleft == -1 ? pk.add(F->u_right, sizeof(float) * F->n) : SIZE_MAX);
    set_off(A.grid_start, pk.add(F->grid_start, sizeof(int32_t) * (OSG_GRID_CELLS + 1)));
    set_off(A.grid_idx, pk.add(F->grid_idx, sizeof(int32_t) * F->grid_start[OSG_GRID_CELLS]));
    if (F->nleft != -1) {
        set_off(A.grid_start_r, pk.add(F->grid_start_r, sizeof(int32_t) * (OSG_GRID_CELLS + 1)));
        set_off(A.grid_idx_r, pk.add(F->grid_idx_r, sizeof(int32_t) * F->grid_start_r[OSG_GRID_CELLS]));
        set_off(A.l2r, pk.add(F->left_to_right, sizeof(int32_t) * F->nleft));
        set_off(A.r2l, pk.add(F->right_to_left, sizeof(int32_t) * (F->n - F->nleft)));
    }
    set_off(A.scale, pk.add(F->scale_factors, sizeof(float) * F->n_levels));
    A.min_x = F->min_x;
    A.max_x = F->max_x;
    A.min_y = F->min_y;
    A.max_y = F->max_y;
    A.inv_w = F->grid_inv_w;
    A.inv_h = F->grid_inv_h;
    A.mb = F->mb;
    A.mbf = F->mbf;
}

// A grid in CSR must index keypoints [0, n_cam) only: the kernels trust it.
static int check_grid(osg_ctx *ctx, const int32_t *gs, const int32_t *gi, int n_cam, const char *which)
{
    OSG_REQUIRE(ctx, gs && (gi || gs[OSG_GRID_CELLS] == 0), "%s grid missing", which);
    OSG_REQUIRE(ctx, gs[0] == 0, "%s grid_start[0] != 0", which);
    for (int c = 0; c < OSG_GRID_CELLS; c++)
        OSG_REQUIRE(ctx, gs[c + 1] >= gs[c], "%s grid_start not monotone at cell %d", which, c);
    const int m = gs[OSG_GRID_CELLS];
    for (int j = 0; j < m; j++)
        OSG_REQUIRE(ctx, gi[j] >= 0 && gi[j] < n_cam, "%s grid_idx[%d] = %d out of range", which, j, gi[j]);
    return OSG_OK;
}

int check_frame(osg_ctx *ctx, const osg_frame *F)
{
    OSG_REQUIRE(ctx, F && F->n >= 0 && F->n <= MAX_SLOTS, "frame n out of range");
    OSG_REQUIRE(ctx, F->nleft == -1 || (F->nleft >= 0 && F->nleft <= F->n), "frame nleft out of range");
    OSG_REQUIRE(ctx, F->n == 0 || (F->desc && F->kp_x && F->kp_y && F->kp_angle && F->kp_octave), "frame arrays");
    OSG_REQUIRE(ctx, F->scale_factors && F->n_levels > 0, "frame scale factors");
    const int nl = F->nleft == -1 ? F->n : F->nleft;
    int rc = check_grid(ctx, F->grid_start, F->grid_idx, nl, "left");
    if (rc < 0) return rc;
    if (F->nleft != -1) {
        rc = check_grid(ctx, F->grid_start_r, F->grid_idx_r, F->n - F->nleft, "right");
        if (rc < 0) return rc;
        for (int i = 0; F->left_to_right && i < F->nleft; i++)
            OSG_REQUIRE(ctx, F->left_to_right[i] >= -1 && F->left_to_right[i] < F->n - F->nleft, "left_to_right[%d]", i);
        for (int i = 0; F->right_to_left && i < F->n - F->nleft; i++)
            OSG_REQUIRE(ctx, F->right_to_left[i] >= -1 && F->right_to_left[i] < F->nleft, "right_to_left[%d]", i);
    }
    return OSG_OK;
}

}  // namespace

extern "C" {

int osg_search_by_projection_mps(osg_ctx *ctx, const osg_frame *F, const osg_mp_queries *Q, float nnratio,
                                 float th, int far_points, float th_far_points, int32_t *slot_mp,
                                 const uint8_t *slot_taken)
{
    if (!ctx) return OSG_E_INVALID;
    int rc = check_frame(ctx, F);
    if (rc < 0) return rc;
    OSG_REQUIRE(ctx, Q && Q->n >= 0 && slot_mp && slot_taken, "null argument");
    if (Q->n == 0) return 0;
    OSG_REQUIRE(ctx, Q->desc && Q->mp_id && Q->usable && Q->has_obs && Q->in_view && Q->proj_x && Q->proj_y &&
                         Q->proj_xr && Q->view_cos && Q->pred_level && Q->track_depth, "query arrays");
    for (int i = 0; i < Q->n; i++)
        if (Q->in_view[i] && (Q->pred_level[i] < 0 || Q->pred_level[i] >= F->n_levels))
            return osg_set_error(ctx, OSG_E_INVALID, "pred_level[%d] = %d out of range", i, Q->pred_level[i]);
    if (F->nleft != -1) {
        OSG_REQUIRE(ctx, Q->in_view_r && Q->proj_yr && Q->view_cos_r && Q->pred_level_r, "right-camera query arrays");
        for (int i = 0; i < Q->n; i++)
            if (Q->in_view_r[i] && (Q->pred_level_r[i] < -1 || Q->pred_level_r[i] >= F->n_levels))
                return osg_set_error(ctx, OSG_E_INVALID, "pred_level_r[%d] = %d out of range", i, Q->pred_level_r[i]);
    }
    MatchArgs A = {};
    osg_packer pk;
    frame_into_args(A, pk, F);
    const int n = Q->n;
    A.nq = n;
    set_off(A.qdesc, pk.add(Q->desc, (size_t)n * 32));
    set_off(A.q_mp, pk.add(Q->mp_id, sizeof(int32_t) * n));
    set_off(A.q_has_obs, pk.add(Q->has_obs, n));
    set_off(A.q_m0, pk.add(Q->in_view, n));
    set_off(A.q_m1, pk.add(Q->usable, n));
    set_off(A.q_x, pk.add(Q->proj_x, sizeof(float) * n));
    set_off(A.q_y, pk.add(Q->proj_y, sizeof(float) * n));
    set_off(A.q_f0, pk.add(Q->view_cos, sizeof(float) * n));
    set_off(A.q_f1, pk.add(Q->proj_xr, sizeof(float) * n));
    set_off(A.q_f2, pk.add(Q->track_depth, sizeof(float) * n));
    set_off(A.q_lvl, pk.add(Q->pred_level, sizeof(int32_t) * n));
    set_off(A.slot_taken, pk.add(slot_taken, F->n));
    if (F->nleft != -1) {
        A.q_xr = A.q_f1;  // mTrackProjXR
        set_off(A.q_yr, pk.add(Q->proj_yr, sizeof(float) * n));
        set_off(A.q_f0r, pk.add(Q->view_cos_r, sizeof(float) * n));
        set_off(A.q_lvl_r, pk.add(Q->pred_level_r, sizeof(int32_t) * n));
        set_off(A.q_m0r, pk.add(Q->in_view_r, n));
    }
    A.nnratio = nnratio;
    A.th = th;
    A.far_points = far_points;
    A.th_far = th_far_points;
    return launch_packed<MODE_MPS>(ctx, A, pk, slot_mp, F->n, nullptr);
}

int osg_search_by_projection_last(osg_ctx *ctx, const osg_frame *CF, const osg_last_queries *L, float th,
                                  int mono, int check_orientation, int32_t *slot_mp, const uint8_t *slot_taken)
{
    if (!ctx) return OSG_E_INVALID;
    int rc = check_frame(ctx, CF);
    if (rc < 0) return rc;
    OSG_REQUIRE(ctx, L && L->n >= 0 && slot_mp && slot_taken, "null argument");
    if (L->n == 0) return 0;
    OSG_REQUIRE(ctx, L->desc && L->mp_id && L->valid && L->has_obs && L->u && L->v && L->invz && L->octave &&
                         L->angle, "query arrays");
    for (int i = 0; i < L->n; i++)
        if (L->valid[i] && (L->octave[i] < 0 || L->octave[i] >= CF->n_levels))
            return osg_set_error(ctx, OSG_E_INVALID, "octave[%d] out of range", i);
    MatchArgs A = {};
    osg_packer pk;
    frame_into_args(A, pk, CF);
    const int n = L->n;
    A.nq = n;
    set_off(A.qdesc, pk.add(L->desc, (size_t)n * 32));
    set_off(A.q_mp, pk.add(L->mp_id, sizeof(int32_t) * n));
    set_off(A.q_has_obs, pk.add(L->has_obs, n));
    set_off(A.q_m0, pk.add(L->valid, n));
    set_off(A.q_x, pk.add(L->u, sizeof(float) * n));
    set_off(A.q_y, pk.add(L->v, sizeof(float) * n));
    set_off(A.q_f0, pk.add(L->invz, sizeof(float) * n));
    set_off(A.q_lvl, pk.add(L->octave, sizeof(int32_t) * n));
    set_off(A.q_angle, pk.add(L->angle, sizeof(float) * n));
    set_off(A.slot_taken, pk.add(slot_taken, CF->n));
    if (CF->nleft != -1) {
        OSG_REQUIRE(ctx, L->u_r && L->v_r, "right-camera projections (u_r, v_r)");
        set_off(A.q_xr, pk.add(L->u_r, sizeof(float) * n));
        set_off(A.q_yr, pk.add(L->v_r, sizeof(float) * n));
    }
    A.th = th;
    A.mono = mono;
    A.tlc_z = L->tlc_z;
    A.check_ori = check_orientation;
    return launch_packed<MODE_LAST>(ctx, A, pk, slot_mp, CF->n, nullptr);
}

int osg_search_by_projection_kf(osg_ctx *ctx, const osg_frame *CF, const osg_kf_queries *K, float th, int orb_dist,
                                int check_orientation, int32_t *slot_mp)
{
    if (!ctx) return OSG_E_INVALID;
    int rc = check_frame(ctx, CF);
    if (rc < 0) return rc;
    OSG_REQUIRE(ctx, K && K->n >= 0 && slot_mp, "null argument");
    if (K->n == 0) return 0;
    OSG_REQUIRE(ctx, K->desc && K->mp_id && K->valid && K->u && K->v && K->pred_level && K->angle, "query arrays");
    for (int i = 0; i < K->n; i++)
        if (K->valid[i] && (K->pred_level[i] < 0 || K->pred_level[i] >= CF->n_levels))
            return osg_set_error(ctx, OSG_E_INVALID, "pred_level[%d] out of range", i);
    MatchArgs A = {};
    osg_packer pk;
    frame_into_args(A, pk, CF);
    const int n = K->n;
    A.nq = n;
    set_off(A.qdesc, pk.add(K->desc, (size_t)n * 32));
    set_off(A.q_mp, pk.add(K->mp_id, sizeof(int32_t) * n));
    set_off(A.q_m0, pk.add(K->valid, n));
    set_off(A.q_x, pk.add(K->u, sizeof(float) * n));
    set_off(A.q_y, pk.add(K->v, sizeof(float) * n));
    set_off(A.q_lvl, pk.add(K->pred_level, sizeof(int32_t) * n));
    set_off(A.q_angle, pk.add(K->angle, sizeof(float) * n));
    A.th = th;
    A.orb_dist = orb_dist;
    A.check_ori = check_orientation;
    return launch_packed<MODE_KF>(ctx, A, pk, slot_mp, CF->n, nullptr);
}

// Host half of SearchByBoW: the FeatureVector merge-walk (ref:src/ORBmatcher.cc:292-467) emits the
// query order (shared nodes ascending, KeyFrame features in node order); each query's candidate
// list is the other side's feature list of the same node.
static int bow_queries(const osg_bow_side *A_, const osg_bow_side *B_, bool guard_nleft_a,
                       std::vector<int32_t> &q_feat, std::vector<int32_t> &q_cb, std::vector<int32_t> &q_ce)
{
    int ia = 0, ib = 0;
    const osg_featvec &fa = A_->fv, &fb = B_->fv;
    while (ia < fa.n_nodes && ib < fb.n_nodes) {
        if (fa.node_id[ia] == fb.node_id[ib]) {
            for (int a = fa.node_start[ia]; a < fa.node_start[ia + 1]; a++) {
                const int idx = fa.feat[a];
                // mvKeysUn.size() == NLeft on a two-camera rig (ref:src/ORBmatcher.cc:934-936)
                if (guard_nleft_a && A_->nleft != -1 && idx >= A_->nleft) continue;
                if (idx < 0 || idx >= A_->n) return -1;
                if (!A_->mp_good[idx]) continue;
                q_feat.push_back(idx);
                q_cb.push_back(fb.node_start[ib]);
                q_ce.push_back(fb.node_start[ib + 1]);
            }
            ia++;
            ib++;
        } else if (fa.node_id[ia] < fb.node_id[ib]) {
            const uint32_t key = fb.node_id[ib];
            int lo = ia, hi = fa.n_nodes;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (fa.node_id[mid] < key) lo = mid + 1; else hi = mid;
            }
            ia = lo;
        } else {
            const uint32_t key = fa.node_id[ia];
            int lo = ib, hi = fb.n_nodes;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (fb.node_id[mid] < key) lo = mid + 1; else hi = mid;
            }
            ib = lo;
        }
    }
    return 0;
}

int osg_search_by_bow_kf_f(osg_ctx *ctx, const osg_bow_side *kf, const osg_bow_side *f, float nnratio,
                           int check_orientation, int32_t *out_mp)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, kf && f && out_mp, "null argument");
    OSG_REQUIRE(ctx, f->n >= 0 && f->n <= MAX_SLOTS && kf->n >= 0, "sizes");
    OSG_REQUIRE(ctx, f->nleft == -1 || (f->nleft >= 0 && f->nleft <= f->n), "frame nleft");
    for (int i = 0; i < f->n; i++) out_mp[i] = -1;
    std::vector<int32_t> q_feat, q_cb, q_ce;
    if (bow_queries(kf, f, false, q_feat, q_cb, q_ce) < 0) return osg_set_error(ctx, OSG_E_INVALID, "feature index");
    const int n = (int)q_feat.size();
    if (n == 0) return 0;
    for (int j = 0; j < f->fv.node_start[f->fv.n_nodes]; j++)
        OSG_REQUIRE(ctx, f->fv.feat[j] >= 0 && f->fv.feat[j] < f->n, "frame feature index");
    std::vector<uint8_t> qdesc((size_t)n * 32);
    std::vector<int32_t> q_mp(n);
    std::vector<float> q_angle(n);
    for (int i = 0; i < n; i++) {
        std::memcpy(&qdesc[(size_t)i * 32], kf->desc + (size_t)q_feat[i] * 32, 32);
        q_mp[i] = kf->mp_id[q_feat[i]];
        q_angle[i] = kf->angle[q_feat[i]];
    }
    MatchArgs A = {};
    osg_packer pk;
    A.nq = n;
    A.n_slots = f->n;
    A.nleft = f->nleft;
    set_off(A.fdesc, pk.add(f->desc, (size_t)f->n * 32));
    set_off(A.slot_angle, pk.add(f->angle, sizeof(float) * f->n));
    set_off(A.qdesc, pk.add(qdesc.data(), qdesc.size()));
    set_off(A.q_mp, pk.add(q_mp.data(), sizeof(int32_t) * n));
    set_off(A.q_angle, pk.add(q_angle.data(), sizeof(float) * n));
    set_off(A.q_cb, pk.add(q_cb.data(), sizeof(int32_t) * n));
    set_off(A.q_ce, pk.add(q_ce.data(), sizeof(int32_t) * n));
    set_off(A.cand_list, pk.add(f->fv.feat, sizeof(int32_t) * f->fv.node_start[f->fv.n_nodes]));
    A.nnratio = nnratio;
    A.check_ori = check_orientation;
    return launch_packed<MODE_BOW_KF_F>(ctx, A, pk, out_mp, f->n, nullptr);
}

int osg_search_by_bow_kf_kf(osg_ctx *ctx, const osg_bow_side *kf1, const osg_bow_side *kf2, float nnratio,
                            int check_orientation, int32_t *out_mp12)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, kf1 && kf2 && out_mp12, "null argument");
    OSG_REQUIRE(ctx, kf2->n >= 0 && kf2->n <= MAX_SLOTS && kf1->n >= 0, "sizes");
    OSG_REQUIRE(ctx, kf1->nleft == -1 || (kf1->nleft >= 0 && kf1->nleft <= kf1->n), "kf1 nleft");
    OSG_REQUIRE(ctx, kf2->nleft == -1 || (kf2->nleft >= 0 && kf2->nleft <= kf2->n), "kf2 nleft");
    for (int i = 0; i < kf1->n; i++) out_mp12[i] = -1;
    std::vector<int32_t> q_feat, q_cb, q_ce;
    if (bow_queries(kf1, kf2, true, q_feat, q_cb, q_ce) < 0) return osg_set_error(ctx, OSG_E_INVALID, "feature index");
    const int n = (int)q_feat.size();
    if (n == 0) return 0;
    for (int j = 0; j < kf2->fv.node_start[kf2->fv.n_nodes]; j++)
        OSG_REQUIRE(ctx, kf2->fv.feat[j] >= 0 && kf2->fv.feat[j] < kf2->n, "keyframe feature index");
    std::vector<uint8_t> qdesc((size_t)n * 32), slot_ok(kf2->n);
    std::vector<float> q_angle(n);
    for (int i = 0; i < n; i++) {
        std::memcpy(&qdesc[(size_t)i * 32], kf1->desc + (size_t)q_feat[i] * 32, 32);
        q_angle[i] = kf1->angle[q_feat[i]];
    }
    // right-camera keypoints of a two-camera KF2 are skipped (ref:src/ORBmatcher.cc:953-955)
    for (int s = 0; s < kf2->n; s++)
        slot_ok[s] = (kf2->mp_id[s] >= 0 && kf2->mp_good[s] && (kf2->nleft == -1 || s < kf2->nleft)) ? 1 : 0;
    MatchArgs A = {};
    osg_packer pk;
    A.nq = n;
    A.n_slots = kf2->n;
    A.nleft = -1;
    set_off(A.fdesc, pk.add(kf2->desc, (size_t)kf2->n * 32));
    set_off(A.slot_angle, pk.add(kf2->angle, sizeof(float) * kf2->n));
    set_off(A.slot_mp2, pk.add(kf2->mp_id, sizeof(int32_t) * kf2->n));
    set_off(A.slot_ok, pk.add(slot_ok.data(), slot_ok.size()));
    set_off(A.qdesc, pk.add(qdesc.data(), qdesc.size()));
    set_off(A.q_angle, pk.add(q_angle.data(), sizeof(float) * n));
    set_off(A.q_cb, pk.add(q_cb.data(), sizeof(int32_t) * n));
    set_off(A.q_ce, pk.add(q_ce.data(), sizeof(int32_t) * n));
    set_off(A.cand_list, pk.add(kf2->fv.feat, sizeof(int32_t) * kf2->fv.node_start[kf2->fv.n_nodes]));
    A.nnratio = nnratio;
    A.check_ori = check_orientation;
    std::vector<int32_t> out_q(n, -1);
    const int nm = launch_packed<MODE_BOW_KF_KF>(ctx, A, pk, nullptr, 0, out_q.data());
    if (nm < 0) return nm;
    for (int i = 0; i < n; i++) out_mp12[q_feat[i]] = out_q[i];
    return nm;
}

}  // extern "C"
