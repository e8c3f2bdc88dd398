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
#include <chrono>
#include <deque>
#include <type_traits>
#include <string>

#include "match_common.h"

// Every MatchArgs array lives in global memory; typing the pointers so (address space 1) makes the
// compiler emit global_load / global_store instead of flat accesses for pointers read from the
// per-problem argument array.
#define GLOBAL __attribute__((address_space(1)))
// native vector types (the HIP vector classes cannot be copied through such pointers on the host pass)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

enum { MODE_MPS = 0, MODE_LAST = 1, MODE_KF = 2, MODE_BOW_KF_F = 3, MODE_BOW_KF_KF = 4 };

constexpr int MT = 1024;               // threads per problem
constexpr int MAX_SLOTS = 8192;        // LDS claim arrays
constexpr int INT_BIG = 0x7FFFFFFF;

struct MatchArgs {
    int nq, n_slots;
    int nleft;                // slot side: Frame::Nleft (-1: one camera / rectified stereo)
    // slot side (Frame F / KeyFrame 2)
    GLOBAL const uint32_t *fdesc;
    GLOBAL const float *kp_x, *kp_y, *slot_angle;
    GLOBAL const int32_t *kp_octave;
    GLOBAL const float *u_right;     // NULL for a two-camera rig (the u_R check needs Nleft == -1)
    GLOBAL const int32_t *grid_start, *grid_idx;
    GLOBAL const int32_t *grid_start_r, *grid_idx_r;   // mGridRight, indices relative to nleft
    GLOBAL const int32_t *l2r, *r2l;                    // mvLeftToRightMatch / mvRightToLeftMatch
    float min_x, max_x, min_y, max_y, inv_w, inv_h;
    GLOBAL const float *scale;
    int n_levels;
    float mb, mbf;
    // queries
    GLOBAL const uint32_t *qdesc;
    GLOBAL const int32_t *q_mp;
    GLOBAL const uint8_t *q_has_obs;
    GLOBAL const float *q_angle;
    GLOBAL const float *q_x, *q_y, *q_f0, *q_f1, *q_f2;
    GLOBAL const int32_t *q_lvl;
    GLOBAL const uint8_t *q_m0, *q_m1;
    // right-camera query fields (two-camera rig)
    GLOBAL const float *q_xr, *q_yr, *q_f0r;
    GLOBAL const int32_t *q_lvl_r;
    GLOBAL const uint8_t *q_m0r;
    GLOBAL const int32_t *q_cb, *q_ce, *cand_list;
    GLOBAL const uint8_t *slot_ok;
    GLOBAL const int32_t *slot_mp2;  // KF-KF: KF2 MapPoint ids
    // parameters
    float nnratio, th, th_far, tlc_z;
    int far_points, orb_dist, check_ori, mono;
    // state / outputs
    GLOBAL int32_t *slot_mp;         // in/out (out_mp for KF-F)
    GLOBAL const uint8_t *slot_taken;
    GLOBAL int32_t *out_q;           // KF-KF: per query result
    // scratch
    GLOBAL int32_t *q_off;           // nq + 1: candidate CSR
    GLOBAL int32_t *q_mid;           // nq: first right-camera candidate of each query
    GLOBAL f32x4 *q_win;            // 4 nq: left / right search windows (grid modes)
    GLOBAL uint32_t *cands;
    GLOBAL int32_t *q_res;           // 2 nq: {left slot, right slot}, -1 = no match
    GLOBAL uint8_t *q_bin;           // 2 nq
    GLOBAL int32_t *status;          // [0] candidates, [1] nmatches, [2] rounds, [3] overflow, [4] serial
    int cap;
    int lds_free;                    // dynamic LDS bytes past the resolve arrays (the staged grid region)
    int prefilled;                   // SearchByBoW: k_bow_fill wrote q_off (host CSR), cands and the first q_res;
                                     // k_bow_claims / k_bow_round ran the first Jacobi round (status[13]: changed)
    GLOBAL int32_t *claim_g;         // SearchByBoW: n_slots claims of the first round (global scratch)
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

__device__ __forceinline__ uint4 ld4(GLOBAL const uint32_t *p)
{
    const u32x4 v = *(GLOBAL const u32x4 *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ld4(const uint32_t *p) { return *(const uint4 *)p; }

template <typename P>
__device__ __forceinline__ uint32_t dist256(const uint32_t (&a)[8], P b)
{
    const uint4 b0 = ld4(b), b1 = ld4(b + 4);
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

// Search window of the left (or only) camera pass.  Every query field is loaded before any test
// (selects, no branches), so a query costs one round of memory latency, not one per field.
template <int MODE>
__device__ __forceinline__ Win query_window(const MatchArgs &A, int q)
{
    Win w;
    w.stereo = false;
    w.sx = 0.f;
    w.sr = 0.f;
    const int nl1 = A.n_levels - 1;
    if (MODE == MODE_MPS) {
        // ref:src/ORBmatcher.cc:55-80
        const bool in_view = A.q_m0[q] != 0, usable = A.q_m1[q] != 0;   // mbTrackInView, !isBad()
        const float depth = A.q_f2[q], vcos = A.q_f0[q];
        const float x = A.q_x[q], y = A.q_y[q], xr = A.q_f1[q];
        const int lvl = A.q_lvl[q];
        const float sc = A.scale[min(max(lvl, 0), nl1)];
        w.valid = in_view && !(A.far_points && depth > A.th_far) && usable;
        float r = radius_by_viewing_cos(vcos);
        if (A.th != 1.0f) r *= A.th;
        w.r = r * sc;
        w.x = x;
        w.y = y;
        w.minL = lvl - 1;
        w.maxL = lvl;
        w.stereo = true;
        w.sx = xr;          // mTrackProjXR
        w.sr = w.r;         // r * mvScaleFactors[nPredictedLevel]
    } else if (MODE == MODE_LAST) {
        // ref:src/ORBmatcher.cc:1984-2030
        const bool valid = A.q_m0[q] != 0;
        const float invzc = A.q_f0[q];
        const float u = A.q_x[q], v = A.q_y[q];
        const int oct = A.q_lvl[q];
        const float sc = A.scale[min(max(oct, 0), nl1)];
        w.valid = valid && !(invzc < 0) && !(u < A.min_x || u > A.max_x) && !(v < A.min_y || v > A.max_y);
        const float radius = A.th * sc;
        const bool bForward = A.tlc_z > A.mb && !A.mono;
        const bool bBackward = -A.tlc_z > A.mb && !A.mono;
        w.minL = bForward ? oct : bBackward ? 0 : oct - 1;
        w.maxL = bForward ? -1 : bBackward ? oct : oct + 1;
        w.x = u;
        w.y = v;
        w.r = radius;
        w.stereo = true;
        const float prod = A.mbf * invzc;
        w.sx = u - prod;   // ur = uv(0) - mbf * invzc
        w.sr = radius;
    } else {
        // MODE_KF, ref:src/ORBmatcher.cc:2262-2265
        const bool valid = A.q_m0[q] != 0;
        const int lvl = A.q_lvl[q];
        const float x = A.q_x[q], y = A.q_y[q];
        const float sc = A.scale[min(max(lvl, 0), nl1)];
        w.valid = valid;
        w.r = A.th * sc;
        w.x = x;
        w.y = y;
        w.minL = lvl - 1;
        w.maxL = lvl + 1;
    }
    return w;
}

// Search window of the right-camera pass of a two-camera rig.  For a6 the pass is also skipped when
// the left window was empty (:2040-2041 'continue'); enumeration applies that rule.
template <int MODE>
__device__ __forceinline__ Win query_window_r(const MatchArgs &A, int q, const Win &wl)
{
    Win w;
    w.valid = false;
    w.stereo = false;
    w.sx = 0.f;
    w.sr = 0.f;
    w.x = w.y = w.r = 0.f;
    w.minL = w.maxL = 0;
    if (A.nleft < 0) return w;
    if (MODE == MODE_MPS) {
        // ref:src/ORBmatcher.cc:185-196: mbTrackInViewR, mnTrackScaleLevelR != -1, radius from
        // mTrackViewCosR (no th factor), levels (lvl-1, lvl), right grid at mTrackProjXR/YR
        const bool in_view_r = A.q_m0r[q] != 0, usable = A.q_m1[q] != 0;
        const float depth = A.q_f2[q], vcos = A.q_f0r[q];
        const float x = A.q_xr[q], y = A.q_yr[q];
        const int lvl = A.q_lvl_r[q];
        const float sc = A.scale[min(max(lvl, 0), A.n_levels - 1)];
        w.valid = in_view_r && !(A.far_points && depth > A.th_far) && usable && lvl != -1;
        w.r = radius_by_viewing_cos(vcos) * sc;
        w.x = x;
        w.y = y;
        w.minL = lvl - 1;
        w.maxL = lvl;
    } else if (MODE == MODE_LAST) {
        // ref:src/ORBmatcher.cc:2096-2110: same radius and levels at the right-camera projection
        const float x = A.q_xr[q], y = A.q_yr[q];
        w = wl;
        w.x = x;
        w.y = y;
        w.stereo = false;
    }
    return w;
}

// Windows are computed once per query (phase 0) and kept as two float4 each.
__device__ __forceinline__ void store_win(GLOBAL f32x4 *dst, const Win &w)
{
    dst[0] = f32x4{w.x, w.y, w.r, w.sx};
    dst[1] = f32x4{w.sr, __int_as_float(w.minL), __int_as_float(w.maxL),
                   __int_as_float((w.valid ? 1 : 0) | (w.stereo ? 2 : 0))};
}
__device__ __forceinline__ Win load_win(GLOBAL const f32x4 *src)
{
    const f32x4 a = src[0], b = src[1];
    Win w;
    w.x = a.x;
    w.y = a.y;
    w.r = a.z;
    w.sx = a.w;
    w.sr = b.x;
    w.minL = __float_as_int(b.y);
    w.maxL = __float_as_int(b.z);
    const int f = __float_as_int(b.w);
    w.valid = (f & 1) != 0;
    w.stereo = (f & 2) != 0;
    return w;
}

// Where a grid walk reads the frame.  STAGE 0: the frame's own arrays in global memory; STAGE 1:
// per-entry records in grid order staged in LDS; STAGE 2: also the descriptors in LDS.
template <int STAGE>
struct GridView {
    using GsPtr = std::conditional_t<(STAGE >= 1), const int32_t *, GLOBAL const int32_t *>;
    using FdPtr = std::conditional_t<(STAGE >= 2), const uint32_t *, GLOBAL const uint32_t *>;
    GsPtr gs;                   // cell offsets, OSG_GRID_CELLS + 1
    GLOBAL const int32_t *gi;   // STAGE 0: keypoint index relative to the camera
    int off;                    // STAGE 0: slot offset (nleft for the right grid)
    const float *rx, *ry, *ru;  // STAGE >= 1: x, y, u_R (or -1) of each grid entry
    const int32_t *rk;          // STAGE >= 1: slot << 8 | octave of each grid entry
    FdPtr fd;                   // descriptors by slot
};

// Frame::GetFeaturesInArea (ref:src/Frame.cc:868-962) + the caller's static per-candidate skips.
// The cells (ix, minCY..maxCY) of one column are consecutive in the CSR (cell = ix*48 + iy), so
// each column is ONE contiguous run in the reference's iy-then-insertion order.  Candidates are
// written as slot indices (right keypoints at nleft + i).
template <bool FILL, int STAGE, bool RIGHT>
__device__ __forceinline__ int enum_grid(const MatchArgs &A, const GridView<STAGE> &G, const Win &w,
                                         const uint32_t (&qd)[8], GLOBAL uint32_t *out)
{
    constexpr bool STAGED = STAGE >= 1;
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
    const bool stereo = !RIGHT && w.stereo && A.u_right;      // u_R check (one-camera frames only)
    int cnt = 0;
    for (int ix = minCX; ix <= maxCX; ix++) {
        const int j0 = G.gs[ix * OSG_GRID_ROWS + minCY], j1 = G.gs[ix * OSG_GRID_ROWS + maxCY + 1];
        for (int j = j0; j < j1; j++) {
            int k, oct;
            float x, y;
            if (STAGED) {
                const int r = G.rk[j];
                k = r >> 8;
                oct = r & 0xFF;
                x = G.rx[j];
                y = G.ry[j];
            } else {
                k = G.gi[j] + G.off;
                oct = A.kp_octave[k];
                x = A.kp_x[k];
                y = A.kp_y[k];
            }
            if (bCheckLevels) {
                if (oct < w.minL) continue;
                if (w.maxL >= 0 && oct > w.maxL) continue;
            }
            const float distx = x - w.x;
            const float disty = y - w.y;
            if (!(fabsf(distx) < factorX && fabsf(disty) < factorY)) continue;
            if (stereo) {
                const float ur = STAGED ? G.ru[j] : A.u_right[k];
                if (ur > 0) {
                    const float er = fabsf(w.sx - ur);
                    if (er > w.sr) continue;
                }
            }
            if (FILL) {
                const uint32_t d = dist256(qd, G.fd + (size_t)k * 8);
                out[cnt] = (uint32_t)k | (d << 16) | ((uint32_t)(oct & 0x7F) << 25);
            }
            cnt++;
        }
    }
    return cnt;
}

__device__ __forceinline__ void load_desc(const MatchArgs &A, int q, uint32_t (&qd)[8])
{
    const uint4 a = ld4(A.qdesc + (size_t)q * 8);
    const uint4 b = ld4(A.qdesc + (size_t)q * 8 + 4);
    qd[0] = a.x; qd[1] = a.y; qd[2] = a.z; qd[3] = a.w;
    qd[4] = b.x; qd[5] = b.y; qd[6] = b.z; qd[7] = b.w;
}

// Candidates of grid-mode query q from its precomputed windows: left-camera ones first, then
// right-camera ones; cl = left count.
template <int MODE, bool FILL, int STAGE>
__device__ __forceinline__ int enum_query(const MatchArgs &A, const GridView<STAGE> &GL, const GridView<STAGE> &GR,
                                          int q, GLOBAL uint32_t *out, int &cl)
{
    uint32_t qd[8];
    if (FILL) load_desc(A, q, qd);
    const Win w = load_win(A.q_win + 4 * (size_t)q);
    const int c0 = w.valid ? enum_grid<FILL, STAGE, false>(A, GL, w, qd, out) : 0;
    cl = c0;
    int c1 = 0;
    if ((MODE == MODE_MPS || MODE == MODE_LAST) && A.nleft >= 0 && (MODE != MODE_LAST || c0 > 0)) {
        const Win wr = load_win(A.q_win + 4 * (size_t)q + 2);
        if (wr.valid) c1 = enum_grid<FILL, STAGE, true>(A, GR, wr, qd, FILL ? out + c0 : nullptr);
    }
    return c0 + c1;
}

// SearchByBoW candidates: the other side's feature list of the query's vocabulary node, in list
// order.  BOW_G lanes share one query.  A KF-KF candidate without a usable MapPoint (or a right-
// camera keypoint) keeps its position with distance 0x1FF, which evaluation skips.
constexpr int BOW_G = 16;

template <int MODE>
__device__ __forceinline__ void fill_bow_group(const MatchArgs &A, int q, int lane)
{
    uint32_t qd[8];
    load_desc(A, q, qd);
    const int cb = A.q_cb[q], ce = A.q_ce[q];
    GLOBAL uint32_t *out = A.cands + A.q_off[q] - cb;
    for (int j = cb + lane; j < ce; j += BOW_G) {
        const int idx = A.cand_list[j];
        uint32_t d = dist256(qd, A.fdesc + (size_t)idx * 8);
        if (MODE == MODE_BOW_KF_KF && !A.slot_ok[idx]) d = 0x1FF;  // !pMP2 || isBad || right camera
        out[j] = (uint32_t)idx | (d << 16);
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

// One grid-mode query in reference order.  blocked(s): is slot s unavailable to q given the
// assignments of the queries before q (Jacobi: claims of the previous round; serial: the live slot
// state).
template <int MODE, typename Blocked>
__device__ __forceinline__ QRes eval_query(const MatchArgs &A, int q, Blocked blocked)
{
    QRes res{-1, -1};
    const int e0 = A.q_off[q], em = A.q_mid[q], e1 = A.q_off[q + 1];
    Top2 L, R;
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
    } else {  // MODE_KF, ref:src/ORBmatcher.cc:2287
        acc = L.best <= A.orb_dist;
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

// top-2 of packed keys (distance << 16 | position in the query's list).  Keys are distinct, and
// their order is the reference loop's (distance, then enumeration order): the first key is
// (bestDist, bestIdx), the second is bestDist2 with multiplicity.
constexpr uint32_t KEY_NONE = (256u << 16) | 0xFFFFu;

__device__ __forceinline__ void push2(uint32_t &a1, uint32_t &a2, uint32_t k)
{
    const uint32_t hi = max(a1, k);
    a1 = min(a1, k);
    a2 = min(a2, hi);
}

__device__ __forceinline__ void merge2(uint32_t &a1, uint32_t &a2, int o)
{
    const uint32_t b1 = (uint32_t)__shfl_xor((int)a1, o), b2 = (uint32_t)__shfl_xor((int)a2, o);
    const uint32_t hi = max(a1, b1);
    a1 = min(a1, b1);
    a2 = min(min(a2, b2), hi);
}

// One SearchByBoW query evaluated by the BOW_G lanes of a group (every lane returns the result).
// ref:src/ORBmatcher.cc:316-441 (KF-F: separate left / right top-2 on a two-camera frame) and
// :960-987 (KF-KF).
template <int MODE, typename Blocked>
__device__ __forceinline__ QRes eval_bow_group(const MatchArgs &A, int q, int lane, Blocked blocked)
{
    const int e0 = A.q_off[q], e1 = A.q_off[q + 1];
    uint32_t l1 = KEY_NONE, l2 = KEY_NONE, r1 = KEY_NONE, r2 = KEY_NONE;
    // BK candidates per lane at a time, all loads issued before the first use: one memory latency
    // per BK x BOW_G candidates instead of one per candidate
    constexpr int BK = 8;
    for (int base = e0 + lane; base < e1; base += BK * BOW_G) {
        uint32_t cv[BK];
#pragma unroll
        for (int k = 0; k < BK; k++) {
            const int e = base + k * BOW_G;
            cv[k] = e < e1 ? A.cands[e] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int k = 0; k < BK; k++) {
            const int e = base + k * BOW_G;
            const uint32_t c = cv[k];
            const int s = (int)(c & 0xFFFFu);
            const uint32_t d = (c >> 16) & 0x1FFu;
            if (e >= e1 || d > 256 || blocked(s)) continue;
            const uint32_t key = (d << 16) | (uint32_t)(e - e0);
            if (MODE == MODE_BOW_KF_KF || A.nleft < 0 || s < A.nleft) push2(l1, l2, key);
            else push2(r1, r2, key);
        }
    }
#pragma unroll
    for (int o = BOW_G / 2; o > 0; o >>= 1) {
        merge2(l1, l2, o);
        if (MODE == MODE_BOW_KF_F) merge2(r1, r2, o);
    }
    const int best = (int)(l1 >> 16), second = (int)(l2 >> 16);
    QRes res{-1, -1};
    if (MODE == MODE_BOW_KF_F) {
        if (best <= OSG_TH_LOW) {
            if ((float)best < A.nnratio * (float)second) res.l = (int)(A.cands[e0 + (l1 & 0xFFFFu)] & 0xFFFFu);
            if ((int)(r1 >> 16) <= OSG_TH_LOW)  // ratio disabled by '|| true' (:425)
                res.r = (int)(A.cands[e0 + (r1 & 0xFFFFu)] & 0xFFFFu);
        }
    } else {
        if (best < OSG_TH_LOW && (float)best < A.nnratio * (float)second)
            res.l = (int)(A.cands[e0 + (l1 & 0xFFFFu)] & 0xFFFFu);
    }
    return res;
}

// SearchByBoW's distances and first evaluation spread over the chip: one BOW_G-lane group per
// query, BFG queries per workgroup, grid (ceil(max nq / BFG), problems).  The candidate CSR (q_off)
// comes from the host's merge-walk, so no count / scan pass is needed; each group writes its
// query's {slot | dist << 16} list and its unclaimed top-2 result, which k_match's resolve starts
// from (no slot is taken before a SearchByBoW call: every first evaluation sees blocked(s) = false).
constexpr int BFG = 16;
template <int MODE>
__global__ __launch_bounds__(BFG *BOW_G) void k_bow_fill(const MatchArgs *__restrict__ args)
{
    const MatchArgs &A = args[blockIdx.y];
    for (int sl = blockIdx.x * blockDim.x + threadIdx.x; sl < A.n_slots; sl += gridDim.x * blockDim.x)
        A.claim_g[sl] = INT_BIG;
    const int lane = threadIdx.x & (BOW_G - 1);
    const int q = blockIdx.x * BFG + threadIdx.x / BOW_G;
    if (q >= A.nq) return;
    uint32_t qd[8];
    load_desc(A, q, qd);
    const int cb = A.q_cb[q], ce = A.q_ce[q];
    GLOBAL uint32_t *out = A.cands + A.q_off[q] - cb;
    for (int j = cb + lane; j < ce; j += BOW_G) {
        const int idx = A.cand_list[j];
        uint32_t d = dist256(qd, A.fdesc + (size_t)idx * 8);
        if (MODE == MODE_BOW_KF_KF && !A.slot_ok[idx]) d = 0x1FF;
        out[j] = (uint32_t)idx | (d << 16);
    }
    // each lane reads back the entries it wrote (the same strides), so no barrier is needed
    const QRes r = eval_bow_group<MODE>(A, q, lane, [](int) { return false; });
    if (lane == 0) {
        A.q_res[2 * q] = r.l;
        A.q_res[2 * q + 1] = r.r;
    }
}

// The first Jacobi round of SearchByBoW's resolve (see k_match) over the chip: every query's
// assigned slots claimed (device-scope atomicMin, order-independent), then every query re-evaluated
// with blocked(s) = claimed by an earlier query.  k_match continues from these results and skips
// its rounds when nothing changed.
template <int MODE>
__global__ __launch_bounds__(256) void k_bow_claims(const MatchArgs *__restrict__ args)
{
    const MatchArgs &A = args[blockIdx.y];
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= A.nq) return;
    const QRes r = QRes{A.q_res[2 * q], A.q_res[2 * q + 1]};
    if (r.l >= 0) atomicMin((int32_t *)&A.claim_g[r.l], q);
    if (r.r >= 0) atomicMin((int32_t *)&A.claim_g[r.r], q);
}
template <int MODE>
__global__ __launch_bounds__(BFG *BOW_G) void k_bow_round(const MatchArgs *__restrict__ args)
{
    const MatchArgs &A = args[blockIdx.y];
    const int lane = threadIdx.x & (BOW_G - 1);
    const int q = blockIdx.x * BFG + threadIdx.x / BOW_G;
    if (q >= A.nq) return;
    const QRes r1 = QRes{A.q_res[2 * q], A.q_res[2 * q + 1]};
    const QRes r2 = eval_bow_group<MODE>(A, q, lane, [&](int s) { return A.claim_g[s] < q; });
    if (lane == 0 && (r2.l != r1.l || r2.r != r1.r)) {
        A.q_res[2 * q] = r2.l;
        A.q_res[2 * q + 1] = r2.r;
        atomicOr((int32_t *)&A.status[13], 1);
    }
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

// SearchByProjection's (a5 / a6 / a7) search windows, candidate counts, candidate fill and first
// evaluation spread over the chip, for launches of a few problems (the drop-in's one-frame call):
// one thread per query, grid (ceil(max nq / GQ), problems), and one workgroup per problem for the
// exclusive scan between them.  k_match then starts its Jacobi rounds from these results
// (prefilled), so a lone frame no longer walks its queries' grids on one CU.  The enumeration and
// the evaluation are k_match's own functions on the frame's global arrays (GridView<0>), so the
// candidate lists and the first results are the ones k_match forms itself.
constexpr int GRID_PREPASS_MAX_B = 64;  // launches of up to this many problems take the prepass
constexpr int GQG = 16;                   // queries per prepass workgroup (BOW_G lanes each)
template <int MODE>
__device__ __forceinline__ bool taken_init(const MatchArgs &A, int s)
{
    if (MODE == MODE_MPS || MODE == MODE_LAST) return A.slot_mp[s] >= 0 && A.slot_taken[s];
    return A.slot_mp[s] >= 0;  // MODE_KF
}
// enum_grid<STAGE 0> with the BOW_G lanes of a group sharing one query: each column run of the
// window is read BOW_G entries at a time, one per lane, and the passing entries keep the run's
// order through a ballot prefix (every lane returns the count; FILL writes the candidates).
template <bool FILL, bool RIGHT>
__device__ __forceinline__ int enum_grid_group(const MatchArgs &A, const Win &w, const uint32_t (&qd)[8],
                                               GLOBAL uint32_t *out, int lane)
{
    GLOBAL const int32_t *gs = RIGHT ? A.grid_start_r : A.grid_start;
    GLOBAL const int32_t *gi = RIGHT ? A.grid_idx_r : A.grid_idx;
    const int koff = RIGHT ? A.nleft : 0;
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
    const bool stereo = !RIGHT && w.stereo && A.u_right;
    const int gshift = (threadIdx.x & 63) & ~(BOW_G - 1);     // the group's first lane in the wave
    int cnt = 0;
    for (int ix = minCX; ix <= maxCX; ix++) {
        const int j0 = gs[ix * OSG_GRID_ROWS + minCY], j1 = gs[ix * OSG_GRID_ROWS + maxCY + 1];
        for (int jb = j0; jb < j1; jb += BOW_G) {
            const int j = jb + lane;
            bool pass = false;
            int k = 0, oct = 0;
            if (j < j1) {
                k = gi[j] + koff;
                oct = A.kp_octave[k];
                const float x = A.kp_x[k], y = A.kp_y[k];
                pass = !(bCheckLevels && (oct < w.minL || (w.maxL >= 0 && oct > w.maxL)));
                const float distx = x - w.x, disty = y - w.y;
                pass = pass && fabsf(distx) < factorX && fabsf(disty) < factorY;
                if (stereo && pass) {
                    const float ur = A.u_right[k];
                    if (ur > 0 && fabsf(w.sx - ur) > w.sr) pass = false;
                }
            }
            const uint32_t m = (uint32_t)(__ballot(pass) >> gshift) & ((1u << BOW_G) - 1);
            if (FILL && pass) {
                const uint32_t d = dist256(qd, A.fdesc + (size_t)k * 8);
                out[cnt + __builtin_popcount(m & ((1u << lane) - 1))] =
                    (uint32_t)k | (d << 16) | ((uint32_t)(oct & 0x7F) << 25);
            }
            cnt += __builtin_popcount(m);
        }
    }
    return cnt;
}
// enum_query for a group, from the query's windows: left-camera candidates, then right-camera ones;
// cl = left count
template <int MODE, bool FILL>
__device__ __forceinline__ int enum_query_group(const MatchArgs &A, int q, const Win &w, const Win &wr,
                                                GLOBAL uint32_t *out, int &cl, int lane)
{
    uint32_t qd[8];
    if (FILL) load_desc(A, q, qd);
    const int c0 = w.valid ? enum_grid_group<FILL, false>(A, w, qd, out, lane) : 0;
    cl = c0;
    int c1 = 0;
    if ((MODE == MODE_MPS || MODE == MODE_LAST) && A.nleft >= 0 && (MODE != MODE_LAST || c0 > 0))
        if (wr.valid) c1 = enum_grid_group<FILL, true>(A, wr, qd, FILL ? out + c0 : nullptr, lane);
    return c0 + c1;
}
// eval_query for a group: each pass's top-2 over the candidates as packed keys (distance << 16 |
// position), merged across the group — the sequential loop's bestDist / bestDist2 with its tie order
// (see push2) — and the levels read back from the best and second candidates
template <int MODE, typename Blocked>
__device__ __forceinline__ QRes eval_query_group(const MatchArgs &A, int q, int e0, int em, int e1, int lane,
                                                 Blocked blocked)
{
    QRes res{-1, -1};
    auto top2 = [&](int b0, int b1, auto skip, int &best, int &bl, int &second, int &sl, int &bslot) {
        uint32_t k1 = KEY_NONE, k2 = KEY_NONE;
        for (int e = b0 + lane; e < b1; e += BOW_G) {
            const uint32_t c = A.cands[e];
            const int s = (int)(c & 0xFFFFu);
            if (skip(s)) continue;
            push2(k1, k2, (((c >> 16) & 0x1FFu) << 16) | (uint32_t)(e - b0));
        }
#pragma unroll
        for (int o = BOW_G / 2; o > 0; o >>= 1) merge2(k1, k2, o);
        best = (int)(k1 >> 16);
        second = (int)(k2 >> 16);
        // Top2::push takes a candidate only below 256: one at 256 leaves the defaults (-1)
        const uint32_t c1 = best < 256 ? A.cands[b0 + (k1 & 0xFFFFu)] : 0u;
        const uint32_t c2 = second < 256 ? A.cands[b0 + (k2 & 0xFFFFu)] : 0u;
        bl = best < 256 ? (int)(c1 >> 25) : -1;
        bslot = best < 256 ? (int)(c1 & 0xFFFFu) : -1;
        sl = second < 256 ? (int)(c2 >> 25) : -1;
        if (best >= 256) best = 256;
        if (second >= 256) second = 256;
    };
    int best, bl, second, sl, bslot;
    top2(e0, em, [&](int s) { return blocked(s); }, best, bl, second, sl, bslot);
    bool acc, skip_r = false;
    if (MODE == MODE_MPS) {  // ref:src/ORBmatcher.cc:147-167
        acc = best <= OSG_TH_HIGH && !(bl == sl && (float)best > A.nnratio * (float)second);
        skip_r = best <= OSG_TH_HIGH && !acc;
    } else if (MODE == MODE_LAST) {  // ref:src/ORBmatcher.cc:2070
        acc = best <= OSG_TH_HIGH;
    } else {  // MODE_KF, ref:src/ORBmatcher.cc:2287
        acc = best <= A.orb_dist;
    }
    res.l = acc ? bslot : -1;
    if ((MODE == MODE_MPS || MODE == MODE_LAST) && em < e1 && !skip_r) {
        int own = -1;
        bool own_blocked = false;
        if (MODE == MODE_MPS && res.l >= 0 && A.l2r) {
            const int t = A.l2r[res.l];
            if (t != -1) {
                own = t + A.nleft;
                own_blocked = A.q_has_obs[q] != 0;
            }
        }
        top2(em, e1, [&](int s) { return s == own ? own_blocked : blocked(s); }, best, bl, second, sl, bslot);
        bool accr;
        if (MODE == MODE_MPS)  // ref:src/ORBmatcher.cc:222-238
            accr = best <= OSG_TH_HIGH && !(bl == sl && (float)best > A.nnratio * (float)second);
        else  // ref:src/ORBmatcher.cc:2133
            accr = best <= OSG_TH_HIGH;
        res.r = accr ? bslot : -1;
    }
    return res;
}
// The prepass in one launch.  Each workgroup counts its queries' candidates and publishes the sum in flags[workgroup] (the call's epoch in the high word, so the
// buffer needs no clearing), then takes its offset as the sum of its predecessors' published counts
// (wave 0 reads 64 flags at a time) and fills and evaluates its queries.  A wait that
// never ends (it cannot, short of a hardware fault) is bounded and reported in status[3] bit 2.
template <int MODE>
__global__ __launch_bounds__(GQG *BOW_G) void k_grid_prepass(const MatchArgs *__restrict__ args,
                                                             unsigned long long *__restrict__ flags, int flag_stride,
                                                             unsigned epoch)
{
    const MatchArgs &A = args[blockIdx.y];
    unsigned long long *F = flags + (size_t)blockIdx.y * flag_stride;
    __shared__ int s_cnt[GQG];
    __shared__ int s_base;
    const int lane = threadIdx.x & (BOW_G - 1), g = threadIdx.x / BOW_G;
    __shared__ int s_wg;
    const int nwg = (A.nq + GQG - 1) / GQG;
    if ((int)blockIdx.x >= nwg) return;  // the whole workgroup
    // the workgroup's place in the order comes from a ticket (status[14], zeroed with the call's
    // status), not blockIdx: a workgroup then only waits for ones that have started
    if (threadIdx.x == 0) s_wg = atomicAdd((int *)&A.status[14], 1);
    __syncthreads();
    const int wg = s_wg;
    const int q = wg * GQG + g;
    const bool valid = q < A.nq;
    const bool two = (MODE == MODE_MPS || MODE == MODE_LAST) && A.nleft >= 0;
    Win wl{}, wr{};
    int c = 0, cl = 0;
    if (valid) {
        wl = query_window<MODE>(A, q);
        wr = two ? query_window_r<MODE>(A, q, wl) : wl;
        if (lane == 0) {  // for k_match's serial redo
            store_win(A.q_win + 4 * (size_t)q, wl);
            if (two) store_win(A.q_win + 4 * (size_t)q + 2, wr);
        }
        c = enum_query_group<MODE, false>(A, q, wl, wr, nullptr, cl, lane);
    }
    if (lane == 0) s_cnt[g] = c;
    __syncthreads();
    int agg = 0;
#pragma unroll
    for (int i = 0; i < GQG; i++) agg += s_cnt[i];
    if (threadIdx.x == 0)
        __hip_atomic_store(&F[wg], ((unsigned long long)epoch << 32) | (unsigned)agg, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 64) {
        int sum = 0;
        bool stuck = false;
        for (int base = 0; base < wg; base += 64) {
            const int i = base + (int)threadIdx.x;
            int v = 0;
            if (i < wg) {
                unsigned long long f;
                int spins = 0;
                do {
                    f = __hip_atomic_load(&F[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                } while ((unsigned)(f >> 32) != epoch && ++spins < (1 << 22));
                stuck |= (unsigned)(f >> 32) != epoch;
                v = (int)(unsigned)f;
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
            sum += v;
        }
        if (__ballot(stuck) && threadIdx.x == 0) atomicOr((int *)&A.status[3], 2);
        if (threadIdx.x == 0) s_base = sum;
    }
    __syncthreads();
    int off = s_base;
    for (int i = 0; i < g; i++) off += s_cnt[i];
    if (valid && lane == 0) A.q_off[q] = off;
    if (wg == nwg - 1 && threadIdx.x == 0) {
        const int total = s_base + agg;
        A.q_off[A.nq] = total;
        if (total > A.cap) {  // the host resizes and retries; k_match skips the problem
            A.status[0] = total;
            atomicOr((int *)&A.status[3], 1);
        }
    }
    if (!valid || off + c > A.cap) return;
    int cl2;
    enum_query_group<MODE, true>(A, q, wl, wr, A.cands + off, cl2, lane);
    if (lane == 0) A.q_mid[q] = off + cl;
    // the group reads back the candidates its lanes wrote: their stores complete first (the lanes
    // share the CU's write-through L1)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const QRes r = eval_query_group<MODE>(A, q, off, off + cl, off + c, lane,
                                          [&](int s) { return taken_init<MODE>(A, s); });
    if (lane == 0) store_res(A, q, r);
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

// The serial redo of a5 on a two-camera rig (see the resolve phase) on LDS copies of its inputs:
// eval_query<MODE_MPS> with blocked(s) = taken[s], then the assigned slots' state, query by query.
struct SerialLds {
    const int *off, *mid, *l2r, *r2l;
    const uint32_t *cands;
    const uint8_t *obs;
};
__device__ __forceinline__ QRes eval_mps_lds(const MatchArgs &A, const SerialLds &V, int q, const uint8_t *taken)
{
    QRes res{-1, -1};
    const int e0 = V.off[q], em = V.mid[q], e1 = V.off[q + 1];
    Top2 L, R;
    for (int e = e0; e < em; e++) {
        const uint32_t c = V.cands[e];
        const int s = (int)(c & 0xFFFFu);
        if (taken[s]) continue;
        L.push((int)((c >> 16) & 0x1FFu), (int)(c >> 25), s);
    }
    const bool acc = L.best <= OSG_TH_HIGH && !(L.bl == L.sl && (float)L.best > A.nnratio * (float)L.second);
    const bool skip_r = L.best <= OSG_TH_HIGH && !acc;
    res.l = acc ? L.bslot : -1;
    if (em < e1 && !skip_r) {
        int own = -1;
        bool own_blocked = false;
        if (res.l >= 0) {
            const int t = V.l2r[res.l];
            if (t != -1) {
                own = t + A.nleft;
                own_blocked = V.obs[q] != 0;
            }
        }
        for (int e = em; e < e1; e++) {
            const uint32_t c = V.cands[e];
            const int s = (int)(c & 0xFFFFu);
            if (s == own ? own_blocked : taken[s] != 0) continue;
            R.push((int)((c >> 16) & 0x1FFu), (int)(c >> 25), s);
        }
        const bool accr = R.best <= OSG_TH_HIGH && !(R.bl == R.sl && (float)R.best > A.nnratio * (float)R.second);
        res.r = accr ? R.bslot : -1;
    }
    return res;
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

// Extra LDS of a staged grid-mode launch: cell offsets (one or two grids) + 4 words per keypoint.
constexpr int GS_PAD = (OSG_GRID_CELLS + 1 + 3) & ~3;
// STAGE 1: cell offsets + per-entry records; STAGE 2: also the descriptors (32 B per slot).
__host__ __device__ inline size_t staged_lds_bytes(int ns, bool two_cam, int stage)
{
    if (stage <= 0) return 0;
    size_t b = sizeof(int) * ((size_t)GS_PAD * (two_cam ? 2 : 1) + 4 * (size_t)ns);
    if (stage >= 2) b = ((b + 15) & ~size_t(15)) + 32 * (size_t)ns;
    return b;
}

template <int MODE, int STAGE>
__global__ __launch_bounds__(MT) void k_match(const MatchArgs *__restrict__ args)
{
    constexpr bool BOW = MODE == MODE_BOW_KF_F || MODE == MODE_BOW_KF_KF;
    constexpr bool STAGED = STAGE >= 1;
    const MatchArgs &A = args[blockIdx.x];  // one problem per workgroup
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
    if (nq == 0) return;  // status was zeroed by the host; the slot arrays stay as they are
    const int per = (nq + MT - 1) / MT;
    const int q0 = min(nq, tid * per), q1 = min(nq, q0 + per);
    const int lane = tid & (BOW_G - 1), grp = tid / BOW_G;  // BoW: BOW_G lanes per query
    constexpr int NGRP = MT / BOW_G;
    // phase clocks (s_memtime) for OSG_MATCH_PROFILE: count, scan, fill, init, rounds, finish
    uint64_t tclk[9];
    tclk[0] = __builtin_amdgcn_s_memtime();

    // prefilled: SearchByBoW's k_bow_* or a grid mode's k_grid_* kernels formed the candidate CSR,
    // the candidate lists and the first results (BoW: also the first Jacobi round)
    const bool pre = A.prefilled != 0;
    // ---- 0. grid views; a staged launch copies the grids into LDS as records in grid order
    GridView<STAGE> GL{}, GR{};
    if (!BOW && !pre) {
        if constexpr (STAGED) {
            const bool two = A.nleft >= 0;
            int *gsL = (int *)(removedS + ((NS + 15) & ~15));
            int *gsR = gsL + GS_PAD;
            float *rx = (float *)(gsL + GS_PAD * (two ? 2 : 1));
            float *ry = rx + NS, *ru = ry + NS;
            int *rk = (int *)(ru + NS);
            const int mL = A.grid_start[OSG_GRID_CELLS];
            for (int c = tid; c <= OSG_GRID_CELLS; c += MT) gsL[c] = A.grid_start[c];
            for (int j = tid; j < mL; j += MT) {
                const int k = A.grid_idx[j];
                rx[j] = A.kp_x[k];
                ry[j] = A.kp_y[k];
                ru[j] = A.u_right ? A.u_right[k] : -1.f;
                rk[j] = (k << 8) | A.kp_octave[k];
            }
            if (two) {
                const int mR = A.grid_start_r[OSG_GRID_CELLS];
                for (int c = tid; c <= OSG_GRID_CELLS; c += MT) gsR[c] = A.grid_start_r[c] + mL;
                for (int j = tid; j < mR; j += MT) {
                    const int k = A.grid_idx_r[j] + A.nleft;
                    rx[mL + j] = A.kp_x[k];
                    ry[mL + j] = A.kp_y[k];
                    ru[mL + j] = -1.f;
                    rk[mL + j] = (k << 8) | A.kp_octave[k];
                }
            }
            typename GridView<STAGE>::FdPtr fd;
            if constexpr (STAGE >= 2) {
                u32x4 *fdl = (u32x4 *)(smem + (((uintptr_t)(rk + NS) - (uintptr_t)smem + 15) & ~uintptr_t(15)));
                GLOBAL const u32x4 *src = (GLOBAL const u32x4 *)A.fdesc;
                for (int i = tid; i < 2 * NS; i += MT) fdl[i] = src[i];
                fd = (const uint32_t *)fdl;
            } else {
                fd = A.fdesc;
            }
            GL = GridView<STAGE>{gsL, nullptr, 0, rx, ry, ru, rk, fd};
            GR = GridView<STAGE>{gsR, nullptr, 0, rx, ry, ru, rk, fd};
            __syncthreads();
        } else {
            if constexpr (STAGE == 0) {
                GL = GridView<STAGE>{A.grid_start, A.grid_idx, 0, nullptr, nullptr, nullptr, nullptr, A.fdesc};
                GR = GridView<STAGE>{A.grid_start_r, A.grid_idx_r, A.nleft, nullptr, nullptr, nullptr, nullptr, A.fdesc};
            }
        }
        tclk[1] = __builtin_amdgcn_s_memtime();
        // search windows, computed once; four queries per thread per step with all loads first
        const bool two = (MODE == MODE_MPS || MODE == MODE_LAST) && A.nleft >= 0;
        for (int qb = tid; qb < nq; qb += 4 * MT) {
            Win wl[4], wr[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int q = min(qb + u * MT, nq - 1);
                wl[u] = query_window<MODE>(A, q);
                if (two) wr[u] = query_window_r<MODE>(A, q, wl[u]);
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int q = qb + u * MT;
                if (q < nq) {
                    store_win(A.q_win + 4 * (size_t)q, wl[u]);
                    if (two) store_win(A.q_win + 4 * (size_t)q + 2, wr[u]);
                }
            }
        }
        __syncthreads();
    }

    else {
        tclk[1] = tclk[0];
    }
    tclk[2] = __builtin_amdgcn_s_memtime();
    int total = pre ? A.q_off[nq] : 0;
    if (pre && total > A.cap) return;  // k_grid_prepass flagged the overflow; the host retries
    if (!pre) {
    // ---- 1. count
    int my = 0;
    for (int q = q0; q < q1; q++) {
        int cl;
        const int c = BOW ? A.q_ce[q] - A.q_cb[q] : enum_query<MODE, false, STAGE>(A, GL, GR, q, nullptr, cl);
        A.q_off[q] = c;  // temporarily the count
        my += c;
    }
    __syncthreads();
    tclk[3] = __builtin_amdgcn_s_memtime();
    // ---- 2. block scan (inclusive, Hillis-Steele)
    s_scan[tid] = my;
    __syncthreads();
    for (int o = 1; o < MT; o <<= 1) {
        const int v = tid >= o ? s_scan[tid - o] : 0;
        __syncthreads();
        s_scan[tid] += v;
        __syncthreads();
    }
    total = s_scan[MT - 1];
    if (total > A.cap) {
        if (tid == 0) {
            A.status[0] = total;
            A.status[3] = 1;
        }
        return;
    }
    tclk[4] = __builtin_amdgcn_s_memtime();
    // ---- 3. fill
    {
        int off = s_scan[tid] - my;
        for (int q = q0; q < q1; q++) {
            const int c = A.q_off[q];
            A.q_off[q] = off;
            if (BOW) {
                A.q_mid[q] = off + c;
            } else {
                int cl;
                enum_query<MODE, true, STAGE>(A, GL, GR, q, A.cands + off, cl);
                A.q_mid[q] = off + cl;
            }
            off += c;
        }
        if (tid == MT - 1) A.q_off[nq] = total;
        if (BOW) {
            __syncthreads();
            for (int q = grp; q < nq; q += NGRP) fill_bow_group<MODE>(A, q, lane);
        }
    }
    }  // !pre
    else {
        tclk[3] = tclk[4] = tclk[2];
    }
    __syncthreads();
    tclk[5] = __builtin_amdgcn_s_memtime();
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
    if (BOW) {
        if (!pre)
            for (int q = grp; q < nq; q += NGRP) {
                const QRes r = eval_bow_group<MODE>(A, q, lane, [&](int s) { return taken0[s] != 0; });
                if (lane == 0) store_res(A, q, r);
            }
    } else if (!pre) {
        for (int q = q0; q < q1; q++)
            store_res(A, q, eval_query<MODE>(A, q, [&](int s) { return taken0[s] != 0; }));
    }
    __syncthreads();
    // Jacobi rounds.  A slot is blocked for q when it was blocked initially or a query p < q
    // whose MapPoint has observations wrote it (SearchByBoW / a7: any earlier write).
    tclk[6] = __builtin_amdgcn_s_memtime();
    int rounds = (BOW && pre) ? 1 : 0;
    int *cur = claimB, *other = claimA;
    // (SearchByBoW's first round ran over the chip; its results are final when it changed nothing)
    if (!(BOW && pre && A.status[13] == 0))
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
        if (BOW) {
            for (int q = grp; q < nq; q += NGRP) {
                const QRes r2 = eval_bow_group<MODE>(A, q, lane, [&](int s) { return taken0[s] || cur[s] < q; });
                if (lane == 0) {
                    const QRes r1 = load_res(A, q);
                    if (r2.l != r1.l || r2.r != r1.r) {
                        changed = 1;
                        store_res(A, q, r2);
                    }
                }
            }
        } else {
            for (int q = q0; q < q1; q++) {
                const QRes r2 = eval_query<MODE>(A, q, [&](int s) { return taken0[s] || cur[s] < q; });
                const QRes r1 = load_res(A, q);
                if (r2.l != r1.l || r2.r != r1.r) {
                    changed = 1;
                    store_res(A, q, r2);
                }
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
    tclk[7] = __builtin_amdgcn_s_memtime();
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
            // The staged grid region is free after the fill phase: when the walk's inputs fit, they
            // are copied there (all threads), so the one-thread walk reads LDS instead of a chain of
            // dependent global loads per query.
            const int nright = NS - A.nleft;
            const size_t o_mid = 4 * ((size_t)nq + 1), o_l2r = o_mid + 4 * (size_t)nq;
            const size_t o_r2l = o_l2r + 4 * (size_t)A.nleft, o_c = o_r2l + 4 * (size_t)nright;
            const size_t o_obs = o_c + 4 * (size_t)total, lds_need = o_obs + (size_t)nq;
            if (STAGED && A.l2r && A.r2l && lds_need <= (size_t)A.lds_free) {
                char *fr = (char *)(removedS + ((NS + 15) & ~15));
                SerialLds V{(const int *)fr, (const int *)(fr + o_mid), (const int *)(fr + o_l2r),
                            (const int *)(fr + o_r2l), (const uint32_t *)(fr + o_c), (const uint8_t *)(fr + o_obs)};
                for (int i = tid; i <= nq; i += MT) ((int *)fr)[i] = A.q_off[i];
                for (int i = tid; i < nq; i += MT) {
                    ((int *)(fr + o_mid))[i] = A.q_mid[i];
                    ((uint8_t *)(fr + o_obs))[i] = A.q_has_obs[i];
                }
                for (int i = tid; i < A.nleft; i += MT) ((int *)(fr + o_l2r))[i] = A.l2r[i];
                for (int i = tid; i < nright; i += MT) ((int *)(fr + o_r2l))[i] = A.r2l[i];
                for (int i = tid; i < total; i += MT) ((uint32_t *)(fr + o_c))[i] = A.cands[i];
                int *mark = cur;  // the Jacobi claim array is free now: earliest writer lane per slot
                for (int i = tid; i < NS; i += MT) mark[i] = INT_BIG;
                __syncthreads();
                // Wave 0 walks the queries 64 at a time, speculatively: every lane evaluates its query
                // on the slot state at the batch start and marks the slots it writes; lane i's result
                // is the sequential one unless a lane j < i wrote one of i's candidate slots.  Lanes
                // below the first such conflict commit, their writes applied in lane order (a slot's
                // state is its last writer's); the next batch starts at the conflict.  Lane 0 always
                // commits, so the walk advances.
                if (tid < 64) {
                    const int ln = tid;
                    for (int qb = 0; qb < nq;) {
                        const int q = qb + ln;
                        const bool valid = q < nq;
                        QRes r{-1, -1};
                        if (valid) r = eval_mps_lds(A, V, q, taken0);
                        int ws[4], n = 0;
                        if (r.l >= 0) {
                            ws[n++] = r.l;
                            const int t = V.l2r[r.l];
                            if (t != -1) ws[n++] = t + A.nleft;
                        }
                        if (r.r >= 0) {
                            const int t = V.r2l[r.r - A.nleft];
                            if (t != -1) ws[n++] = t;
                            ws[n++] = r.r;
                        }
                        for (int i = 0; i < n; i++) atomicMin(&mark[ws[i]], ln);
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        bool conf = false;
                        if (valid)
                            for (int e = V.off[q], e1 = V.off[q + 1]; e < e1; e++)
                                conf |= mark[V.cands[e] & 0xFFFFu] < ln;
                        const unsigned long long cm = __ballot(conf);
                        const int nvalid = min(64, nq - qb);
                        const int first = cm ? min((int)__builtin_ctzll(cm), nvalid) : nvalid;
                        const uint8_t o = valid ? V.obs[q] : (uint8_t)0;
                        for (int j = 0; j < first; j++) {
                            if (ln == j)
                                for (int i = 0; i < n; i++) taken0[ws[i]] = o;
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        }
                        if (ln < first) store_res(A, q, r);
                        for (int i = 0; i < n; i++) mark[ws[i]] = INT_BIG;
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        qb += first;
                    }
                }
            } else if (tid == 0) {
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
        A.status[3] &= 2;  // keep k_grid_prepass's wait-bound flag
        A.status[4] = serial;
        tclk[8] = __builtin_amdgcn_s_memtime();
        if (BOW) tclk[1] = tclk[2] = tclk[0];
        for (int i = 0; i < 8; i++) A.status[5 + i] = (int32_t)(tclk[i + 1] - tclk[i]);
    }
}

size_t match_lds_bytes(int ns)
{
    return (size_t)ns * 3 * sizeof(int) + 2 * (((size_t)ns + 15) & ~size_t(15));
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

// One problem of a launch: its packed arguments plus host-side bookkeeping.  The vectors hold
// host-built inputs (BoW query arrays) that must stay alive until the packer copies them.
struct Problem {
    MatchArgs A = {};
    int32_t *host_slot = nullptr;  // slot array (in/out), n_slot entries
    int n_slot = 0;
    std::vector<int32_t> q_feat, q_cb, q_ce, q_mp, q_off;  // q_off: SearchByBoW's candidate CSR
    std::vector<uint8_t> qdesc, slot_ok;
    std::vector<float> q_angle;
    int32_t *out_mp12 = nullptr;   // KF-KF: result indexed by KF1 keypoint
    // a new call's problem: the arrays are emptied but keep their capacity (a 256-frame batch would
    // otherwise allocate and page in tens of MB of host memory per call)
    void reset()
    {
        A = {};
        host_slot = nullptr;
        n_slot = 0;
        out_mp12 = nullptr;
        for (auto *v : {&q_feat, &q_cb, &q_ce, &q_mp, &q_off}) v->clear();
        qdesc.clear();
        slot_ok.clear();
        q_angle.clear();
    }
};
// the context's problems and packer, reused call to call (one context per host thread)
struct MatchCache {
    std::deque<Problem> P;
    osg_packer pk;
};

constexpr int STATUS_INTS = 16;

// Upload every problem's packed inputs and slot arrays, launch one workgroup per problem (growing
// a problem's candidate buffer when its count pass reports more than the capacity), and download
// the slot arrays / KF-KF results and the per-problem match counts.
template <int MODE>
int run_batch(osg_ctx *ctx, std::deque<Problem> &P, int B, const osg_packer &pk, int32_t *nmatches)
{
    if (B == 0) return OSG_OK;
    // host phase stamps for OSG_MATCH_PROFILE=2: setup, sync + pack, launches, wait, results
    using hclock = std::chrono::steady_clock;
    hclock::time_point hs[6], hx[4];
    hs[0] = hclock::now();
    std::vector<size_t> slot_off(B + 1, 0), q_base(B + 1, 0);
    size_t lds = 0;
    for (int b = 0; b < B; b++) {
        OSG_REQUIRE(ctx, P[b].A.n_slots <= MAX_SLOTS, "problem %d: %d slots exceed the %d supported", b,
                    P[b].A.n_slots, MAX_SLOTS);
        slot_off[b + 1] = slot_off[b] + (size_t)P[b].n_slot;
        q_base[b + 1] = q_base[b] + (size_t)P[b].A.nq + 1;
        lds = std::max(lds, match_lds_bytes(P[b].A.n_slots));
    }
    // grid modes stage the frames' grids (and descriptors) in LDS when every problem's fits
    constexpr bool BOW = MODE == MODE_BOW_KF_F || MODE == MODE_BOW_KF_KF;
    static const int stage_env = getenv("OSG_MATCH_STAGE") ? atoi(getenv("OSG_MATCH_STAGE")) : 2;
    const size_t lds_budget = (size_t)std::max(0, ctx->lds_per_block - 8 * 1024);  // static LDS ~4.3 KB
    int stage = 0;
    if (!BOW)
        for (int st = std::min(stage_env, 2); st >= 1 && stage == 0; st--) {
            size_t need = lds;
            for (int b = 0; b < B; b++)
                need = std::max(need, match_lds_bytes(P[b].A.n_slots) +
                                          staged_lds_bytes(P[b].A.n_slots, P[b].A.nleft >= 0, st));
            if (need <= lds_budget) {
                stage = st;
                lds = need;
            }
        }
    // (dynamic LDS up to the 160 KiB of a CU launches without a function attribute on gfx950:
    // tools/micro/lds_limit.hip)
    const size_t n_slot_total = slot_off[B], nq_total = q_base[B];
    // device io block: [status B x 16 ints][slot arrays][out_q]
    const size_t status_bytes = sizeof(int32_t) * STATUS_INTS * (size_t)B;
    const size_t io_in_bytes = status_bytes + sizeof(int32_t) * n_slot_total;
    const size_t io_bytes = io_in_bytes + sizeof(int32_t) * nq_total + 64;
    const size_t in_bytes = (pk.total + 255) & ~size_t(255);
    const size_t io_pad = (io_bytes + 255) & ~size_t(255);
    const size_t args_bytes = sizeof(MatchArgs) * (size_t)B;
    char *pin = (char *)osg_pinned(ctx, in_bytes + io_pad + args_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    hs[1] = hclock::now();
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    hx[0] = hclock::now();
    pk.fill(pin);
    char *pin_io = pin + in_bytes;
    MatchArgs *pin_args = (MatchArgs *)(pin_io + io_pad);
    std::memset(pin_io, 0, status_bytes);
    for (int b = 0; b < B; b++)
        if (P[b].n_slot > 0)
            std::memcpy(pin_io + status_bytes + sizeof(int32_t) * slot_off[b], P[b].host_slot,
                        sizeof(int32_t) * P[b].n_slot);
    // one device block with the pinned block's layout [inputs | io | args]: the first attempt uploads
    // it with one copy, and one copy brings status, slots and KF-KF results back (a single call's
    // host cost is mostly HIP API calls and synchronisations, not bytes)
    char *dev_in = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, in_bytes + io_pad + args_bytes + 256);
    char *dev_io = dev_in + in_bytes;
    MatchArgs *dev_args = (MatchArgs *)(dev_io + io_pad);
    // grid modes: the k_grid_* prepass for launches of a few problems (OSG_MATCH_PREPASS=0 / 1 pins it)
    const char *pe = getenv("OSG_MATCH_PREPASS");  // read per call: tests switch it
    const int prepass_env = pe ? atoi(pe) : -1;
    const bool grid_pre = !BOW && (prepass_env >= 0 ? prepass_env != 0 : B <= GRID_PREPASS_MAX_B);
    for (int b = 0; b < B; b++) {
        MatchArgs &A = P[b].A;
        OSG_RELOCATE_ALL(A, dev_in);
        if (BOW && A.prefilled) relocate(A.q_off, dev_in);  // the host CSR (packed input)
        if (grid_pre) A.prefilled = 1;
        A.status = (GLOBAL int32_t *)dev_io + STATUS_INTS * b;
        A.slot_mp = (GLOBAL int32_t *)(dev_io + status_bytes) + slot_off[b];
        A.out_q = (GLOBAL int32_t *)(dev_io + io_in_bytes) + q_base[b];
    }
    for (int b = 0; b < B; b++) P[b].A.lds_free = (int)(lds - match_lds_bytes(P[b].A.n_slots));
    std::vector<size_t> cap(B), cand_off(B + 1);
    for (int b = 0; b < B; b++)
        cap[b] = (BOW && P[b].A.prefilled) ? (size_t)std::max(P[b].q_off.back(), 1)
                                            : std::max<size_t>((size_t)P[b].A.nq * 32, 1024);
    std::vector<int32_t> st((size_t)STATUS_INTS * B);
    for (int attempt = 0; attempt < 2; attempt++) {
        cand_off[0] = 0;
        for (int b = 0; b < B; b++) cand_off[b + 1] = cand_off[b] + cap[b];
        int32_t *q_off, *q_mid, *q_res;
        uint8_t *q_bin;
        uint32_t *cands;
        OSG_ALLOC(ctx, q_off, SLOT_TMP2, sizeof(int32_t) * nq_total);
        OSG_ALLOC(ctx, q_res, SLOT_TMP3, sizeof(int32_t) * 2 * nq_total);
        OSG_ALLOC(ctx, q_bin, SLOT_TMP4, 2 * nq_total + 16);
        OSG_ALLOC(ctx, q_mid, SLOT_TMP6, sizeof(int32_t) * nq_total);
        float4 *q_win = nullptr;
        if (!BOW) OSG_ALLOC(ctx, q_win, SLOT_TMP8, sizeof(float4) * 4 * nq_total);
        OSG_ALLOC(ctx, cands, SLOT_TMP5, sizeof(uint32_t) * cand_off[B]);
        int32_t *claim_g = nullptr;
        if (BOW) OSG_ALLOC(ctx, claim_g, SLOT_TMP9, sizeof(int32_t) * (n_slot_total + 1));
        for (int b = 0; b < B; b++) {
            MatchArgs &A = P[b].A;
            if (!(BOW && A.prefilled)) A.q_off = (GLOBAL int32_t *)(q_off + q_base[b]);
            A.q_mid = (GLOBAL int32_t *)(q_mid + q_base[b]);
            A.q_win = q_win ? (GLOBAL f32x4 *)(q_win + 4 * q_base[b]) : nullptr;
            A.q_res = (GLOBAL int32_t *)(q_res + 2 * q_base[b]);
            A.q_bin = (GLOBAL uint8_t *)(q_bin + 2 * q_base[b]);
            A.cands = (GLOBAL uint32_t *)(cands + cand_off[b]);
            A.claim_g = claim_g ? (GLOBAL int32_t *)(claim_g + slot_off[b]) : nullptr;
            A.cap = (int)std::min<size_t>(cap[b], INT_BIG);
            pin_args[b] = A;
        }
        // the inputs, the status block, the input slot state and the arguments in one copy; a retry
        // re-uploads [io | args] (it must not see the slot arrays written by the problems that fitted
        // the first time)
        if (attempt == 0) hs[2] = hclock::now();
        if (attempt == 0) OSG_RC(osg_upload(ctx, dev_in, pin, in_bytes + io_pad + args_bytes));
        if (attempt == 0) hx[1] = hclock::now();
        else OSG_RC(osg_upload(ctx, dev_io, pin_io, io_pad + args_bytes));
        hipEvent_t *ev = osg_ctx_events(ctx);
        if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
        OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
        if (attempt == 0) hx[2] = hclock::now();
        if (BOW) {
            int max_nq = 0;
            for (int b = 0; b < B; b++) max_nq = std::max(max_nq, P[b].A.prefilled ? P[b].A.nq : 0);
            if (max_nq > 0) {
                hipLaunchKernelGGL((k_bow_fill<MODE>), dim3((max_nq + BFG - 1) / BFG, B), dim3(BFG * BOW_G), 0, ctx->stream,
                                   dev_args);
                hipLaunchKernelGGL((k_bow_claims<MODE>), dim3((max_nq + 255) / 256, B), dim3(256), 0, ctx->stream,
                                   dev_args);
                hipLaunchKernelGGL((k_bow_round<MODE>), dim3((max_nq + BFG - 1) / BFG, B), dim3(BFG * BOW_G), 0, ctx->stream,
                                   dev_args);
            }
        }
        if (grid_pre) {
            int max_nq = 0;
            for (int b = 0; b < B; b++) max_nq = std::max(max_nq, P[b].A.nq);
            if (max_nq > 0) {
                const int nwg = (max_nq + GQG - 1) / GQG;
                const size_t need = (size_t)nwg * B;
                if (ctx->lb_cap < need) {  // zeroed once: epoch 0 is never a call's
                    if (ctx->lb_flags) OSG_HIP_CHECK(ctx, hipFree(ctx->lb_flags));
                    ctx->lb_flags = nullptr;
                    ctx->lb_cap = 0;
                    OSG_HIP_CHECK(ctx, hipMalloc(&ctx->lb_flags, sizeof(unsigned long long) * need));
                    OSG_HIP_CHECK(ctx, hipMemsetAsync(ctx->lb_flags, 0, sizeof(unsigned long long) * need, ctx->stream));
                    ctx->lb_cap = need;
                }
                if (++ctx->lb_epoch == 0) ++ctx->lb_epoch;
                hipLaunchKernelGGL((k_grid_prepass<MODE>), dim3(nwg, B), dim3(GQG * BOW_G), 0, ctx->stream, dev_args,
                                   ctx->lb_flags, nwg, ctx->lb_epoch);
            }
        }
        if (stage == 2)
            hipLaunchKernelGGL((k_match<MODE, 2>), dim3(B), dim3(MT), lds, ctx->stream, dev_args);
        else if (stage == 1)
            hipLaunchKernelGGL((k_match<MODE, 1>), dim3(B), dim3(MT), lds, ctx->stream, dev_args);
        else
            hipLaunchKernelGGL((k_match<MODE, 0>), dim3(B), dim3(MT), lds, ctx->stream, dev_args);
        OSG_HIP_CHECK(ctx, hipGetLastError());
        if (attempt == 0) hx[3] = hclock::now();
        OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
        // status, slot arrays and KF-KF results in one copy (the pinned io block is re-filled from the
        // callers' slots before a retry)
        OSG_RC(osg_download(ctx, pin_io, dev_io, io_bytes));
        hs[3] = hclock::now();
        OSG_RC(osg_wait(ctx));
        hs[4] = hclock::now();
        std::memcpy(st.data(), pin_io, status_bytes);
        bool overflow = false;
        for (int b = 0; b < B; b++)
            if (st[(size_t)STATUS_INTS * b + 3] & 2)
                return osg_set_error(ctx, OSG_E_HIP, "problem %d: k_grid_prepass wait bound exceeded", b);
        for (int b = 0; b < B; b++)
            if (st[(size_t)STATUS_INTS * b + 3]) {
                overflow = true;
                cap[b] = (size_t)st[(size_t)STATUS_INTS * b] + 256;
            }
        if (!overflow) break;
        if (attempt == 1) return osg_set_error(ctx, OSG_E_HIP, "candidate buffer overflow after resize");
        std::memset(pin_io, 0, status_bytes);
        for (int b = 0; b < B; b++)
            if (P[b].n_slot > 0)
                std::memcpy(pin_io + status_bytes + sizeof(int32_t) * slot_off[b], P[b].host_slot,
                            sizeof(int32_t) * P[b].n_slot);
    }
    int64_t cand_sum = 0, nm_sum = 0;
    int rounds_max = 0, serial_n = 0;
    for (int b = 0; b < B; b++) {
        const int32_t *sb = &st[(size_t)STATUS_INTS * b];
        nmatches[b] = sb[1];
        cand_sum += sb[0];
        nm_sum += sb[1];
        rounds_max = std::max(rounds_max, (int)sb[2]);
        serial_n += sb[4] ? 1 : 0;
        if (P[b].n_slot > 0)
            std::memcpy(P[b].host_slot, pin_io + status_bytes + sizeof(int32_t) * slot_off[b],
                        sizeof(int32_t) * P[b].n_slot);
        if (MODE == MODE_BOW_KF_KF) {
            const int32_t *oq = (const int32_t *)(pin_io + io_in_bytes) + q_base[b];
            for (size_t i = 0; i < P[b].q_feat.size(); i++) P[b].out_mp12[P[b].q_feat[i]] = oq[i];
        }
    }
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]));
    ctx->last_kernel_ms = ms;
    static const int prof_level = getenv("OSG_MATCH_PROFILE") ? atoi(getenv("OSG_MATCH_PROFILE")) : 0;
    const bool prof = prof_level > 0;
    hs[5] = hclock::now();
    if (prof_level >= 2) {
        auto us = [&](int a, int b) { return std::chrono::duration<double, std::micro>(hs[b] - hs[a]).count(); };
        auto ux = [&](hclock::time_point a, hclock::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        fprintf(stderr, "[osg match host] mode %d B %d: setup %.1f | sync+pack %.1f | launches %.1f | wait %.1f | results %.1f us"
                        " || sync %.1f fill %.1f | upload %.1f event %.1f kernels %.1f event+download %.1f (pack %zu B)\n",
                MODE, B, us(0, 1), us(1, 2), us(2, 3), us(3, 4), us(4, 5), ux(hs[1], hx[0]), ux(hx[0], hs[2]),
                ux(hs[2], hx[1]), ux(hx[1], hx[2]), ux(hx[2], hx[3]), ux(hx[3], hs[3]), (size_t)pk.total);
    }
    if (prof)
        fprintf(stderr, "[osg match] mode %d B %d kernel %.3f ms | problem 0: nq %d cands %d rounds %d serial %d | "
                        "clk stage %d windows %d count %d scan %d fill %d init %d rounds %d finish %d (stage %d)\n",
                MODE, B, ms, P[0].A.nq, st[0], st[2], st[4], st[5], st[6], st[7], st[8], st[9], st[10], st[11], st[12], stage);
    ctx->match_stats[0] = (int32_t)std::min<int64_t>(cand_sum, INT_BIG);
    ctx->match_stats[1] = rounds_max;
    ctx->match_stats[2] = serial_n;
    ctx->match_stats[3] = (int32_t)std::min<int64_t>(nm_sum, INT_BIG);
    return OSG_OK;
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
    A.n_levels = F->n_levels;
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
int check_grid(osg_ctx *ctx, const int32_t *gs, const int32_t *gi, int n_cam, const char *which)
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
    for (int i = 0; i < F->n; i++)  // octaves are packed in 7 bits
        OSG_REQUIRE(ctx, F->kp_octave[i] >= 0 && F->kp_octave[i] < 128, "kp_octave[%d] = %d", i, F->kp_octave[i]);
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

// ---- per-operator problem setup (validation + packing); ref lines are the operators' own

int prep_mps(osg_ctx *ctx, Problem &P, osg_packer &pk, const osg_frame *F, const osg_mp_queries *Q, float nnratio,
             float th, int far_points, float th_far_points, int32_t *slot_mp, const uint8_t *slot_taken)
{
    int rc = check_frame(ctx, F);
    if (rc < 0) return rc;
    OSG_REQUIRE(ctx, Q && Q->n >= 0 && slot_mp && slot_taken, "null argument");
    MatchArgs &A = P.A;
    frame_into_args(A, pk, F);
    P.host_slot = slot_mp;
    P.n_slot = F->n;
    const int n = Q->n;
    A.nq = n;
    A.nnratio = nnratio;
    A.th = th;
    A.far_points = far_points;
    A.th_far = th_far_points;
    if (n == 0) return OSG_OK;
    OSG_REQUIRE(ctx, Q->desc && Q->mp_id && Q->usable && Q->has_obs && Q->in_view && Q->proj_x && Q->proj_y &&
                         Q->proj_xr && Q->view_cos && Q->pred_level && Q->track_depth, "query arrays");
    for (int i = 0; i < n; i++)
        if (Q->in_view[i] && (Q->pred_level[i] < 0 || Q->pred_level[i] >= F->n_levels))
            return osg_set_error(ctx, OSG_E_INVALID, "pred_level[%d] = %d out of range", i, Q->pred_level[i]);
    if (F->nleft != -1) {
        OSG_REQUIRE(ctx, Q->in_view_r && Q->proj_yr && Q->view_cos_r && Q->pred_level_r, "right-camera query arrays");
        for (int i = 0; i < n; i++)
            if (Q->in_view_r[i] && (Q->pred_level_r[i] < -1 || Q->pred_level_r[i] >= F->n_levels))
                return osg_set_error(ctx, OSG_E_INVALID, "pred_level_r[%d] = %d out of range", i, Q->pred_level_r[i]);
    }
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
    return OSG_OK;
}

int prep_last(osg_ctx *ctx, Problem &P, osg_packer &pk, const osg_frame *CF, const osg_last_queries *L, float th,
              int mono, int check_orientation, int32_t *slot_mp, const uint8_t *slot_taken)
{
    int rc = check_frame(ctx, CF);
    if (rc < 0) return rc;
    OSG_REQUIRE(ctx, L && L->n >= 0 && slot_mp && slot_taken, "null argument");
    MatchArgs &A = P.A;
    frame_into_args(A, pk, CF);
    P.host_slot = slot_mp;
    P.n_slot = CF->n;
    const int n = L->n;
    A.nq = n;
    A.th = th;
    A.mono = mono;
    A.tlc_z = L->tlc_z;
    A.check_ori = check_orientation;
    if (n == 0) return OSG_OK;
    OSG_REQUIRE(ctx, L->desc && L->mp_id && L->valid && L->has_obs && L->u && L->v && L->invz && L->octave &&
                         L->angle, "query arrays");
    for (int i = 0; i < n; i++)
        if (L->valid[i] && (L->octave[i] < 0 || L->octave[i] >= CF->n_levels))
            return osg_set_error(ctx, OSG_E_INVALID, "octave[%d] out of range", i);
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
    return OSG_OK;
}

int prep_kf(osg_ctx *ctx, Problem &P, osg_packer &pk, const osg_frame *CF, const osg_kf_queries *K, float th,
            int orb_dist, int check_orientation, int32_t *slot_mp)
{
    int rc = check_frame(ctx, CF);
    if (rc < 0) return rc;
    OSG_REQUIRE(ctx, K && K->n >= 0 && slot_mp, "null argument");
    MatchArgs &A = P.A;
    frame_into_args(A, pk, CF);
    P.host_slot = slot_mp;
    P.n_slot = CF->n;
    const int n = K->n;
    A.nq = n;
    A.th = th;
    A.orb_dist = orb_dist;
    A.check_ori = check_orientation;
    if (n == 0) return OSG_OK;
    OSG_REQUIRE(ctx, K->desc && K->mp_id && K->valid && K->u && K->v && K->pred_level && K->angle, "query arrays");
    for (int i = 0; i < n; i++)
        if (K->valid[i] && (K->pred_level[i] < 0 || K->pred_level[i] >= CF->n_levels))
            return osg_set_error(ctx, OSG_E_INVALID, "pred_level[%d] out of range", i);
    set_off(A.qdesc, pk.add(K->desc, (size_t)n * 32));
    set_off(A.q_mp, pk.add(K->mp_id, sizeof(int32_t) * n));
    set_off(A.q_m0, pk.add(K->valid, n));
    set_off(A.q_x, pk.add(K->u, sizeof(float) * n));
    set_off(A.q_y, pk.add(K->v, sizeof(float) * n));
    set_off(A.q_lvl, pk.add(K->pred_level, sizeof(int32_t) * n));
    set_off(A.q_angle, pk.add(K->angle, sizeof(float) * n));
    return OSG_OK;
}

// Host half of SearchByBoW: the FeatureVector merge-walk (ref:src/ORBmatcher.cc:292-467) emits the
// query order (shared nodes ascending, KeyFrame features in node order); each query's candidate
// list is the other side's feature list of the same node.
int bow_queries(const osg_bow_side *A_, const osg_bow_side *B_, bool guard_nleft_a, std::vector<int32_t> &q_feat,
                std::vector<int32_t> &q_cb, std::vector<int32_t> &q_ce)
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

int check_bow_side(osg_ctx *ctx, const osg_bow_side *S, const char *which, bool slot_side)
{
    OSG_REQUIRE(ctx, S->n >= 0 && (!slot_side || S->n <= MAX_SLOTS), "%s: n out of range", which);
    OSG_REQUIRE(ctx, S->nleft == -1 || (S->nleft >= 0 && S->nleft <= S->n), "%s: nleft out of range", which);
    OSG_REQUIRE(ctx, S->fv.n_nodes >= 0 && (S->fv.n_nodes == 0 || (S->fv.node_id && S->fv.node_start)),
                "%s: FeatureVector", which);
    if (S->fv.n_nodes > 0) {
        const int m = S->fv.node_start[S->fv.n_nodes];
        OSG_REQUIRE(ctx, m == 0 || S->fv.feat, "%s: FeatureVector features", which);
        for (int j = 0; j < m; j++)
            OSG_REQUIRE(ctx, S->fv.feat[j] >= 0 && S->fv.feat[j] < S->n, "%s: feature index %d", which, S->fv.feat[j]);
    }
    return OSG_OK;
}

int prep_bow_kf_f(osg_ctx *ctx, Problem &P, osg_packer &pk, const osg_bow_side *kf, const osg_bow_side *f,
                  float nnratio, int check_orientation, int32_t *out_mp)
{
    OSG_REQUIRE(ctx, kf && f && out_mp, "null argument");
    int rc = check_bow_side(ctx, kf, "keyframe", false);
    if (rc < 0) return rc;
    rc = check_bow_side(ctx, f, "frame", true);
    if (rc < 0) return rc;
    OSG_REQUIRE(ctx, kf->n == 0 || (kf->desc && kf->angle && kf->mp_id && kf->mp_good), "keyframe arrays");
    OSG_REQUIRE(ctx, f->n == 0 || (f->desc && f->angle), "frame arrays");
    for (int i = 0; i < f->n; i++) out_mp[i] = -1;
    if (bow_queries(kf, f, false, P.q_feat, P.q_cb, P.q_ce) < 0) return osg_set_error(ctx, OSG_E_INVALID, "feature index");
    const int n = (int)P.q_feat.size();
    MatchArgs &A = P.A;
    A.nq = n;
    A.n_slots = f->n;
    A.nleft = f->nleft;
    P.host_slot = out_mp;
    P.n_slot = f->n;
    A.nnratio = nnratio;
    A.check_ori = check_orientation;
    if (n == 0) return OSG_OK;
    set_off(A.fdesc, pk.add(f->desc, (size_t)f->n * 32));
    set_off(A.slot_angle, pk.add(f->angle, sizeof(float) * f->n));
    // the queries' descriptor rows, MapPoint ids and angles are gathered from the KeyFrame's arrays
    // straight into the pinned block (P.q_feat lives until the fill)
    set_off(A.qdesc, pk.add_rows(kf->desc, P.q_feat.data(), n, 32));
    set_off(A.q_mp, pk.add_rows(kf->mp_id, P.q_feat.data(), n, sizeof(int32_t)));
    set_off(A.q_angle, pk.add_rows(kf->angle, P.q_feat.data(), n, sizeof(float)));
    set_off(A.q_cb, pk.add(P.q_cb.data(), sizeof(int32_t) * n));
    set_off(A.q_ce, pk.add(P.q_ce.data(), sizeof(int32_t) * n));
    set_off(A.cand_list, pk.add(f->fv.feat, sizeof(int32_t) * f->fv.node_start[f->fv.n_nodes]));
    P.q_off.assign(n + 1, 0);
    for (int i = 0; i < n; i++) P.q_off[i + 1] = P.q_off[i] + (P.q_ce[i] - P.q_cb[i]);
    set_off(A.q_off, pk.add(P.q_off.data(), sizeof(int32_t) * (n + 1)));
    A.prefilled = 1;
    return OSG_OK;
}

int prep_bow_kf_kf(osg_ctx *ctx, Problem &P, osg_packer &pk, const osg_bow_side *kf1, const osg_bow_side *kf2,
                   float nnratio, int check_orientation, int32_t *out_mp12)
{
    OSG_REQUIRE(ctx, kf1 && kf2 && out_mp12, "null argument");
    int rc = check_bow_side(ctx, kf1, "keyframe 1", false);
    if (rc < 0) return rc;
    rc = check_bow_side(ctx, kf2, "keyframe 2", true);
    if (rc < 0) return rc;
    OSG_REQUIRE(ctx, kf1->n == 0 || (kf1->desc && kf1->angle && kf1->mp_good), "keyframe 1 arrays");
    OSG_REQUIRE(ctx, kf2->n == 0 || (kf2->desc && kf2->angle && kf2->mp_id && kf2->mp_good), "keyframe 2 arrays");
    for (int i = 0; i < kf1->n; i++) out_mp12[i] = -1;
    if (bow_queries(kf1, kf2, true, P.q_feat, P.q_cb, P.q_ce) < 0) return osg_set_error(ctx, OSG_E_INVALID, "feature index");
    const int n = (int)P.q_feat.size();
    P.slot_ok.resize(kf2->n);
    // right-camera keypoints of a two-camera KF2 are skipped (ref:src/ORBmatcher.cc:953-955)
    for (int s = 0; s < kf2->n; s++)
        P.slot_ok[s] = (kf2->mp_id[s] >= 0 && kf2->mp_good[s] && (kf2->nleft == -1 || s < kf2->nleft)) ? 1 : 0;
    MatchArgs &A = P.A;
    A.nq = n;
    A.n_slots = kf2->n;
    A.nleft = -1;
    P.out_mp12 = out_mp12;
    A.nnratio = nnratio;
    A.check_ori = check_orientation;
    if (n == 0) return OSG_OK;
    set_off(A.fdesc, pk.add(kf2->desc, (size_t)kf2->n * 32));
    set_off(A.slot_angle, pk.add(kf2->angle, sizeof(float) * kf2->n));
    set_off(A.slot_mp2, pk.add(kf2->mp_id, sizeof(int32_t) * kf2->n));
    set_off(A.slot_ok, pk.add(P.slot_ok.data(), P.slot_ok.size()));
    // KF1's query rows and angles gathered straight into the pinned block (as prep_bow_kf_f)
    set_off(A.qdesc, pk.add_rows(kf1->desc, P.q_feat.data(), n, 32));
    set_off(A.q_angle, pk.add_rows(kf1->angle, P.q_feat.data(), n, sizeof(float)));
    set_off(A.q_cb, pk.add(P.q_cb.data(), sizeof(int32_t) * n));
    set_off(A.q_ce, pk.add(P.q_ce.data(), sizeof(int32_t) * n));
    set_off(A.cand_list, pk.add(kf2->fv.feat, sizeof(int32_t) * kf2->fv.node_start[kf2->fv.n_nodes]));
    P.q_off.assign(n + 1, 0);
    for (int i = 0; i < n; i++) P.q_off[i + 1] = P.q_off[i] + (P.q_ce[i] - P.q_cb[i]);
    set_off(A.q_off, pk.add(P.q_off.data(), sizeof(int32_t) * (n + 1)));
    A.prefilled = 1;
    return OSG_OK;
}

// Single and batched entry points share one path: prepare B problems, one launch.
template <int MODE, typename Prep>
int run_problems(osg_ctx *ctx, int B, int32_t *nmatches, Prep prep)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, B >= 0 && (B == 0 || nmatches), "batch size / nmatches");
    if (!ctx->match_cache) ctx->match_cache = std::make_shared<MatchCache>();
    MatchCache &mc = *static_cast<MatchCache *>(ctx->match_cache.get());
    std::deque<Problem> &P = mc.P;
    osg_packer &pk = mc.pk;
    pk.items.clear();
    pk.total = 0;
    while ((int)P.size() < B) P.emplace_back();
    static const int prof_level = getenv("OSG_MATCH_PROFILE") ? atoi(getenv("OSG_MATCH_PROFILE")) : 0;
    const auto tp = std::chrono::steady_clock::now();
    for (int b = 0; b < B; b++) {
        P[b].reset();
        const int rc = prep(P[b], pk, b);
        if (rc < 0) {
            if (B > 1) {
                const std::string msg = ctx->last_error;
                return osg_set_error(ctx, rc, "problem %d: %s", b, msg.c_str());
            }
            return rc;
        }
    }
    if (prof_level >= 2)
        fprintf(stderr, "[osg match prep] mode %d B %d: %.1f us\n", MODE, B,
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tp).count());
    return run_batch<MODE>(ctx, P, B, pk, nmatches);
}

template <int MODE, typename Prep>
int run_single(osg_ctx *ctx, Prep prep)
{
    int32_t nm = 0;
    const int rc = run_problems<MODE>(ctx, 1, &nm, [&](Problem &P, osg_packer &pk, int) { return prep(P, pk); });
    return rc < 0 ? rc : nm;
}

}  // namespace

int osg_check_frame(osg_ctx *ctx, const osg_frame *F) { return check_frame(ctx, F); }

extern "C" {

int osg_search_by_projection_mps(osg_ctx *ctx, const osg_frame *F, const osg_mp_queries *Q, float nnratio,
                                 float th, int far_points, float th_far_points, int32_t *slot_mp,
                                 const uint8_t *slot_taken)
{
    return run_single<MODE_MPS>(ctx, [&](Problem &P, osg_packer &pk) {
        return prep_mps(ctx, P, pk, F, Q, nnratio, th, far_points, th_far_points, slot_mp, slot_taken);
    });
}

int osg_search_by_projection_last(osg_ctx *ctx, const osg_frame *CF, const osg_last_queries *L, float th,
                                  int mono, int check_orientation, int32_t *slot_mp, const uint8_t *slot_taken)
{
    return run_single<MODE_LAST>(ctx, [&](Problem &P, osg_packer &pk) {
        return prep_last(ctx, P, pk, CF, L, th, mono, check_orientation, slot_mp, slot_taken);
    });
}

int osg_search_by_projection_kf(osg_ctx *ctx, const osg_frame *CF, const osg_kf_queries *K, float th, int orb_dist,
                                int check_orientation, int32_t *slot_mp)
{
    return run_single<MODE_KF>(ctx, [&](Problem &P, osg_packer &pk) {
        return prep_kf(ctx, P, pk, CF, K, th, orb_dist, check_orientation, slot_mp);
    });
}

int osg_search_by_bow_kf_f(osg_ctx *ctx, const osg_bow_side *kf, const osg_bow_side *f, float nnratio,
                           int check_orientation, int32_t *out_mp)
{
    return run_single<MODE_BOW_KF_F>(ctx, [&](Problem &P, osg_packer &pk) {
        return prep_bow_kf_f(ctx, P, pk, kf, f, nnratio, check_orientation, out_mp);
    });
}

int osg_search_by_bow_kf_kf(osg_ctx *ctx, const osg_bow_side *kf1, const osg_bow_side *kf2, float nnratio,
                            int check_orientation, int32_t *out_mp12)
{
    return run_single<MODE_BOW_KF_KF>(ctx, [&](Problem &P, osg_packer &pk) {
        return prep_bow_kf_kf(ctx, P, pk, kf1, kf2, nnratio, check_orientation, out_mp12);
    });
}

// ---- batched forms: problem b's slot array starts at the sum of the earlier problems' sizes

int osg_search_by_projection_mps_batch(osg_ctx *ctx, const osg_frame *F, const osg_mp_queries *Q, int32_t B,
                                       float nnratio, float th, int far_points, float th_far_points,
                                       int32_t *slot_mp, const uint8_t *slot_taken, int32_t *nmatches)
{
    size_t off = 0;
    return run_problems<MODE_MPS>(ctx, B, nmatches, [&](Problem &P, osg_packer &pk, int b) {
        OSG_REQUIRE(ctx, F && Q && slot_mp && slot_taken, "null argument");
        const int rc = prep_mps(ctx, P, pk, &F[b], &Q[b], nnratio, th, far_points, th_far_points, slot_mp + off,
                                slot_taken + off);
        off += F[b].n;
        return rc;
    });
}

int osg_search_by_projection_last_batch(osg_ctx *ctx, const osg_frame *CF, const osg_last_queries *L, int32_t B,
                                        float th, int mono, int check_orientation, int32_t *slot_mp,
                                        const uint8_t *slot_taken, int32_t *nmatches)
{
    size_t off = 0;
    return run_problems<MODE_LAST>(ctx, B, nmatches, [&](Problem &P, osg_packer &pk, int b) {
        OSG_REQUIRE(ctx, CF && L && slot_mp && slot_taken, "null argument");
        const int rc = prep_last(ctx, P, pk, &CF[b], &L[b], th, mono, check_orientation, slot_mp + off,
                                 slot_taken + off);
        off += CF[b].n;
        return rc;
    });
}

int osg_search_by_projection_kf_batch(osg_ctx *ctx, const osg_frame *CF, const osg_kf_queries *K, int32_t B,
                                      float th, int orb_dist, int check_orientation, int32_t *slot_mp,
                                      int32_t *nmatches)
{
    size_t off = 0;
    return run_problems<MODE_KF>(ctx, B, nmatches, [&](Problem &P, osg_packer &pk, int b) {
        OSG_REQUIRE(ctx, CF && K && slot_mp, "null argument");
        const int rc = prep_kf(ctx, P, pk, &CF[b], &K[b], th, orb_dist, check_orientation, slot_mp + off);
        off += CF[b].n;
        return rc;
    });
}

int osg_search_by_bow_kf_f_batch(osg_ctx *ctx, const osg_bow_side *kf, const osg_bow_side *f, int32_t B,
                                 float nnratio, int check_orientation, int32_t *out_mp, int32_t *nmatches)
{
    size_t off = 0;
    return run_problems<MODE_BOW_KF_F>(ctx, B, nmatches, [&](Problem &P, osg_packer &pk, int b) {
        OSG_REQUIRE(ctx, kf && f && out_mp, "null argument");
        const int rc = prep_bow_kf_f(ctx, P, pk, &kf[b], &f[b], nnratio, check_orientation, out_mp + off);
        off += f[b].n;
        return rc;
    });
}

int osg_search_by_bow_kf_kf_batch(osg_ctx *ctx, const osg_bow_side *kf1, const osg_bow_side *kf2, int32_t B,
                                  float nnratio, int check_orientation, int32_t *out_mp12, int32_t *nmatches)
{
    size_t off = 0;
    return run_problems<MODE_BOW_KF_KF>(ctx, B, nmatches, [&](Problem &P, osg_packer &pk, int b) {
        OSG_REQUIRE(ctx, kf1 && kf2 && out_mp12, "null argument");
        const int rc = prep_bow_kf_kf(ctx, P, pk, &kf1[b], &kf2[b], nnratio, check_orientation, out_mp12 + off);
        off += kf1[b].n;
        return rc;
    });
}

}  // extern "C"
