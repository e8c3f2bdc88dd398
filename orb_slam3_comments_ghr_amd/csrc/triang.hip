// triang.hip — ORBmatcher::SearchForTriangulation on gfx950 (ref:src/ORBmatcher.cc:1045-1328).
//
// LocalMapping::CreateNewMapPoints (ref:src/LocalMapping.cc:630) calls it for the new keyframe
// against each of its ~10-20 covisible neighbours; the batched entry point takes all of those
// pairs in one launch, one workgroup per pair.
//
// In this fork the claim `vbMatched2[bestIdx2] = true` is commented out (ref:src/ORBmatcher.cc:1262),
// so a KF1 keypoint's choice never depends on another's: the search is one lane per query with no
// cross-lane resolve.  Per query the lane walks the KF2 feature list of the shared vocabulary node
// in node order with the reference's tests, in its order and float arithmetic (built with
// -ffp-contract=off):
//   skip a KF2 keypoint with a MapPoint (and, bOnlyStereo, a monocular one)      :1161-1172
//   dist > TH_LOW || dist > bestDist -> skip ('<=': the last of equal distances wins) :1180
//   epipole distance^2 < 100 * mvScaleFactors[octave2] -> skip (both monocular)    :1189-1203
//   bCoarse || Pinhole::epipolarConstrain (F12 of the camera pair)  :1246, Pinhole.cpp:189-219
//            || KannalaBrandt8::epipolarConstrain (triangulate + reproject, kb8_epipolar.h)
// then the rotation histogram (bin of kp1.angle - kp2.angle, factor 1/30 kept) and
// ComputeThreeMaxima in LDS (:1266-1316).  The FeatureVector merge-walk that pairs the nodes
// (:1113-1287) is host work (node lists are std::map-ordered already).
#include <algorithm>
#include <vector>

#include "kb8_epipolar.h"
#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int TT = 256;  // lanes per workgroup (one workgroup per keyframe pair)

struct TriArgs {
    int nq, check_ori, coarse, two_cam1, pinhole;
    float ep_x, ep_y;
    float F[4][9];
    float R12[4][9], t12[4][3], kb[4][8];  // KannalaBrandt8 (pinhole = 0)
    GLOBAL const float *qsig;       // KF1 mvLevelSigma2[kp1.octave] per query (KannalaBrandt8)
    GLOBAL const uint32_t *qdesc;   // nq x 32 B: KF1 descriptors of the queries
    GLOBAL const float *qx, *qy, *qang;
    GLOBAL const uint8_t *qflag;    // bit0 bStereo1, bit1 bRight1
    GLOBAL const int32_t *q_cb, *q_ce;  // the node's range in cand
    GLOBAL const int32_t *cand;     // KF2 FeatureVector features (CSR feat)
    GLOBAL const uint32_t *desc2;
    GLOBAL const float *x2, *y2, *ang2;
    GLOBAL const int32_t *oct2;
    GLOBAL const uint8_t *flag2;    // bit0 eligible (no MapPoint, stereo filter), bit1 bStereo2, bit2 bRight2
    GLOBAL const float *scale2, *sigma2_2;  // KF2 mvScaleFactors, mvLevelSigma2
    GLOBAL int32_t *out;            // nq: best KF2 index after the histogram, -1
    GLOBAL int32_t *nmatch;         // 1
};

__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int rot_bin(float a, float b)
{  // ref:src/ORBmatcher.cc:1269-1276, factor = 1.0f/HISTO_LENGTH (kept upstream bug)
    const float factor = 1.0f / OSG_HISTO_LENGTH;
    float rot = a - b;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == OSG_HISTO_LENGTH) bin = 0;
    return bin;
}

// Pinhole::epipolarConstrain, ref:src/CameraModels/Pinhole.cpp:203-218 (F row-major, F(r,c) = F[3r+c])
__device__ __forceinline__ bool epipolar_ok(const float *F, float x1, float y1, float x2, float y2, float unc)
{
    const float a = x1 * F[0] + y1 * F[3] + F[6];
    const float b = x1 * F[1] + y1 * F[4] + F[7];
    const float c = x1 * F[2] + y1 * F[5] + F[8];
    const float num = a * x2 + b * y2 + c;
    const float den = a * a + b * b;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return (double)dsqr < 3.84 * (double)unc;
}

__global__ __launch_bounds__(TT) void k_triang(const TriArgs *__restrict__ args)
{
    const TriArgs &A = args[blockIdx.x];
    __shared__ int s_hist[OSG_HISTO_LENGTH];
    __shared__ int s_keep[3];
    __shared__ int s_cnt;
    const int tid = threadIdx.x;
    if (tid < OSG_HISTO_LENGTH) s_hist[tid] = 0;
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    for (int q = tid; q < A.nq; q += TT) {
        const u32x4 qa = *(GLOBAL const u32x4 *)(A.qdesc + 8 * q), qb = *(GLOBAL const u32x4 *)(A.qdesc + 8 * q + 4);
        const float x1 = A.qx[q], y1 = A.qy[q];
        const int qf = A.qflag[q];
        const bool stereo1 = qf & 1, right1 = qf & 2;
        int best_dist = OSG_TH_LOW, best = -1;
        const int ce = A.q_ce[q];
        for (int c = A.q_cb[q]; c < ce; c++) {
            const int idx2 = A.cand[c];
            const int f2 = A.flag2[idx2];
            if (!(f2 & 1)) continue;  // MapPoint / bOnlyStereo, :1161-1172
            const u32x4 ka = *(GLOBAL const u32x4 *)(A.desc2 + 8 * idx2), kb = *(GLOBAL const u32x4 *)(A.desc2 + 8 * idx2 + 4);
            uint32_t d = __popc(qa.x ^ ka.x);
            d = bcnt_acc(qa.y ^ ka.y, d);
            d = bcnt_acc(qa.z ^ ka.z, d);
            d = bcnt_acc(qa.w ^ ka.w, d);
            d = bcnt_acc(qb.x ^ kb.x, d);
            d = bcnt_acc(qb.y ^ kb.y, d);
            d = bcnt_acc(qb.z ^ kb.z, d);
            d = bcnt_acc(qb.w ^ kb.w, d);
            const int dist = (int)d;
            if (dist > OSG_TH_LOW || dist > best_dist) continue;  // :1180
            const float x2 = A.x2[idx2], y2 = A.y2[idx2];
            const int oct2 = A.oct2[idx2];
            const bool stereo2 = f2 & 2, right2 = f2 & 4;
            if (!stereo1 && !stereo2 && !A.two_cam1) {  // :1189-1203
                const float distex = A.ep_x - x2;
                const float distey = A.ep_y - y2;
                if (distex * distex + distey * distey < 100 * A.scale2[oct2]) continue;
            }
            const int k = A.two_cam1 ? (right1 ? 2 : 0) + (right2 ? 1 : 0) : 0;  // :1205-1244
            bool ok = A.coarse;  // :1246
            if (!ok && A.pinhole) ok = epipolar_ok(A.F[k], x1, y1, x2, y2, A.sigma2_2[oct2]);
            else if (!ok)  // pCamera1 = KF1 mpCamera / mpCamera2 by bRight1, pCamera2 likewise for KF2
                ok = kb8::epipolar_constrain(A.kb[right1 ? 1 : 0], A.kb[right2 ? 3 : 2], x1, y1, x2, y2, A.R12[k],
                                             A.t12[k], A.qsig[q], A.sigma2_2[oct2]);
            if (ok) {
                best = idx2;
                best_dist = dist;
            }
        }
        A.out[q] = best;
        if (best >= 0 && A.check_ori) atomicAdd(&s_hist[rot_bin(A.qang[q], A.ang2[best])], 1);
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
    }
    __syncthreads();
    int cnt = 0;
    for (int q = tid; q < A.nq; q += TT) {  // the same lane re-reads its own stores
        int best = A.out[q];
        if (best < 0) continue;
        if (A.check_ori) {  // :1303-1316
            const int bin = rot_bin(A.qang[q], A.ang2[best]);
            if (!(bin == s_keep[0] || bin == s_keep[1] || bin == s_keep[2])) {
                A.out[q] = -1;
                continue;
            }
        }
        cnt++;
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if ((tid & 63) == 0) atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (tid == 0) A.nmatch[0] = s_cnt;
}

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

int check_side(osg_ctx *ctx, const osg_kf_side *S, const char *which, int b)
{
    OSG_REQUIRE(ctx, S->n >= 0, "problem %d: %s n", b, which);
    OSG_REQUIRE(ctx, S->nleft == -1 || (S->nleft >= 0 && S->nleft <= S->n), "problem %d: %s nleft", b, which);
    OSG_REQUIRE(ctx, S->n == 0 || (S->desc && S->kp_x && S->kp_y && S->kp_angle && S->kp_octave && S->has_mp),
                "problem %d: %s keypoint arrays", b, which);
    OSG_REQUIRE(ctx, S->n_levels > 0 && S->n_levels <= 128 && S->level_sigma2 && S->scale_factors,
                "problem %d: %s level tables", b, which);
    for (int i = 0; i < S->n; i++)
        OSG_REQUIRE(ctx, S->kp_octave[i] >= 0 && S->kp_octave[i] < S->n_levels, "problem %d: %s octave[%d]", b,
                    which, i);
    const osg_featvec &fv = S->fv;
    OSG_REQUIRE(ctx, fv.n_nodes >= 0 && (fv.n_nodes == 0 || (fv.node_id && fv.node_start)),
                "problem %d: %s FeatureVector", b, which);
    if (fv.n_nodes > 0) {
        const int m = fv.node_start[fv.n_nodes];
        OSG_REQUIRE(ctx, m == 0 || fv.feat, "problem %d: %s FeatureVector features", b, which);
        for (int j = 0; j < m; j++)
            OSG_REQUIRE(ctx, fv.feat[j] >= 0 && fv.feat[j] < S->n, "problem %d: %s feature index %d", b, which,
                        fv.feat[j]);
    }
    return OSG_OK;
}

struct Problem {
    std::vector<int32_t> q_feat, q_cb, q_ce;
    std::vector<uint32_t> qdesc;
    std::vector<float> qx, qy, qang, qsig;
    std::vector<uint8_t> qflag, flag2;
};

// The FeatureVector merge-walk, ref:src/ORBmatcher.cc:1113-1287: shared nodes ascending, KF1 features
// in node order, with the per-KF1-keypoint filters (MapPoint present, bOnlyStereo) of :1129-1140.
void walk(const osg_kf_side *k1, const osg_kf_side *k2, int only_stereo, Problem &P)
{
    const osg_featvec &fa = k1->fv, &fb = k2->fv;
    int ia = 0, ib = 0;
    while (ia < fa.n_nodes && ib < fb.n_nodes) {
        if (fa.node_id[ia] == fb.node_id[ib]) {
            for (int a = fa.node_start[ia]; a < fa.node_start[ia + 1]; a++) {
                const int idx1 = fa.feat[a];
                if (k1->has_mp[idx1]) continue;
                const bool stereo1 = !k1->two_cam && k1->u_right && k1->u_right[idx1] >= 0;
                if (only_stereo && !stereo1) continue;
                const bool right1 = !(k1->nleft == -1 || idx1 < k1->nleft);
                P.q_feat.push_back(idx1);
                P.q_cb.push_back(fb.node_start[ib]);
                P.q_ce.push_back(fb.node_start[ib + 1]);
                P.qflag.push_back((uint8_t)((stereo1 ? 1 : 0) | (right1 ? 2 : 0)));
            }
            ia++;
            ib++;
        } else if (fa.node_id[ia] < fb.node_id[ib]) {  // lower_bound(f2it->first)
            ia = (int)(std::lower_bound(fa.node_id + ia, fa.node_id + fa.n_nodes, fb.node_id[ib]) - fa.node_id);
        } else {
            ib = (int)(std::lower_bound(fb.node_id + ib, fb.node_id + fb.n_nodes, fa.node_id[ia]) - fb.node_id);
        }
    }
}

int triang_run(osg_ctx *ctx, const osg_kf_side *K1, const osg_kf_side *K2, const osg_triang_geom *G, int B,
               int only_stereo, int coarse, int check_ori, int32_t *match12, int32_t *nmatches)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, B >= 0 && (B == 0 || (K1 && K2 && G && nmatches)), "null argument");
    std::vector<Problem> P(B);
    std::vector<TriArgs> args(B);
    std::vector<size_t> q_base(B + 1, 0), o_base(B + 1, 0);
    osg_packer pk;
    for (int b = 0; b < B; b++) {
        const osg_kf_side *k1 = &K1[b], *k2 = &K2[b];
        int rc = check_side(ctx, k1, "kf1", b);
        if (rc < 0) return rc;
        rc = check_side(ctx, k2, "kf2", b);
        if (rc < 0) return rc;
        OSG_REQUIRE(ctx, (k1->two_cam != 0) == (k2->two_cam != 0),
                    "problem %d: both keyframes need the same rig (R12 is undefined otherwise)", b);
        o_base[b + 1] = o_base[b] + (size_t)k1->n;
        Problem &p = P[b];
        walk(k1, k2, only_stereo, p);
        const int nq = (int)p.q_feat.size();
        q_base[b + 1] = q_base[b] + nq;
        TriArgs &A = args[b];
        A = TriArgs{};
        A.nq = nq;
        A.check_ori = check_ori;
        A.coarse = coarse;
        A.two_cam1 = k1->two_cam != 0;
        A.ep_x = G[b].ep_x;
        A.ep_y = G[b].ep_y;
        std::memcpy(A.F, G[b].F12, sizeof(A.F));
        A.pinhole = G[b].pinhole != 0;
        std::memcpy(A.R12, G[b].R12, sizeof(A.R12));
        std::memcpy(A.t12, G[b].t12, sizeof(A.t12));
        std::memcpy(A.kb, G[b].kb, sizeof(A.kb));
        if (nq == 0) continue;
        p.qdesc.resize((size_t)nq * 8);
        p.qx.resize(nq);
        p.qy.resize(nq);
        p.qang.resize(nq);
        p.qsig.resize(nq);
        for (int i = 0; i < nq; i++) {
            const int f = p.q_feat[i];
            std::memcpy(&p.qdesc[(size_t)i * 8], k1->desc + (size_t)f * 32, 32);
            p.qx[i] = k1->kp_x[f];
            p.qy[i] = k1->kp_y[f];
            p.qang[i] = k1->kp_angle[f];
            const int o1 = k1->kp_octave[f];
            p.qsig[i] = (o1 >= 0 && o1 < k1->n_levels) ? k1->level_sigma2[o1] : 0.f;
        }
        p.flag2.resize(k2->n);
        for (int j = 0; j < k2->n; j++) {
            const bool stereo2 = !k2->two_cam && k2->u_right && k2->u_right[j] >= 0;
            const bool right2 = !(k2->nleft == -1 || j < k2->nleft);
            const bool ok = !k2->has_mp[j] && (!only_stereo || stereo2);
            p.flag2[j] = (uint8_t)((ok ? 1 : 0) | (stereo2 ? 2 : 0) | (right2 ? 4 : 0));
        }
        set_off(A.qdesc, pk.add(p.qdesc.data(), sizeof(uint32_t) * p.qdesc.size()));
        set_off(A.qx, pk.add(p.qx.data(), sizeof(float) * nq));
        set_off(A.qy, pk.add(p.qy.data(), sizeof(float) * nq));
        set_off(A.qang, pk.add(p.qang.data(), sizeof(float) * nq));
        set_off(A.qsig, pk.add(p.qsig.data(), sizeof(float) * nq));
        set_off(A.qflag, pk.add(p.qflag.data(), nq));
        set_off(A.q_cb, pk.add(p.q_cb.data(), sizeof(int32_t) * nq));
        set_off(A.q_ce, pk.add(p.q_ce.data(), sizeof(int32_t) * nq));
        set_off(A.cand, pk.add(k2->fv.feat, sizeof(int32_t) * k2->fv.node_start[k2->fv.n_nodes]));
        set_off(A.desc2, pk.add(k2->desc, (size_t)k2->n * 32));
        set_off(A.x2, pk.add(k2->kp_x, sizeof(float) * k2->n));
        set_off(A.y2, pk.add(k2->kp_y, sizeof(float) * k2->n));
        set_off(A.ang2, pk.add(k2->kp_angle, sizeof(float) * k2->n));
        set_off(A.oct2, pk.add(k2->kp_octave, sizeof(int32_t) * k2->n));
        set_off(A.flag2, pk.add(p.flag2.data(), k2->n));
        set_off(A.scale2, pk.add(k2->scale_factors, sizeof(float) * k2->n_levels));
        set_off(A.sigma2_2, pk.add(k2->level_sigma2, sizeof(float) * k2->n_levels));
    }
    if (B > 0) OSG_REQUIRE(ctx, match12 || o_base[B] == 0, "null match12");
    for (size_t i = 0; i < o_base[B]; i++) match12[i] = -1;
    for (int b = 0; b < B; b++) nmatches[b] = 0;
    const size_t nq_total = q_base[B];
    if (nq_total == 0) return OSG_OK;
    const size_t in_bytes = (pk.total + 255) & ~size_t(255);
    const size_t args_bytes = (sizeof(TriArgs) * (size_t)B + 255) & ~size_t(255);
    const size_t out_bytes = sizeof(int32_t) * (nq_total + B);
    char *pin = (char *)osg_pinned(ctx, in_bytes + args_bytes + out_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    pk.fill_parallel(pin, 8);
    TriArgs *pin_args = (TriArgs *)(pin + in_bytes);
    int32_t *pin_out = (int32_t *)((char *)pin_args + args_bytes);
    char *dev_in = nullptr;
    TriArgs *dev_args = nullptr;
    int32_t *dev_out = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dev_args, SLOT_TMP1, args_bytes);
    OSG_ALLOC(ctx, dev_out, SLOT_TMP2, out_bytes);
    for (int b = 0; b < B; b++) {
        TriArgs &A = args[b];
        relocate(A.qdesc, dev_in);
        relocate(A.qx, dev_in);
        relocate(A.qy, dev_in);
        relocate(A.qang, dev_in);
        relocate(A.qsig, dev_in);
        relocate(A.qflag, dev_in);
        relocate(A.q_cb, dev_in);
        relocate(A.q_ce, dev_in);
        relocate(A.cand, dev_in);
        relocate(A.desc2, dev_in);
        relocate(A.x2, dev_in);
        relocate(A.y2, dev_in);
        relocate(A.ang2, dev_in);
        relocate(A.oct2, dev_in);
        relocate(A.flag2, dev_in);
        relocate(A.scale2, dev_in);
        relocate(A.sigma2_2, dev_in);
        A.out = (GLOBAL int32_t *)(dev_out + q_base[b]);
        A.nmatch = (GLOBAL int32_t *)(dev_out + nq_total + b);
        pin_args[b] = A;
    }
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_in, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_args, pin_args, sizeof(TriArgs) * (size_t)B, hipMemcpyHostToDevice,
                                      ctx->stream));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_triang, dim3(B), dim3(TT), 0, ctx->stream, dev_args);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    OSG_RC(osg_download(ctx, pin_out, dev_out, out_bytes));
    OSG_RC(osg_wait(ctx));
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    for (int b = 0; b < B; b++) {
        const Problem &p = P[b];
        int32_t *m = match12 + o_base[b];
        for (size_t i = 0; i < p.q_feat.size(); i++) m[p.q_feat[i]] = pin_out[q_base[b] + i];
        nmatches[b] = pin_out[nq_total + b];
    }
    return OSG_OK;
}


// ---- Frame::ComputeStereoFishEyeMatches (ref:src/Frame.cc:1546-1603) ---------------------------------
// BFMatcher(NORM_HAMMING).knnMatch(k = 2) of the left stereo rows [monoLeft, Nleft) against the right stereo
// rows [monoRight, Nright) (ref:src/Frame.cc:47, :1569), Lowe's ratio d0 < d1 * 0.7 (float * double),
// then KannalaBrandt8::TriangulateMatches with sigma2 of both octaves and depth > 0.0001f.  One
// left row's wave walks every right row (knn's insertion order: a tie never displaces the first neighbour,
// it becomes the second).  mvRightToLeftMatch is written in query order by the reference, so the last
// accepted query wins: atomicMax over the query index.
struct FishArgs {
    const uint4 *dl, *dr;
    const float2 *kl, *kr;
    const int32_t *ol, *orr;
    const float *sig2;
    float caml[8], camr[8], R[9], t[3];
    int nl, ml, nr, mr;
    GLOBAL int32_t *l2r, *r2l, *nmatch;
    GLOBAL float *depth, *p3d;
};

__global__ __launch_bounds__(256) void k_stereo_fisheye(const FishArgs A)
{
    // one wave per left row: lanes stride over the right rows, each keeps its own (first, second) in row
    // order, then a butterfly merges them: first = the least (distance, row), second = the least of the
    // other summary's first and the winner's second (the multiset's second smallest, as knn's insertion)
    const int lane = threadIdx.x & 63;
    const int i = A.ml + (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (i >= A.nl) return;  // wave-uniform
    const uint4 q0 = A.dl[2 * i], q1 = A.dl[2 * i + 1];
    unsigned long long k1 = ~0ull;  // (distance << 32) | row
    unsigned int b2 = 0x7fffffffu;
    for (int j = A.mr + lane; j < A.nr; j += 64) {
        const uint4 t0 = A.dr[2 * j], t1 = A.dr[2 * j + 1];
        const unsigned int d = __popc(q0.x ^ t0.x) + __popc(q0.y ^ t0.y) + __popc(q0.z ^ t0.z) +
                               __popc(q0.w ^ t0.w) + __popc(q1.x ^ t1.x) + __popc(q1.y ^ t1.y) +
                               __popc(q1.z ^ t1.z) + __popc(q1.w ^ t1.w);
        const unsigned long long k = ((unsigned long long)d << 32) | (unsigned int)j;
        if (k < k1) {
            b2 = (unsigned int)(k1 >> 32) < b2 ? (unsigned int)(k1 >> 32) : b2;
            k1 = k;
        } else if (d < b2) {
            b2 = d;
        }
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const unsigned long long ok1 = __shfl_xor(k1, m);
        const unsigned int ob2 = __shfl_xor(b2, m);
        const unsigned int w1 = (unsigned int)((k1 < ok1 ? ok1 : k1) >> 32);  // the loser's first
        const unsigned int wb2 = k1 < ok1 ? b2 : ob2;                          // the winner's second
        k1 = k1 < ok1 ? k1 : ok1;
        b2 = w1 < wb2 ? w1 : wb2;
    }
    const int b1 = (int)(k1 >> 32), j1 = (int)(k1 & 0xffffffffu);  // every lane holds the merged result
    if (A.nr - A.mr < 2 || !((double)(float)b1 < (double)(float)(int)b2 * 0.7)) return;  // wave-uniform
    // lanes 0 and 1 unproject the left and the right keypoint side by side, lane 0 triangulates
    const float2 a = A.kl[i], b = A.kr[j1];
    float r[3] = {0.f, 0.f, 0.f};
    if (lane < 2) kb8::unproject(lane ? A.camr : A.caml, lane ? b.x : a.x, lane ? b.y : a.y, r);
    const float r1[3] = {r[0], r[1], r[2]};
    const float r2[3] = {__shfl(r[0], 1), __shfl(r[1], 1), __shfl(r[2], 1)};
    if (lane != 0) return;
    float p[3];
    const float z = kb8::triangulate_rays(A.caml, A.camr, r1, r2, a.x, a.y, b.x, b.y, A.R, A.t, A.sig2[A.ol[i]],
                                          A.sig2[A.orr[j1]], p);
    if (!(z > 0.0001f)) return;
    A.l2r[i] = j1;
    A.depth[i] = z;
    A.p3d[3 * i] = p[0];
    A.p3d[3 * i + 1] = p[1];
    A.p3d[3 * i + 2] = p[2];
    atomicMax((int32_t *)&A.r2l[j1], i);
    atomicAdd((int32_t *)A.nmatch, 1);
}

int stereo_fisheye_run(osg_ctx *ctx, int32_t n_left, int32_t mono_left, const uint8_t *desc_left,
                       const float *kp_left, const int32_t *oct_left, int32_t n_right, int32_t mono_right,
                       const uint8_t *desc_right, const float *kp_right, const int32_t *oct_right,
                       const float *level_sigma2, int32_t n_levels, const float *cam_left, const float *cam_right,
                       const float *Rlr, const float *tlr, int32_t *left_to_right, int32_t *right_to_left,
                       float *depth, float *points3d)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, n_left >= 0 && n_right >= 0 && mono_left >= 0 && mono_left <= n_left && mono_right >= 0 &&
                         mono_right <= n_right && n_levels >= 1,
                "sizes (Nleft %d, monoLeft %d, Nright %d, monoRight %d, %d levels)", n_left, mono_left, n_right,
                mono_right, n_levels);
    OSG_REQUIRE(ctx, level_sigma2 && cam_left && cam_right && Rlr && tlr, "null camera / rig / level argument");
    OSG_REQUIRE(ctx, (n_left == 0 || (left_to_right && depth && points3d)) && (n_right == 0 || right_to_left),
                "null output");
    for (int i = 0; i < n_left; i++) {
        left_to_right[i] = -1;
        depth[i] = -1.0f;
        points3d[3 * i] = points3d[3 * i + 1] = points3d[3 * i + 2] = 0.f;
    }
    for (int j = 0; j < n_right; j++) right_to_left[j] = -1;
    const int nq = n_left - mono_left, nt = n_right - mono_right;
    if (nq == 0 || nt < 2) return 0;
    OSG_REQUIRE(ctx, desc_left && kp_left && oct_left && desc_right && kp_right && oct_right, "null keypoint input");
    for (int i = mono_left; i < n_left; i++)
        OSG_REQUIRE(ctx, oct_left[i] >= 0 && oct_left[i] < n_levels, "left octave %d of row %d", oct_left[i], i);
    for (int j = mono_right; j < n_right; j++)
        OSG_REQUIRE(ctx, oct_right[j] >= 0 && oct_right[j] < n_levels, "right octave %d of row %d", oct_right[j],
                    j);
    osg_packer pk;
    const size_t o_dl = pk.add(desc_left, 32 * (size_t)n_left), o_dr = pk.add(desc_right, 32 * (size_t)n_right);
    const size_t o_kl = pk.add(kp_left, 8 * (size_t)n_left), o_kr = pk.add(kp_right, 8 * (size_t)n_right);
    const size_t o_ol = pk.add(oct_left, 4 * (size_t)n_left), o_or = pk.add(oct_right, 4 * (size_t)n_right);
    const size_t o_sg = pk.add(level_sigma2, 4 * (size_t)n_levels);
    const size_t int_bytes = 4 * ((size_t)n_left + n_right + 1);
    const size_t out_bytes = int_bytes + 16 * (size_t)n_left;
    const size_t in_bytes = (pk.total + 255) & ~size_t(255);
    char *pin = (char *)osg_pinned(ctx, in_bytes + out_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    pk.fill(pin);
    char *pin_out = pin + in_bytes;
    char *dev_in = nullptr, *dev_out = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dev_out, SLOT_TMP2, out_bytes);
    FishArgs A{};
    A.dl = (const uint4 *)(dev_in + o_dl);
    A.dr = (const uint4 *)(dev_in + o_dr);
    A.kl = (const float2 *)(dev_in + o_kl);
    A.kr = (const float2 *)(dev_in + o_kr);
    A.ol = (const int32_t *)(dev_in + o_ol);
    A.orr = (const int32_t *)(dev_in + o_or);
    A.sig2 = (const float *)(dev_in + o_sg);
    std::copy(cam_left, cam_left + 8, A.caml);
    std::copy(cam_right, cam_right + 8, A.camr);
    std::copy(Rlr, Rlr + 9, A.R);
    std::copy(tlr, tlr + 3, A.t);
    A.nl = n_left;
    A.ml = mono_left;
    A.nr = n_right;
    A.mr = mono_right;
    A.l2r = (GLOBAL int32_t *)dev_out;
    A.r2l = A.l2r + n_left;
    A.nmatch = A.r2l + n_right;
    A.depth = (GLOBAL float *)(dev_out + int_bytes);
    A.p3d = A.depth + n_left;
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_in, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemsetAsync(dev_out, 0xff, 4 * ((size_t)n_left + n_right), ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemsetAsync(dev_out + 4 * ((size_t)n_left + n_right), 0, 4, ctx->stream));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_stereo_fisheye, dim3((nq + 3) / 4), dim3(256), 0, ctx->stream, A);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    OSG_RC(osg_download(ctx, pin_out, dev_out, out_bytes));
    OSG_RC(osg_wait(ctx));
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    const int32_t *o_l2r = (const int32_t *)pin_out, *o_r2l = o_l2r + n_left;
    const float *o_depth = (const float *)(pin_out + int_bytes), *o_p3d = o_depth + n_left;
    for (int i = mono_left; i < n_left; i++) {
        if (o_l2r[i] < 0) continue;
        left_to_right[i] = o_l2r[i];
        depth[i] = o_depth[i];
        for (int k = 0; k < 3; k++) points3d[3 * i + k] = o_p3d[3 * i + k];
    }
    for (int j = mono_right; j < n_right; j++) right_to_left[j] = o_r2l[j];
    return o_r2l[n_right];
}

}  // namespace

extern "C" {

int osg_compute_stereo_fisheye_matches(osg_ctx *ctx, int32_t n_left, int32_t mono_left, const uint8_t *desc_left,
                                       const float *kp_left, const int32_t *oct_left, int32_t n_right,
                                       int32_t mono_right, const uint8_t *desc_right, const float *kp_right,
                                       const int32_t *oct_right, const float *level_sigma2, int32_t n_levels,
                                       const float *cam_left, const float *cam_right, const float *Rlr,
                                       const float *tlr, int32_t *left_to_right, int32_t *right_to_left,
                                       float *depth, float *points3d)
{
    return stereo_fisheye_run(ctx, n_left, mono_left, desc_left, kp_left, oct_left, n_right, mono_right, desc_right,
                              kp_right, oct_right, level_sigma2, n_levels, cam_left, cam_right, Rlr, tlr,
                              left_to_right, right_to_left, depth, points3d);
}

int osg_search_for_triangulation(osg_ctx *ctx, const osg_kf_side *kf1, const osg_kf_side *kf2,
                                 const osg_triang_geom *geom, int only_stereo, int coarse, int check_orientation,
                                 int32_t *match12)
{
    int32_t n = 0;
    const int rc = triang_run(ctx, kf1, kf2, geom, 1, only_stereo, coarse, check_orientation, match12, &n);
    return rc < 0 ? rc : n;
}

int osg_search_for_triangulation_batch(osg_ctx *ctx, const osg_kf_side *kf1, const osg_kf_side *kf2,
                                       const osg_triang_geom *geom, int32_t B, int only_stereo, int coarse,
                                       int check_orientation, int32_t *match12, int32_t *nmatches)
{
    return triang_run(ctx, kf1, kf2, geom, B, only_stereo, coarse, check_orientation, match12, nmatches);
}

}  // extern "C"
