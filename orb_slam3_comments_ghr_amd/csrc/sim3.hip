// sim3.hip — the Sim3 projection matchers of LoopClosing on gfx950:
//   SearchByProjection(KeyFrame*, Sim3f& Scw, const vector<MapPoint*>&, vector<MapPoint*>& vpMatched, th, ratioHamming)
//                                                                     ref:src/ORBmatcher.cc:498-621
//   and its vpPointsKFs / vpMatchedKF overload                         ref:src/ORBmatcher.cc:623-733
// (LoopClosing calls them at ref:src/LoopClosing.cc:1062, 1091, 1368), and
//   SearchBySim3(KeyFrame*, KeyFrame*, vector<MapPoint*>& vpMatches12, Sim3f& S12, th)
//                                                                     ref:src/ORBmatcher.cc:1696-1939
// whose two projection searches (KF1's MapPoints into KF2, KF2's into KF1) take no slots: each
// query's strict-'<' minimum over its window is final after one round (`once`), accepted iff
// bestDist <= TH_HIGH, and the host keeps the mutual pairs.
//
// Per MapPoint (query, list order): KeyFrame::GetFeaturesInArea (ix outer, iy inner, strict window;
// ref:src/KeyFrame.cc:859-907), skip slots already in vpMatched, level window [pred - 1, pred], the
// strict-'<' minimum distance; accept iff bestDist <= TH_LOW * ratioHamming (float), and then the
// slot is taken: vpMatched[bestIdx] = pMP, seen by every later MapPoint.  That sequential claim is
// solved as a fixed point (as k_match does for SearchByProjection): every query re-walks its window
// against the claims of lower-indexed queries (LDS atomicMin table) until no choice changes; the
// fixed point is the sequential result (induction on the query index).  One 1024-lane workgroup per
// keyframe; grid = keyframes.
#include <algorithm>
#include <vector>

#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int ST = 1024;
constexpr int MAX_SLOTS = 8192;  // claim table in LDS

struct Sim3Args {
    int nq, n_slots;
    float min_x, min_y, inv_w, inv_h, th, thr;
    GLOBAL const uint32_t *kdesc;
    GLOBAL const float *kp_x, *kp_y;
    GLOBAL const int32_t *kp_octave;
    GLOBAL const int32_t *gs, *gi;
    GLOBAL const float *scale;
    GLOBAL const uint8_t *taken0;  // vpMatched[idx] != NULL before the call
    GLOBAL const uint32_t *qdesc;
    GLOBAL const uint8_t *valid;
    GLOBAL const float *u, *v;
    GLOBAL const int32_t *lvl;
    GLOBAL int32_t *best;          // per query: matched slot or -1
    GLOBAL int32_t *stats;         // per problem: rounds
    int once;                      // SearchBySim3: no slot claims, one round
};

__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// The query's choice given the claim table: the first minimum over unblocked candidates in area order.
__device__ int choose(const Sim3Args &A, int q, const int *claim, const uint8_t *taken0)
{
    const int lvl = A.lvl[q];
    const float u = A.u[q], v = A.v[q];
    const float r = A.th * A.scale[lvl];  // ref:src/ORBmatcher.cc:574 / 690
    int minCX = (int)floorf((u - A.min_x - r) * A.inv_w);
    minCX = minCX < 0 ? 0 : minCX;
    int maxCX = (int)ceilf((u - A.min_x + r) * A.inv_w);
    maxCX = maxCX > OSG_GRID_COLS - 1 ? OSG_GRID_COLS - 1 : maxCX;
    int minCY = (int)floorf((v - A.min_y - r) * A.inv_h);
    minCY = minCY < 0 ? 0 : minCY;
    int maxCY = (int)ceilf((v - A.min_y + r) * A.inv_h);
    maxCY = maxCY > OSG_GRID_ROWS - 1 ? OSG_GRID_ROWS - 1 : maxCY;
    const bool empty = minCX >= OSG_GRID_COLS || maxCX < 0 || minCY >= OSG_GRID_ROWS || maxCY < 0;
    const u32x4 qa = *(GLOBAL const u32x4 *)(A.qdesc + 8 * q), qb = *(GLOBAL const u32x4 *)(A.qdesc + 8 * q + 4);
    int bd = 256, bi = -1;  // :585-586
    for (int ix = empty ? maxCX + 1 : minCX; ix <= maxCX; ix++) {
        const int j1 = A.gs[ix * OSG_GRID_ROWS + maxCY + 1];
        for (int j = A.gs[ix * OSG_GRID_ROWS + minCY]; j < j1; j++) {
            const int idx = A.gi[j];
            const float kx = A.kp_x[idx], ky = A.kp_y[idx];
            if (!(fabsf(kx - u) < r && fabsf(ky - v) < r)) continue;  // ref:src/KeyFrame.cc:897-900
            if (taken0[idx] || claim[idx] < q) continue;              // vpMatched[idx], :591-592
            const int oct = A.kp_octave[idx];
            if (oct < lvl - 1 || oct > lvl) continue;                  // :597-598
            const u32x4 ka = *(GLOBAL const u32x4 *)(A.kdesc + 8 * idx), kb = *(GLOBAL const u32x4 *)(A.kdesc + 8 * idx + 4);
            uint32_t d = __popc(qa.x ^ ka.x);
            d = bcnt_acc(qa.y ^ ka.y, d);
            d = bcnt_acc(qa.z ^ ka.z, d);
            d = bcnt_acc(qa.w ^ ka.w, d);
            d = bcnt_acc(qb.x ^ kb.x, d);
            d = bcnt_acc(qb.y ^ kb.y, d);
            d = bcnt_acc(qb.z ^ kb.z, d);
            d = bcnt_acc(qb.w ^ kb.w, d);
            if ((int)d < bd) {  // :604-608
                bd = (int)d;
                bi = idx;
            }
        }
    }
    return ((float)bd <= A.thr) ? bi : -1;  // bestDist <= TH_LOW * ratioHamming, :612 / :724
}

__global__ __launch_bounds__(ST) void k_sim3(const Sim3Args *__restrict__ args)
{
    const Sim3Args &A = args[blockIdx.x];
    __shared__ int claim[MAX_SLOTS];
    __shared__ uint8_t taken0[MAX_SLOTS];
    __shared__ int s_changed;
    const int tid = threadIdx.x;
    for (int s = tid; s < A.n_slots; s += ST) {
        claim[s] = 0x7FFFFFFF;
        taken0[s] = A.taken0[s];
    }
    for (int q = tid; q < A.nq; q += ST) A.best[q] = -1;
    __syncthreads();
    int rounds = 0;
    for (;;) {  // terminates: after round r the first r queries are final
        if (tid == 0) s_changed = 0;
        __syncthreads();
        bool changed = false;
        for (int q = tid; q < A.nq; q += ST) {
            if (!A.valid[q]) continue;
            const int b = choose(A, q, claim, taken0);
            if (b != A.best[q]) {
                A.best[q] = b;
                changed = true;
            }
        }
        if (changed) s_changed = 1;
        rounds++;
        __syncthreads();
        if (!s_changed || A.once) break;
        for (int s = tid; s < A.n_slots; s += ST) claim[s] = 0x7FFFFFFF;
        __syncthreads();
        for (int q = tid; q < A.nq; q += ST) {
            const int b = A.best[q];
            if (b >= 0) atomicMin(&claim[b], q);
        }
        __syncthreads();
    }
    if (tid == 0) A.stats[0] = rounds;
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

// once = 0: the Sim3 projections (slot claims, thr = TH_LOW * ratio, results into slot_query);
// once = 1: SearchBySim3's searches (thr = TH_HIGH, per-query results into query_best)
int sim3_run(osg_ctx *ctx, const osg_frame *KF, const osg_fuse_queries *Q, int B, float th, float ratio,
             int32_t *slot_query, int32_t *nmatches, int once = 0, int32_t *query_best = nullptr)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, B >= 0 && (B == 0 || (KF && Q && nmatches && slot_query)), "null argument");
    osg_packer pk;
    std::vector<Sim3Args> args(B);
    std::vector<std::vector<uint8_t>> taken(B);
    std::vector<size_t> q_base(B + 1, 0), s_base(B + 1, 0);
    for (int b = 0; b < B; b++) {
        const osg_frame *F = &KF[b];
        const osg_fuse_queries *S = &Q[b];
        int rc = osg_check_frame(ctx, F);
        if (rc < 0) return osg_set_error(ctx, rc, "problem %d: %s", b, osg_ctx_last_error(ctx));
        OSG_REQUIRE(ctx, S->n >= 0, "problem %d: query count", b);
        OSG_REQUIRE(ctx, F->n <= MAX_SLOTS, "problem %d: %d keypoints > %d", b, F->n, MAX_SLOTS);
        q_base[b + 1] = q_base[b] + (size_t)S->n;
        s_base[b + 1] = s_base[b] + (size_t)F->n;
        Sim3Args &A = args[b];
        A = Sim3Args{};
        A.nq = S->n;
        A.n_slots = F->n;
        A.min_x = F->min_x;
        A.min_y = F->min_y;
        A.inv_w = F->grid_inv_w;
        A.inv_h = F->grid_inv_h;
        A.th = th;
        A.thr = once ? (float)OSG_TH_HIGH : (float)OSG_TH_LOW * ratio;
        A.once = once;
        const int32_t *sq = slot_query + s_base[b];
        taken[b].resize(F->n);
        for (int i = 0; i < F->n; i++) {
            OSG_REQUIRE(ctx, sq[i] == -1 || sq[i] == -2, "problem %d: slot_query[%d] must be -1 (free) or -2 (taken)", b, i);
            taken[b][i] = sq[i] == -2;
        }
        if (S->n == 0) continue;
        OSG_REQUIRE(ctx, S->desc && S->valid && S->u && S->v && S->pred_level, "problem %d: query arrays", b);
        for (int i = 0; i < S->n; i++)
            if (S->valid[i] && (S->pred_level[i] < 0 || S->pred_level[i] >= F->n_levels))
                return osg_set_error(ctx, OSG_E_INVALID, "problem %d: pred_level[%d] = %d out of range", b, i,
                                     S->pred_level[i]);
        set_off(A.kdesc, pk.add(F->desc, (size_t)F->n * 32));
        set_off(A.kp_x, pk.add(F->kp_x, sizeof(float) * F->n));
        set_off(A.kp_y, pk.add(F->kp_y, sizeof(float) * F->n));
        set_off(A.kp_octave, pk.add(F->kp_octave, sizeof(int32_t) * F->n));
        set_off(A.gs, pk.add(F->grid_start, sizeof(int32_t) * (OSG_GRID_CELLS + 1)));
        set_off(A.gi, pk.add(F->grid_idx, sizeof(int32_t) * F->grid_start[OSG_GRID_CELLS]));
        set_off(A.scale, pk.add(F->scale_factors, sizeof(float) * F->n_levels));
        set_off(A.taken0, pk.add(taken[b].data(), F->n));
        set_off(A.qdesc, pk.add(S->desc, (size_t)S->n * 32));
        set_off(A.valid, pk.add(S->valid, S->n));
        set_off(A.u, pk.add(S->u, sizeof(float) * S->n));
        set_off(A.v, pk.add(S->v, sizeof(float) * S->n));
        set_off(A.lvl, pk.add(S->pred_level, sizeof(int32_t) * S->n));
    }
    for (int b = 0; b < B; b++) nmatches[b] = 0;
    const size_t nq_total = q_base[B];
    if (query_best)
        for (size_t i = 0; i < nq_total; i++) query_best[i] = -1;
    if (nq_total == 0) return OSG_OK;
    const size_t in_bytes = (pk.total + 255) & ~size_t(255);
    const size_t args_bytes = (sizeof(Sim3Args) * (size_t)B + 255) & ~size_t(255);
    const size_t out_bytes = sizeof(int32_t) * (nq_total + B);
    char *pin = (char *)osg_pinned(ctx, in_bytes + args_bytes + out_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    pk.fill_parallel(pin, 8);
    Sim3Args *pin_args = (Sim3Args *)(pin + in_bytes);
    int32_t *pin_out = (int32_t *)((char *)pin_args + args_bytes);
    char *dev_in = nullptr;
    Sim3Args *dev_args = nullptr;
    int32_t *dev_out = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dev_args, SLOT_TMP1, args_bytes);
    OSG_ALLOC(ctx, dev_out, SLOT_TMP2, out_bytes);
    for (int b = 0; b < B; b++) {
        Sim3Args &A = args[b];
        relocate(A.kdesc, dev_in);
        relocate(A.kp_x, dev_in);
        relocate(A.kp_y, dev_in);
        relocate(A.kp_octave, dev_in);
        relocate(A.gs, dev_in);
        relocate(A.gi, dev_in);
        relocate(A.scale, dev_in);
        relocate(A.taken0, dev_in);
        relocate(A.qdesc, dev_in);
        relocate(A.valid, dev_in);
        relocate(A.u, dev_in);
        relocate(A.v, dev_in);
        relocate(A.lvl, dev_in);
        A.best = (GLOBAL int32_t *)(dev_out + q_base[b]);
        A.stats = (GLOBAL int32_t *)(dev_out + nq_total + b);
        pin_args[b] = A;
    }
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_in, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_args, pin_args, sizeof(Sim3Args) * (size_t)B, hipMemcpyHostToDevice,
                                      ctx->stream));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_sim3, dim3(B), dim3(ST), 0, ctx->stream, dev_args);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    OSG_RC(osg_download(ctx, pin_out, dev_out, out_bytes));
    OSG_RC(osg_wait(ctx));
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    int32_t rounds_max = 0;
    if (query_best) {
        for (size_t i = 0; i < nq_total; i++) query_best[i] = pin_out[i];
        for (int b = 0; b < B; b++) rounds_max = std::max(rounds_max, pin_out[nq_total + b]);
        ctx->match_stats[1] = rounds_max;
        return OSG_OK;
    }
    for (int b = 0; b < B; b++) {
        int32_t *sq = slot_query + s_base[b];
        int nm = 0;
        for (size_t i = q_base[b]; i < q_base[b + 1]; i++) {
            const int s = pin_out[i];
            if (s >= 0) {
                sq[s] = (int32_t)(i - q_base[b]);
                nm++;
            }
        }
        nmatches[b] = nm;
        rounds_max = std::max(rounds_max, pin_out[nq_total + b]);
    }
    ctx->match_stats[1] = rounds_max;
    return OSG_OK;
}

}  // namespace

extern "C" {

int osg_search_by_projection_sim3(osg_ctx *ctx, const osg_frame *KF, const osg_fuse_queries *Q, float th,
                                  float ratio_hamming, int32_t *slot_query)
{
    int32_t n = 0;
    const int rc = sim3_run(ctx, KF, Q, 1, th, ratio_hamming, slot_query, &n);
    return rc < 0 ? rc : n;
}

int osg_search_by_projection_sim3_batch(osg_ctx *ctx, const osg_frame *KF, const osg_fuse_queries *Q, int32_t B,
                                        float th, float ratio_hamming, int32_t *slot_query, int32_t *nmatches)
{
    return sim3_run(ctx, KF, Q, B, th, ratio_hamming, slot_query, nmatches);
}

// SearchBySim3: both directions in one launch (problem 0: q12 against KF2, problem 1: q21 against
// KF1), then the mutual check of ref:src/ORBmatcher.cc:1920-1936 in KF1 slot order.
int osg_search_by_sim3(osg_ctx *ctx, const osg_frame *kf1, const osg_frame *kf2, const osg_fuse_queries *q12,
                       const osg_fuse_queries *q21, float th, int32_t *match12)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, kf1 && kf2 && q12 && q21 && match12, "null argument");
    OSG_REQUIRE(ctx, q12->n == kf1->n && q21->n == kf2->n,
                "q12 needs one query per KF1 keypoint (%d vs %d), q21 one per KF2 keypoint (%d vs %d)", q12->n,
                kf1->n, q21->n, kf2->n);
    const osg_frame F[2] = {*kf2, *kf1};
    const osg_fuse_queries Q[2] = {*q12, *q21};
    std::vector<int32_t> slots((size_t)kf1->n + kf2->n, -1), best((size_t)q12->n + q21->n, -1);
    int32_t nm[2] = {0, 0};
    const int rc = sim3_run(ctx, F, Q, 2, th, 1.0f, slots.data(), nm, 1, best.data());
    if (rc < 0) return rc;
    const int32_t *vnMatch1 = best.data(), *vnMatch2 = best.data() + q12->n;
    int nFound = 0;
    for (int i1 = 0; i1 < kf1->n; i1++) {
        const int idx2 = vnMatch1[i1];
        match12[i1] = -1;
        if (idx2 >= 0 && vnMatch2[idx2] == i1) {
            match12[i1] = idx2;
            nFound++;
        }
    }
    return nFound;
}

}  // extern "C"
