// fuse.hip — the search half of ORBmatcher::Fuse on gfx950.
//
//   osg_fuse_search[_batch]  gated = 1: Fuse(KeyFrame*, vector<MapPoint*>, th, bRight)  ref:src/ORBmatcher.cc:1330-1541
//                            gated = 0: Fuse(KeyFrame*, Sim3f, vector<MapPoint*>, th, vpReplacePoint)
//                                                                                      ref:src/ORBmatcher.cc:1553-1694
//
// Unlike the SearchByProjection family there is no claim inside the search: the best keypoint of a
// MapPoint does not depend on what earlier MapPoints matched (the replace / add that follows is the
// caller's, in MapPoint order).  So the kernel is one lane per MapPoint with no cross-lane step:
// KeyFrame::GetFeaturesInArea's walk (ix outer, iy inner; the cells iy = minCY..maxCY of one
// column are one contiguous CSR run, cell = ix*48 + iy), the level window, the chi2 reprojection
// gate and the strict-'<' minimum distance, in the reference's candidate order and float
// arithmetic (built with -ffp-contract=off).  grid = (query blocks, problems).
#include <algorithm>
#include <vector>

#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int FT = 256;  // lanes (MapPoints) per workgroup

struct FuseArgs {
    int nq, off, n_levels, gated;
    float min_x, min_y, inv_w, inv_h, th;
    GLOBAL const uint32_t *kdesc;
    GLOBAL const float *kp_x, *kp_y;
    GLOBAL const int32_t *kp_octave;
    GLOBAL const float *u_right;  // mvuRight indexed by the camera-local keypoint index; NULL = all < 0
    GLOBAL const int32_t *gs, *gi;
    GLOBAL const float *scale, *inv_s2;
    GLOBAL const uint32_t *qdesc;
    GLOBAL const uint8_t *valid;
    GLOBAL const float *u, *v, *ur;
    GLOBAL const int32_t *lvl;
    GLOBAL int32_t *out;  // per query {best_idx, best_dist}
};

__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(FT) void k_fuse(const FuseArgs *__restrict__ args)
{
    const FuseArgs &A = args[blockIdx.y];
    const int q = blockIdx.x * FT + threadIdx.x;
    if (q >= A.nq) return;
    int best = 256, best_idx = -1;
    if (A.valid[q]) {
        const int lvl = A.lvl[q];
        const float u = A.u[q], v = A.v[q];
        const float ur = A.ur ? A.ur[q] : 0.f;
        const float r = A.th * A.scale[lvl];  // ref:src/ORBmatcher.cc:1437 / :1626
        const u32x4 qa = *(GLOBAL const u32x4 *)(A.qdesc + 8 * q), qb = *(GLOBAL const u32x4 *)(A.qdesc + 8 * q + 4);
        // KeyFrame::GetFeaturesInArea bounds, ref:src/KeyFrame.cc:865-884
        int minCX = (int)floorf((u - A.min_x - r) * A.inv_w);
        minCX = minCX < 0 ? 0 : minCX;
        int maxCX = (int)ceilf((u - A.min_x + r) * A.inv_w);
        maxCX = maxCX > OSG_GRID_COLS - 1 ? OSG_GRID_COLS - 1 : maxCX;
        int minCY = (int)floorf((v - A.min_y - r) * A.inv_h);
        minCY = minCY < 0 ? 0 : minCY;
        int maxCY = (int)ceilf((v - A.min_y + r) * A.inv_h);
        maxCY = maxCY > OSG_GRID_ROWS - 1 ? OSG_GRID_ROWS - 1 : maxCY;
        const bool empty = minCX >= OSG_GRID_COLS || maxCX < 0 || minCY >= OSG_GRID_ROWS || maxCY < 0;
        int bd = A.gated ? 256 : 0x7FFFFFFF;  // ref:src/ORBmatcher.cc:1451 / :1638
        for (int ix = empty ? maxCX + 1 : minCX; ix <= maxCX; ix++) {
            const int j1 = A.gs[ix * OSG_GRID_ROWS + maxCY + 1];
            for (int j = A.gs[ix * OSG_GRID_ROWS + minCY]; j < j1; j++) {
                const int idx = A.gi[j];
                const int k = idx + A.off;  // mvKeysUn / mvKeys / mvKeysRight[idx]
                const float kx = A.kp_x[k], ky = A.kp_y[k];
                const int oct = A.kp_octave[k];
                if (!(fabsf(kx - u) < r && fabsf(ky - v) < r)) continue;   // ref:src/KeyFrame.cc:897-900
                if (oct < lvl - 1 || oct > lvl) continue;                  // ref:src/ORBmatcher.cc:1462 / :1645
                if (A.gated) {
                    const float kpr = A.u_right ? A.u_right[idx] : -1.f;   // mvuRight[idx], :1466
                    const float ex = u - kx;
                    const float ey = v - ky;
                    if (kpr >= 0) {
                        const float er = ur - kpr;
                        const float e2 = ex * ex + ey * ey + er * er;
                        if ((double)(e2 * A.inv_s2[oct]) > 7.8) continue;  // :1480
                    } else {
                        const float e2 = ex * ex + ey * ey;
                        if ((double)(e2 * A.inv_s2[oct]) > 5.99) continue; // :1493
                    }
                }
                const u32x4 ka = *(GLOBAL const u32x4 *)(A.kdesc + 8 * k), kb = *(GLOBAL const u32x4 *)(A.kdesc + 8 * k + 4);
                uint32_t d = __popc(qa.x ^ ka.x);
                d = bcnt_acc(qa.y ^ ka.y, d);
                d = bcnt_acc(qa.z ^ ka.z, d);
                d = bcnt_acc(qa.w ^ ka.w, d);
                d = bcnt_acc(qb.x ^ kb.x, d);
                d = bcnt_acc(qb.y ^ kb.y, d);
                d = bcnt_acc(qb.z ^ kb.z, d);
                d = bcnt_acc(qb.w ^ kb.w, d);
                if ((int)d < bd) {  // strict: the first candidate in area order wins
                    bd = (int)d;
                    best_idx = k;   // :1498 idx += NLeft
                }
            }
        }
        best = bd < 256 ? bd : 256;
        if (bd > OSG_TH_LOW) best_idx = -1;  // :1514 / :1661
    }
    A.out[2 * q] = best_idx;
    A.out[2 * q + 1] = best;
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

int fuse_run(osg_ctx *ctx, const osg_frame *KF, const osg_fuse_queries *Q, int B, float th, int right, int gated,
             int32_t *best_idx, int32_t *best_dist, int32_t *nfused)
{
    OSG_REQUIRE(ctx, B >= 0 && (B == 0 || (KF && Q && nfused)), "null argument");
    osg_packer pk;
    std::vector<FuseArgs> args(B);
    std::vector<size_t> q_base(B + 1, 0);
    int maxq = 0;
    for (int b = 0; b < B; b++) {
        const osg_frame *F = &KF[b];
        const osg_fuse_queries *S = &Q[b];
        int rc = osg_check_frame(ctx, F);
        if (rc < 0) return osg_set_error(ctx, rc, "problem %d: %s", b, osg_ctx_last_error(ctx));
        OSG_REQUIRE(ctx, S->n >= 0, "problem %d: query count", b);
        OSG_REQUIRE(ctx, !right || F->nleft != -1, "problem %d: bRight needs a two-camera keyframe (nleft != -1)", b);
        q_base[b + 1] = q_base[b] + (size_t)S->n;
        maxq = std::max(maxq, S->n);
        FuseArgs &A = args[b];
        A = FuseArgs{};
        A.nq = S->n;
        A.off = right ? F->nleft : 0;
        A.n_levels = F->n_levels;
        A.gated = gated;
        A.min_x = F->min_x;
        A.min_y = F->min_y;
        A.inv_w = F->grid_inv_w;
        A.inv_h = F->grid_inv_h;
        A.th = th;
        if (S->n == 0) continue;
        OSG_REQUIRE(ctx, S->desc && S->valid && S->u && S->v && S->pred_level, "problem %d: query arrays", b);
        for (int i = 0; i < S->n; i++)
            if (S->valid[i] && (S->pred_level[i] < 0 || S->pred_level[i] >= F->n_levels))
                return osg_set_error(ctx, OSG_E_INVALID, "problem %d: pred_level[%d] = %d out of range", b, i,
                                     S->pred_level[i]);
        if (gated) {
            OSG_REQUIRE(ctx, S->inv_level_sigma2, "problem %d: inv_level_sigma2 (gated)", b);
            bool any_ur = false;
            for (int i = 0; F->u_right && i < F->n && !any_ur; i++) any_ur = F->u_right[i] >= 0;
            OSG_REQUIRE(ctx, S->ur || !any_ur, "problem %d: ur needed (keyframe has u_right >= 0)", b);
        }
        set_off(A.kdesc, pk.add(F->desc, (size_t)F->n * 32));
        set_off(A.kp_x, pk.add(F->kp_x, sizeof(float) * F->n));
        set_off(A.kp_y, pk.add(F->kp_y, sizeof(float) * F->n));
        set_off(A.kp_octave, pk.add(F->kp_octave, sizeof(int32_t) * F->n));
        if (gated) set_off(A.u_right, pk.add(F->u_right, sizeof(float) * F->n));
        const int32_t *gs = right ? F->grid_start_r : F->grid_start;
        const int32_t *gi = right ? F->grid_idx_r : F->grid_idx;
        set_off(A.gs, pk.add(gs, sizeof(int32_t) * (OSG_GRID_CELLS + 1)));
        set_off(A.gi, pk.add(gi, sizeof(int32_t) * gs[OSG_GRID_CELLS]));
        set_off(A.scale, pk.add(F->scale_factors, sizeof(float) * F->n_levels));
        if (gated) set_off(A.inv_s2, pk.add(S->inv_level_sigma2, sizeof(float) * F->n_levels));
        set_off(A.qdesc, pk.add(S->desc, (size_t)S->n * 32));
        set_off(A.valid, pk.add(S->valid, S->n));
        set_off(A.u, pk.add(S->u, sizeof(float) * S->n));
        set_off(A.v, pk.add(S->v, sizeof(float) * S->n));
        if (gated) set_off(A.ur, pk.add(S->ur, sizeof(float) * S->n));
        set_off(A.lvl, pk.add(S->pred_level, sizeof(int32_t) * S->n));
    }
    const size_t nq_total = q_base[B];
    for (int b = 0; b < B; b++) nfused[b] = 0;
    if (nq_total == 0) return OSG_OK;
    OSG_REQUIRE(ctx, best_idx && best_dist, "null output");
    const size_t in_bytes = (pk.total + 255) & ~size_t(255);
    const size_t args_bytes = sizeof(FuseArgs) * (size_t)B;
    const size_t out_bytes = sizeof(int32_t) * 2 * nq_total;
    char *pin = (char *)osg_pinned(ctx, in_bytes + ((args_bytes + 255) & ~size_t(255)) + out_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    pk.fill_parallel(pin, 8);
    FuseArgs *pin_args = (FuseArgs *)(pin + in_bytes);
    int32_t *pin_out = (int32_t *)((char *)pin_args + ((args_bytes + 255) & ~size_t(255)));
    char *dev_in = nullptr;
    FuseArgs *dev_args = nullptr;
    int32_t *dev_out = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dev_args, SLOT_TMP1, args_bytes);
    OSG_ALLOC(ctx, dev_out, SLOT_TMP2, out_bytes);
    for (int b = 0; b < B; b++) {
        FuseArgs &A = args[b];
        relocate(A.kdesc, dev_in);
        relocate(A.kp_x, dev_in);
        relocate(A.kp_y, dev_in);
        relocate(A.kp_octave, dev_in);
        relocate(A.u_right, dev_in);
        relocate(A.gs, dev_in);
        relocate(A.gi, dev_in);
        relocate(A.scale, dev_in);
        relocate(A.inv_s2, dev_in);
        relocate(A.qdesc, dev_in);
        relocate(A.valid, dev_in);
        relocate(A.u, dev_in);
        relocate(A.v, dev_in);
        relocate(A.ur, dev_in);
        relocate(A.lvl, dev_in);
        A.out = (GLOBAL int32_t *)(dev_out + 2 * q_base[b]);
        pin_args[b] = A;
    }
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_in, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_args, pin_args, args_bytes, hipMemcpyHostToDevice, ctx->stream));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_fuse, dim3((maxq + FT - 1) / FT, B), dim3(FT), 0, ctx->stream, dev_args);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    OSG_RC(osg_download(ctx, pin_out, dev_out, out_bytes));
    OSG_RC(osg_wait(ctx));
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    for (int b = 0; b < B; b++) {
        int nf = 0;
        for (size_t i = q_base[b]; i < q_base[b + 1]; i++) {
            best_idx[i] = pin_out[2 * i];
            best_dist[i] = pin_out[2 * i + 1];
            nf += best_idx[i] >= 0;
        }
        nfused[b] = nf;
    }
    return OSG_OK;
}

}  // namespace

extern "C" {

int osg_fuse_search(osg_ctx *ctx, const osg_frame *KF, const osg_fuse_queries *Q, float th, int right, int gated,
                    int32_t *best_idx, int32_t *best_dist)
{
    if (!ctx) return OSG_E_INVALID;
    int32_t nf = 0;
    const int rc = fuse_run(ctx, KF, Q, 1, th, right, gated, best_idx, best_dist, &nf);
    return rc < 0 ? rc : nf;
}

int osg_fuse_search_batch(osg_ctx *ctx, const osg_frame *KF, const osg_fuse_queries *Q, int32_t B, float th,
                          int right, int gated, int32_t *best_idx, int32_t *best_dist, int32_t *nfused)
{
    if (!ctx) return OSG_E_INVALID;
    return fuse_run(ctx, KF, Q, B, th, right, gated, best_idx, best_dist, nfused);
}

}  // extern "C"
