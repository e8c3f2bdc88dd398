// init.hip — ORBmatcher::SearchForInitialization on gfx950 (ref:src/ORBmatcher.cc:735-878), the
// matcher of monocular initialisation (Tracking::MonocularInitialization, ref:src/Tracking.cc:2956).
//
// The reference walks F1's level-0 keypoints in order and carries state across them: a candidate
// i2 is skipped when vMatchedDistance[i2] <= dist (i2 already matched at least as well), and an
// accepted match steals i2 from its earlier owner (vnMatches21).  Each keypoint's decision depends
// on every earlier one, so the walk stays sequential — in ONE wave per frame pair, with the work of
// each step spread over the 64 lanes: the lanes take the window's candidates (F2::GetFeaturesInArea
// order, ix outer / iy inner: the CSR positions of one column's cells are contiguous and increase
// with ix, so the CSR position IS the enumeration order), test the window and level, compute the
// distance, apply the vMatchedDistance skip (LDS), and a wave reduction of packed keys
// (dist << 23 | CSR position) gives the best (first minimum) and the second distance (with
// multiplicity).  Lane 0 then applies the accept / steal / histogram step.  grid = frame pairs.
#include <algorithm>
#include <vector>

#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int MAX_N2 = 8192;
constexpr uint32_t KEY_NONE = 0xFFFFFFFFu;

struct InitArgs {
    int n1, n2, window, check_ori;
    float nnratio, min_x, min_y, inv_w, inv_h;
    GLOBAL const uint32_t *desc1;
    GLOBAL const int32_t *oct1;
    GLOBAL const float *ang1;
    GLOBAL const float *prev;      // n1 x 2 (vbPrevMatched)
    GLOBAL const uint32_t *desc2;
    GLOBAL const float *x2, *y2, *ang2;
    GLOBAL const int32_t *oct2;
    GLOBAL const int32_t *gs, *gi;
    GLOBAL int32_t *m12;           // n1 out
    GLOBAL int32_t *nmatch;        // 1 out
};

__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int rot_bin(float a, float b)
{  // ref:src/ORBmatcher.cc:831-838, factor = 1.0f/HISTO_LENGTH (kept upstream bug)
    const float factor = 1.0f / OSG_HISTO_LENGTH;
    float rot = a - b;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == OSG_HISTO_LENGTH) bin = 0;
    return bin;
}

__global__ __launch_bounds__(64) void k_init(const InitArgs *__restrict__ args)
{
    const InitArgs &A = args[blockIdx.x];
    __shared__ int s_md[MAX_N2];    // vMatchedDistance
    __shared__ int s_21[MAX_N2];    // vnMatches21
    __shared__ int s_hist[OSG_HISTO_LENGTH];
    const int lane = threadIdx.x;
    for (int i = lane; i < A.n2; i += 64) {
        s_md[i] = 0x7FFFFFFF;
        s_21[i] = -1;
    }
    if (lane < OSG_HISTO_LENGTH) s_hist[lane] = 0;
    for (int i = lane; i < A.n1; i += 64) A.m12[i] = -1;
    __syncthreads();
    int nmatches = 0;  // lane 0's count
    const float r = (float)A.window;
    for (int i1 = 0; i1 < A.n1; i1++) {
        if (A.oct1[i1] > 0) continue;  // :760-762
        const float x = A.prev[2 * i1], y = A.prev[2 * i1 + 1];
        // Frame::GetFeaturesInArea(x, y, windowSize, 0, 0), ref:src/Frame.cc:868-962
        int minCX = (int)floorf((x - A.min_x - r) * A.inv_w);
        minCX = minCX < 0 ? 0 : minCX;
        int maxCX = (int)ceilf((x - A.min_x + r) * A.inv_w);
        maxCX = maxCX > OSG_GRID_COLS - 1 ? OSG_GRID_COLS - 1 : maxCX;
        int minCY = (int)floorf((y - A.min_y - r) * A.inv_h);
        minCY = minCY < 0 ? 0 : minCY;
        int maxCY = (int)ceilf((y - A.min_y + r) * A.inv_h);
        maxCY = maxCY > OSG_GRID_ROWS - 1 ? OSG_GRID_ROWS - 1 : maxCY;
        if (minCX >= OSG_GRID_COLS || maxCX < 0 || minCY >= OSG_GRID_ROWS || maxCY < 0) continue;
        const u32x4 qa = *(GLOBAL const u32x4 *)(A.desc1 + 8 * i1), qb = *(GLOBAL const u32x4 *)(A.desc1 + 8 * i1 + 4);
        uint32_t k1 = KEY_NONE, k2 = KEY_NONE;
        for (int ix = minCX; ix <= maxCX; ix++) {
            const int j0 = A.gs[ix * OSG_GRID_ROWS + minCY], j1 = A.gs[ix * OSG_GRID_ROWS + maxCY + 1];
            for (int jb = j0; jb < j1; jb += 64) {
                const int j = jb + lane;
                if (j < j1) {
                    const int i2 = A.gi[j];
                    const float dx = A.x2[i2] - x, dy = A.y2[i2] - y;
                    if (A.oct2[i2] == 0 && fabsf(dx) < r && fabsf(dy) < r) {  // level filter (0, 0) and window
                        const u32x4 ka = *(GLOBAL const u32x4 *)(A.desc2 + 8 * i2),
                                    kb = *(GLOBAL const u32x4 *)(A.desc2 + 8 * i2 + 4);
                        uint32_t d = __popc(qa.x ^ ka.x);
                        d = bcnt_acc(qa.y ^ ka.y, d);
                        d = bcnt_acc(qa.z ^ ka.z, d);
                        d = bcnt_acc(qa.w ^ ka.w, d);
                        d = bcnt_acc(qb.x ^ kb.x, d);
                        d = bcnt_acc(qb.y ^ kb.y, d);
                        d = bcnt_acc(qb.z ^ kb.z, d);
                        d = bcnt_acc(qb.w ^ kb.w, d);
                        if (!(s_md[i2] <= (int)d)) {  // :781-782
                            const uint32_t key = (d << 23) | (uint32_t)j;
                            const uint32_t hi = max(k1, key);
                            k1 = min(k1, key);
                            k2 = min(k2, hi);
                        }
                    }
                }
            }
        }
        for (int o = 32; o > 0; o >>= 1) {  // wave top-2 of packed keys
            const uint32_t a1 = __shfl_xor(k1, o), a2 = __shfl_xor(k2, o);
            const uint32_t hi = max(k1, a1);
            k1 = min(k1, a1);
            k2 = min(min(k2, a2), hi);
        }
        if (k1 == KEY_NONE) continue;
        const int bestDist = (int)(k1 >> 23);
        const int bestDist2 = k2 == KEY_NONE ? 0x7FFFFFFF : (int)(k2 >> 23);
        if (bestDist <= OSG_TH_LOW && bestDist < (float)bestDist2 * A.nnratio) {  // :794-797
            const int s = A.gi[k1 & ((1u << 23) - 1)];
            if (lane == 0) {
                const int prev_owner = s_21[s];
                if (prev_owner >= 0) {  // :798-802: steal
                    A.m12[prev_owner] = -1;
                    nmatches--;
                }
                A.m12[i1] = s;
                s_21[s] = i1;
                s_md[s] = bestDist;
                nmatches++;
                if (A.check_ori) s_hist[rot_bin(A.ang1[i1], A.ang2[s])]++;  // every accepted event counts
            }
            __syncthreads();  // LDS state visible to every lane before the next keypoint
        }
    }
    __syncthreads();
    if (A.check_ori) {
        // ComputeThreeMaxima (ref:src/ORBmatcher.cc:2341-2383), then drop the matches outside the
        // three bins (:849-866): the bin of keypoint i1 is recomputed from its surviving match
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
        int removed = 0;
        for (int i = lane; i < A.n1; i += 64) {
            const int s = A.m12[i];
            if (s < 0) continue;
            const int bin = rot_bin(A.ang1[i], A.ang2[s]);
            if (!(bin == ind1 || bin == ind2 || bin == ind3)) {
                A.m12[i] = -1;
                removed++;
            }
        }
        for (int o = 32; o > 0; o >>= 1) removed += __shfl_xor(removed, o);
        nmatches -= removed;
    }
    if (lane == 0) A.nmatch[0] = nmatches;
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

int init_run(osg_ctx *ctx, const osg_frame *F1, const osg_frame *F2, float *prev_xy, int B, int window, float nnratio,
             int check_ori, int32_t *m12, int32_t *nmatches)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, B >= 0 && (B == 0 || (F1 && F2 && prev_xy && m12 && nmatches)), "null argument");
    OSG_REQUIRE(ctx, window >= 0, "windowSize < 0");
    osg_packer pk;
    std::vector<InitArgs> args(B);
    std::vector<size_t> o_base(B + 1, 0);
    for (int b = 0; b < B; b++) {
        const osg_frame *a = &F1[b], *c = &F2[b];
        OSG_REQUIRE(ctx, a->n >= 0 && (a->n == 0 || (a->desc && a->kp_octave && a->kp_angle)), "problem %d: F1", b);
        int rc = osg_check_frame(ctx, c);
        if (rc < 0) return osg_set_error(ctx, rc, "problem %d: F2: %s", b, osg_ctx_last_error(ctx));
        OSG_REQUIRE(ctx, a->nleft == -1 && c->nleft == -1, "problem %d: monocular frames only (Nleft == -1)", b);
        OSG_REQUIRE(ctx, c->n <= MAX_N2, "problem %d: F2 has %d keypoints > %d", b, c->n, MAX_N2);
        o_base[b + 1] = o_base[b] + (size_t)a->n;
        InitArgs &A = args[b];
        A = InitArgs{};
        A.n1 = a->n;
        A.n2 = c->n;
        A.window = window;
        A.check_ori = check_ori;
        A.nnratio = nnratio;
        A.min_x = c->min_x;
        A.min_y = c->min_y;
        A.inv_w = c->grid_inv_w;
        A.inv_h = c->grid_inv_h;
        if (a->n == 0) continue;
        set_off(A.desc1, pk.add(a->desc, (size_t)a->n * 32));
        set_off(A.oct1, pk.add(a->kp_octave, sizeof(int32_t) * a->n));
        set_off(A.ang1, pk.add(a->kp_angle, sizeof(float) * a->n));
        set_off(A.prev, pk.add(prev_xy + 2 * o_base[b], sizeof(float) * 2 * a->n));
        set_off(A.desc2, pk.add(c->desc, (size_t)c->n * 32));
        set_off(A.x2, pk.add(c->kp_x, sizeof(float) * c->n));
        set_off(A.y2, pk.add(c->kp_y, sizeof(float) * c->n));
        set_off(A.ang2, pk.add(c->kp_angle, sizeof(float) * c->n));
        set_off(A.oct2, pk.add(c->kp_octave, sizeof(int32_t) * c->n));
        set_off(A.gs, pk.add(c->grid_start, sizeof(int32_t) * (OSG_GRID_CELLS + 1)));
        set_off(A.gi, pk.add(c->grid_idx, sizeof(int32_t) * c->grid_start[OSG_GRID_CELLS]));
    }
    for (size_t i = 0; i < o_base[B]; i++) m12[i] = -1;
    for (int b = 0; b < B; b++) nmatches[b] = 0;
    if (o_base[B] == 0) return OSG_OK;
    const size_t in_bytes = (pk.total + 255) & ~size_t(255);
    const size_t args_bytes = (sizeof(InitArgs) * (size_t)B + 255) & ~size_t(255);
    const size_t out_bytes = sizeof(int32_t) * (o_base[B] + B);
    char *pin = (char *)osg_pinned(ctx, in_bytes + args_bytes + out_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));  // the pinned block may still be in use
    pk.fill_parallel(pin, 8);
    InitArgs *pin_args = (InitArgs *)(pin + in_bytes);
    int32_t *pin_out = (int32_t *)((char *)pin_args + args_bytes);
    char *dev_in = nullptr;
    InitArgs *dev_args = nullptr;
    int32_t *dev_out = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dev_args, SLOT_TMP1, args_bytes);
    OSG_ALLOC(ctx, dev_out, SLOT_TMP2, out_bytes);
    for (int b = 0; b < B; b++) {
        InitArgs &A = args[b];
        relocate(A.desc1, dev_in);
        relocate(A.oct1, dev_in);
        relocate(A.ang1, dev_in);
        relocate(A.prev, dev_in);
        relocate(A.desc2, dev_in);
        relocate(A.x2, dev_in);
        relocate(A.y2, dev_in);
        relocate(A.ang2, dev_in);
        relocate(A.oct2, dev_in);
        relocate(A.gs, dev_in);
        relocate(A.gi, dev_in);
        A.m12 = (GLOBAL int32_t *)(dev_out + o_base[b]);
        A.nmatch = (GLOBAL int32_t *)(dev_out + o_base[B] + b);
        pin_args[b] = A;
    }
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_in, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_args, pin_args, sizeof(InitArgs) * (size_t)B, hipMemcpyHostToDevice,
                                      ctx->stream));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_init, dim3(B), dim3(64), 0, ctx->stream, dev_args);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(pin_out, dev_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    for (int b = 0; b < B; b++) {
        const osg_frame *c = &F2[b];
        for (size_t i = o_base[b]; i < o_base[b + 1]; i++) {
            m12[i] = pin_out[i];
            if (m12[i] >= 0) {  // vbPrevMatched[i1] = F2.mvKeysUn[vnMatches12[i1]].pt, :870-872
                prev_xy[2 * i] = c->kp_x[m12[i]];
                prev_xy[2 * i + 1] = c->kp_y[m12[i]];
            }
        }
        nmatches[b] = pin_out[o_base[B] + b];
    }
    return OSG_OK;
}

}  // namespace

extern "C" {

int osg_search_for_initialization(osg_ctx *ctx, const osg_frame *F1, const osg_frame *F2, float *prev_xy,
                                  int window_size, float nnratio, int check_orientation, int32_t *matches12)
{
    int32_t n = 0;
    const int rc = init_run(ctx, F1, F2, prev_xy, 1, window_size, nnratio, check_orientation, matches12, &n);
    return rc < 0 ? rc : n;
}

int osg_search_for_initialization_batch(osg_ctx *ctx, const osg_frame *F1, const osg_frame *F2, int32_t B,
                                        float *prev_xy, int window_size, float nnratio, int check_orientation,
                                        int32_t *matches12, int32_t *nmatches)
{
    return init_run(ctx, F1, F2, prev_xy, B, window_size, nnratio, check_orientation, matches12, nmatches);
}

}  // extern "C"
