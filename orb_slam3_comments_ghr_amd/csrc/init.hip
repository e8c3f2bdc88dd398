// init.hip — ORBmatcher::SearchForInitialization on gfx950 (ref:src/ORBmatcher.cc:735-878), the
// matcher of monocular initialisation (Tracking::MonocularInitialization, ref:src/Tracking.cc:2956).
//
// The reference walks F1's level-0 keypoints in order and carries state across them: a candidate
// i2 is skipped when vMatchedDistance[i2] <= dist, an accepted match steals i2 from its earlier
// owner (vnMatches21), and every accepted event enters the rotation histogram.  The state a
// keypoint q sees is vMatchedDistance[s] = the distance of the last accepted earlier keypoint at s,
// which (accepted distances at a slot strictly decrease) is the SMALLEST distance among the
// accepted earlier keypoints at s.  So the walk is a fixed point, as the SearchByProjection claim
// is: every level-0 keypoint re-decides against the claims (q, dist) of the keypoints currently
// accepted, counting only claims with a lower index, until no decision changes; after round r the
// first r keypoints are final, and the fixed point is the sequential result.  Claims live in LDS
// (FP_K per slot per round); on overflow, or with more level-0 keypoints than the LDS tables hold,
// one wave walks the keypoints in order instead (lanes over each window's candidates).
//
// Candidate lists (window + level filter, GetFeaturesInArea's ix-outer / iy-inner order) are built
// once: the host hands over a grid of F2's level-0 keypoints only (same cell order, so the CSR
// position is the enumeration order), the kernel counts, scans and fills {slot | dist << 16}.
#include <algorithm>
#include <vector>

#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int IT = 1024;            // threads per workgroup (one workgroup per frame pair)
constexpr int FP_SLOTS = 4096;      // level-0 F2 keypoints the fixed point keeps claim lists for
constexpr int FP_K = 4;             // claimants per slot and round before the serial fallback
constexpr int MAX_Q = 8192;         // level-0 F1 keypoints
constexpr int MAX_L0 = 8192;        // level-0 F2 keypoints (serial path)
constexpr int LDS_WORDS = FP_SLOTS + FP_SLOTS * FP_K + MAX_Q + IT;  // 29 696 words = 116 KiB
constexpr uint32_t KEY_NONE = 0xFFFFFFFFu;
constexpr int MD_NONE = 0x7FFFFFFF;

struct InitArgs {
    int nq, m0, window, check_ori;
    float nnratio, min_x, min_y, inv_w, inv_h;
    GLOBAL const int32_t *q_i1;    // nq: the level-0 F1 keypoints, ascending
    GLOBAL const uint32_t *desc1;  // F1 descriptors (indexed by i1)
    GLOBAL const float *ang1;
    GLOBAL const float *prev;      // F1.n x 2 (vbPrevMatched)
    GLOBAL const uint32_t *desc2;  // F2 descriptors (indexed by i2)
    GLOBAL const float *x2, *y2, *ang2;
    GLOBAL const int32_t *gs0, *gi0;  // level-0 F2 grid: CSR of level-0 ranks (cell order kept)
    GLOBAL const int32_t *l0_i2;   // m0: rank -> F2 index
    GLOBAL uint32_t *cand;         // candidate lists {slot | dist << 16}, capacity nq * m0
    GLOBAL int32_t *qoff;          // nq + 1 list offsets
    GLOBAL int32_t *m12;           // F1.n out (host prefills -1 for every keypoint)
    GLOBAL int32_t *stats;         // {nmatches, rounds (0 = serial path)}
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

__device__ __forceinline__ uint32_t dist_to(const u32x4 &qa, const u32x4 &qb, GLOBAL const uint32_t *d2, int i2)
{
    const u32x4 ka = *(GLOBAL const u32x4 *)(d2 + 8 * i2), kb = *(GLOBAL const u32x4 *)(d2 + 8 * i2 + 4);
    uint32_t d = __popc(qa.x ^ ka.x);
    d = bcnt_acc(qa.y ^ ka.y, d);
    d = bcnt_acc(qa.z ^ ka.z, d);
    d = bcnt_acc(qa.w ^ ka.w, d);
    d = bcnt_acc(qb.x ^ kb.x, d);
    d = bcnt_acc(qb.y ^ kb.y, d);
    d = bcnt_acc(qb.z ^ kb.z, d);
    d = bcnt_acc(qb.w ^ kb.w, d);
    return d;
}

struct Window {
    int minCX, maxCX, minCY, maxCY;
    bool empty;
};

// Frame::GetFeaturesInArea(x, y, windowSize, 0, 0) cell range, ref:src/Frame.cc:868-962
__device__ __forceinline__ Window window_of(const InitArgs &A, float x, float y, float r)
{
    Window w;
    w.minCX = (int)floorf((x - A.min_x - r) * A.inv_w);
    w.minCX = w.minCX < 0 ? 0 : w.minCX;
    w.maxCX = (int)ceilf((x - A.min_x + r) * A.inv_w);
    w.maxCX = w.maxCX > OSG_GRID_COLS - 1 ? OSG_GRID_COLS - 1 : w.maxCX;
    w.minCY = (int)floorf((y - A.min_y - r) * A.inv_h);
    w.minCY = w.minCY < 0 ? 0 : w.minCY;
    w.maxCY = (int)ceilf((y - A.min_y + r) * A.inv_h);
    w.maxCY = w.maxCY > OSG_GRID_ROWS - 1 ? OSG_GRID_ROWS - 1 : w.maxCY;
    w.empty = w.minCX >= OSG_GRID_COLS || w.maxCX < 0 || w.minCY >= OSG_GRID_ROWS || w.maxCY < 0;
    return w;
}

__device__ __forceinline__ bool accept(uint32_t k1, uint32_t k2, float nnratio)
{  // bestDist <= TH_LOW && bestDist < (float)bestDist2 * mfNNratio, ref:src/ORBmatcher.cc:794-797
    if (k1 == KEY_NONE) return false;
    const int d1 = (int)(k1 >> 16);
    const int d2 = k2 == KEY_NONE ? 0x7FFFFFFF : (int)(k2 >> 16);
    return d1 <= OSG_TH_LOW && d1 < (float)d2 * nnratio;
}

// LDS and global writes of one lane visible to the rest of its wave (the serial path runs in one wave
// while the others wait at the workgroup barrier after it)
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// The reference's sequential walk, one wave, lanes over each window's candidates (used when the
// fixed point's claim lists overflow or there are too many level-0 keypoints).  md / m21 in LDS.
__device__ void serial_walk(const InitArgs &A, int *md, int *m21, int *hist, int lane)
{
    for (int i = lane; i < A.m0; i += 64) {
        md[i] = MD_NONE;
        m21[i] = -1;
    }
    for (int q = lane; q < A.nq; q += 64) A.m12[A.q_i1[q]] = -1;
    if (lane < OSG_HISTO_LENGTH) hist[lane] = 0;
    wave_sync();
    const float r = (float)A.window;
    for (int q = 0; q < A.nq; q++) {
        const int i1 = A.q_i1[q];
        const Window w = window_of(A, A.prev[2 * i1], A.prev[2 * i1 + 1], r);
        if (w.empty) continue;
        const float x = A.prev[2 * i1], y = A.prev[2 * i1 + 1];
        const u32x4 qa = *(GLOBAL const u32x4 *)(A.desc1 + 8 * i1), qb = *(GLOBAL const u32x4 *)(A.desc1 + 8 * i1 + 4);
        uint32_t k1 = KEY_NONE, k2 = KEY_NONE;
        for (int ix = w.minCX; ix <= w.maxCX; ix++) {
            const int j0 = A.gs0[ix * OSG_GRID_ROWS + w.minCY], j1 = A.gs0[ix * OSG_GRID_ROWS + w.maxCY + 1];
            for (int jb = j0; jb < j1; jb += 64) {
                const int j = jb + lane;
                if (j >= j1) continue;
                const int s = A.gi0[j], i2 = A.l0_i2[s];
                if (!(fabsf(A.x2[i2] - x) < r && fabsf(A.y2[i2] - y) < r)) continue;
                const uint32_t d = dist_to(qa, qb, A.desc2, i2);
                if (md[s] <= (int)d) continue;  // :781-782
                const uint32_t key = (d << 16) | (uint32_t)j;  // j < 65536: the enumeration order
                const uint32_t hi = max(k1, key);
                k1 = min(k1, key);
                k2 = min(k2, hi);
            }
        }
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t a1 = __shfl_xor(k1, o), a2 = __shfl_xor(k2, o);
            const uint32_t hi = max(k1, a1);
            k1 = min(k1, a1);
            k2 = min(min(k2, a2), hi);
        }
        if (!accept(k1, k2, A.nnratio)) continue;
        const int s = A.gi0[k1 & 0xFFFF];
        if (lane == 0) {
            if (m21[s] >= 0) A.m12[m21[s]] = -1;  // :798-802: steal
            const int i2 = A.l0_i2[s];
            A.m12[i1] = i2;
            m21[s] = i1;
            md[s] = (int)(k1 >> 16);
            if (A.check_ori) hist[rot_bin(A.ang1[i1], A.ang2[i2])]++;  // every accepted event counts
        }
        wave_sync();
    }
}

__global__ __launch_bounds__(IT) void k_init(const InitArgs *__restrict__ args)
{
    const InitArgs &A = args[blockIdx.x];
    __shared__ int lds[LDS_WORDS];
    __shared__ int s_hist[OSG_HISTO_LENGTH];
    __shared__ int s_flag[3];  // changed, overflow, nmatches
    const int tid = threadIdx.x, lane = tid & 63;
    int *cnt = lds;                          // FP_SLOTS: claims per slot this round
    int *claim = lds + FP_SLOTS;             // FP_SLOTS * FP_K: q << 9 | dist
    int *dec = claim + FP_SLOTS * FP_K;      // MAX_Q: q's decision (slot << 9 | dist) or -1
    int *scan = dec + MAX_Q;                 // IT
    if (tid < OSG_HISTO_LENGTH) s_hist[tid] = 0;
    if (tid < 3) s_flag[tid] = 0;
    const float r = (float)A.window;
    const int QPT = (A.nq + IT - 1) / IT;  // queries of thread tid: [tid * QPT, tid * QPT + QPT)
    const bool fits = A.m0 <= FP_SLOTS && A.nq <= MAX_Q;
    int rounds = 0;
    if (fits) {
        // ---- candidate lists: count, scan, fill ----
        int my = 0;
        for (int k = 0; k < QPT; k++) {
            const int q = tid * QPT + k;
            if (q >= A.nq) break;
            const int i1 = A.q_i1[q];
            const float x = A.prev[2 * i1], y = A.prev[2 * i1 + 1];
            const Window w = window_of(A, x, y, r);
            if (w.empty) continue;
            for (int ix = w.minCX; ix <= w.maxCX; ix++) {
                const int j1 = A.gs0[ix * OSG_GRID_ROWS + w.maxCY + 1];
                for (int j = A.gs0[ix * OSG_GRID_ROWS + w.minCY]; j < j1; j++) {
                    const int i2 = A.l0_i2[A.gi0[j]];
                    my += (fabsf(A.x2[i2] - x) < r && fabsf(A.y2[i2] - y) < r);
                }
            }
        }
        scan[tid] = my;
        __syncthreads();
        for (int o = 1; o < IT; o <<= 1) {  // inclusive scan
            const int v = tid >= o ? scan[tid - o] : 0;
            __syncthreads();
            scan[tid] += v;
            __syncthreads();
        }
        int pos = scan[tid] - my;
        for (int k = 0; k < QPT; k++) {
            const int q = tid * QPT + k;
            if (q >= A.nq) break;
            A.qoff[q] = pos;
            dec[q] = -1;
            const int i1 = A.q_i1[q];
            const float x = A.prev[2 * i1], y = A.prev[2 * i1 + 1];
            const Window w = window_of(A, x, y, r);
            if (w.empty) continue;
            const u32x4 qa = *(GLOBAL const u32x4 *)(A.desc1 + 8 * i1), qb = *(GLOBAL const u32x4 *)(A.desc1 + 8 * i1 + 4);
            for (int ix = w.minCX; ix <= w.maxCX; ix++) {
                const int j1 = A.gs0[ix * OSG_GRID_ROWS + w.maxCY + 1];
                for (int j = A.gs0[ix * OSG_GRID_ROWS + w.minCY]; j < j1; j++) {
                    const int sl = A.gi0[j], i2 = A.l0_i2[sl];
                    if (fabsf(A.x2[i2] - x) < r && fabsf(A.y2[i2] - y) < r)
                        A.cand[pos++] = (uint32_t)sl | (dist_to(qa, qb, A.desc2, i2) << 16);
                }
            }
        }
        if (tid == IT - 1) A.qoff[A.nq] = scan[IT - 1];
        for (int sl = tid; sl < A.m0; sl += IT) cnt[sl] = 0;
        __syncthreads();
        // ---- fixed point: every keypoint against the claims of lower-indexed keypoints ----
        for (;;) {
            bool changed = false;
            for (int k = 0; k < QPT; k++) {
                const int q = tid * QPT + k;
                if (q >= A.nq) break;
                const int e0 = A.qoff[q], e1 = A.qoff[q + 1];
                uint32_t k1 = KEY_NONE, k2 = KEY_NONE;
                for (int e = e0; e < e1; e++) {
                    const uint32_t c = A.cand[e];
                    const int sl = (int)(c & 0xFFFF), d = (int)(c >> 16);
                    int md = MD_NONE;  // vMatchedDistance[sl] before q
                    const int nc = min(cnt[sl], FP_K);
                    for (int t = 0; t < nc; t++) {
                        const int cl = claim[sl * FP_K + t];
                        if ((cl >> 9) < q) md = min(md, cl & 511);
                    }
                    if (md <= d) continue;  // :781-782
                    const uint32_t key = ((uint32_t)d << 16) | (uint32_t)(e - e0);
                    const uint32_t hi = max(k1, key);
                    k1 = min(k1, key);
                    k2 = min(k2, hi);
                }
                int nd = -1;
                if (accept(k1, k2, A.nnratio))
                    nd = ((int)(A.cand[e0 + (k1 & 0xFFFF)] & 0xFFFF) << 9) | (int)(k1 >> 16);
                if (nd != dec[q]) {
                    dec[q] = nd;
                    changed = true;
                }
            }
            if (changed) s_flag[0] = 1;
            rounds++;
            __syncthreads();
            const bool any = s_flag[0] != 0;
            __syncthreads();
            if (!any) break;  // uniform: every thread read the same flag between the barriers
            if (tid == 0) s_flag[0] = 0;
            for (int sl = tid; sl < A.m0; sl += IT) cnt[sl] = 0;
            __syncthreads();
            for (int q = tid; q < A.nq; q += IT) {
                const int dq = dec[q];
                if (dq < 0) continue;
                const int sl = dq >> 9;
                const int at = atomicAdd(&cnt[sl], 1);
                if (at < FP_K) claim[sl * FP_K + at] = (q << 9) | (dq & 511);
                else s_flag[1] = 1;
            }
            __syncthreads();
            if (s_flag[1]) break;  // uniform
        }
        if (!s_flag[1]) {
            // an accepted keypoint keeps its match unless a later accepted keypoint took the slot
            for (int q = tid; q < A.nq; q += IT) {
                const int i1 = A.q_i1[q];
                const int dq = dec[q];
                int out = -1;
                if (dq >= 0) {
                    const int sl = dq >> 9;
                    const int i2 = A.l0_i2[sl];
                    bool stolen = false;
                    const int nc = min(cnt[sl], FP_K);
                    for (int t = 0; t < nc; t++) stolen |= (claim[sl * FP_K + t] >> 9) > q;
                    if (!stolen) out = i2;
                    if (A.check_ori) atomicAdd(&s_hist[rot_bin(A.ang1[i1], A.ang2[i2])], 1);
                }
                A.m12[i1] = out;
            }
        }
    }
    const bool serial = !fits || s_flag[1] != 0;  // uniform
    __syncthreads();
    if (serial) {  // the reference's order, one wave; the fixed point's state is discarded
        rounds = 0;
        if (tid < 64) serial_walk(A, lds, lds + MAX_L0, s_hist, lane);
    }
    __syncthreads();
    int nm = 0;
    if (A.check_ori) {
        // ComputeThreeMaxima (ref:src/ORBmatcher.cc:2341-2383), then drop matches outside the three
        // bins (:849-866); a surviving match's bin is the bin it was counted in
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
        for (int q = tid; q < A.nq; q += IT) {
            const int i1 = A.q_i1[q];
            const int i2 = A.m12[i1];
            if (i2 < 0) continue;
            const int bin = rot_bin(A.ang1[i1], A.ang2[i2]);
            if (!(bin == ind1 || bin == ind2 || bin == ind3)) A.m12[i1] = -1;
            else nm++;
        }
    } else {
        for (int q = tid; q < A.nq; q += IT) nm += A.m12[A.q_i1[q]] >= 0;
    }
    for (int o = 32; o > 0; o >>= 1) nm += __shfl_xor(nm, o);
    if (lane == 0) atomicAdd(&s_flag[2], nm);
    __syncthreads();
    if (tid == 0) {
        A.stats[0] = s_flag[2];
        A.stats[1] = rounds;
    }
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

struct Problem {
    std::vector<int32_t> q_i1, gs0, gi0, l0_i2;
};

int init_run(osg_ctx *ctx, const osg_frame *F1, const osg_frame *F2, float *prev_xy, int B, int window, float nnratio,
             int check_ori, int32_t *m12, int32_t *nmatches)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, B >= 0 && (B == 0 || (F1 && F2 && prev_xy && m12 && nmatches)), "null argument");
    OSG_REQUIRE(ctx, window >= 0, "windowSize < 0");
    osg_packer pk;
    std::vector<InitArgs> args(B);
    std::vector<Problem> P(B);
    std::vector<size_t> o_base(B + 1, 0), c_base(B + 1, 0), q_base(B + 1, 0);
    for (int b = 0; b < B; b++) {
        const osg_frame *a = &F1[b], *c = &F2[b];
        OSG_REQUIRE(ctx, a->n >= 0 && (a->n == 0 || (a->desc && a->kp_octave && a->kp_angle)), "problem %d: F1", b);
        int rc = osg_check_frame(ctx, c);
        if (rc < 0) return osg_set_error(ctx, rc, "problem %d: F2: %s", b, osg_ctx_last_error(ctx));
        OSG_REQUIRE(ctx, a->nleft == -1 && c->nleft == -1, "problem %d: monocular frames only (Nleft == -1)", b);
        o_base[b + 1] = o_base[b] + (size_t)a->n;
        Problem &p = P[b];
        // level-0 F1 keypoints in order (:758-762); level-0 F2 keypoints as a grid of their own (the
        // level filter of GetFeaturesInArea(.., 0, 0), cell order and in-cell order kept)
        for (int i = 0; i < a->n; i++)
            if (a->kp_octave[i] <= 0) p.q_i1.push_back(i);
        std::vector<int32_t> rank(c->n, -1);
        for (int i = 0; i < c->n; i++)
            if (c->kp_octave[i] == 0) {
                rank[i] = (int)p.l0_i2.size();
                p.l0_i2.push_back(i);
            }
        p.gs0.assign(OSG_GRID_CELLS + 1, 0);
        for (int cell = 0; cell < OSG_GRID_CELLS; cell++) {
            for (int j = c->grid_start[cell]; j < c->grid_start[cell + 1]; j++)
                if (rank[c->grid_idx[j]] >= 0) p.gi0.push_back(rank[c->grid_idx[j]]);
            p.gs0[cell + 1] = (int32_t)p.gi0.size();
        }
        const int nq = (int)p.q_i1.size(), m0 = (int)p.l0_i2.size();
        OSG_REQUIRE(ctx, m0 <= MAX_L0 && nq <= 65535, "problem %d: %d level-0 F2 keypoints > %d", b, m0, MAX_L0);
        q_base[b + 1] = q_base[b] + (size_t)nq + 1;
        c_base[b + 1] = c_base[b] + (m0 <= FP_SLOTS && nq <= MAX_Q ? (size_t)nq * m0 : 0);
        InitArgs &A = args[b];
        A = InitArgs{};
        A.nq = nq;
        A.m0 = m0;
        A.window = window;
        A.check_ori = check_ori;
        A.nnratio = nnratio;
        A.min_x = c->min_x;
        A.min_y = c->min_y;
        A.inv_w = c->grid_inv_w;
        A.inv_h = c->grid_inv_h;
        if (nq == 0 || m0 == 0) continue;
        set_off(A.q_i1, pk.add(p.q_i1.data(), sizeof(int32_t) * nq));
        set_off(A.desc1, pk.add(a->desc, (size_t)a->n * 32));
        set_off(A.ang1, pk.add(a->kp_angle, sizeof(float) * a->n));
        set_off(A.prev, pk.add(prev_xy + 2 * o_base[b], sizeof(float) * 2 * a->n));
        set_off(A.desc2, pk.add(c->desc, (size_t)c->n * 32));
        set_off(A.x2, pk.add(c->kp_x, sizeof(float) * c->n));
        set_off(A.y2, pk.add(c->kp_y, sizeof(float) * c->n));
        set_off(A.ang2, pk.add(c->kp_angle, sizeof(float) * c->n));
        set_off(A.gs0, pk.add(p.gs0.data(), sizeof(int32_t) * (OSG_GRID_CELLS + 1)));
        set_off(A.gi0, pk.add(p.gi0.data(), sizeof(int32_t) * m0));
        set_off(A.l0_i2, pk.add(p.l0_i2.data(), sizeof(int32_t) * m0));
    }
    for (size_t i = 0; i < o_base[B]; i++) m12[i] = -1;
    for (int b = 0; b < B; b++) nmatches[b] = 0;
    if (pk.total == 0) return OSG_OK;
    const size_t in_bytes = (pk.total + 255) & ~size_t(255);
    const size_t args_bytes = (sizeof(InitArgs) * (size_t)B + 255) & ~size_t(255);
    const size_t out_bytes = sizeof(int32_t) * (o_base[B] + 2 * (size_t)B);
    char *pin = (char *)osg_pinned(ctx, in_bytes + args_bytes + out_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    pk.fill_parallel(pin, 8);
    InitArgs *pin_args = (InitArgs *)(pin + in_bytes);
    int32_t *pin_out = (int32_t *)((char *)pin_args + args_bytes);
    char *dev_in = nullptr;
    InitArgs *dev_args = nullptr;
    int32_t *dev_out = nullptr, *dev_qoff = nullptr;
    uint32_t *dev_cand = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dev_args, SLOT_TMP1, args_bytes);
    OSG_ALLOC(ctx, dev_out, SLOT_TMP2, out_bytes);
    OSG_ALLOC(ctx, dev_cand, SLOT_TMP3, sizeof(uint32_t) * (c_base[B] + 1));
    OSG_ALLOC(ctx, dev_qoff, SLOT_TMP4, sizeof(int32_t) * (q_base[B] + 1));
    for (int b = 0; b < B; b++) {
        InitArgs &A = args[b];
        relocate(A.q_i1, dev_in);
        relocate(A.desc1, dev_in);
        relocate(A.ang1, dev_in);
        relocate(A.prev, dev_in);
        relocate(A.desc2, dev_in);
        relocate(A.x2, dev_in);
        relocate(A.y2, dev_in);
        relocate(A.ang2, dev_in);
        relocate(A.gs0, dev_in);
        relocate(A.gi0, dev_in);
        relocate(A.l0_i2, dev_in);
        A.cand = (GLOBAL uint32_t *)(dev_cand + c_base[b]);
        A.qoff = (GLOBAL int32_t *)(dev_qoff + q_base[b]);
        A.m12 = (GLOBAL int32_t *)(dev_out + o_base[b]);
        A.stats = (GLOBAL int32_t *)(dev_out + o_base[B] + 2 * b);
        if (A.nq == 0 || A.m0 == 0) A.nq = 0;  // nothing to match: the kernel only writes the stats
        pin_args[b] = A;
    }
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_in, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_args, pin_args, sizeof(InitArgs) * (size_t)B, hipMemcpyHostToDevice,
                                      ctx->stream));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_init, dim3(B), dim3(IT), 0, ctx->stream, dev_args);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    OSG_RC(osg_download(ctx, pin_out, dev_out, out_bytes));
    OSG_RC(osg_wait(ctx));
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    int32_t rounds_max = 0, serial = 0;
    for (int b = 0; b < B; b++) {
        const osg_frame *c = &F2[b];
        const Problem &p = P[b];
        if (args[b].nq == 0) continue;
        for (int q : p.q_i1) {
            const size_t i = o_base[b] + (size_t)q;
            m12[i] = pin_out[i];
            if (m12[i] >= 0) {  // vbPrevMatched[i1] = F2.mvKeysUn[vnMatches12[i1]].pt, :869-871
                prev_xy[2 * i] = c->kp_x[m12[i]];
                prev_xy[2 * i + 1] = c->kp_y[m12[i]];
            }
        }
        nmatches[b] = pin_out[o_base[B] + 2 * b];
        const int32_t rb = pin_out[o_base[B] + 2 * b + 1];
        rounds_max = std::max(rounds_max, rb);
        serial += rb == 0;
    }
    ctx->match_stats[1] = rounds_max;
    ctx->match_stats[2] = serial;
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
