// stereo.hip — Frame::ComputeStereoMatches on gfx950 (ref:src/Frame.cc:1117-1373).
//
// Rectified stereo: every left keypoint looks for a right keypoint on its row, then refines the
// disparity with an 11 x 11 SAD block match at its pyramid level and a parabola fit; matches whose
// SAD is >= 1.5 * 1.4 * the median SAD are dropped.  Three kernels:
//  * k_stereo_rows — one workgroup per frame builds vRowIndices (ref:src/Frame.cc:1150-1170) as CSR
//    in HBM: per-row counts in LDS, a block scan, then an atomic fill.  The fill order within a row
//    is free because the matcher breaks distance ties by the right index itself (since late r05;
//    before, the host built the lists, 40 us per frame).
//  * k_stereo_match — one wave per left keypoint (grid = (ceil(max n / 4), frames)).  The lanes
//    take the row's candidates and a wave min of (dist << 24 | right index) gives the reference's
//    first minimum (its candidate vector is in ascending right index); then the left 11 x 11 patch and the right
//    11 x 21 strip are staged in LDS, the 121 (offset, row) pairs are summed across the lanes and
//    lanes 0..10 add the rows of one offset each; lane 0 finishes the reference's float arithmetic
//    (built with -ffp-contract=off).
//  * k_stereo_filter — one workgroup per frame: the median SAD of the accepted matches by a
//    two-pass radix select in LDS (the vDistIdx sort only ever yields that element), then the
//    removal and the count.
// Host pyramids are packed row-contiguous into the per-call upload; device-resident pyramids
// (osg_image_pyramid.on_device) are read in place with their own row step.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <vector>

#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int SW = 5;  // half window (w)
constexpr int SL = 5;  // half search range (L)
constexpr int PATCH = 2 * SW + 1;            // 11
constexpr int STRIP = 2 * SW + 2 * SL + 1;   // 21
constexpr int NOFF = 2 * SL + 1;             // 11 offsets incR = -L..L
constexpr int MAX_LEVELS = 32;
constexpr int MAX_ROW_LIST = 1 << 24;        // right-index field of the wave-min key
constexpr int MAX_ROWS0 = 8192;              // level-0 image rows: k_stereo_rows' LDS counters

struct StereoArgs {
    int n, n_levels, rows0, n_right;
    float mb, mbf;
    GLOBAL const float *x, *y;
    GLOBAL const int32_t *oct;
    GLOBAL const uint32_t *desc;
    GLOBAL const float *xr, *yr;
    GLOBAL const int32_t *oct_r;
    GLOBAL const uint32_t *desc_r;
    GLOBAL int32_t *row_start, *row_list;        // vRowIndices as CSR over rows0 rows (k_stereo_rows)
    GLOBAL const float *scale, *inv_scale;
    GLOBAL const uint8_t *img_l[MAX_LEVELS];
    GLOBAL const uint8_t *img_r[MAX_LEVELS];
    int rows_l[MAX_LEVELS], cols_l[MAX_LEVELS], step_l[MAX_LEVELS];
    int rows_r[MAX_LEVELS], cols_r[MAX_LEVELS], step_r[MAX_LEVELS];
    GLOBAL float *ur, *depth;                    // n
    GLOBAL int32_t *sad;                         // n: bestDist of an accepted match, -1
    GLOBAL int32_t *nmatch;
};

__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// rows floor(y - r) .. ceil(y + r) of right keypoint iR, r = 2 mvScaleFactors[octave], clipped to the
// image (ref:src/Frame.cc:1158-1169; the reference would index past vRowIndices)
__device__ __forceinline__ void right_rows(const StereoArgs &A, int iR, int &lo, int &hi)
{
    const float kpY = A.yr[iR];
    const float r = 2.0f * A.scale[A.oct_r[iR]];
    hi = min((int)ceilf(kpY + r), A.rows0 - 1);
    lo = max((int)floorf(kpY - r), 0);
}

__global__ __launch_bounds__(1024) void k_stereo_rows(const StereoArgs *__restrict__ args)
{
    const StereoArgs &A = args[blockIdx.x];
    __shared__ int s_cnt[MAX_ROWS0];
    __shared__ int s_wave[16];
    if (A.n == 0) return;
    const int tid = threadIdx.x, R = A.rows0, nr = A.n_right;
    for (int y = tid; y < R; y += 1024) s_cnt[y] = 0;
    __syncthreads();
    for (int iR = tid; iR < nr; iR += 1024) {
        int lo, hi;
        right_rows(A, iR, lo, hi);
        for (int y = lo; y <= hi; y++) atomicAdd(&s_cnt[y], 1);
    }
    __syncthreads();
    // exclusive scan: thread t owns rows [t seg, (t + 1) seg)
    const int seg = (R + 1023) / 1024, y0 = min(tid * seg, R), y1 = min(y0 + seg, R);
    int sum = 0;
    for (int y = y0; y < y1; y++) sum += s_cnt[y];
    int incl = sum;
    const int lane = tid & 63, w = tid >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) s_wave[w] = incl;
    __syncthreads();
    int base = incl - sum;
    for (int i = 0; i < w; i++) base += s_wave[i];
    __syncthreads();   // every thread has read its rows' counts
    for (int y = y0; y < y1; y++) {
        const int c = s_cnt[y];
        A.row_start[y] = base;
        s_cnt[y] = base;   // the fill cursor
        base += c;
    }
    if (tid == 1023) A.row_start[R] = base;
    __syncthreads();
    for (int iR = tid; iR < nr; iR += 1024) {
        int lo, hi;
        right_rows(A, iR, lo, hi);
        for (int y = lo; y <= hi; y++) A.row_list[atomicAdd(&s_cnt[y], 1)] = iR;
    }
}

__global__ __launch_bounds__(256) void k_stereo_match(const StereoArgs *__restrict__ args)
{
    const StereoArgs &A = args[blockIdx.y];
    __shared__ uint8_t s_pl[4][PATCH * PATCH];
    __shared__ uint8_t s_pr[4][PATCH * STRIP];
    __shared__ int s_part[4][NOFF * PATCH];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int iL = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + w);
    if (iL >= A.n) return;
    float out_ur = -1.0f, out_depth = -1.0f;
    int out_sad = -1;
    const float uL = A.x[iL], vL = A.y[iL];
    const int levelL = A.oct[iL];
    const float minZ = A.mb;
    const float minD = 0;
    const float maxD = A.mbf / minZ;                       // :1176-1178
    const bool row_ok = vL >= 0 && (int)vL < A.rows0;      // vRowIndices[vL], :1190
    const int row = row_ok ? (int)vL : 0;
    const float minU = uL - maxD;
    const float maxU = uL - minD;
    const int c0 = row_ok ? A.row_start[row] : 0;
    const int c1 = row_ok ? A.row_start[row + 1] : 0;
    if (c1 > c0 && !(maxU < 0)) {
        const u32x4 qa = *(GLOBAL const u32x4 *)(A.desc + 8 * iL), qb = *(GLOBAL const u32x4 *)(A.desc + 8 * iL + 4);
        uint32_t best = 0xFFFFFFFFu;
        for (int c = c0 + lane; c < c1; c += 64) {         // :1214-1245
            const uint32_t iR = (uint32_t)A.row_list[c];
            const int o = A.oct_r[iR];
            if (o < levelL - 1 || o > levelL + 1) continue;
            const float uR = A.xr[iR];
            if (!(uR >= minU && uR <= maxU)) continue;
            const u32x4 ka = *(GLOBAL const u32x4 *)(A.desc_r + 8 * iR), kb = *(GLOBAL const u32x4 *)(A.desc_r + 8 * iR + 4);
            uint32_t d = __popc(qa.x ^ ka.x);
            d = bcnt_acc(qa.y ^ ka.y, d);
            d = bcnt_acc(qa.z ^ ka.z, d);
            d = bcnt_acc(qa.w ^ ka.w, d);
            d = bcnt_acc(qb.x ^ kb.x, d);
            d = bcnt_acc(qb.y ^ kb.y, d);
            d = bcnt_acc(qb.z ^ kb.z, d);
            d = bcnt_acc(qb.w ^ kb.w, d);
            if ((int)d < OSG_TH_HIGH) best = min(best, (d << 24) | iR);  // bestDist = TH_HIGH, '<'
        }
        for (int o = 32; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor(best, o));
        const int thOrbDist = (OSG_TH_HIGH + OSG_TH_LOW) / 2;  // :1138
        if (best != 0xFFFFFFFFu && (int)(best >> 24) < thOrbDist) {  // :1248
            const int bestIdxR = (int)(best & 0xFFFFFF);
            const float uR0 = A.xr[bestIdxR];
            const float scaleFactor = A.inv_scale[levelL];
            const float scaleduL = roundf(uL * scaleFactor);
            const float scaledvL = roundf(vL * scaleFactor);
            const float scaleduR0 = roundf(uR0 * scaleFactor);
            const float iniu = scaleduR0 + SL - SW;          // :1280-1284 (the reference's own bound)
            const float endu = scaleduR0 + SL + SW + 1;
            const int cl = A.cols_l[levelL], rl = A.rows_l[levelL], cr = A.cols_r[levelL], rr = A.rows_r[levelL];
            const int pu = (int)scaleduL, pv = (int)scaledvL, pr = (int)scaleduR0;
            // patches inside both level images (the reference's rowRange / colRange would throw otherwise)
            const bool inside = pv - SW >= 0 && pv + SW < rl && pv + SW < rr && pu - SW >= 0 && pu + SW < cl &&
                                pr - SW - SL >= 0 && pr + SW + SL < cr;
            if (!(iniu < 0 || endu >= cr) && inside) {
                GLOBAL const uint8_t *L0 = A.img_l[levelL], *R0 = A.img_r[levelL];
                const size_t sl = (size_t)A.step_l[levelL], sr = (size_t)A.step_r[levelL];
                for (int i = lane; i < PATCH * PATCH; i += 64)
                    s_pl[w][i] = L0[(size_t)(pv - SW + i / PATCH) * sl + (pu - SW + i % PATCH)];
                for (int i = lane; i < PATCH * STRIP; i += 64)
                    s_pr[w][i] = R0[(size_t)(pv - SW + i / STRIP) * sr + (pr - SW - SL + i % STRIP)];
                wave_lds_sync();
                // pair p = (offset k, patch row r): one row of cv::norm(IL, IR, NORM_L1) for incR = k - L
                for (int p = lane; p < NOFF * PATCH; p += 64) {
                    const int k = p / PATCH, r = p % PATCH;
                    int s = 0;
#pragma unroll
                    for (int c = 0; c < PATCH; c++) s += abs((int)s_pl[w][r * PATCH + c] - (int)s_pr[w][r * STRIP + c + k]);
                    s_part[w][p] = s;
                }
                wave_lds_sync();
                int sum = 0;  // lane k < 11: the SAD of offset incR = k - L, :1288-1298
                if (lane < NOFF) {
#pragma unroll
                    for (int r = 0; r < PATCH; r++) sum += s_part[w][lane * PATCH + r];
                }
                int bestDist = 0x7FFFFFFF, bestincR = 0;
                float vDists[NOFF];
#pragma unroll
                for (int k = 0; k < NOFF; k++) {
                    const float dist = (float)__shfl(sum, k);
                    if (dist < bestDist) {
                        bestDist = (int)dist;
                        bestincR = k - SL;
                    }
                    vDists[k] = dist;
                }
                if (!(bestincR == -SL || bestincR == SL)) {  // :1306-1307
                    float dist1 = 0, dist2 = 0, dist3 = 0;
#pragma unroll
                    for (int k = 1; k < NOFF - 1; k++)
                        if (k == SL + bestincR) {
                            dist1 = vDists[k - 1];
                            dist2 = vDists[k];
                            dist3 = vDists[k + 1];
                        }
                    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));  // :1324
                    if (!(deltaR < -1 || deltaR > 1)) {
                        float bestuR = A.scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);  // :1332
                        float disparity = (uL - bestuR);
                        if (disparity >= minD && disparity < maxD) {  // :1336-1351
                            if (disparity <= 0) {
                                disparity = 0.01;
                                bestuR = (float)((double)uL - 0.01);
                            }
                            out_depth = A.mbf / disparity;
                            out_ur = bestuR;
                            out_sad = bestDist;
                        }
                    }
                }
            }
        }
    }
    if (lane == 0) {
        A.ur[iL] = out_ur;
        A.depth[iL] = out_depth;
        A.sad[iL] = out_sad;
    }
}

// median of the accepted SADs (vDistIdx[size / 2].first after sort, ref:src/Frame.cc:1357-1359) by
// a radix select (SAD <= 121 * 255 < 2^15), then the removal loop (:1361-1372)
__global__ __launch_bounds__(1024) void k_stereo_filter(const StereoArgs *__restrict__ args)
{
    const StereoArgs &A = args[blockIdx.x];
    __shared__ int hist[256];
    __shared__ int s_m, s_sel, s_k, s_cnt;
    const int tid = threadIdx.x;
    if (tid < 256) hist[tid] = 0;
    if (tid == 0) s_m = s_cnt = 0;
    __syncthreads();
    int m = 0;
    for (int i = tid; i < A.n; i += 1024) {
        const int s = A.sad[i];
        if (s >= 0) {
            m++;
            atomicAdd(&hist[s >> 7], 1);
        }
    }
    atomicAdd(&s_m, m);
    __syncthreads();
    const int M = s_m;
    if (M == 0) {  // (the reference indexes an empty vDistIdx here)
        if (tid == 0) A.nmatch[0] = 0;
        return;
    }
    if (tid == 0) {
        int k = M / 2, b = 0;
        while (k >= hist[b]) k -= hist[b++];
        s_sel = b;
        s_k = k;
    }
    __syncthreads();
    const int hi = s_sel;
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < A.n; i += 1024) {
        const int s = A.sad[i];
        if (s >= 0 && (s >> 7) == hi) atomicAdd(&hist[s & 127], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int k = s_k, b = 0;
        while (k >= hist[b]) k -= hist[b++];
        s_sel = (hi << 7) | b;
    }
    __syncthreads();
    const float median = (float)s_sel;
    const float thDist = 1.5f * 1.4f * median;
    int cnt = 0;
    for (int i = tid; i < A.n; i += 1024) {
        const int s = A.sad[i];
        if (s < 0) continue;
        if (!((float)s < thDist)) {
            A.ur[i] = -1;
            A.depth[i] = -1;
        } else {
            cnt++;
        }
    }
    atomicAdd(&s_cnt, cnt);
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

struct Problem {
    std::vector<std::vector<uint8_t>> lv;  // packed host levels (left 0..L-1, right 0..L-1)
    bool dev[2] = {false, false};          // pyramid read in place (left, right)
    size_t rs_off = 0, rl_off = 0;         // this frame's vRowIndices CSR in the device row buffer (ints)
};

int check_pyr(osg_ctx *ctx, const osg_image_pyramid &P, int n_levels, const char *which, int b)
{
    OSG_REQUIRE(ctx, P.n_levels >= n_levels && P.data && P.rows && P.cols && P.step,
                "problem %d: %s pyramid needs %d levels", b, which, n_levels);
    for (int l = 0; l < n_levels; l++)
        OSG_REQUIRE(ctx, P.data[l] && P.rows[l] > 0 && P.cols[l] > 0 && P.step[l] >= P.cols[l],
                    "problem %d: %s level %d", b, which, l);
    return OSG_OK;
}

int stereo_run(osg_ctx *ctx, const osg_stereo_frame *F, int B, float *u_right, float *depth, int32_t *nmatches)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, B >= 0 && B <= 65535 && (B == 0 || (F && nmatches)), "batch arguments");
    // OSG_STEREO_PROFILE=1: host phase times per call on stderr (probe runs)
    static const bool prof = getenv("OSG_STEREO_PROFILE") && atoi(getenv("OSG_STEREO_PROFILE")) == 1;
    using hclock = std::chrono::steady_clock;
    const hclock::time_point t0 = hclock::now();
    osg_packer pk;
    std::vector<StereoArgs> args(B);
    std::vector<Problem> P(B);
    std::vector<size_t> o_base(B + 1, 0);
    size_t row_ints = 0;   // device vRowIndices of all frames (row_start + row_list capacity)
    int maxn = 0;
    for (int b = 0; b < B; b++) {
        const osg_stereo_frame &S = F[b];
        OSG_REQUIRE(ctx, S.n >= 0 && S.n_right >= 0 && S.n_right < MAX_ROW_LIST, "problem %d: sizes", b);
        OSG_REQUIRE(ctx, S.n_levels > 0 && S.n_levels <= MAX_LEVELS && S.scale_factors && S.inv_scale_factors,
                    "problem %d: levels", b);
        OSG_REQUIRE(ctx, S.n == 0 || (S.x && S.y && S.octave && S.desc), "problem %d: left keypoints", b);
        OSG_REQUIRE(ctx, S.n_right == 0 || (S.xr && S.yr && S.octave_r && S.desc_r), "problem %d: right keypoints", b);
        o_base[b + 1] = o_base[b] + (size_t)S.n;
        maxn = std::max(maxn, S.n);
        StereoArgs &A = args[b];
        A = StereoArgs{};
        A.n = S.n;
        A.n_levels = S.n_levels;
        A.mb = S.mb;
        A.mbf = S.mbf;
        if (S.n == 0) continue;
        int rc = check_pyr(ctx, S.left, S.n_levels, "left", b);
        if (rc < 0) return rc;
        rc = check_pyr(ctx, S.right, S.n_levels, "right", b);
        if (rc < 0) return rc;
        for (int i = 0; i < S.n; i++)
            OSG_REQUIRE(ctx, S.octave[i] >= 0 && S.octave[i] < S.n_levels, "problem %d: octave[%d]", b, i);
        for (int i = 0; i < S.n_right; i++)
            OSG_REQUIRE(ctx, S.octave_r[i] >= 0 && S.octave_r[i] < S.n_levels, "problem %d: right octave[%d]", b, i);
        // vRowIndices (ref:src/Frame.cc:1150-1170) is built on the device by k_stereo_rows; a right
        // keypoint covers at most 2 r + 3 <= 4 max(mvScaleFactors) + 3 rows
        const int nRows = S.left.rows[0];
        OSG_REQUIRE(ctx, nRows <= MAX_ROWS0, "problem %d: %d image rows above %d", b, nRows, MAX_ROWS0);
        float smax = 1.0f;
        for (int l = 0; l < S.n_levels; l++) smax = std::max(smax, S.scale_factors[l]);
        OSG_REQUIRE(ctx, smax < 1e6f, "problem %d: scale factors", b);
        Problem &p = P[b];
        p.rs_off = row_ints;
        p.rl_off = row_ints + (size_t)nRows + 1;
        row_ints = p.rl_off + (size_t)S.n_right * (size_t)((int)std::ceil(4.0f * smax) + 3);
        A.rows0 = nRows;
        A.n_right = S.n_right;
        set_off(A.x, pk.add(S.x, sizeof(float) * S.n));
        set_off(A.y, pk.add(S.y, sizeof(float) * S.n));
        set_off(A.oct, pk.add(S.octave, sizeof(int32_t) * S.n));
        set_off(A.desc, pk.add(S.desc, (size_t)S.n * 32));
        set_off(A.xr, pk.add(S.xr, sizeof(float) * S.n_right));
        set_off(A.yr, pk.add(S.yr, sizeof(float) * S.n_right));
        set_off(A.oct_r, pk.add(S.octave_r, sizeof(int32_t) * S.n_right));
        set_off(A.desc_r, pk.add(S.desc_r, (size_t)S.n_right * 32));
        set_off(A.scale, pk.add(S.scale_factors, sizeof(float) * S.n_levels));
        set_off(A.inv_scale, pk.add(S.inv_scale_factors, sizeof(float) * S.n_levels));
        p.lv.resize(2 * S.n_levels);
        for (int side = 0; side < 2; side++) {
            const osg_image_pyramid &Y = side ? S.right : S.left;
            p.dev[side] = Y.on_device != 0;
            for (int l = 0; l < S.n_levels; l++) {
                const int rows = Y.rows[l], cols = Y.cols[l];
                (side ? A.rows_r : A.rows_l)[l] = rows;
                (side ? A.cols_r : A.cols_l)[l] = cols;
                GLOBAL const uint8_t *&img = side ? A.img_r[l] : A.img_l[l];
                int &step = side ? A.step_r[l] : A.step_l[l];
                if (p.dev[side]) {  // device address, kept as is
                    img = (GLOBAL const uint8_t *)Y.data[l];
                    step = Y.step[l];
                    continue;
                }
                step = cols;
                const uint8_t *src = Y.data[l];
                if (Y.step[l] == cols) {
                    set_off(img, pk.add(src, (size_t)rows * cols));
                } else {
                    std::vector<uint8_t> &buf = p.lv[side * S.n_levels + l];
                    buf.resize((size_t)rows * cols);
                    for (int r = 0; r < rows; r++) std::memcpy(&buf[(size_t)r * cols], src + (size_t)r * Y.step[l], cols);
                    set_off(img, pk.add(buf.data(), buf.size()));
                }
            }
        }
    }
    for (size_t i = 0; i < o_base[B]; i++) {
        if (u_right) u_right[i] = -1.0f;
        if (depth) depth[i] = -1.0f;
    }
    for (int b = 0; b < B; b++) nmatches[b] = 0;
    if (o_base[B] == 0) return OSG_OK;
    OSG_REQUIRE(ctx, u_right && depth, "null output");
    const size_t in_bytes = (pk.total + 255) & ~size_t(255);
    const size_t args_bytes = (sizeof(StereoArgs) * (size_t)B + 255) & ~size_t(255);
    const size_t out_bytes = sizeof(int32_t) * (3 * o_base[B] + B);
    char *pin = (char *)osg_pinned(ctx, in_bytes + args_bytes + out_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    const hclock::time_point t1 = hclock::now();
    pk.fill_parallel(pin, 8);
    const hclock::time_point t2 = hclock::now();
    StereoArgs *pin_args = (StereoArgs *)(pin + in_bytes);
    int32_t *pin_out = (int32_t *)((char *)pin_args + args_bytes);
    char *dev_in = nullptr;
    StereoArgs *dev_args = nullptr;
    int32_t *dev_out = nullptr, *dev_rows = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dev_args, SLOT_TMP1, args_bytes);
    OSG_ALLOC(ctx, dev_out, SLOT_TMP2, out_bytes);
    OSG_ALLOC(ctx, dev_rows, SLOT_TMP3, sizeof(int32_t) * row_ints + 256);
    const size_t N = o_base[B];
    for (int b = 0; b < B; b++) {
        StereoArgs &A = args[b];
        relocate(A.x, dev_in);
        relocate(A.y, dev_in);
        relocate(A.oct, dev_in);
        relocate(A.desc, dev_in);
        relocate(A.xr, dev_in);
        relocate(A.yr, dev_in);
        relocate(A.oct_r, dev_in);
        relocate(A.desc_r, dev_in);
        A.row_start = (GLOBAL int32_t *)(dev_rows + P[b].rs_off);
        A.row_list = (GLOBAL int32_t *)(dev_rows + P[b].rl_off);
        relocate(A.scale, dev_in);
        relocate(A.inv_scale, dev_in);
        for (int l = 0; l < MAX_LEVELS; l++) {
            if (!P[b].dev[0]) relocate(A.img_l[l], dev_in);
            if (!P[b].dev[1]) relocate(A.img_r[l], dev_in);
        }
        A.ur = (GLOBAL float *)(dev_out + o_base[b]);
        A.depth = (GLOBAL float *)(dev_out + N + o_base[b]);
        A.sad = (GLOBAL int32_t *)(dev_out + 2 * N + o_base[b]);
        A.nmatch = (GLOBAL int32_t *)(dev_out + 3 * N + b);
        pin_args[b] = A;
    }
    if (pk.total) OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_in, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_args, pin_args, sizeof(StereoArgs) * (size_t)B, hipMemcpyHostToDevice,
                                      ctx->stream));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_stereo_rows, dim3(B), dim3(1024), 0, ctx->stream, dev_args);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_stereo_match, dim3((maxn + 3) / 4, B), dim3(256), 0, ctx->stream, dev_args);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_stereo_filter, dim3(B), dim3(1024), 0, ctx->stream, dev_args);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    OSG_RC(osg_download(ctx, pin_out, dev_out, out_bytes));
    const hclock::time_point t3 = hclock::now();
    OSG_RC(osg_wait(ctx));
    const hclock::time_point t4 = hclock::now();
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    std::memcpy(u_right, pin_out, sizeof(float) * N);
    std::memcpy(depth, pin_out + N, sizeof(float) * N);
    for (int b = 0; b < B; b++) nmatches[b] = pin_out[3 * N + b];
    if (prof) {
        auto us = [](hclock::time_point a, hclock::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        fprintf(stderr, "[osg stereo host] B %d: prep %.1f | fill %.1f | launch %.1f | wait %.1f | results %.1f us (kernel %.3f ms, pack %zu B)\n",
                B, us(t0, t1), us(t1, t2), us(t2, t3), us(t3, t4), us(t4, hclock::now()), ms, (size_t)pk.total);
    }
    return OSG_OK;
}

}  // namespace

extern "C" {

int osg_compute_stereo_matches(osg_ctx *ctx, const osg_stereo_frame *F, float *u_right, float *depth)
{
    int32_t n = 0;
    const int rc = stereo_run(ctx, F, 1, u_right, depth, &n);
    return rc < 0 ? rc : n;
}

int osg_compute_stereo_matches_batch(osg_ctx *ctx, const osg_stereo_frame *F, int32_t B, float *u_right,
                                     float *depth, int32_t *nmatches)
{
    return stereo_run(ctx, F, B, u_right, depth, nmatches);
}

}  // extern "C"
