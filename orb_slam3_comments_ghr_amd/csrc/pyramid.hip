// pyramid.hip — ORBextractor::ComputePyramid (ref:src/ORBextractor.cc:1692-1743) and the per-level
// GaussianBlur of ORBextractor::operator() (ref:src/ORBextractor.cc:1628-1636) on gfx950, writing
// straight into one caller-owned device buffer that osg_orb_detect / osg_orb_describe /
// osg_compute_stereo_matches then read in place.
//  * k_pyr_group (OSG_PYR_FUSED=1) — GROUP = 4 levels per launch, each pixel of level l evaluated from the
//    last stored level by applying the resize formula recursively (4^D stored pixels for D levels
//    up), with the previous group's blur tiles in the same launch: 3 launches for 8 levels.
//  * k_pyr_level (default) — one launch per level (level l reads level l - 1),
//    one thread per pixel of the bordered level (cols + 38) x (rows + 38).  A border pixel is the
//    reflect-101 image of an interior one (copyMakeBorder BORDER_REFLECT_101 [+ ISOLATED], :1717,
//    :1738), so each thread maps its coordinates back into the ROI and evaluates that pixel: level 0
//    copies the input image, level l >= 1 evaluates cv::resize INTER_LINEAR's 8-bit fixed-point
//    formula at it — the per-column (sx, sx + 1, 11-bit weights) and per-row tables are OpenCV's,
//    built on the host with its float/double expressions, and the vertical rounding follows the
//    columns its 128-bit vector loop covers (see oracle/oracle_pyramid.c for the restated algorithm).
//  * k_pyr_blur (with k_pyr_level) and the blur parts of k_pyr_group — 64 x 16 output tiles: the (70 x 22)-byte source tile
//    (reflect-101 at the level edges, as on the reference's continuous clone) and the 22 x 64
//    horizontal sums stay in LDS; the 7-tap fixed-point kernel [18 34 48 56 48 34 18] / 256 of OpenCV's
//    bit-exact 8-bit GaussianBlur, rows then columns, every sum exact, one rounding (+2^15) >> 16.
// Everything is integer arithmetic on bytes: HBM/latency-bound, no MFMA.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int EDGE = 19;           // EDGE_THRESHOLD (ref:src/ORBextractor.cc:80)
constexpr int MAX_LEVELS = 32;
constexpr int BT_W = 64, BT_H = 16, KR = 3;  // blur tile and kernel radius

__device__ __forceinline__ int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

struct LevelArgs {
    GLOBAL const uint8_t *src;  // level 0: the image; else the previous level's ROI
    int sstep;
    GLOBAL uint8_t *dst;        // bordered level (top-left of the border)
    int w, h, bstep;
    const int4 *xt;             // per output column: sx, sx + 1 (clamped), alpha0, alpha1
    const int4 *yt;             // per output row: r0, r1, beta0, beta1
    int xv;                     // columns of the vector loop (rounding of the vertical pass)
    int copy;                   // level 0
    long long src_bstride, dst_bstride;  // batch (blockIdx.z = image): bytes between images' src / dst
};

__global__ __launch_bounds__(256) void k_pyr_level(const LevelArgs A)
{
    const int bx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int by = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (bx >= A.w + 2 * EDGE || by >= A.h + 2 * EDGE) return;
    const int x = reflect101(bx - EDGE, A.w), y = reflect101(by - EDGE, A.h);
    GLOBAL const uint8_t *src = A.src + (long long)blockIdx.z * A.src_bstride;
    int v;
    if (A.copy) {
        v = src[(long long)y * A.sstep + x];
    } else {
        const int4 X = A.xt[x], Y = A.yt[y];
        GLOBAL const uint8_t *S0 = src + (long long)Y.x * A.sstep;
        GLOBAL const uint8_t *S1 = src + (long long)Y.y * A.sstep;
        const int d0 = S0[X.x] * X.z + S0[X.y] * X.w;  // HResizeLinear: exact int
        const int d1 = S1[X.x] * X.z + S1[X.y] * X.w;
        if (x < A.xv)  // VResizeLinearVec_32s8u: mulhi of (d >> 4) by the weight, (+2) >> 2
            v = ((((d0 >> 4) * Y.z) >> 16) + (((d1 >> 4) * Y.w) >> 16) + 2) >> 2;
        else           // FixedPtCast<int, uchar, 22>
            v = (d0 * Y.z + d1 * Y.w + (1 << 21)) >> 22;
        v = v < 0 ? 0 : v > 255 ? 255 : v;
    }
    A.dst[(long long)blockIdx.z * A.dst_bstride + (long long)by * A.bstep + bx] = (uint8_t)v;
}

struct BlurArgs {
    int n_levels;
    int k[2 * KR + 1];
    GLOBAL const uint8_t *roi[MAX_LEVELS];
    GLOBAL uint8_t *out[MAX_LEVELS];
    int w[MAX_LEVELS], h[MAX_LEVELS], bstep[MAX_LEVELS];
    int tiles_x[MAX_LEVELS], block0[MAX_LEVELS + 1];
    long long bstride;  // batch (blockIdx.y = image): bytes between the images' pyramid buffers
};

__global__ __launch_bounds__(256) void k_pyr_blur(const BlurArgs A)
{
    constexpr int SW = BT_W + 2 * KR, SH = BT_H + 2 * KR;
    __shared__ uint8_t s_src[SH][SW + 2];
    __shared__ uint16_t s_h[SH][BT_W];
    int l = 0;
    while (l + 1 < A.n_levels && (int)blockIdx.x >= A.block0[l + 1]) l++;
    const int b = blockIdx.x - A.block0[l];
    const int w = A.w[l], h = A.h[l], bstep = A.bstep[l];
    const int tx0 = (b % A.tiles_x[l]) * BT_W, ty0 = (b / A.tiles_x[l]) * BT_H;
    GLOBAL const uint8_t *roi = A.roi[l] + (long long)blockIdx.y * A.bstride;
    for (int i = threadIdx.x; i < SH * SW; i += 256) {
        const int r = i / SW, c = i - r * SW;
        const int y = reflect101(ty0 + r - KR, h), x = reflect101(tx0 + c - KR, w);
        s_src[r][c] = roi[(long long)y * bstep + x];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < SH * BT_W; i += 256) {
        const int r = i / BT_W, c = i - r * BT_W;
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j <= 2 * KR; j++) s += (uint32_t)s_src[r][c + j] * (uint32_t)A.k[j];
        s_h[r][c] = (uint16_t)s;  // <= 255 * 256: exact (ufixedpoint16)
    }
    __syncthreads();
    for (int i = threadIdx.x; i < BT_H * BT_W; i += 256) {
        const int r = i / BT_W, c = i - r * BT_W;
        const int y = ty0 + r, x = tx0 + c;
        if (y >= h || x >= w) continue;
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j <= 2 * KR; j++) s += (uint32_t)s_h[r + j][c] * (uint32_t)A.k[j];
        A.out[l][(long long)blockIdx.y * A.bstride + (long long)y * w + x] = (uint8_t)((s + (1u << 15)) >> 16);
    }
}

// ---- the fused form (default): GROUP levels per launch, each from the last stored level ----------
// A level-l pixel needs the 2 x 2 level-(l - 1) pixels of its resize tables, so a pixel D levels
// above the stored one is the same integer formula applied recursively over 4^D stored pixels
// (D <= GROUP): no value changes, only where it is computed.  Launch k computes level group k and
// blurs group k - 1 (stored by launch k - 1); a last launch blurs the last group.
constexpr int GROUP = 4;  // the largest group; OSG_PYR_GROUP=1..4 picks it per call
constexpr bool PYR_FUSED_DEFAULT = false;
constexpr int PYR_GROUP_DEFAULT = 4;
constexpr int GMAX = 16;  // levels a fused call handles (the level-wise path takes up to MAX_LEVELS)

struct PyrLevelDev {
    const int4 *xt, *yt;        // resize tables of this level from the previous one
    GLOBAL uint8_t *dst;        // bordered level
    GLOBAL uint8_t *blur_out;   // blurred level
    int xv, w, h, bstep;
};

struct GroupArgs {
    GLOBAL const uint8_t *src;  // the stored level src_level (the image for level 0, else an ROI)
    int sstep, src_level, n_parts;
    int k[2 * KR + 1];
    PyrLevelDev L[GMAX];
    int part_level[2 * GROUP], part_kind[2 * GROUP], part_tiles_x[2 * GROUP], part_block0[2 * GROUP + 1];
};

template <int D>
__device__ __forceinline__ int level_px(const GroupArgs &A, int l, int x, int y)
{
    if constexpr (D == 0) {
        return A.src[(long long)y * A.sstep + x];
    } else {
        const int4 X = A.L[l].xt[x], Y = A.L[l].yt[y];
        const int s00 = level_px<D - 1>(A, l - 1, X.x, Y.x), s01 = level_px<D - 1>(A, l - 1, X.y, Y.x);
        const int s10 = level_px<D - 1>(A, l - 1, X.x, Y.y), s11 = level_px<D - 1>(A, l - 1, X.y, Y.y);
        const int d0 = s00 * X.z + s01 * X.w, d1 = s10 * X.z + s11 * X.w;
        int v;
        if (x < A.L[l].xv)
            v = ((((d0 >> 4) * Y.z) >> 16) + (((d1 >> 4) * Y.w) >> 16) + 2) >> 2;
        else
            v = (d0 * Y.z + d1 * Y.w + (1 << 21)) >> 22;
        return v < 0 ? 0 : v > 255 ? 255 : v;
    }
}

// depth d of the level above the stored one, dispatched over the instantiations up to DMAX only (the
// kernel is instantiated per group size: the deep recursion's code stays out of the shallow launches)
template <int D, int DMAX>
__device__ __forceinline__ int level_at(const GroupArgs &A, int d, int l, int x, int y)
{
    if constexpr (D == DMAX)
        return level_px<D>(A, l, x, y);
    else
        return d == D ? level_px<D>(A, l, x, y) : level_at<D + 1, DMAX>(A, d, l, x, y);
}

template <int DMAX>
__global__ __launch_bounds__(256) void k_pyr_group(const GroupArgs *__restrict__ Ad)
{
    const GroupArgs &A = *Ad;
    constexpr int SW = BT_W + 2 * KR, SH = BT_H + 2 * KR;
    __shared__ uint8_t s_src[SH][SW + 2];
    __shared__ uint16_t s_h[SH][BT_W];
    int p = 0;
    while (p + 1 < A.n_parts && (int)blockIdx.x >= A.part_block0[p + 1]) p++;
    const int b = blockIdx.x - A.part_block0[p];
    const int l = A.part_level[p], tx = A.part_tiles_x[p];
    const int w = A.L[l].w, h = A.L[l].h, bstep = A.L[l].bstep;
    if (A.part_kind[p] == 0) {  // a 64 x 4 patch of the bordered level
        const int bx = (b % tx) * 64 + (threadIdx.x & 63), by = (b / tx) * 4 + (threadIdx.x >> 6);
        if (bx >= w + 2 * EDGE || by >= h + 2 * EDGE) return;
        const int x = reflect101(bx - EDGE, w), y = reflect101(by - EDGE, h);
        const int v = level_at<0, DMAX>(A, l - A.src_level, l, x, y);
        A.L[l].dst[(long long)by * bstep + bx] = (uint8_t)v;
        return;
    }
    // a 64 x 16 blur tile (block-uniform branch: the barriers below are reached by every thread)
    const int tx0 = (b % tx) * BT_W, ty0 = (b / tx) * BT_H;
    GLOBAL const uint8_t *roi = A.L[l].dst + (long long)EDGE * bstep + EDGE;
    for (int i = threadIdx.x; i < SH * SW; i += 256) {
        const int r = i / SW, c = i - r * SW;
        s_src[r][c] = roi[(long long)reflect101(ty0 + r - KR, h) * bstep + reflect101(tx0 + c - KR, w)];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < SH * BT_W; i += 256) {
        const int r = i / BT_W, c = i - r * BT_W;
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j <= 2 * KR; j++) s += (uint32_t)s_src[r][c + j] * (uint32_t)A.k[j];
        s_h[r][c] = (uint16_t)s;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < BT_H * BT_W; i += 256) {
        const int r = i / BT_W, c = i - r * BT_W;
        const int y = ty0 + r, x = tx0 + c;
        if (y >= h || x >= w) continue;
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j <= 2 * KR; j++) s += (uint32_t)s_h[r + j][c] * (uint32_t)A.k[j];
        A.L[l].blur_out[(long long)y * w + x] = (uint8_t)((s + (1u << 15)) >> 16);
    }
}

int16_t sat_short(float v)
{
    const long r = lrintf(v);  // cvRound
    return (int16_t)(r < -32768 ? -32768 : r > 32767 ? 32767 : r);
}

// cv::resize's INTER_LINEAR coefficient tables (imgproc/resize.cpp) for one axis; xmax semantics on x
void axis_table(int sn, int dn, bool is_x, std::vector<int4> &t)
{
    const double scale = 1.0 / ((double)dn / sn);
    t.resize(dn);
    for (int d = 0; d < dn; d++) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s = (int)std::floor(f);
        f -= (float)s;
        int s1;
        if (is_x) {
            if (s < 0) f = 0, s = 0;
            if (s + 1 >= sn && s >= sn - 1) f = 0, s = sn - 1;
            s1 = std::min(s + 1, sn - 1);  // from xmax on the weight of sx + 1 is 0
        } else {
            s1 = std::min(std::max(s + 1, 0), sn - 1);  // rows are clipped, weights kept
            s = std::min(std::max(s, 0), sn - 1);
        }
        t[d] = make_int4(s, s1, sat_short((1.f - f) * 2048), sat_short(f * 2048));
    }
}

int vector_columns(int w)
{
    int x = 0;
    while (x <= w - 16) x += 16;
    while (x < w - 8) x += 8;
    return x;
}

// getGaussianKernelBitExact(7, 2) quantised by getGaussianKernelFixedPoint_ED to 8 fraction bits
void gaussian_kernel7(int k[7])
{
    const double scale2X = -0.125 / (2.0 * 2.0);
    double v[3], sum = 0;
    for (int i = 0, x = -6; i < 3; i++, x += 2) {
        v[i] = std::exp((double)(x * x) * scale2X);
        sum += v[i];
    }
    const double mul1 = 1.0 / (sum * 2 + 1);
    double err = 0;
    long s = 0;
    for (int i = 0; i < 3; i++) {
        const double adj = v[i] * mul1 * 256.0 + err;
        const long v0 = std::lrint(adj);
        err = adj - (double)v0;
        k[i] = k[6 - i] = (int)v0;
        s += v0;
    }
    k[3] = (int)(256 - 2 * s);
}

int64_t layout(int32_t rows, int32_t cols, int32_t n_levels, const float *inv_scale, int32_t *lrows, int32_t *lcols,
               int64_t *bordered_off, int64_t *blurred_off)
{
    if (rows < 1 || cols < 1 || n_levels < 1 || n_levels > MAX_LEVELS || !inv_scale || !lrows || !lcols ||
        !bordered_off || !blurred_off)
        return OSG_E_INVALID;
    int64_t at = 0;
    for (int l = 0; l < n_levels; l++) {
        if (!(inv_scale[l] > 0.f) || !(inv_scale[l] <= 1.f)) return OSG_E_INVALID;
        lcols[l] = (int32_t)std::lrint((float)cols * inv_scale[l]);  // cvRound((float)cols * scale), :1697
        lrows[l] = (int32_t)std::lrint((float)rows * inv_scale[l]);
        if (lcols[l] < 1 || lrows[l] < 1) return OSG_E_INVALID;
        bordered_off[l] = at;
        at += ((int64_t)(lrows[l] + 2 * EDGE) * (lcols[l] + 2 * EDGE) + 255) & ~(int64_t)255;
    }
    for (int l = 0; l < n_levels; l++) {
        blurred_off[l] = at;
        at += ((int64_t)lrows[l] * lcols[l] + 255) & ~(int64_t)255;
    }
    return at;
}

// B images (B > 1: device images img_bstride bytes apart, pyramids out_bstride bytes apart in dev_out,
// the level-wise launches with the image in the grid's last dimension)
int pyramid_run(osg_ctx *ctx, const uint8_t *image, int32_t rows, int32_t cols, int32_t step, int32_t on_device,
                int32_t n_levels, const float *inv_scale, uint8_t *dev_out, int64_t dev_bytes, int32_t blur,
                int32_t B = 1, int64_t img_bstride = 0, int64_t out_bstride = 0)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, B >= 1 && B <= 65535 && (B == 1 || on_device), "batch of %d images (device images only)", B);
    OSG_REQUIRE(ctx, image && dev_out && step >= cols, "null argument or step < cols");
    int32_t lr[MAX_LEVELS], lc[MAX_LEVELS];
    int64_t bo[MAX_LEVELS], bl[MAX_LEVELS];
    const int64_t total = layout(rows, cols, n_levels, inv_scale, lr, lc, bo, bl);
    OSG_REQUIRE(ctx, total > 0, "pyramid layout (%d x %d, %d levels; 0 < mvInvScaleFactor <= 1)", cols, rows,
                n_levels);
    OSG_REQUIRE(ctx, B == 1 || out_bstride >= total, "pyramid stride %lld < %lld bytes", (long long)out_bstride,
                (long long)total);
    const int64_t need = (int64_t)(B - 1) * out_bstride + (blur ? total : bl[0]);
    OSG_REQUIRE(ctx, dev_bytes >= need, "output buffer of %lld bytes, %lld needed", (long long)dev_bytes,
                (long long)need);
    osg_packer pk;
    std::vector<uint8_t> packed;
    size_t img_off = SIZE_MAX;
    if (!on_device) {
        if (step == cols) {
            img_off = pk.add(image, (size_t)rows * cols);
        } else {
            packed.resize((size_t)rows * cols);
            for (int r = 0; r < rows; r++) std::memcpy(&packed[(size_t)r * cols], image + (size_t)r * step, cols);
            img_off = pk.add(packed.data(), packed.size());
        }
    }
    std::vector<std::vector<int4>> xt(n_levels), yt(n_levels);
    std::vector<size_t> xo(n_levels, SIZE_MAX), yo(n_levels, SIZE_MAX);
    for (int l = 1; l < n_levels; l++) {
        axis_table(lc[l - 1], lc[l], true, xt[l]);
        axis_table(lr[l - 1], lr[l], false, yt[l]);
        xo[l] = pk.add(xt[l].data(), sizeof(int4) * xt[l].size());
        yo[l] = pk.add(yt[l].data(), sizeof(int4) * yt[l].size());
    }
    // OSG_PYR_FUSED=0/1 picks the launch form per call (the tests compare both); default below
    const char *fz = getenv("OSG_PYR_FUSED");
    const bool levelwise = fz ? atoi(fz) == 0 : !PYR_FUSED_DEFAULT;
    const char *gz = getenv("OSG_PYR_GROUP");
    const int grp = gz ? std::min(GROUP, std::max(1, atoi(gz))) : PYR_GROUP_DEFAULT;
    const bool fused = !levelwise && n_levels <= GMAX && B == 1;
    const int ng = fused ? (n_levels + grp - 1) / grp : 0;
    // the fused launches' descriptors travel in the staging upload and the kernel reads them from HBM:
    // as kernel arguments (~1 KB, indexed by the block's part and level) each dependent read was a
    // round trip to the host-resident kernarg segment
    std::vector<GroupArgs> groups(fused ? ng + 1 : 0);
    std::vector<int> group_blocks(groups.size(), 0);
    const size_t go = fused ? pk.add(groups.data(), sizeof(GroupArgs) * groups.size()) : SIZE_MAX;
    char *din = nullptr;
    if (pk.total) {
        char *pin = (char *)osg_pinned(ctx, pk.total + 256);
        if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
        OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
        OSG_ALLOC(ctx, din, SLOT_TMP0, pk.total + 256);
        if (fused) {
            GroupArgs G{};
            gaussian_kernel7(G.k);
            for (int l = 0; l < n_levels; l++) {
                PyrLevelDev &V = G.L[l];
                V.w = lc[l];
                V.h = lr[l];
                V.bstep = lc[l] + 2 * EDGE;
                V.dst = (GLOBAL uint8_t *)(dev_out + bo[l]);
                V.blur_out = (GLOBAL uint8_t *)(dev_out + bl[l]);
                if (l > 0) {
                    V.xt = (const int4 *)(din + xo[l]);
                    V.yt = (const int4 *)(din + yo[l]);
                    V.xv = vector_columns(lc[l]);
                }
            }
            for (int k = 0; k <= ng; k++) {
                G.n_parts = 0;
                int nb = 0;
                auto add_part = [&](int l, int kind, int tiles_x, int tiles) {
                    G.part_level[G.n_parts] = l;
                    G.part_kind[G.n_parts] = kind;
                    G.part_tiles_x[G.n_parts] = tiles_x;
                    G.part_block0[G.n_parts] = nb;
                    G.n_parts++;
                    nb += tiles;
                };
                if (k < ng) {
                    if (k == 0) {
                        G.src = on_device ? (GLOBAL const uint8_t *)image : (GLOBAL const uint8_t *)(din + img_off);
                        G.sstep = on_device ? step : cols;
                        G.src_level = 0;
                    } else {
                        const int s0 = grp * k - 1;
                        G.src = (GLOBAL const uint8_t *)(dev_out + bo[s0] + (int64_t)EDGE * G.L[s0].bstep + EDGE);
                        G.sstep = G.L[s0].bstep;
                        G.src_level = s0;
                    }
                    for (int l = grp * k; l < std::min(n_levels, grp * (k + 1)); l++) {
                        const int tx = (lc[l] + 2 * EDGE + 63) / 64;
                        add_part(l, 0, tx, tx * ((lr[l] + 2 * EDGE + 3) / 4));
                    }
                }
                if (blur && k >= 1)
                    for (int l = grp * (k - 1); l < std::min(n_levels, grp * k); l++) {
                        const int tx = (lc[l] + BT_W - 1) / BT_W;
                        add_part(l, 1, tx, tx * ((lr[l] + BT_H - 1) / BT_H));
                    }
                G.part_block0[G.n_parts] = nb;
                groups[k] = G;
                group_blocks[k] = G.n_parts ? nb : 0;
            }
        }
        pk.fill(pin);
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(din, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    }
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    if (fused) {
        auto *kern = grp == 1 ? k_pyr_group<1> : grp == 2 ? k_pyr_group<2> : grp == 3 ? k_pyr_group<3>
                                                                             : k_pyr_group<4>;
        for (int k = 0; k <= ng; k++) {
            if (!group_blocks[k]) continue;
            const GroupArgs *gd = (const GroupArgs *)(din + go + sizeof(GroupArgs) * k);
            hipLaunchKernelGGL(kern, dim3(group_blocks[k]), dim3(256), 0, ctx->stream, gd);
            OSG_HIP_CHECK(ctx, hipGetLastError());
        }
        OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
        OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));  // (a polled wait measured slower here)
        float ms = 0.f;
        OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
        ctx->last_kernel_ms = ms;
        return OSG_OK;
    }
    for (int l = 0; l < n_levels; l++) {
        LevelArgs A{};
        A.w = lc[l];
        A.h = lr[l];
        A.bstep = lc[l] + 2 * EDGE;
        A.dst = (GLOBAL uint8_t *)(dev_out + bo[l]);
        if (l == 0) {
            A.copy = 1;
            A.src = on_device ? (GLOBAL const uint8_t *)image : (GLOBAL const uint8_t *)(din + img_off);
            A.sstep = on_device ? step : cols;
        } else {
            const int pstep = lc[l - 1] + 2 * EDGE;
            A.src = (GLOBAL const uint8_t *)(dev_out + bo[l - 1] + (int64_t)EDGE * pstep + EDGE);
            A.sstep = pstep;
            A.xt = (const int4 *)(din + xo[l]);
            A.yt = (const int4 *)(din + yo[l]);
            A.xv = vector_columns(lc[l]);
        }
        A.src_bstride = l == 0 ? img_bstride : out_bstride;
        A.dst_bstride = out_bstride;
        const dim3 grid((A.w + 2 * EDGE + 63) / 64, (A.h + 2 * EDGE + 3) / 4, B);
        hipLaunchKernelGGL(k_pyr_level, grid, dim3(256), 0, ctx->stream, A);
        OSG_HIP_CHECK(ctx, hipGetLastError());
    }
    if (blur) {
        const int nimg = B;
        BlurArgs B{};
        B.n_levels = n_levels;
        gaussian_kernel7(B.k);
        int nb = 0;
        for (int l = 0; l < n_levels; l++) {
            B.w[l] = lc[l];
            B.h[l] = lr[l];
            B.bstep[l] = lc[l] + 2 * EDGE;
            B.roi[l] = (GLOBAL const uint8_t *)(dev_out + bo[l] + (int64_t)EDGE * B.bstep[l] + EDGE);
            B.out[l] = (GLOBAL uint8_t *)(dev_out + bl[l]);
            B.tiles_x[l] = (lc[l] + BT_W - 1) / BT_W;
            B.block0[l] = nb;
            nb += B.tiles_x[l] * ((lr[l] + BT_H - 1) / BT_H);
        }
        B.block0[n_levels] = nb;
        B.bstride = out_bstride;
        hipLaunchKernelGGL(k_pyr_blur, dim3(nb, nimg), dim3(256), 0, ctx->stream, B);
        OSG_HIP_CHECK(ctx, hipGetLastError());
    }
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    if (B > 1) return OSG_OK;  // the batched extractor goes on in the same stream (detection waits for it)
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));  // (a polled wait measured slower here)
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    return OSG_OK;
}

}  // namespace

// internal (orb.hip's batched extractor): B device images -> B pyramids out_bstride bytes apart
int osg_pyramid_batch(osg_ctx *ctx, const uint8_t *d_images, int64_t img_bstride, int32_t rows, int32_t cols,
                      int32_t step, int32_t B, int32_t n_levels, const float *inv_scale, uint8_t *dev_out,
                      int64_t out_bstride, int64_t dev_bytes)
{
    return pyramid_run(ctx, d_images, rows, cols, step, 1, n_levels, inv_scale, dev_out, dev_bytes, 1, B, img_bstride,
                       out_bstride);
}

extern "C" {

int64_t osg_orb_pyramid_layout(int32_t rows, int32_t cols, int32_t n_levels, const float *inv_scale_factors,
                               int32_t *level_rows, int32_t *level_cols, int64_t *bordered_offset,
                               int64_t *blurred_offset)
{
    return layout(rows, cols, n_levels, inv_scale_factors, level_rows, level_cols, bordered_offset, blurred_offset);
}

int osg_orb_pyramid(osg_ctx *ctx, const uint8_t *image, int32_t rows, int32_t cols, int32_t step,
                    int32_t image_on_device, int32_t n_levels, const float *inv_scale_factors, uint8_t *dev_out,
                    int64_t dev_bytes, int32_t blur)
{
    return pyramid_run(ctx, image, rows, cols, step, image_on_device, n_levels, inv_scale_factors, dev_out,
                       dev_bytes, blur);
}

void osg_debug_gaussian_kernel7(int32_t *k7)
{
    int k[7];
    gaussian_kernel7(k);
    for (int i = 0; i < 7; i++) k7[i] = k[i];
}

}  // extern "C"
