// fast.hip — ORBextractor::ComputeKeyPointsOctTree (ref:src/ORBextractor.cc:1065-1198) on gfx950.
//
// The reference FASTs every W = 35 cell of every pyramid level as its own image (rowRange /
// colRange ROI, :1139-1155), once with iniThFAST and, when that finds nothing, with minThFAST, then
// thins each level's keypoints with DistributeOctTree (:716-1050).  The FAST corner test and score
// of a pixel read only its 16-pixel circle, so they do not depend on the cell; what does is the
// tested range (3 px inside the cell) and the non-maximum suppression, whose neighbours outside
// that range count as score 0.  So:
//   k_fast_score   every pixel of every level, both thresholds: the 9-of-16 arc test on the circle's
//                  darker / brighter bit masks and cornerScore<16> (OpenCV's FAST_t / cornerScore,
//                  restated: cv::FAST is not in the reference tree) -> 2 bytes per pixel
//   k_fast_cells   one workgroup per cell: the cell's two score planes staged in LDS with a zero
//                  ring (suppression neighbours outside the tested range), the strict 3x3 maximum at
//                  iniThFAST, the minThFAST pass when it keeps nothing, and the kept keypoints written
//                  in row-major order to the cell's own slot range, with their count
//   k_cell_gather  one workgroup per cell: its offset = the sum of the counts of the cells before it
//                  (cells in the reference's level / row / column order, so the keypoints come out in
//                  vToDistributeKeys order), then its keypoints copied there
// DistributeOctTree is a short sequential tree walk per level (a few thousand keypoints): it runs
// on the host over the downloaded keypoints, with the reference's node-list order (push_front,
// erase by the stored position) and its std::sort of (size, UL.x) for the final expansions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int MAX_LEVELS = 32;
constexpr int EDGE_THRESHOLD = 19;
constexpr int PATCH_SIZE = 31;
constexpr float CELL_W = 35.f;

struct FastArgs {
    int block0[MAX_LEVELS + 1];         // first 64 x 4 pixel block of each level (flattened grid)
    int bx[MAX_LEVELS];                 // blocks per row of 64 pixels
    int n_levels;
    GLOBAL const uint8_t *img[MAX_LEVELS];
    GLOBAL uint8_t *score[MAX_LEVELS];  // per pixel: (score at min_th, score at ini_th)
    int rows[MAX_LEVELS], cols[MAX_LEVELS], step[MAX_LEVELS];
    int ini_th, min_th;
    long long img_bstride, score_bstride;  // batch (blockIdx.y = image): bytes between images
};

struct Cell {
    int level, r0, r1, c0, c1;  // the cell image: rows r0 .. r1 - 1, columns c0 .. c1 - 1 of the level
    int dx, dy;                 // (j wCell, i hCell): the shift :1168-1169 adds
    int slot;                   // first slot of the cell's keypoint range (one per tested pixel)
};
constexpr int MAX_T = 72;       // tested rows / columns of a cell + the zero ring: hCell, wCell <= 70

struct CellArgs {
    const Cell *cells;
    int n_cells;
    GLOBAL uint8_t *score[MAX_LEVELS];
    int cols[MAX_LEVELS];
    GLOBAL int32_t *count;        // per cell
    float4 *slots;                // (x, y, response, 0) per cell slot range
    float4 *keys;                 // compacted, in cell order
    GLOBAL int32_t *total;
    long long score_bstride;      // batch (blockIdx.y = image): score planes, count[n_cells], slots /
    int max_keys;                 // keys [max_keys], total[1] per image
};

// cornerScore<16> (OpenCV fast_score.cpp) with d[k] = v - circle[k] (circle index k mod 16) works
// out to max(threshold, best_dark, best_bright) - 1, where best_dark = the largest min(d) over the 16
// arcs of 9 and best_bright = the largest min(-d): its early "a <= a0: continue" skips only arcs that
// cannot raise the maximum.  A pixel is a FAST corner at threshold t exactly when best_dark > t or
// best_bright > t (a 9-arc strictly darker than v - t / brighter than v + t), so with
// s0 = max(best_dark, best_bright) - 1:
//     corner at t  <=>  s0 >= t,   and then  cornerScore(t) = s0.
// One branch-free s0 per pixel gives both thresholds' scores (the oracle keeps OpenCV's literal
// test + cornerScore; the GPU tests compare the two on every pixel of their frames).
__device__ __forceinline__ int fast_s0(const int (&d)[16])
{
    int bd = -1024, bb = -1024;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        int mn = d[k], mx = d[k];
#pragma unroll
        for (int j = 1; j < 9; j++) {
            mn = min(mn, d[(k + j) & 15]);
            mx = max(mx, d[(k + j) & 15]);
        }
        bd = max(bd, mn);
        bb = max(bb, -mx);
    }
    return max(bd, bb) - 1;
}

// one 64 x 4 pixel block per workgroup, the levels' blocks one after the other (no idle blocks of a
// grid sized for level 0)
__global__ __launch_bounds__(256) void k_fast_score(const FastArgs A)
{
    const int b = blockIdx.x;
    int l = 0;
    while (l + 1 < A.n_levels && b >= A.block0[l + 1]) l++;
    const int bl = b - A.block0[l];
    const int x = (bl % A.bx[l]) * 64 + (threadIdx.x & 63), y = (bl / A.bx[l]) * 4 + (threadIdx.x >> 6);
    const int rows = A.rows[l], cols = A.cols[l];
    if (x >= cols || y >= rows) return;
    const long long bi = blockIdx.y;
    uint8_t s_lo = 0, s_hi = 0;
    if (x >= 3 && y >= 3 && x < cols - 3 && y < rows - 3) {
        const int step = A.step[l];
        GLOBAL const uint8_t *p = A.img[l] + bi * A.img_bstride + (size_t)y * step + x;
        // the circle (x, y) offsets of OpenCV's offsets16, in order
        const int ox[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
        const int oy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
        const int v = p[0];
        int d[16];
#pragma unroll
        for (int k = 0; k < 16; k++) d[k] = v - (int)p[ox[k] + oy[k] * step];
        const int s0 = fast_s0(d);
        s_lo = (uint8_t)(s0 >= A.min_th ? s0 : 0);
        s_hi = (uint8_t)(s0 >= A.ini_th ? s0 : 0);
    }
    GLOBAL uint8_t *o = A.score[l] + bi * A.score_bstride + 2 * ((size_t)y * cols + x);
    *(GLOBAL uint16_t *)o = (uint16_t)(s_lo | (s_hi << 8));
}

// one 256-thread workgroup per cell
__global__ __launch_bounds__(256) void k_fast_cells(const CellArgs A)
{
    const int c = blockIdx.x;
    if (c >= A.n_cells) return;
    const long long bi = blockIdx.y;
    const Cell C = A.cells[c];
    const int h = C.r1 - C.r0 - 6, w = C.c1 - C.c0 - 6;  // tested rows / columns of the cell image
    const int cols = A.cols[C.level];
    GLOBAL const uint16_t *S = (GLOBAL const uint16_t *)(A.score[C.level] + bi * A.score_bstride);
    GLOBAL int32_t *count = A.count + bi * A.n_cells;
    float4 *slots = A.slots + bi * A.max_keys;
    __shared__ uint16_t s_sc[MAX_T * MAX_T];  // (score at min_th, score at ini_th), zero ring
    __shared__ int s_cnt[4];
    __shared__ int s_total;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int n = (h > 0 && w > 0) ? h * w : 0;
    const int tw = w + 2, nt = (h + 2) * tw;
    for (int i = threadIdx.x; i < nt; i += 256) {
        const int rr = i / tw - 1, cc = i % tw - 1;
        const bool in = rr >= 0 && rr < h && cc >= 0 && cc < w;
        s_sc[i] = in ? S[(size_t)(C.r0 + 3 + rr) * cols + C.c0 + 3 + cc] : (uint16_t)0;
    }
    __syncthreads();
    const int sh = 8;  // the ini_th score is the high byte
    auto keep_at = [&](int idx, int shift, int &sc) -> bool {
        const int rr = idx / w, cc = idx - rr * w;
        const uint16_t *p = s_sc + (rr + 1) * tw + cc + 1;
        sc = (p[0] >> shift) & 0xff;
        if (!sc) return false;
        const int n8[8] = {p[-tw - 1], p[-tw], p[-tw + 1], p[-1], p[1], p[tw - 1], p[tw], p[tw + 1]};
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (!(sc > ((n8[k] >> shift) & 0xff))) return false;
        return true;
    };
    auto count_pass = [&](int shift) -> int {
        int k = 0;
        for (int i = threadIdx.x; i < n; i += 256) {
            int sc;
            k += keep_at(i, shift, sc) ? 1 : 0;
        }
        for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o);
        if (lane == 0) s_cnt[wv] = k;
        __syncthreads();
        const int t = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        __syncthreads();
        return t;
    };
    int shift = sh;  // iniThFAST
    int total = count_pass(sh);
    if (total == 0) {  // :1146-1155
        shift = 0;
        total = count_pass(0);
    }
    if (threadIdx.x == 0) {
        count[c] = total;
        s_total = 0;
    }
    if (total == 0) return;
    __syncthreads();
    // ordered compaction into the cell's slots, 256 pixels per round: wave ballots, then 4 wave counts
    for (int base = 0; base < n; base += 256) {
        const int i = base + threadIdx.x;
        int sc = 0;
        const bool k = i < n && keep_at(i, shift, sc);
        const unsigned long long m = __ballot(k);
        if (lane == 0) s_cnt[wv] = __popcll(m);
        __syncthreads();
        int off = s_total;
        for (int q = 0; q < wv; q++) off += s_cnt[q];
        off += __popcll(m & ((1ull << lane) - 1));
        if (k) {
            const int rr = i / w, cc = i - rr * w;
            slots[C.slot + off] = make_float4((float)(cc + 3 + C.dx), (float)(rr + 3 + C.dy), (float)sc, 0.f);
        }
        __syncthreads();
        if (threadIdx.x == 0) s_total += s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        __syncthreads();
    }
}

// one 256-thread workgroup per cell: offset = sum of the earlier cells' counts (a few hundred loads),
// then the cell's keypoints moved to it; the last cell writes the total
__global__ __launch_bounds__(256) void k_cell_gather(const CellArgs A)
{
    const int c = blockIdx.x;
    if (c >= A.n_cells) return;
    const long long bi = blockIdx.y;
    GLOBAL const int32_t *count = A.count + bi * A.n_cells;
    __shared__ int s_part[4];
    int t = 0;
    for (int i = threadIdx.x; i < c; i += 256) t += count[i];
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = t;
    __syncthreads();
    const int off = s_part[0] + s_part[1] + s_part[2] + s_part[3];
    const int cnt = count[c];
    const int slot = A.cells[c].slot;
    float4 *keys = A.keys + bi * A.max_keys;
    const float4 *slots = A.slots + bi * A.max_keys;
    for (int i = threadIdx.x; i < cnt; i += 256) keys[off + i] = slots[slot + i];
    if (c == A.n_cells - 1 && threadIdx.x == 0) A.total[bi] = off + cnt;
}

// A batch's keys made contiguous for one download: image b's total keys move to the sum of the totals
// before it (the slot area is free once k_cell_gather has run)
__global__ __launch_bounds__(256) void k_keys_compact(const float4 *keys, int max_keys, const GLOBAL int32_t *total,
                                                      float4 *out)
{
    const int b = blockIdx.y;
    int base = 0;
    for (int i = 0; i < b; i++) base += total[i];
    const int n = total[b];
    const float4 *src = keys + (size_t)b * max_keys;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) out[base + i] = src[i];
}

#include "octree.h"
using osg_oct::Key4;
using osg_oct::distribute_oct_tree;

struct LevelGeom {
    int minBX, minBY, maxBX, maxBY, cell0, cell1;
};

// B images (B > 1: device pyramids pyr_bstride bytes apart, image b's levels at P's pointers + b
// pyr_bstride); image b's keypoints go to x / y / response / size + b cap and level_start + b (L + 1).
// Returns the keypoints of all images.
int detect_run(osg_ctx *ctx, const osg_image_pyramid *P, int ini_th, int min_th, const int32_t *n_features,
               const float *scale_factors, int cap, float *x, float *y, float *response, float *size,
               int32_t *level_start, int B = 1, int64_t pyr_bstride = 0)
{
    if (!ctx) return OSG_E_INVALID;
    static const bool prof = getenv("OSG_ORB_PROFILE") != nullptr;  // host phase times to stderr
    const auto tp0 = std::chrono::steady_clock::now();
    auto ms_since = [](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    OSG_REQUIRE(ctx, P && P->n_levels >= 1 && P->n_levels <= MAX_LEVELS && P->data && P->rows && P->cols && P->step,
                "pyramid (1 .. %d levels)", MAX_LEVELS);
    OSG_REQUIRE(ctx, n_features && scale_factors && level_start && (cap == 0 || (x && y && response && size)),
                "null argument");
    OSG_REQUIRE(ctx, B >= 1 && B <= 65535 && (B == 1 || P->on_device), "batch of %d images (device pyramids only)", B);
    const int L = P->n_levels;
    // cells in the reference's order (:1071-1175); geometry per level
    std::vector<Cell> cells;
    std::vector<LevelGeom> lg(L);
    FastArgs FA{};
    FA.ini_th = std::min(std::max(ini_th, 0), 255);  // FAST_t clamps the threshold
    FA.min_th = std::min(std::max(min_th, 0), 255);
    for (int l = 0; l < L; l++) {
        const int rows = P->rows[l], cols = P->cols[l];
        OSG_REQUIRE(ctx, P->data[l] && rows > 0 && cols > 0 && P->step[l] >= cols, "level %d", l);
        LevelGeom &g = lg[l];
        g.minBX = EDGE_THRESHOLD - 3;
        g.minBY = g.minBX;
        g.maxBX = cols - EDGE_THRESHOLD + 3;
        g.maxBY = rows - EDGE_THRESHOLD + 3;
        const float width = (g.maxBX - g.minBX), height = (g.maxBY - g.minBY);
        const int nCols = (int)(width / CELL_W), nRows = (int)(height / CELL_W);
        OSG_REQUIRE(ctx, nCols >= 1 && nRows >= 1 && (int)std::round(width / height) >= 1,
                    "level %d (%d x %d) is too small for one %g px cell", l, cols, rows, (double)CELL_W);
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        g.cell0 = (int)cells.size();
        for (int i = 0; i < nRows; i++) {
            const float iniY = g.minBY + i * hCell;
            float maxY = iniY + hCell + 6;
            if (iniY >= g.maxBY - 3) continue;
            if (maxY > g.maxBY) maxY = g.maxBY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = g.minBX + j * wCell;
                float maxX = iniX + wCell + 6;
                if (iniX >= g.maxBX - 6) continue;
                if (maxX > g.maxBX) maxX = g.maxBX;
                cells.push_back(Cell{l, (int)iniY, (int)maxY, (int)iniX, (int)maxX, j * wCell, i * hCell, 0});
            }
        }
        g.cell1 = (int)cells.size();
        FA.rows[l] = rows;
        FA.cols[l] = cols;
    }
    const int nc = (int)cells.size();
    // device: packed inputs (host levels row-contiguous, cells), score planes, counts, keys
    osg_packer pk;
    std::vector<std::vector<uint8_t>> keep;
    std::vector<size_t> img_off(L, SIZE_MAX);
    for (int l = 0; l < L; l++) {
        if (P->on_device) {
            FA.img[l] = (GLOBAL const uint8_t *)P->data[l];
            FA.step[l] = P->step[l];
            continue;
        }
        FA.step[l] = P->cols[l];
        if (P->step[l] == P->cols[l]) {
            img_off[l] = pk.add(P->data[l], (size_t)P->rows[l] * P->cols[l]);
        } else {
            keep.emplace_back((size_t)P->rows[l] * P->cols[l]);
            for (int r = 0; r < P->rows[l]; r++)
                std::memcpy(&keep.back()[(size_t)r * P->cols[l]], P->data[l] + (size_t)r * P->step[l], P->cols[l]);
            img_off[l] = pk.add(keep.back().data(), keep.back().size());
        }
    }
    size_t score_bytes = 0;  // one image's score planes
    std::vector<size_t> score_off(L);
    for (int l = 0; l < L; l++) {
        score_off[l] = score_bytes;
        score_bytes += ((size_t)P->rows[l] * P->cols[l] * 2 + 255) & ~size_t(255);
    }
    // slots per cell: a kept pixel is a strict maximum of its 8 neighbours, so no two kept pixels are
    // adjacent and an h x w cell holds at most ceil(h / 2) ceil(w / 2) of them (a quarter of the tested
    // pixels, where one slot per pixel sized a 64-image batch's staging at ~2.4 GB: ADVICE r04)
    size_t max_keys = 0;
    for (Cell &c : cells) {
        const int h = std::max(0, c.r1 - c.r0 - 6), w = std::max(0, c.c1 - c.c0 - 6);
        OSG_REQUIRE(ctx, h + 2 <= MAX_T && w + 2 <= MAX_T, "cell of %d x %d tested pixels", h, w);
        c.slot = (int)max_keys;
        max_keys += (size_t)((h + 1) / 2) * (size_t)((w + 1) / 2);
    }
    max_keys = (max_keys + 15) & ~size_t(15);
    OSG_REQUIRE(ctx, (size_t)B * max_keys < (size_t(1) << 31), "batch too large");
    const size_t cell_off = pk.add(cells.data(), sizeof(Cell) * cells.size());
    char *din = nullptr, *dsc = nullptr, *dcnt = nullptr, *dkeys = nullptr;
    OSG_ALLOC(ctx, din, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dsc, SLOT_TMP1, score_bytes * B + 256);
    OSG_ALLOC(ctx, dcnt, SLOT_TMP2, sizeof(int32_t) * ((size_t)nc * B + B + 64));
    OSG_ALLOC(ctx, dkeys, SLOT_TMP3, sizeof(float4) * (2 * max_keys * B + 2));
    for (int l = 0; l < L; l++) {
        if (!P->on_device) FA.img[l] = (GLOBAL const uint8_t *)(din + img_off[l]);
        FA.score[l] = (GLOBAL uint8_t *)(dsc + score_off[l]);
    }
    FA.img_bstride = pyr_bstride;
    FA.score_bstride = (long long)score_bytes;
    CellArgs CA{};
    CA.cells = (const Cell *)(din + cell_off);
    CA.n_cells = nc;
    for (int l = 0; l < L; l++) {
        CA.score[l] = FA.score[l];
        CA.cols[l] = P->cols[l];
    }
    CA.score_bstride = (long long)score_bytes;
    CA.max_keys = (int)max_keys;
    CA.count = (GLOBAL int32_t *)dcnt;
    CA.slots = (float4 *)dkeys;
    CA.keys = (float4 *)dkeys + max_keys * B;
    GLOBAL int32_t *d_total = (GLOBAL int32_t *)(dcnt + sizeof(int32_t) * ((size_t)nc * B + 32));
    CA.total = d_total;
    // flattened score grid: the levels' 64 x 4 pixel blocks one after another
    FA.n_levels = L;
    FA.block0[0] = 0;
    for (int l = 0; l < L; l++) {
        FA.bx[l] = (P->cols[l] + 63) / 64;
        FA.block0[l + 1] = FA.block0[l] + FA.bx[l] * ((P->rows[l] + 3) / 4);
    }
    // pinned: inputs, then the totals and counts, then the keys
    const size_t in_pad = (pk.total + 255) & ~size_t(255);
    const size_t cnt_pad = (sizeof(int32_t) * ((size_t)nc * B + B) + 255) & ~size_t(255);
    // (a batch's keys get their own staging request once the totals are known: max_keys is a quarter of
    // an image's tested pixels, ~25x the keypoints)
    const size_t keys_pin = B == 1 ? sizeof(float4) * (max_keys + 1) : 0;
    char *pin = (char *)osg_pinned(ctx, in_pad + cnt_pad + keys_pin + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    pk.fill_parallel(pin, 8);
    int32_t *pin_tot = (int32_t *)(pin + in_pad);                 // B totals
    int32_t *pin_cnt = pin_tot + B;                                // B x nc counts
    char *pin_keys = pin + in_pad + cnt_pad;                       // image b's keys at kbase[b]
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(din, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_fast_score, dim3(FA.block0[L], B), dim3(256), 0, ctx->stream, FA);
    if (nc > 0) {
        hipLaunchKernelGGL(k_fast_cells, dim3(nc, B), dim3(256), 0, ctx->stream, CA);
        hipLaunchKernelGGL(k_cell_gather, dim3(nc, B), dim3(256), 0, ctx->stream, CA);
        if (B > 1) hipLaunchKernelGGL(k_keys_compact, dim3(32, B), dim3(256), 0, ctx->stream, CA.keys, CA.max_keys, CA.total,
                                      CA.slots);
    }
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    std::vector<int32_t> tot(B, 0), cnt_copy;
    std::vector<size_t> kbase(B + 1, 0);
    const int32_t *cnt_src = pin_cnt;
    if (nc > 0) {
        OSG_RC(osg_download(ctx, pin_tot, (const void *)d_total, sizeof(int32_t) * B));
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(pin_cnt, dcnt, sizeof(int32_t) * (size_t)nc * B, hipMemcpyDeviceToHost,
                                          ctx->stream));
        OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));  // (a polled wait measured slower here)
        for (int b = 0; b < B; b++) {
            tot[b] = pin_tot[b];
            kbase[b + 1] = kbase[b] + (size_t)tot[b];
        }
        if (B > 1) {  // the counts leave the staging block, which the keys may now reuse (stream idle)
            cnt_copy.assign(pin_cnt, pin_cnt + (size_t)nc * B);
            cnt_src = cnt_copy.data();
            pin_keys = (char *)osg_pinned(ctx, sizeof(float4) * (kbase[B] + 1) + 256);
            if (!pin_keys) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
        }
        if (B > 1) {  // compacted on the device (k_keys_compact): one copy
            if (kbase[B] > 0)
                OSG_HIP_CHECK(ctx, hipMemcpyAsync(pin_keys, CA.slots, sizeof(float4) * kbase[B], hipMemcpyDeviceToHost,
                                                  ctx->stream));
        } else if (tot[0] > 0) {
            OSG_HIP_CHECK(ctx, hipMemcpyAsync(pin_keys, CA.keys, sizeof(float4) * (size_t)tot[0], hipMemcpyDeviceToHost,
                                              ctx->stream));
        }
    }
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));  // (a polled wait measured slower here)
    const double t_gpu = ms_since(tp0);
    const auto tp1 = std::chrono::steady_clock::now();
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    // the keypoints leave the pinned staging block once: the tree walk reads each of them several
    // times, from ordinary cached memory
    thread_local std::vector<Key4> hkeys;
    thread_local std::vector<int32_t> hoffs;
    size_t ntot = 0;
    for (int b = 0; b < B; b++) ntot += (size_t)tot[b];
    hkeys.resize(ntot + 1);
    hoffs.assign((size_t)B * (nc + 1), 0);
    if (ntot > 0) {  // a batch's keys (~10 MB) in 1 MiB pieces on the worker pool
        const size_t bytes = sizeof(Key4) * ntot, piece = size_t(1) << 20;
        char *dst = (char *)hkeys.data();
        osg_parallel_for((int)((bytes + piece - 1) / piece), B > 1 ? 16 : 1, [&](int p) {
            const size_t lo = (size_t)p * piece;
            std::memcpy(dst + lo, pin_keys + lo, std::min(piece, bytes - lo));
        });
    }
    for (int b = 0; b < B; b++) {
        int32_t *o = hoffs.data() + (size_t)b * (nc + 1);
        for (int c = 0; c < nc; c++) o[c + 1] = o[c] + cnt_src[(size_t)b * nc + c];  // counts -> offsets
    }
    const double t_copy = ms_since(tp1);
    // DistributeOctTree per (image, level) over that level's cells' keypoints (:1180-1196).  The tasks
    // are independent: a batch spreads them over host threads; one image keeps its ~12k FAST keypoints
    // on the calling thread unless the frame is very large (contiguous level ranges of about equal
    // keypoint counts; a thread started per call pays its tree buffers' page faults)
    std::vector<std::vector<Key4>> kept((size_t)B * L);
    // the calling thread's buffers by pointer: inside a lambda run on a worker thread the names
    // hkeys / hoffs would denote that worker's own (empty) thread_local instances
    const Key4 *keys_all = hkeys.data();
    const int32_t *offs_all = hoffs.data();
    auto run_task = [&](int task) {
        const int b = task / L, l = task % L;
        const LevelGeom &g = lg[l];
        const int32_t *o = offs_all + (size_t)b * (nc + 1);
        const int k0 = o[g.cell0], k1 = o[g.cell1];
        distribute_oct_tree(keys_all + kbase[b] + k0, k1 - k0, g.minBX, g.maxBX, g.minBY, g.maxBY, n_features[l],
                            kept[task]);
    };
    if (B > 1) {
        osg_parallel_for(B * L, 16, run_task);
    } else {
        const int total = tot[0];
        const int32_t *offs = hoffs.data();
        auto run_levels = [&](int l0, int l1) {
            for (int l = l0; l < l1; l++) run_task(l);
        };
        const int nthr = total > 60000 ? std::min(L, 3) : 1;
        if (nthr <= 1) {
            run_levels(0, L);
        } else {
            std::vector<int> cut(nthr + 1, L);
            cut[0] = 0;
            for (int t = 1, l = 0; t < nthr; t++) {  // level ranges of ~total / nthr keypoints
                while (l < L && offs[lg[l].cell1] < (int64_t)total * t / nthr) l++;
                cut[t] = std::max(cut[t - 1] + 1, std::min(l + 1, L - (nthr - t)));
            }
            std::vector<std::thread> th;
            for (int t = 1; t < nthr; t++) th.emplace_back(run_levels, cut[t], cut[t + 1]);
            run_levels(cut[0], cut[1]);
            for (auto &x : th) x.join();
        }
    }
    int n_all = 0;
    for (int b = 0; b < B; b++) {
        int n_out = 0;
        int32_t *ls = level_start + (size_t)b * (L + 1);
        const size_t o = (size_t)b * cap;
        ls[0] = 0;
        for (int l = 0; l < L; l++) {
            const LevelGeom &g = lg[l];
            const std::vector<Key4> &kl = kept[(size_t)b * L + l];
            const int scaledPatchSize = (int)(PATCH_SIZE * scale_factors[l]);
            if (n_out + (int)kl.size() > cap)
                return osg_set_error(ctx, OSG_E_INVALID, "keypoint capacity %d exceeded at level %d (image %d)", cap, l, b);
            for (const Key4 &k : kl) {
                x[o + n_out] = k.x + g.minBX;
                y[o + n_out] = k.y + g.minBY;
                response[o + n_out] = k.z;
                size[o + n_out] = (float)scaledPatchSize;
                n_out++;
            }
            ls[l + 1] = n_out;
        }
        n_all += n_out;
    }
    if (prof)
        fprintf(stderr, "[osg orb detect] %d images x %d cells, %zu FAST keypoints -> %d: setup + GPU + download %.3f ms "
                        "(kernels %.3f ms), key copy %.3f ms, octree %.3f ms\n", B, nc, ntot, n_all, t_gpu, (double)ms, t_copy,
                ms_since(tp1) - t_copy);
    return n_all;
}

}  // namespace

extern "C" int osg_debug_distribute_oct_tree(const float *keys4, int32_t nk, int32_t minX, int32_t maxX, int32_t minY,
                                             int32_t maxY, int32_t N, float *out4, int32_t cap)
{  // diagnostics: the host octree alone on (x, y, response, 0) keypoints (timing, no GPU needed)
    if (!keys4 || !out4 || nk < 0 || maxY <= minY || maxX <= minX) return OSG_E_INVALID;
    thread_local std::vector<Key4> kept;
    distribute_oct_tree((const Key4 *)keys4, nk, minX, maxX, minY, maxY, N, kept);
    if ((int)kept.size() > cap) return OSG_E_INVALID;
    std::memcpy(out4, kept.data(), sizeof(Key4) * kept.size());
    return (int)kept.size();
}

// internal (orb.hip's batched extractor): B device pyramids pyr_bstride bytes apart
int osg_detect_batch(osg_ctx *ctx, const osg_image_pyramid *raw0, int32_t B, int64_t pyr_bstride, int32_t ini_th_fast,
                     int32_t min_th_fast, const int32_t *n_features_per_level, const float *scale_factors,
                     int32_t capacity, float *x, float *y, float *response, float *size, int32_t *level_start)
{
    return detect_run(ctx, raw0, ini_th_fast, min_th_fast, n_features_per_level, scale_factors, capacity, x, y,
                      response, size, level_start, B, pyr_bstride);
}

extern "C" int osg_orb_detect(osg_ctx *ctx, const osg_image_pyramid *raw, int32_t ini_th_fast, int32_t min_th_fast,
                              const int32_t *n_features_per_level, const float *scale_factors, int32_t capacity,
                              float *x, float *y, float *response, float *size, int32_t *level_start)
{
    return detect_run(ctx, raw, ini_th_fast, min_th_fast, n_features_per_level, scale_factors, capacity, x, y,
                      response, size, level_start);
}
