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
//   k_fast_cells   one workgroup per cell: the strict 3x3 maximum at iniThFAST inside the cell's
//                  tested range, the minThFAST pass when it keeps nothing; pass 0 counts, pass 1
//                  writes the keypoints in the cell's row-major order at the cell's offset
//   k_cell_scan    exclusive scan of the cell counts (cells in the reference's level / row / column
//                  order, so the keypoints come out in vToDistributeKeys order)
// DistributeOctTree is a short sequential tree walk per level (a few thousand keypoints): it runs
// on the host over the downloaded keypoints, with the reference's node-list order (push_front,
// erase by the stored position) and its std::sort of (size, UL.x) for the final expansions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int MAX_LEVELS = 32;
constexpr int EDGE_THRESHOLD = 19;
constexpr int PATCH_SIZE = 31;
constexpr float CELL_W = 35.f;

struct FastArgs {
    GLOBAL const uint8_t *img[MAX_LEVELS];
    GLOBAL uint8_t *score[MAX_LEVELS];  // per pixel: (score at min_th, score at ini_th)
    int rows[MAX_LEVELS], cols[MAX_LEVELS], step[MAX_LEVELS];
    int ini_th, min_th;
};

struct Cell {
    int level, r0, r1, c0, c1;  // the cell image: rows r0 .. r1 - 1, columns c0 .. c1 - 1 of the level
    int dx, dy;                 // (j wCell, i hCell): the shift :1168-1169 adds
};

struct CellArgs {
    const Cell *cells;
    int n_cells;
    GLOBAL uint8_t *score[MAX_LEVELS];
    int cols[MAX_LEVELS];
    GLOBAL int32_t *count;        // per cell (pass 0), then the exclusive scan (k_cell_scan)
    float4 *keys;                 // (x, y, response, 0) in cell order (pass 1)
};

// 9 contiguous set bits in a circular 16-bit mask
__device__ __forceinline__ bool arc9(uint32_t m)
{
    uint32_t r = m | (m << 16);  // rotate by doubling
    uint32_t a = r;
#pragma unroll
    for (int k = 1; k < 9; k++) a &= r >> k;
    return (a & 0xffffu) != 0;
}

// cornerScore<16> (OpenCV fast_score.cpp), d[k] = v - circle[k], k < 25 (circle index k mod 16)
__device__ __forceinline__ int corner_score(const int (&d)[16], int threshold)
{
#define D(k) d[(k) & 15]
    int a0 = threshold;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int a = min(D(k + 1), D(k + 2));
        a = min(a, D(k + 3));
        if (a <= a0) continue;
        a = min(a, D(k + 4));
        a = min(a, D(k + 5));
        a = min(a, D(k + 6));
        a = min(a, D(k + 7));
        a = min(a, D(k + 8));
        a0 = max(a0, min(a, D(k)));
        a0 = max(a0, min(a, D(k + 9)));
    }
    int b0 = -a0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int b = max(D(k + 1), D(k + 2));
        b = max(b, D(k + 3));
        b = max(b, D(k + 4));
        b = max(b, D(k + 5));
        if (b >= b0) continue;
        b = max(b, D(k + 6));
        b = max(b, D(k + 7));
        b = max(b, D(k + 8));
        b0 = min(b0, max(b, D(k)));
        b0 = min(b0, max(b, D(k + 9)));
    }
#undef D
    return -b0 - 1;
}

// FAST_t<16>'s test at one threshold: a 9-of-16 arc strictly darker than v - t or brighter than v + t
__device__ __forceinline__ int fast_at(const int (&d)[16], int t)
{
    uint32_t dark = 0, bright = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        dark |= (uint32_t)(d[k] > t) << k;     // circle < v - t
        bright |= (uint32_t)(d[k] < -t) << k;  // circle > v + t
    }
    return (arc9(dark) || arc9(bright)) ? corner_score(d, t) : 0;
}

// grid (ceil(max cols / 64), ceil(max rows / 4), levels), 64 x 4 threads: one pixel each
__global__ __launch_bounds__(256) void k_fast_score(const FastArgs A)
{
    const int l = blockIdx.z;
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int rows = A.rows[l], cols = A.cols[l];
    if (x >= cols || y >= rows) return;
    uint8_t s_lo = 0, s_hi = 0;
    if (x >= 3 && y >= 3 && x < cols - 3 && y < rows - 3) {
        const int step = A.step[l];
        GLOBAL const uint8_t *p = A.img[l] + (size_t)y * step + x;
        // the circle (x, y) offsets of OpenCV's offsets16, in order
        const int ox[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
        const int oy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
        const int v = p[0];
        int d[16];
#pragma unroll
        for (int k = 0; k < 16; k++) d[k] = v - (int)p[ox[k] + oy[k] * step];
        s_lo = (uint8_t)fast_at(d, A.min_th);
        s_hi = (uint8_t)fast_at(d, A.ini_th);
    }
    GLOBAL uint8_t *o = A.score[l] + 2 * ((size_t)y * cols + x);
    *(GLOBAL uint16_t *)o = (uint16_t)(s_lo | (s_hi << 8));
}

// one 256-thread workgroup per cell; PASS 0: count (the ini_th pass, else the min_th pass), PASS 1:
// write the keypoints at the scanned offset in row-major order
template <int PASS>
__global__ __launch_bounds__(256) void k_fast_cells(const CellArgs A)
{
    const int c = blockIdx.x;
    if (c >= A.n_cells) return;
    const Cell C = A.cells[c];
    const int h = C.r1 - C.r0 - 6, w = C.c1 - C.c0 - 6;  // tested rows / columns of the cell image
    const int cols = A.cols[C.level];
    GLOBAL const uint8_t *S = A.score[C.level];
    __shared__ int s_cnt[4];
    __shared__ int s_total;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int n = (h > 0 && w > 0) ? h * w : 0;
    auto keep_at = [&](int idx, int sel, int &s) -> bool {
        const int rr = idx / w, cc = idx - rr * w;
        const int y = C.r0 + 3 + rr, x = C.c0 + 3 + cc;
        s = S[2 * ((size_t)y * cols + x) + sel];
        if (!s) return false;
#pragma unroll
        for (int dy = -1; dy <= 1; dy++)
#pragma unroll
            for (int dx = -1; dx <= 1; dx++) {
                if (!dy && !dx) continue;
                const int r2 = rr + dy, c2 = cc + dx;
                const int t = (r2 >= 0 && r2 < h && c2 >= 0 && c2 < w) ? S[2 * ((size_t)(y + dy) * cols + x + dx) + sel] : 0;
                if (!(s > t)) return false;
            }
        return true;
    };
    auto count_pass = [&](int sel) -> int {
        int k = 0;
        for (int i = threadIdx.x; i < n; i += 256) {
            int s;
            k += keep_at(i, sel, s) ? 1 : 0;
        }
        for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o);
        if (lane == 0) s_cnt[wv] = k;
        __syncthreads();
        const int t = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        __syncthreads();
        return t;
    };
    int sel = 1;  // iniThFAST
    int total = count_pass(1);
    if (total == 0) {  // :1146-1155
        sel = 0;
        total = count_pass(0);
    }
    if (PASS == 0) {
        if (threadIdx.x == 0) A.count[c] = total;
        return;
    }
    if (total == 0) return;
    // ordered compaction, 256 pixels per round: wave ballots, then the 4 wave counts
    if (threadIdx.x == 0) s_total = A.count[c];  // this cell's offset (scanned)
    __syncthreads();
    for (int base = 0; base < n; base += 256) {
        const int i = base + threadIdx.x;
        int s = 0;
        const bool k = i < n && keep_at(i, sel, s);
        const unsigned long long m = __ballot(k);
        if (lane == 0) s_cnt[wv] = __popcll(m);
        __syncthreads();
        int off = s_total;
        for (int q = 0; q < wv; q++) off += s_cnt[q];
        off += __popcll(m & ((1ull << lane) - 1));
        if (k) {
            const int rr = i / w, cc = i - rr * w;
            A.keys[off] = make_float4((float)(cc + 3 + C.dx), (float)(rr + 3 + C.dy), (float)s, 0.f);
        }
        __syncthreads();
        if (threadIdx.x == 0) s_total += s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        __syncthreads();
    }
}

// exclusive scan of the cell counts in place (one workgroup); out_total[0] = the sum
__global__ __launch_bounds__(1024) void k_cell_scan(GLOBAL int32_t *count, int n, GLOBAL int32_t *out_total)
{
    __shared__ int s[1024];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 1024) {
        const int i = base + threadIdx.x;
        const int v = i < n ? count[i] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const int t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < n) count[i] = carry + s[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += s[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) out_total[0] = carry;
}

// ---- DistributeOctTree (ref:src/ORBextractor.cc:716-1050) on the host ------------------------------
// Nodes live in a pool and form a doubly linked list in the reference's list order; a node's
// keypoints are a range of an index pool (DivideNode copies them to its children in order).
struct OctNode {
    int ulx, uly, urx, ury, blx, bly, brx, bry;
    int kbeg, kcnt;
    bool no_more;
    int prev, next;
};

struct OctTree {
    const float4 *keys;
    std::vector<OctNode> nodes;
    std::vector<int> kidx;
    int head = -1, size = 0;

    int new_node()
    {
        nodes.push_back(OctNode{});
        OctNode &n = nodes.back();
        n.prev = n.next = -1;
        n.no_more = false;
        return (int)nodes.size() - 1;
    }
    void push_front(int id)
    {
        nodes[id].prev = -1;
        nodes[id].next = head;
        if (head >= 0) nodes[head].prev = id;
        head = id;
        size++;
    }
    void push_back_after(int tail, int id)
    {
        nodes[id].prev = tail;
        nodes[id].next = -1;
        if (tail >= 0) nodes[tail].next = id;
        else head = id;
        size++;
    }
    int erase(int id)  // returns the next node
    {
        const int p = nodes[id].prev, n = nodes[id].next;
        if (p >= 0) nodes[p].next = n;
        else head = n;
        if (n >= 0) nodes[n].prev = p;
        size--;
        return n;
    }
    // ExtractorNode::DivideNode (:607-654): the four children's geometry and keypoints (in the
    // parent's order), pushed to the list front as the caller does (n1, n2, n3, n4, non-empty
    // only); children with > 1 keypoint are appended to `expand`
    void divide(int id, std::vector<std::pair<int, int>> &expand, int *n_expand)
    {
        const OctNode P = nodes[id];
        const int halfX = (int)std::ceil(static_cast<float>(P.urx - P.ulx) / 2);
        const int halfY = (int)std::ceil(static_cast<float>(P.bry - P.uly) / 2);
        int ch[4];
        for (int q = 0; q < 4; q++) ch[q] = new_node();
        OctNode *c = &nodes[0];
        OctNode &n1 = c[ch[0]], &n2 = c[ch[1]], &n3 = c[ch[2]], &n4 = c[ch[3]];
        n1.ulx = P.ulx, n1.uly = P.uly, n1.urx = P.ulx + halfX, n1.ury = P.uly;
        n1.blx = P.ulx, n1.bly = P.uly + halfY, n1.brx = P.ulx + halfX, n1.bry = P.uly + halfY;
        n2.ulx = n1.urx, n2.uly = n1.ury, n2.urx = P.urx, n2.ury = P.ury;
        n2.blx = n1.brx, n2.bly = n1.bry, n2.brx = P.urx, n2.bry = P.uly + halfY;
        n3.ulx = n1.blx, n3.uly = n1.bly, n3.urx = n1.brx, n3.ury = n1.bry;
        n3.blx = P.blx, n3.bly = P.bly, n3.brx = n1.brx, n3.bry = P.bly;
        n4.ulx = n3.urx, n4.uly = n3.ury, n4.urx = n2.brx, n4.ury = n2.bry;
        n4.blx = n3.brx, n4.bly = n3.bry, n4.brx = P.brx, n4.bry = P.bry;
        // classify into four runs of the index pool, each in the parent's order
        int cnt[4] = {0, 0, 0, 0};
        std::vector<uint8_t> q(P.kcnt);
        for (int k = 0; k < P.kcnt; k++) {
            const float4 kp = keys[kidx[P.kbeg + k]];
            const int qq = (kp.x < n1.urx) ? ((kp.y < n1.bry) ? 0 : 2) : ((kp.y < n1.bry) ? 1 : 3);
            q[k] = (uint8_t)qq;
            cnt[qq]++;
        }
        int beg[4];
        beg[0] = (int)kidx.size();
        for (int t = 1; t < 4; t++) beg[t] = beg[t - 1] + cnt[t - 1];
        kidx.resize(kidx.size() + P.kcnt);
        int fill[4] = {beg[0], beg[1], beg[2], beg[3]};
        for (int k = 0; k < P.kcnt; k++) kidx[fill[q[k]]++] = kidx[P.kbeg + k];
        for (int t = 0; t < 4; t++) {
            OctNode &n = nodes[ch[t]];
            n.kbeg = beg[t];
            n.kcnt = cnt[t];
            n.no_more = cnt[t] == 1;
            if (cnt[t] > 0) {
                push_front(ch[t]);
                if (cnt[t] > 1) {
                    if (n_expand) (*n_expand)++;
                    expand.push_back(std::make_pair(cnt[t], ch[t]));
                }
            }
        }
    }
};

// keys[0 .. nk) in vToDistributeKeys order (relative to (minX, minY)); out: the kept keypoints
void distribute_oct_tree(const float4 *keys, int nk, int minX, int maxX, int minY, int maxY, int N,
                         std::vector<float4> &out)
{
    out.clear();
    OctTree T;
    T.keys = keys;
    T.nodes.reserve(4 * (size_t)nk + 64);
    T.kidx.reserve(8 * (size_t)nk + 64);
    const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
    const float hX = static_cast<float>(maxX - minX) / nIni;
    std::vector<int> ini(nIni);
    int tail = -1;
    for (int i = 0; i < nIni; i++) {
        const int id = T.new_node();
        OctNode &n = T.nodes[id];
        n.ulx = (int)(hX * static_cast<float>(i));
        n.uly = 0;
        n.urx = (int)(hX * static_cast<float>(i + 1));
        n.ury = 0;
        n.blx = n.ulx;
        n.bly = maxY - minY;
        n.brx = n.urx;
        n.bry = maxY - minY;
        T.push_back_after(tail, id);
        tail = id;
        ini[i] = id;
    }
    // keypoints to the initial nodes (:739-745), in order
    std::vector<int> cnt(nIni, 0), which(nk);
    for (int k = 0; k < nk; k++) {
        which[k] = (int)(keys[k].x / hX);
        cnt[which[k]]++;
    }
    int off = 0;
    for (int i = 0; i < nIni; i++) {
        T.nodes[ini[i]].kbeg = off;
        T.nodes[ini[i]].kcnt = 0;
        off += cnt[i];
    }
    T.kidx.resize(nk);
    for (int k = 0; k < nk; k++) {
        OctNode &n = T.nodes[ini[which[k]]];
        T.kidx[n.kbeg + n.kcnt++] = k;
    }
    for (int id = T.head; id >= 0;) {
        OctNode &n = T.nodes[id];
        if (n.kcnt == 1) {
            n.no_more = true;
            id = n.next;
        } else if (n.kcnt == 0)
            id = T.erase(id);
        else
            id = n.next;
    }
    bool finish = false;
    std::vector<std::pair<int, int>> expand, prev;
    auto cmp = [&](const std::pair<int, int> &a, const std::pair<int, int> &b) {  // compareNodes (:656-676)
        if (a.first < b.first) return true;
        if (a.first > b.first) return false;
        return T.nodes[a.second].ulx < T.nodes[b.second].ulx;
    };
    while (!finish) {
        const int prevSize = T.size;
        int nToExpand = 0;
        expand.clear();
        for (int id = T.head; id >= 0;) {
            if (T.nodes[id].no_more) {
                id = T.nodes[id].next;
                continue;
            }
            T.divide(id, expand, &nToExpand);
            id = T.erase(id);
        }
        if (T.size >= N || T.size == prevSize) {
            finish = true;
        } else if (T.size + nToExpand * 3 > N) {
            while (!finish) {
                const int prevSize2 = T.size;
                prev = expand;
                expand.clear();
                std::sort(prev.begin(), prev.end(), cmp);
                for (int j = (int)prev.size() - 1; j >= 0; j--) {
                    T.divide(prev[j].second, expand, nullptr);
                    T.erase(prev[j].second);
                    if (T.size >= N) break;
                }
                if (T.size >= N || T.size == prevSize2) finish = true;
            }
        }
    }
    // the strongest keypoint of every node, first maximum, in list order (:1033-1048)
    for (int id = T.head; id >= 0; id = T.nodes[id].next) {
        const OctNode &n = T.nodes[id];
        int best = T.kidx[n.kbeg];
        float r = keys[best].z;
        for (int k = 1; k < n.kcnt; k++) {
            const int kk = T.kidx[n.kbeg + k];
            if (keys[kk].z > r) {
                best = kk;
                r = keys[kk].z;
            }
        }
        out.push_back(keys[best]);
    }
}

struct LevelGeom {
    int minBX, minBY, maxBX, maxBY, cell0, cell1;
};

int detect_run(osg_ctx *ctx, const osg_image_pyramid *P, int ini_th, int min_th, const int32_t *n_features,
               const float *scale_factors, int cap, float *x, float *y, float *response, float *size,
               int32_t *level_start)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, P && P->n_levels >= 1 && P->n_levels <= MAX_LEVELS && P->data && P->rows && P->cols && P->step,
                "pyramid (1 .. %d levels)", MAX_LEVELS);
    OSG_REQUIRE(ctx, n_features && scale_factors && level_start && (cap == 0 || (x && y && response && size)),
                "null argument");
    const int L = P->n_levels;
    // cells in the reference's order (:1071-1175); geometry per level
    std::vector<Cell> cells;
    std::vector<LevelGeom> lg(L);
    FastArgs FA{};
    FA.ini_th = std::min(std::max(ini_th, 0), 255);  // FAST_t clamps the threshold
    FA.min_th = std::min(std::max(min_th, 0), 255);
    int max_rows = 0, max_cols = 0;
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
                cells.push_back(Cell{l, (int)iniY, (int)maxY, (int)iniX, (int)maxX, j * wCell, i * hCell});
            }
        }
        g.cell1 = (int)cells.size();
        FA.rows[l] = rows;
        FA.cols[l] = cols;
        max_rows = std::max(max_rows, rows);
        max_cols = std::max(max_cols, cols);
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
    const size_t cell_off = pk.add(cells.data(), sizeof(Cell) * cells.size());
    size_t score_bytes = 0;
    std::vector<size_t> score_off(L);
    for (int l = 0; l < L; l++) {
        score_off[l] = score_bytes;
        score_bytes += ((size_t)P->rows[l] * P->cols[l] * 2 + 255) & ~size_t(255);
    }
    size_t max_keys = 0;  // bound: the tested pixels of every cell
    for (const Cell &c : cells) max_keys += (size_t)std::max(0, c.r1 - c.r0 - 6) * std::max(0, c.c1 - c.c0 - 6);
    char *din = nullptr, *dsc = nullptr, *dcnt = nullptr, *dkeys = nullptr;
    OSG_ALLOC(ctx, din, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dsc, SLOT_TMP1, score_bytes + 256);
    OSG_ALLOC(ctx, dcnt, SLOT_TMP2, sizeof(int32_t) * (nc + 64));
    OSG_ALLOC(ctx, dkeys, SLOT_TMP3, sizeof(float4) * (max_keys + 1));
    for (int l = 0; l < L; l++) {
        if (!P->on_device) FA.img[l] = (GLOBAL const uint8_t *)(din + img_off[l]);
        FA.score[l] = (GLOBAL uint8_t *)(dsc + score_off[l]);
    }
    CellArgs CA{};
    CA.cells = (const Cell *)(din + cell_off);
    CA.n_cells = nc;
    for (int l = 0; l < L; l++) {
        CA.score[l] = FA.score[l];
        CA.cols[l] = P->cols[l];
    }
    CA.count = (GLOBAL int32_t *)dcnt;
    CA.keys = (float4 *)dkeys;
    GLOBAL int32_t *d_total = (GLOBAL int32_t *)(dcnt + sizeof(int32_t) * (nc + 32));
    // pinned: inputs, then the total (and later the keys)
    char *pin = (char *)osg_pinned(ctx, pk.total + 256 + sizeof(float4) * (max_keys + 1) + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));  // the pinned block may still be in use
    pk.fill_parallel(pin, 8);
    char *pin_out = pin + ((pk.total + 255) & ~size_t(255));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(din, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_fast_score, dim3((max_cols + 63) / 64, (max_rows + 3) / 4, L), dim3(256), 0, ctx->stream, FA);
    if (nc > 0) {
        hipLaunchKernelGGL(k_fast_cells<0>, dim3(nc), dim3(256), 0, ctx->stream, CA);
        hipLaunchKernelGGL(k_cell_scan, dim3(1), dim3(1024), 0, ctx->stream, CA.count, nc, d_total);
        hipLaunchKernelGGL(k_fast_cells<1>, dim3(nc), dim3(256), 0, ctx->stream, CA);
    }
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    int32_t total = 0;
    std::vector<int32_t> offs(nc + 1, 0);
    if (nc > 0) {
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(pin_out, (const void *)d_total, sizeof(int32_t), hipMemcpyDeviceToHost,
                                          ctx->stream));
        OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
        total = *(int32_t *)pin_out;
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(pin_out, dkeys, sizeof(float4) * (size_t)total, hipMemcpyDeviceToHost,
                                          ctx->stream));
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(offs.data(), dcnt, sizeof(int32_t) * nc, hipMemcpyDeviceToHost, ctx->stream));
    }
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    offs[nc] = total;
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    const float4 *keys = (const float4 *)pin_out;
    // DistributeOctTree per level over that level's cells' keypoints (:1180-1196)
    int n_out = 0;
    level_start[0] = 0;
    std::vector<float4> kept;
    for (int l = 0; l < L; l++) {
        const LevelGeom &g = lg[l];
        const int k0 = offs[g.cell0], k1 = offs[g.cell1];
        distribute_oct_tree(keys + k0, k1 - k0, g.minBX, g.maxBX, g.minBY, g.maxBY, n_features[l], kept);
        const int scaledPatchSize = (int)(PATCH_SIZE * scale_factors[l]);
        if (n_out + (int)kept.size() > cap)
            return osg_set_error(ctx, OSG_E_INVALID, "keypoint capacity %d exceeded at level %d", cap, l);
        for (const float4 &k : kept) {
            x[n_out] = k.x + g.minBX;
            y[n_out] = k.y + g.minBY;
            response[n_out] = k.z;
            size[n_out] = (float)scaledPatchSize;
            n_out++;
        }
        level_start[l + 1] = n_out;
    }
    return n_out;
}

}  // namespace

extern "C" int osg_orb_detect(osg_ctx *ctx, const osg_image_pyramid *raw, int32_t ini_th_fast, int32_t min_th_fast,
                              const int32_t *n_features_per_level, const float *scale_factors, int32_t capacity,
                              float *x, float *y, float *response, float *size, int32_t *level_start)
{
    return detect_run(ctx, raw, ini_th_fast, min_th_fast, n_features_per_level, scale_factors, capacity, x, y,
                      response, size, level_start);
}
