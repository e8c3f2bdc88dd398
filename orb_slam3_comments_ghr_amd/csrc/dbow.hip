// dbow.hip — DBoW2 TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup) on
// gfx950 (ref:Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1256; caller Frame::ComputeBoW,
// ref:src/Frame.cc:995-1010).
//
// Vocabulary layout: the tree is renumbered breadth-first (children in the reference's children
// order, ref:TemplatedVocabulary.h:1334-1415), so the children of a node are consecutive ids and
// their descriptors one contiguous run: a descent step is one dependent load of the node's meta
// {first child, child count, leaf, word} and one batch of child-descriptor loads.
//
//   k_voc_descend   one lane per feature: L levels of "nearest child" (FORB distance, strict '<':
//                   the first child in order wins), the node at level L - levelsup, the word and
//                   its weight                                             (latency / L2-MALL)
//   k_bow_assemble  one workgroup per descriptor set: bitonic sort of (word, feature) and
//                   (node rank, feature) keys in LDS — packed into 32 bits when they fit (ORBvoc:
//                   20 + 11 bits at 2048 features), 64 otherwise — BowVector sums in feature order
//                   (addWeight) or the first weight (addIfNotExist), the reference's normalisation
//                   summed in ascending word order, FeatureVector CSR in feature order
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/osg_dbow.h"
#include "match_common.h"

struct osg_vocabulary {
    osg_ctx *ctx = nullptr;
    int k = 0, L = 0, scoring = 0, weighting = 0, n_nodes = 0, n_words = 0;
    int4 *meta = nullptr;        // per BFS node: {first child, child count, leaf, word}
    uint4 *desc = nullptr;       // per BFS node: 2 x uint4
    double *weight = nullptr;    // per BFS node
    uint32_t *old_id = nullptr;  // per BFS node: the reference's node id
    uint32_t *lvl_rank = nullptr;  // per BFS node: rank of its old id among the nodes of its depth
    int level_count[16] = {};      // nodes per depth
};

namespace {

constexpr int DT = 256;        // descend threads per workgroup
constexpr int AT = 1024;       // assemble threads per workgroup
constexpr int MAX_SET = 8192;  // features per descriptor set (LDS sort)
constexpr int KCH = 10;        // children evaluated per unrolled step (ORBvoc: k = 10)

__device__ __forceinline__ uint32_t bcnt(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

__device__ __forceinline__ uint32_t dist256(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1)
{
    uint32_t d = __popc(a0.x ^ b0.x);
    d = bcnt(a0.y ^ b0.y, d);
    d = bcnt(a0.z ^ b0.z, d);
    d = bcnt(a0.w ^ b0.w, d);
    d = bcnt(a1.x ^ b1.x, d);
    d = bcnt(a1.y ^ b1.y, d);
    d = bcnt(a1.z ^ b1.z, d);
    d = bcnt(a1.w ^ b1.w, d);
    return d;
}

// ref:TemplatedVocabulary.h:1214-1256 for every feature of the batch
__global__ __launch_bounds__(DT) void k_voc_descend(const int4 *__restrict__ meta, const uint4 *__restrict__ vdesc,
                                                    const double *__restrict__ vweight,
                                                    const uint32_t *__restrict__ old_id,
                                                    const uint32_t *__restrict__ lvl_rank,
                                                    const uint4 *__restrict__ feat, int nf, int nid_level,
                                                    int32_t *__restrict__ o_word, double *__restrict__ o_w,
                                                    uint32_t *__restrict__ o_nid, uint32_t *__restrict__ o_nrank)
{
    const int f = blockIdx.x * DT + threadIdx.x;
    if (f >= nf) return;
    const uint4 a0 = feat[2 * f], a1 = feat[2 * f + 1];
    int node = 0, level = 0;
    uint32_t nid = 0, nrank = 0;  // the root when nid_level <= 0 (and if no descent step reaches it)
    int4 m = meta[0];
    while (!m.z) {
        ++level;
        const int cs = m.x, nc = m.y;
        uint32_t best_d = 0xFFFFFFFFu;
        int best = cs;
        for (int c0 = 0; c0 < nc; c0 += KCH) {
            uint4 b[KCH][2];
#pragma unroll
            for (int u = 0; u < KCH; u++) {  // clamped, unconditional: all loads in flight at once
                const int id = cs + min(c0 + u, nc - 1);
                b[u][0] = vdesc[2 * id];
                b[u][1] = vdesc[2 * id + 1];
            }
#pragma unroll
            for (int u = 0; u < KCH; u++) {
                const uint32_t d = dist256(a0, a1, b[u][0], b[u][1]);
                if (c0 + u < nc && d < best_d) {  // strict '<': the first child wins ties
                    best_d = d;
                    best = cs + c0 + u;
                }
            }
        }
        node = best;
        m = meta[node];
        if (level == nid_level) {
            nid = old_id[node];
            nrank = 1 + lvl_rank[node];  // sorts like nid: ranks follow old ids, the root (0) first
        }
    }
    o_word[f] = m.w;
    o_w[f] = vweight[node];
    o_nid[f] = nid;
    o_nrank[f] = nrank;
}

struct SetArgs {
    int first, n;          // feature rows of this set
    int32_t *word;         // out, capacity n
    double *value;
    uint32_t *node_id;
    int32_t *node_start;   // n + 1
    int32_t *feat;
    int32_t *counts;       // [0] n_words, [1] n_nodes
};

// bitonic sort of 64-bit keys in LDS (n2 a power of two, padded with ~0).  Compare-exchange pair i
// (lo, lo + stride) is handled by thread i % AT, so for stride <= 64 every wave touches only its
// own 128-key segments: those stages are ordered by the wave's in-order LDS queue and need no
// workgroup barrier (only a compiler fence).  n2 = 2048 has 10 barrier stages instead of 66.
template <typename K>
__device__ void lds_sort(K *k, int n2)
{
    __syncthreads();
    int prev = 0;
    for (int size = 2; size <= n2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride > 64 || prev > 64) {
                __syncthreads();
            } else {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            prev = stride;
            for (int i = threadIdx.x; i < n2 / 2; i += AT) {
                const int lo = ((i & ~(stride - 1)) << 1) | (i & (stride - 1)), hi = lo + stride;  // stride: 2^k
                const bool up = ((lo & size) == 0);
                const K a = k[lo], b = k[hi];
                if ((a > b) == up) {
                    k[lo] = b;
                    k[hi] = a;
                }
            }
        }
    __syncthreads();
}

// Exclusive prefix count of one flag per thread (thread order) over the workgroup; *total gets the
// count of all flags.  Two barriers; s_wtot holds AT / 64 ints.
__device__ int block_scan_flag(bool f, int *s_wtot, int *total)
{
    const unsigned long long mask = __ballot(f);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int before = __popcll(mask & ((1ull << lane) - 1ull));
    if (lane == 0) s_wtot[w] = __popcll(mask);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < AT / 64; i++) {
        const int c = s_wtot[i];
        off += (i < w) ? c : 0;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return off + before;
}

// BowVector + FeatureVector of one descriptor set, ref:TemplatedVocabulary.h:1126-1192,
// BowVector.cpp:35-85, FeatureVector.cpp:32-46.  Sorting (word, feature) makes every word's
// features one run in feature order, so each run head sums its run sequentially (addWeight: the
// reference's += in feature order; addIfNotExist: the first value) and a flag scan gives the run's
// output slot.  Only the norm — one sum in ascending word order — stays serial, in wave 0.
// K: key type (uint32_t when word / node-rank bits + fbits fit in 31, else 64-bit with fbits 32).
template <typename K>
__device__ void assemble(const SetArgs &S, K *key, double *val, int *s_wtot, int *s_m, double *s_norm,
                         const int32_t *__restrict__ i_word, const double *__restrict__ i_w,
                         const uint32_t *__restrict__ i_nid, const uint32_t *__restrict__ i_nrank, int fbits,
                         bool add, bool must, bool l2, unsigned long long *prof)
{
    constexpr int PER = MAX_SET / AT;
    const K PAD = ~K(0), FMASK = (K(1) << fbits) - 1;
#define STAMP(k)                                                                    \
    if (prof && blockIdx.x == 0 && threadIdx.x == 0) prof[k] = __builtin_amdgcn_s_memtime()
    const int n = S.n;
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    // ---- BowVector: sort (word, feature) of the non-stopped features
    for (int i = threadIdx.x; i < n2; i += AT) {
        K v = PAD;
        if (i < n && i_w[S.first + i] > 0) {
            v = ((K)(uint32_t)i_word[S.first + i] << fbits) | (K)i;
            atomicAdd(s_m, 1);
        }
        key[i] = v;
    }
    STAMP(1);
    lds_sort(key, n2);
    STAMP(2);
    const int m = *s_m;  // valid keys, sorted to the front
    for (int i = threadIdx.x; i < m; i += AT) val[i] = i_w[S.first + (uint32_t)(key[i] & FMASK)];
    __syncthreads();
    STAMP(3);
    double rsum[PER];
    int rslot[PER];
    uint32_t rword[PER];
    int nw = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        rslot[k] = -1;
        if (k * AT >= m) continue;  // uniform
        const int i = k * AT + threadIdx.x;
        const uint32_t w = i < m ? (uint32_t)(key[i] >> fbits) : 0u;
        const bool head = i < m && (i == 0 || (uint32_t)(key[i - 1] >> fbits) != w);
        int tot;
        const int pos = nw + block_scan_flag(head, s_wtot, &tot);
        nw += tot;
        if (head) {
            double acc = val[i];
            for (int j = i + 1; j < m && (uint32_t)(key[j] >> fbits) == w; j++)
                if (add) acc += val[j];
            rsum[k] = acc;
            rslot[k] = pos;
            rword[k] = w;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; k++)
        if (rslot[k] >= 0) {
            val[rslot[k]] = (add && !must) ? rsum[k] / (double)nw : rsum[k];  // DOT_PRODUCT: v / n_words
            key[rslot[k]] = (K)rword[k] << fbits;
        }
    __syncthreads();
    STAMP(4);
    if (must && threadIdx.x < 64) {
        // ascending word order, one add at a time: the wave loads 64 values, then every lane adds
        // them in lane order through readlane (the zero padding past nw adds +0.0 to a
        // non-negative sum: exact)
        const int lane = threadIdx.x;
        double norm = 0.0;
        for (int j0 = 0; j0 < nw; j0 += 64) {
            const int j = j0 + lane;
            double x = j < nw ? val[j] : 0.0;
            x = l2 ? x * x : fabs(x);
            const unsigned long long bits = (unsigned long long)__double_as_longlong(x);
            const int lo = (int)(uint32_t)bits, hi = (int)(uint32_t)(bits >> 32);
#pragma unroll
            for (int u = 0; u < 64; u++) {
                const unsigned long long y = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(hi, u) << 32) |
                                             (uint32_t)__builtin_amdgcn_readlane(lo, u);
                norm += __longlong_as_double((long long)y);
            }
        }
        if (lane == 0) *s_norm = l2 ? sqrt(norm) : norm;
    }
    if (threadIdx.x == 0) S.counts[0] = nw;
    __syncthreads();
    STAMP(5);
    {
        const double norm = must ? *s_norm : 0.0;
        for (int j = threadIdx.x; j < nw; j += AT) {
            S.word[j] = (int32_t)(uint32_t)(key[j] >> fbits);
            S.value[j] = norm > 0.0 ? val[j] / norm : val[j];
        }
    }
    __syncthreads();
    // ---- FeatureVector: sort (node rank, feature); a node's features are one run, pushed in
    // feature order
    for (int i = threadIdx.x; i < n2; i += AT) {
        K v = PAD;
        if (i < n && i_w[S.first + i] > 0) v = ((K)i_nrank[S.first + i] << fbits) | (K)i;
        key[i] = v;
    }
    STAMP(6);
    lds_sort(key, n2);
    STAMP(7);
    int nn = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        if (k * AT >= m) continue;
        const int i = k * AT + threadIdx.x;
        const uint32_t r = i < m ? (uint32_t)(key[i] >> fbits) : 0u;
        const bool head = i < m && (i == 0 || (uint32_t)(key[i - 1] >> fbits) != r);
        int tot;
        const int pos = nn + block_scan_flag(head, s_wtot, &tot);
        nn += tot;
        const int f = i < m ? (int)(uint32_t)(key[i] & FMASK) : 0;
        if (i < m) S.feat[i] = f;
        if (head) {
            S.node_id[pos] = i_nid[S.first + f];
            S.node_start[pos] = i;
        }
    }
    if (threadIdx.x == 0) {
        S.node_start[nn] = m;
        S.counts[1] = nn;
    }
    STAMP(8);
#undef STAMP
}

__global__ __launch_bounds__(AT) void k_bow_assemble(const SetArgs *__restrict__ sets, const int32_t *__restrict__ i_word,
                                                     const double *__restrict__ i_w, const uint32_t *__restrict__ i_nid,
                                                     const uint32_t *__restrict__ i_nrank, int wbits, int rbits,
                                                     int weighting, int scoring, unsigned long long *prof)
{
    // OSG_DBOW_PROFILE: s_memtime per phase of workgroup 0
    if (prof && blockIdx.x == 0 && threadIdx.x == 0) prof[0] = __builtin_amdgcn_s_memtime();
    const SetArgs S = sets[blockIdx.x];
    __shared__ unsigned long long key[MAX_SET];
    __shared__ double val[MAX_SET];
    __shared__ int s_m, s_wtot[AT / 64];
    __shared__ double s_norm;
    const bool add = (weighting == OSG_W_TF || weighting == OSG_W_TF_IDF);
    const bool must = scoring != OSG_S_DOT, l2 = scoring == OSG_S_L2;
    if (threadIdx.x == 0) s_m = 0;
    __syncthreads();
    int fbits = 1;
    while ((1 << fbits) < S.n) fbits++;
    if (max(wbits, rbits) + fbits <= 31)
        assemble<uint32_t>(S, (uint32_t *)key, val, s_wtot, &s_m, &s_norm, i_word, i_w, i_nid, i_nrank, fbits, add,
                           must, l2, prof);
    else
        assemble<unsigned long long>(S, key, val, s_wtot, &s_m, &s_norm, i_word, i_w, i_nid, i_nrank, 32, add, must,
                                     l2, prof);
}

int voc_upload(osg_ctx *ctx, const osg_vocabulary_desc *V, osg_vocabulary **out)
{
    OSG_REQUIRE(ctx, V && out, "null argument");
    const int n = V->n_nodes;
    OSG_REQUIRE(ctx, n >= 1 && V->k >= 1 && V->k <= 32 && V->L >= 1 && V->L <= 10, "vocabulary sizes");
    OSG_REQUIRE(ctx, V->scoring >= 0 && V->scoring <= 5 && V->weighting >= 0 && V->weighting <= 3, "vocabulary types");
    OSG_REQUIRE(ctx, n == 1 || (V->parent && V->is_leaf && V->desc && V->weight), "vocabulary arrays");
    // children in id order (loadFromTextFile appends each node to its parent's children)
    std::vector<int> cstart(n + 1, 0), child(std::max(n - 1, 1));
    for (int i = 1; i < n; i++) {
        OSG_REQUIRE(ctx, V->parent[i] >= 0 && V->parent[i] < i, "node %d: parent %d must precede it", i, V->parent[i]);
        cstart[V->parent[i] + 1]++;
    }
    for (int i = 0; i < n; i++) cstart[i + 1] += cstart[i];
    {
        std::vector<int> fill(cstart.begin(), cstart.end() - 1);
        for (int i = 1; i < n; i++) child[fill[V->parent[i]]++] = i;
    }
    std::vector<int> word(n, -1);
    int nw = 0;
    for (int i = 1; i < n; i++)
        if (V->is_leaf[i]) word[i] = nw++;
    for (int i = 0; i < n; i++) {
        const int nc = cstart[i + 1] - cstart[i];
        OSG_REQUIRE(ctx, (i > 0 && V->is_leaf[i]) ? nc == 0 : true, "leaf %d has children", i);
        OSG_REQUIRE(ctx, (i == 0 || !V->is_leaf[i]) ? (nc > 0 || n == 1) : true,
                    "internal node %d has no children (the descent would read past its child list)", i);
        OSG_REQUIRE(ctx, nc <= 1024, "node %d: %d children", i, nc);
    }
    // breadth-first renumbering: children of a node become consecutive
    std::vector<int> order;  // BFS position -> old id
    order.reserve(n);
    order.push_back(0);
    for (size_t h = 0; h < order.size(); h++) {
        const int o = order[h];
        for (int c = cstart[o]; c < cstart[o + 1]; c++) order.push_back(child[c]);
    }
    OSG_REQUIRE(ctx, (int)order.size() == n, "vocabulary is not a tree rooted at node 0");
    std::vector<int> pos(n);
    for (int p = 0; p < n; p++) pos[order[p]] = p;
    std::vector<int4> meta(n);
    std::vector<uint8_t> desc(32 * (size_t)n, 0);
    std::vector<double> weight(n, 0.0);
    std::vector<uint32_t> old(n), rank(n);
    // depth of every node, and its rank by old id among the nodes of that depth
    std::vector<int> depth(n, 0), per_depth(1, 0);
    for (int p = 1; p < n; p++) depth[order[p]] = depth[V->parent[order[p]]] + 1;
    std::vector<uint32_t> rank_old(n);
    for (int o = 0; o < n; o++) {
        if (depth[o] >= (int)per_depth.size()) per_depth.resize(depth[o] + 1, 0);
        rank_old[o] = (uint32_t)per_depth[depth[o]]++;
    }
    for (int p = 0; p < n; p++) {
        const int o = order[p];
        const int nc = cstart[o + 1] - cstart[o];
        const bool leaf = (o == 0) ? (n == 1) : V->is_leaf[o] != 0;
        meta[p] = make_int4(nc > 0 ? pos[child[cstart[o]]] : 0, nc, leaf ? 1 : 0, word[o]);
        if (o > 0) {
            std::memcpy(&desc[32 * (size_t)p], V->desc + 32 * (size_t)o, 32);
            weight[p] = V->weight[o];
        }
        old[p] = (uint32_t)o;
        rank[p] = rank_old[o];
    }
    osg_vocabulary *voc = new osg_vocabulary();
    voc->ctx = ctx;
    voc->k = V->k;
    voc->L = V->L;
    voc->scoring = V->scoring;
    voc->weighting = V->weighting;
    voc->n_nodes = n;
    voc->n_words = nw;
    for (int d = 0; d < (int)per_depth.size() && d < 16; d++) voc->level_count[d] = per_depth[d];
    bool ok = hipMalloc(&voc->meta, sizeof(int4) * n) == hipSuccess && hipMalloc(&voc->desc, 32 * (size_t)n) == hipSuccess &&
              hipMalloc(&voc->weight, sizeof(double) * n) == hipSuccess && hipMalloc(&voc->old_id, 4 * (size_t)n) == hipSuccess &&
              hipMalloc(&voc->lvl_rank, 4 * (size_t)n) == hipSuccess;
    if (ok)
        ok = hipMemcpy(voc->meta, meta.data(), sizeof(int4) * n, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(voc->desc, desc.data(), 32 * (size_t)n, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(voc->weight, weight.data(), sizeof(double) * n, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(voc->old_id, old.data(), 4 * (size_t)n, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(voc->lvl_rank, rank.data(), 4 * (size_t)n, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) {
        osg_vocabulary_destroy(voc);
        return osg_set_error(ctx, OSG_E_NOMEM, "vocabulary upload failed");
    }
    *out = voc;
    return OSG_OK;
}

}  // namespace

extern "C" {

int osg_vocabulary_create(osg_ctx *ctx, const osg_vocabulary_desc *v, osg_vocabulary **out)
{
    if (!ctx) return OSG_E_INVALID;
    return voc_upload(ctx, v, out);
}

// TemplatedVocabulary::loadFromTextFile (ref:TemplatedVocabulary.h:1334-1415): header
// "k L scoring weighting", then one node per line "parent isLeaf d0 .. d31 weight".  Empty lines are
// skipped (the reference's eof loop turns a trailing empty line into an extra childless root child).
int osg_vocabulary_load_text(osg_ctx *ctx, const char *path, osg_vocabulary **out)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, path && out, "null argument");
    std::ifstream f(path);
    if (!f.is_open()) return osg_set_error(ctx, OSG_E_INVALID, "cannot open %s", path);
    std::string line;
    if (!std::getline(f, line)) return osg_set_error(ctx, OSG_E_INVALID, "%s: empty", path);
    osg_vocabulary_desc V{};
    {
        std::stringstream ss(line);
        ss >> V.k >> V.L >> V.scoring >> V.weighting;
        if (!ss || V.k < 0 || V.k > 20 || V.L < 1 || V.L > 10 || V.scoring < 0 || V.scoring > 5 || V.weighting < 0 ||
            V.weighting > 3)
            return osg_set_error(ctx, OSG_E_INVALID, "%s: not a DBoW2 text vocabulary", path);
    }
    std::vector<int32_t> parent(1, 0);
    std::vector<uint8_t> leaf(1, 0), desc(32, 0);
    std::vector<double> weight(1, 0.0);
    while (std::getline(f, line)) {
        if (line.find_first_not_of(" \t\r") == std::string::npos) continue;
        std::stringstream ss(line);
        int pid, is_leaf;
        ss >> pid >> is_leaf;
        uint8_t d[32];
        for (int i = 0; i < 32; i++) {
            int v;
            ss >> v;
            d[i] = (uint8_t)v;
        }
        double w;
        ss >> w;
        if (!ss) return osg_set_error(ctx, OSG_E_INVALID, "%s: malformed node line %zu", path, parent.size());
        parent.push_back(pid);
        leaf.push_back(is_leaf > 0 ? 1 : 0);
        desc.insert(desc.end(), d, d + 32);
        weight.push_back(w);
    }
    V.n_nodes = (int32_t)parent.size();
    V.parent = parent.data();
    V.is_leaf = leaf.data();
    V.desc = desc.data();
    V.weight = weight.data();
    return voc_upload(ctx, &V, out);
}

int osg_vocabulary_destroy(osg_vocabulary *voc)
{
    if (!voc) return OSG_E_INVALID;
    if (voc->meta) (void)hipFree(voc->meta);
    if (voc->desc) (void)hipFree(voc->desc);
    if (voc->weight) (void)hipFree(voc->weight);
    if (voc->old_id) (void)hipFree(voc->old_id);
    if (voc->lvl_rank) (void)hipFree(voc->lvl_rank);
    delete voc;
    return OSG_OK;
}

int osg_vocabulary_info(const osg_vocabulary *voc, int32_t *out4)
{
    if (!voc || !out4) return OSG_E_INVALID;
    out4[0] = voc->k;
    out4[1] = voc->L;
    out4[2] = voc->n_nodes;
    out4[3] = voc->n_words;
    return OSG_OK;
}

int osg_vocabulary_transform_batch(osg_ctx *ctx, const osg_vocabulary *voc, const uint8_t *desc, const int32_t *n,
                                   int32_t B, int32_t levelsup, osg_bow_out *out)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, voc && (B == 0 || (n && out)) && B >= 0, "null argument");
    int total = 0;
    for (int b = 0; b < B; b++) {
        OSG_REQUIRE(ctx, n[b] >= 0 && n[b] <= MAX_SET, "set %d: %d features (at most %d)", b, n[b], MAX_SET);
        OSG_REQUIRE(ctx, out[b].word && out[b].value && out[b].node_id && out[b].node_start && out[b].feat,
                    "set %d: output arrays", b);
        out[b].n_words = 0;
        out[b].n_nodes = 0;
        out[b].node_start[0] = 0;
        total += n[b];
    }
    OSG_REQUIRE(ctx, total == 0 || desc, "descriptors");
    // empty(): nothing to do (ref:TemplatedVocabulary.h:1133-1136)
    if (total == 0 || voc->n_nodes <= 1) return OSG_OK;
    // device layout: [features 32 total][word 4 total][w 8 total][nid 4 total] | per set outputs | SetArgs
    osg_packer pk;
    const size_t o_feat = pk.add(desc, 32 * (size_t)total);
    char *pin = (char *)osg_pinned(ctx, pk.total + 64 * (size_t)total + 256 * (size_t)B + 4096);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    pk.fill(pin);
    char *din = nullptr, *dmid = nullptr, *dout = nullptr;
    SetArgs *dsets = nullptr;
    OSG_ALLOC(ctx, din, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dmid, SLOT_TMP1, 20 * (size_t)total + 256);
    // per set: word 4n, value 8n, node_id 4n, node_start 4(n+1), feat 4n, counts 8 -> padded
    std::vector<size_t> so(B + 1, 0);
    for (int b = 0; b < B; b++) so[b + 1] = so[b] + ((24 * (size_t)n[b] + 4 + 8 + 255) & ~size_t(255)) + 256;
    OSG_ALLOC(ctx, dout, SLOT_TMP2, so[B] + 256);
    OSG_ALLOC(ctx, dsets, SLOT_TMP3, sizeof(SetArgs) * (size_t)B + 64);
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(din, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    int32_t *d_word = (int32_t *)dmid;
    double *d_w = (double *)(dmid + ((4 * (size_t)total + 15) & ~size_t(15)));
    uint32_t *d_nid = (uint32_t *)((char *)d_w + 8 * (size_t)total);
    uint32_t *d_nrank = d_nid + total;
    // key widths: word ids < n_words; node ranks 0 (root) .. level_count[nid_level]
    const int nid_level = voc->L - levelsup;
    const int lvl_n = (nid_level >= 1 && nid_level < 16) ? voc->level_count[nid_level] : 0;
    int wbits = 1, rbits = 1;
    while ((1ll << wbits) < voc->n_words) wbits++;
    while ((1ll << rbits) <= lvl_n) rbits++;
    std::vector<SetArgs> hs(B);
    int first = 0;
    for (int b = 0; b < B; b++) {
        char *base = dout + so[b];
        SetArgs &S = hs[b];
        S.first = first;
        S.n = n[b];
        S.value = (double *)base;
        S.word = (int32_t *)(base + 8 * (size_t)n[b]);
        S.node_id = (uint32_t *)((char *)S.word + 4 * (size_t)n[b]);
        S.node_start = (int32_t *)((char *)S.node_id + 4 * (size_t)n[b]);
        S.feat = (int32_t *)((char *)S.node_start + 4 * ((size_t)n[b] + 1));
        S.counts = (int32_t *)((char *)S.feat + 4 * (size_t)n[b]);
        first += n[b];
    }
    SetArgs *pin_sets = (SetArgs *)(pin + ((pk.total + 255) & ~size_t(255)));
    std::memcpy(pin_sets, hs.data(), sizeof(SetArgs) * B);
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dsets, pin_sets, sizeof(SetArgs) * B, hipMemcpyHostToDevice, ctx->stream));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_voc_descend, dim3((total + DT - 1) / DT), dim3(DT), 0, ctx->stream, voc->meta, voc->desc,
                       voc->weight, voc->old_id, voc->lvl_rank, (const uint4 *)(din + o_feat), total, nid_level,
                       d_word, d_w, d_nid, d_nrank);
    static const bool prof_on = getenv("OSG_DBOW_PROFILE") != nullptr;
    unsigned long long *dprof = nullptr;
    if (prof_on) OSG_ALLOC(ctx, dprof, SLOT_TMP4, 16 * sizeof(unsigned long long));
    hipLaunchKernelGGL(k_bow_assemble, dim3(B), dim3(AT), 0, ctx->stream, dsets, d_word, d_w, d_nid, d_nrank, wbits,
                       rbits, voc->weighting, voc->scoring, dprof);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    char *pout = (char *)pin_sets + ((sizeof(SetArgs) * B + 255) & ~size_t(255));
    OSG_RC(osg_download(ctx, pout, dout, so[B]));
    OSG_RC(osg_wait(ctx));
    float kms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&kms, ev[0], ev[1]));
    ctx->last_kernel_ms = kms;
    if (prof_on) {
        unsigned long long st[16];
        OSG_HIP_CHECK(ctx, hipMemcpy(st, dprof, sizeof(st), hipMemcpyDeviceToHost));
        fprintf(stderr, "[dbow] B=%d kernels %.1f us; assemble wg0 phases (cycles):", B, kms * 1e3);
        for (int k = 1; k <= 8; k++) fprintf(stderr, " %llu", st[k] - st[k - 1]);
        fprintf(stderr, "\n");
    }
    for (int b = 0; b < B; b++) {
        const char *base = pout + so[b];
        const int nb = n[b];
        const double *value = (const double *)base;
        const int32_t *word = (const int32_t *)(base + 8 * (size_t)nb);
        const uint32_t *node_id = (const uint32_t *)((const char *)word + 4 * (size_t)nb);
        const int32_t *node_start = (const int32_t *)((const char *)node_id + 4 * (size_t)nb);
        const int32_t *feat = (const int32_t *)((const char *)node_start + 4 * ((size_t)nb + 1));
        const int32_t *counts = (const int32_t *)((const char *)feat + 4 * (size_t)nb);
        const int nw = nb ? counts[0] : 0, nn = nb ? counts[1] : 0;
        out[b].n_words = nw;
        out[b].n_nodes = nn;
        std::memcpy(out[b].word, word, 4 * (size_t)nw);
        std::memcpy(out[b].value, value, 8 * (size_t)nw);
        std::memcpy(out[b].node_id, node_id, 4 * (size_t)nn);
        std::memcpy(out[b].node_start, node_start, 4 * ((size_t)nn + 1));
        if (nn == 0) out[b].node_start[0] = 0;
        const int m = nn ? node_start[nn] : 0;
        std::memcpy(out[b].feat, feat, 4 * (size_t)m);
    }
    return OSG_OK;
}

int osg_vocabulary_transform(osg_ctx *ctx, const osg_vocabulary *voc, const uint8_t *desc, int32_t n, int32_t levelsup,
                             osg_bow_out *out)
{
    return osg_vocabulary_transform_batch(ctx, voc, desc, &n, 1, levelsup, out);
}

}  // extern "C"
