// hamming.hip — 256-bit Hamming distance and brute-force top-2 kernels for gfx950.
//
// Replaces ORBmatcher::DescriptorDistance (ref:src/ORBmatcher.cc:2388-2408) evaluated inside the
// top-2 candidate loop every matcher runs (ref:src/ORBmatcher.cc:316-355 is the canonical form):
//   bestDist1 = bestDist2 = 256, bestIdx = -1;
//   for each candidate j: d = dist(q, t_j);
//       if (d < bestDist1) { bestDist2 = bestDist1; bestDist1 = d; bestIdx = j; }
//       else if (d < bestDist2) bestDist2 = d;
// which is: best = smallest distance, first index among ties; second = 2nd smallest distance
// counted with multiplicity; a distance of 256 never enters.  On the GPU this is an
// order-independent min over packed keys  key = dist << 23 | local_index  (smaller key = smaller
// distance, then earlier index), kept as (k1 = smallest key, k2 = second smallest key) with
// k2' = min(k2, max(k1, key)), k1' = min(k1, key) — 2 VALU ops (v_max/v_min3 or v_med3).
//
// Three shapes (same semantics, chosen by osg_launch_top2):
//  * qsplit — small query sets (nq <= 32 x CUs, e.g. C2 2000 x 2000): a workgroup owns a few
//             queries against the whole train set staged through LDS; no cross-workgroup merge.
//  * tile   — large query sets: lane = query (its 8 words in VGPRs); every train row is
//             wave-uniform (scalar loads or LDS broadcast), so a pair costs 8 v_xor +
//             8 v_bcnt(accumulate) + 1 v_lshl_or + 2 min = 19 VALU.  INT32-VALU bound.  Train rows
//             split over WAVES waves (merged in LDS) and over G workgroups (merged by the
//             last-arriving workgroup through a self-resetting counter).
//  * stream — few queries (<= 8) against a huge train set (C2', M = 2^24): a lane pair per train
//             row, queries in VGPRs, every row read once with fully coalesced 16-B loads.  HBM bound.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "osg_internal.h"

namespace {

constexpr int KEY_SHIFT = 23;
constexpr uint32_t IDX_MASK = (1u << KEY_SHIFT) - 1u;
constexpr uint32_t KEY_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t D_EMPTY = 511u;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// v_bcnt_u32_b32 with its accumulate operand chained (hipcc otherwise splits the sum into
// bcnt(x,0) + v_add3, 3 extra VALU per pair).
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ uint32_t hamming8(const uint32_t (&a)[8], const uint32_t *__restrict__ b)
{
    uint32_t d = __popc(a[0] ^ b[0]);
    d = bcnt_acc(a[1] ^ b[1], d);
    d = bcnt_acc(a[2] ^ b[2], d);
    d = bcnt_acc(a[3] ^ b[3], d);
    d = bcnt_acc(a[4] ^ b[4], d);
    d = bcnt_acc(a[5] ^ b[5], d);
    d = bcnt_acc(a[6] ^ b[6], d);
    d = bcnt_acc(a[7] ^ b[7], d);
    return d;
}

// (k1, k2) = two smallest keys seen; k1 <= k2 always, so the new second is med3(k1, key, k2).
__device__ __forceinline__ void key_push(uint32_t &k1, uint32_t &k2, uint32_t key)
{
    k2 = med3_u32(k1, key, k2);
    k1 = min(k1, key);
}

__device__ __forceinline__ void key_merge(uint32_t &k1, uint32_t &k2, uint32_t a1, uint32_t a2)
{
    const uint32_t hi = max(k1, a1);
    k1 = min(k1, a1);
    k2 = min(min(k2, a2), hi);
}

// partial = {global idx of best, d1 << 16 | d2}
__device__ __forceinline__ uint2 key_to_part(uint32_t k1, uint32_t k2, uint32_t base)
{
    const uint32_t d1 = k1 >> KEY_SHIFT, d2 = k2 >> KEY_SHIFT;
    const uint32_t i1 = (k1 == KEY_EMPTY) ? 0xFFFFFFFFu : base + (k1 & IDX_MASK);
    return make_uint2(i1, (d1 << 16) | d2);
}

__device__ __forceinline__ void part_merge(uint32_t &D1, uint32_t &I1, uint32_t &D2, uint2 p)
{
    const uint32_t d1 = p.y >> 16, d2 = p.y & 0xFFFFu, i1 = p.x;
    if (d1 < D1 || (d1 == D1 && i1 < I1)) {
        D2 = min(D1, d2);
        D1 = d1;
        I1 = i1;
    } else {
        D2 = min(D2, d1);
    }
}

__device__ __forceinline__ void write_result(int32_t *__restrict__ out, int q, uint32_t D1, uint32_t I1,
                                             uint32_t D2)
{
    const int32_t d1 = (int32_t)min(D1, 256u);
    out[3 * q + 0] = (D1 < 256u) ? (int32_t)I1 : -1;
    out[3 * q + 1] = d1;
    out[3 * q + 2] = (int32_t)min(D2, 256u);
}

// ------------------------------------------------------------------------------- tile kernel
// STAGE 0: train rows come straight from memory through scalar loads (wave-uniform address).
// STAGE 1: the workgroup first copies its chunk into LDS with one coalesced 16-B load per thread,
//          then every wave reads rows with wave-uniform (broadcast) ds_read_b128.
// MERGE 0: partials published with plain stores + agent release, consumed after agent acquire.
// MERGE 1: partials published with write-through (sc1) 8-B stores, drained (vmcnt(0)) before a
//          relaxed agent-scope counter add; the last arriver reads them with sc1 loads
//          (MI355X_MICROARCH.md "Valid forms", first table row).
constexpr int TILE_MAX_ROWS = 512;  // STAGE 1 chunk capacity (16 KiB of LDS)
constexpr int TILE_MAX_G = 64;      // partials staged in LDS by the merging workgroup

template <int WAVES, int STAGE, int MERGE>
__global__ __launch_bounds__(WAVES * 64) void k_top2_tile(const uint4 *__restrict__ query, int nq,
                                                          const uint32_t *__restrict__ train, int nt,
                                                          int rows_per_chunk, int G,
                                                          uint2 *__restrict__ part,
                                                          uint32_t *__restrict__ counters,
                                                          int32_t *__restrict__ out, int dbg)
{
    __shared__ uint32_t s_k1[WAVES][64];
    __shared__ uint32_t s_k2[WAVES][64];
    __shared__ uint4 s_rows[STAGE ? 2 * TILE_MAX_ROWS : 1];
    __shared__ uint2 s_part[TILE_MAX_G * 64];
    __shared__ int s_last;

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int qb = blockIdx.x;
    const int c = blockIdx.y;
    const int qi = qb * 64 + lane;
    const int r0 = c * rows_per_chunk;
    const int r1 = min(nt, r0 + rows_per_chunk);

    if (STAGE) {
        const uint4 *tv = (const uint4 *)train + 2 * (size_t)r0;
        for (int i = threadIdx.x; i < 2 * (r1 - r0); i += WAVES * 64) s_rows[i] = tv[i];
    }
    uint32_t qd[8];
    {
        const int qq = qi < nq ? qi : nq - 1;
        const uint4 a = query[2 * qq], b = query[2 * qq + 1];
        qd[0] = a.x; qd[1] = a.y; qd[2] = a.z; qd[3] = a.w;
        qd[4] = b.x; qd[5] = b.y; qd[6] = b.z; qd[7] = b.w;
    }
    uint32_t k1 = KEY_EMPTY, k2 = KEY_EMPTY;
    if (STAGE) {
        __syncthreads();
        const int nr = (dbg & 1) ? 0 : r1 - r0;
        int j = w;
        for (; j + 3 * WAVES < nr; j += 4 * WAVES) {
            uint32_t t[4][8];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint4 a = s_rows[2 * (j + u * WAVES)], b = s_rows[2 * (j + u * WAVES) + 1];
                t[u][0] = a.x; t[u][1] = a.y; t[u][2] = a.z; t[u][3] = a.w;
                t[u][4] = b.x; t[u][5] = b.y; t[u][6] = b.z; t[u][7] = b.w;
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
                key_push(k1, k2, (hamming8(qd, t[u]) << KEY_SHIFT) | (uint32_t)(j + u * WAVES));
        }
        for (; j < nr; j += WAVES) {
            const uint4 a = s_rows[2 * j], b = s_rows[2 * j + 1];
            const uint32_t t[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            key_push(k1, k2, (hamming8(qd, t) << KEY_SHIFT) | (uint32_t)j);
        }
    } else {
        // rows r0 + w + WAVES*j: wave-uniform, consumed from SGPRs (scalar loads)
        int r = r0 + w;
        for (; r + 3 * WAVES < r1; r += 4 * WAVES) {
            const uint32_t *t0 = train + (size_t)r * 8;
            const uint32_t *t1 = t0 + 8 * WAVES;
            const uint32_t *t2 = t1 + 8 * WAVES;
            const uint32_t *t3 = t2 + 8 * WAVES;
            const uint32_t l = (uint32_t)(r - r0);
            key_push(k1, k2, (hamming8(qd, t0) << KEY_SHIFT) | l);
            key_push(k1, k2, (hamming8(qd, t1) << KEY_SHIFT) | (l + WAVES));
            key_push(k1, k2, (hamming8(qd, t2) << KEY_SHIFT) | (l + 2 * WAVES));
            key_push(k1, k2, (hamming8(qd, t3) << KEY_SHIFT) | (l + 3 * WAVES));
        }
        for (; r < r1; r += WAVES) {
            const uint32_t *t0 = train + (size_t)r * 8;
            key_push(k1, k2, (hamming8(qd, t0) << KEY_SHIFT) | (uint32_t)(r - r0));
        }
    }

    if (WAVES > 1) {
        s_k1[w][lane] = k1;
        s_k2[w][lane] = k2;
        __syncthreads();
        if (w == 0) {
#pragma unroll
            for (int o = 1; o < WAVES; o++) key_merge(k1, k2, s_k1[o][lane], s_k2[o][lane]);
        }
    }
    if (G == 1) {
        if (w == 0 && qi < nq) {
            const uint2 p = key_to_part(k1, k2, (uint32_t)r0);
            write_result(out, qi, p.y >> 16, p.x, p.y & 0xFFFFu);
        }
        return;
    }
    // publish this chunk's partial; the last-arriving workgroup of this query block merges
    if (w == 0 && qi < nq) {
        const uint2 p = key_to_part(k1, k2, (uint32_t)r0);
        if (MERGE == 1) {
            const unsigned long long v = ((unsigned long long)p.y << 32) | p.x;
            __hip_atomic_store((unsigned long long *)&part[(size_t)c * nq + qi], v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        } else {
            part[(size_t)c * nq + qi] = p;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t prev;
        if (MERGE == 1)
            prev = __hip_atomic_fetch_add(&counters[qb], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            prev = __hip_atomic_fetch_add(&counters[qb], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (prev == (uint32_t)(G - 1));
    }
    __syncthreads();
    if (s_last && (dbg & 2) && threadIdx.x == 0)
        __hip_atomic_store(&counters[qb], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!s_last || (dbg & 2)) return;
    // stage all G partials of this query block in LDS with one round of parallel loads
    for (int i = threadIdx.x; i < G * 64; i += WAVES * 64) {
        const int cc = i >> 6, l = i & 63, qq = qb * 64 + l;
        if (qq < nq) {
            if (MERGE == 1) {
                const unsigned long long v = __hip_atomic_load(
                    (unsigned long long *)&part[(size_t)cc * nq + qq], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_part[i] = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
            } else {
                s_part[i] = part[(size_t)cc * nq + qq];
            }
        }
    }
    __syncthreads();
    if (w == 0 && qi < nq) {
        uint32_t D1 = D_EMPTY, I1 = 0xFFFFFFFFu, D2 = D_EMPTY;
        for (int cc = 0; cc < G; cc++) part_merge(D1, I1, D2, s_part[cc * 64 + lane]);
        write_result(out, qi, D1, I1, D2);
    }
    if (threadIdx.x == 0) __hip_atomic_store(&counters[qb], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------- query-split (qsplit) kernel
// Small query sets (C2: 2000 x 2000): one workgroup owns QB queries against the WHOLE train set,
// staged through LDS in chunks of QS_ROWS rows, so no partial keys leave the workgroup (no
// cross-workgroup merge, no atomics).  Thread t handles query t % QB over train rows
// r = t / QB + k * (1024 / QB); a wave therefore reads 64 / QB distinct rows per step (each
// broadcast to QB lanes, conflict-free ds_read_b128).  Reduction: xor-shuffles over the lanes of
// one query inside the wave, then across the 16 waves in LDS.  Keys carry the global row index
// (nt <= 2^23).
constexpr int QS_ROWS = 2048;  // 64 KiB of LDS per chunk

// rows [0, n) of the staged chunk, slice sl of S; keys carry row index base + r
template <int S>
__device__ __forceinline__ void qs_scan(const uint4 *rows, int n, int sl, uint32_t base, const uint32_t (&qd)[8],
                                        uint32_t &k1, uint32_t &k2)
{
    int r = sl;
    for (; r + 3 * S < n; r += 4 * S) {
        uint32_t tr[4][8];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint4 a = rows[2 * (r + u * S)], b = rows[2 * (r + u * S) + 1];
            tr[u][0] = a.x; tr[u][1] = a.y; tr[u][2] = a.z; tr[u][3] = a.w;
            tr[u][4] = b.x; tr[u][5] = b.y; tr[u][6] = b.z; tr[u][7] = b.w;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) key_push(k1, k2, (hamming8(qd, tr[u]) << KEY_SHIFT) | (base + r + u * S));
    }
    for (; r < n; r += S) {
        const uint4 a = rows[2 * r], b = rows[2 * r + 1];
        const uint32_t tr[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        key_push(k1, k2, (hamming8(qd, tr) << KEY_SHIFT) | (base + r));
    }
}

// Query-split with QT queries per thread: a row read from LDS once serves QT queries, so the
// per-workgroup LDS read volume drops QT-fold (the QT = 1 form reads 16 x 32 B per thread at
// C2).  G = QB / QT query groups, S = 1024 / G row slices; thread t: group t % G, slice t / G.
// dbg (sweeps only): 1 = no compute, 2 = no global staging loads, 4 = no reduction.
template <int QB, int QT>
__global__ __launch_bounds__(1024) void k_top2_qsplit_mq(const uint4 *__restrict__ query, int nq,
                                                         const uint4 *__restrict__ train, int nt,
                                                         int32_t *__restrict__ out, int dbg)
{
    constexpr int G = QB / QT;
    constexpr int S = 1024 / G;
    __shared__ uint4 s_rows[2 * QS_ROWS];
    __shared__ uint32_t s_k1[16][QB], s_k2[16][QB];
    const int t = threadIdx.x;
    const int w = t >> 6, lane = t & 63;
    const int g = t % G;
    const int sl = t / G;
    uint32_t qd[QT][8];
#pragma unroll
    for (int j = 0; j < QT; j++) {
        int qq = blockIdx.x * QB + g * QT + j;
        qq = qq < nq ? qq : nq - 1;
        const uint4 a = query[2 * qq], b = query[2 * qq + 1];
        qd[j][0] = a.x; qd[j][1] = a.y; qd[j][2] = a.z; qd[j][3] = a.w;
        qd[j][4] = b.x; qd[j][5] = b.y; qd[j][6] = b.z; qd[j][7] = b.w;
    }
    uint32_t k1[QT], k2[QT];
#pragma unroll
    for (int j = 0; j < QT; j++) k1[j] = k2[j] = KEY_EMPTY;
    for (int c0 = 0; c0 < nt; c0 += QS_ROWS) {
        const int n = min(QS_ROWS, nt - c0);
        const uint4 *src = train + 2 * (size_t)c0;
        const int last = 2 * n - 1;
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0, v2 = v0, v3 = v0;
        if (!(dbg & 2)) {
            v0 = src[min(t, last)];
            v1 = src[min(1024 + t, last)];
            v2 = src[min(2048 + t, last)];
            v3 = src[min(3072 + t, last)];
        }
        if (c0 > 0) __syncthreads();
        s_rows[t] = v0;
        s_rows[1024 + t] = v1;
        s_rows[2048 + t] = v2;
        s_rows[3072 + t] = v3;
        __syncthreads();
        if (dbg & 1) continue;
        int r = sl;
        for (; r + S < n; r += 2 * S) {
            uint32_t tr[2][8];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint4 a = s_rows[2 * (r + u * S)], b = s_rows[2 * (r + u * S) + 1];
                tr[u][0] = a.x; tr[u][1] = a.y; tr[u][2] = a.z; tr[u][3] = a.w;
                tr[u][4] = b.x; tr[u][5] = b.y; tr[u][6] = b.z; tr[u][7] = b.w;
            }
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
                for (int j = 0; j < QT; j++)
                    key_push(k1[j], k2[j], (hamming8(qd[j], tr[u]) << KEY_SHIFT) | (uint32_t)(c0 + r + u * S));
        }
        for (; r < n; r += S) {
            const uint4 a = s_rows[2 * r], b = s_rows[2 * r + 1];
            const uint32_t tr[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int j = 0; j < QT; j++) key_push(k1[j], k2[j], (hamming8(qd[j], tr) << KEY_SHIFT) | (uint32_t)(c0 + r));
        }
    }
    if (!(dbg & 4)) {
        // lanes of one query group inside the wave: lane ^ G, ^ 2G, ... < 64
#pragma unroll
        for (int off = G; off < 64; off <<= 1)
#pragma unroll
            for (int j = 0; j < QT; j++) {
                const uint32_t a1 = __shfl_xor(k1[j], off), a2 = __shfl_xor(k2[j], off);
                key_merge(k1[j], k2[j], a1, a2);
            }
    }
    if (lane < G) {
#pragma unroll
        for (int j = 0; j < QT; j++) {
            s_k1[w][lane * QT + j] = k1[j];
            s_k2[w][lane * QT + j] = k2[j];
        }
    }
    __syncthreads();
    const int q = blockIdx.x * QB + t;
    if (t < QB && q < nq) {
        uint32_t a1 = s_k1[0][t], a2 = s_k2[0][t];
#pragma unroll
        for (int o = 1; o < 16; o++) key_merge(a1, a2, s_k1[o][t], s_k2[o][t]);
        const uint2 p = key_to_part(a1, a2, 0u);
        write_result(out, q, p.y >> 16, p.x, p.y & 0xFFFFu);
    }
}

// (Measured on MI355X at 2000 x 2000, kernel average over back-to-back launches: this register
// staging 5.75 us; LDS-DMA staging (global_load_lds_dwordx4) with per-quarter counted waits
// 6.1 us, whether the rows are then read with compiler-scheduled or inline-asm ds_reads.)
template <int QB>
__global__ __launch_bounds__(1024) void k_top2_qsplit(const uint4 *__restrict__ query, int nq,
                                                      const uint4 *__restrict__ train, int nt,
                                                      int32_t *__restrict__ out)
{
    constexpr int S = 1024 / QB;  // row slices
    __shared__ uint4 s_rows[2 * QS_ROWS];
    __shared__ uint32_t s_k1[16][QB], s_k2[16][QB];
    const int t = threadIdx.x;
    const int w = t >> 6, lane = t & 63;
    const int qi = t % QB;
    const int sl = t / QB;
    const int q = blockIdx.x * QB + qi;
    uint32_t qd[8];
    {
        const int qq = q < nq ? q : nq - 1;
        const uint4 a = query[2 * qq], b = query[2 * qq + 1];
        qd[0] = a.x; qd[1] = a.y; qd[2] = a.z; qd[3] = a.w;
        qd[4] = b.x; qd[5] = b.y; qd[6] = b.z; qd[7] = b.w;
    }
    uint32_t k1 = KEY_EMPTY, k2 = KEY_EMPTY;
    for (int c0 = 0; c0 < nt; c0 += QS_ROWS) {
        const int n = min(QS_ROWS, nt - c0);
        const uint4 *src = train + 2 * (size_t)c0;
        const int last = 2 * n - 1;  // past n: clamped copies, never read
        const uint4 v0 = src[min(t, last)], v1 = src[min(1024 + t, last)];
        const uint4 v2 = src[min(2048 + t, last)], v3 = src[min(3072 + t, last)];
        if (c0 > 0) __syncthreads();  // previous chunk fully consumed
        s_rows[t] = v0;
        s_rows[1024 + t] = v1;
        s_rows[2048 + t] = v2;
        s_rows[3072 + t] = v3;
        __syncthreads();
        qs_scan<S>(s_rows, n, sl, (uint32_t)c0, qd, k1, k2);
    }
    // lanes of one query inside the wave: lane ^ QB, ^ 2QB, ... < 64
#pragma unroll
    for (int off = QB; off < 64; off <<= 1) {
        const uint32_t a1 = __shfl_xor(k1, off), a2 = __shfl_xor(k2, off);
        key_merge(k1, k2, a1, a2);
    }
    if (lane < QB) {
        s_k1[w][lane] = k1;
        s_k2[w][lane] = k2;
    }
    __syncthreads();
    if (t < QB && q < nq) {
        uint32_t a1 = s_k1[0][t], a2 = s_k2[0][t];
#pragma unroll
        for (int o = 1; o < 16; o++) key_merge(a1, a2, s_k1[o][t], s_k2[o][t]);
        const uint2 p = key_to_part(a1, a2, 0u);
        write_result(out, q, p.y >> 16, p.x, p.y & 0xFFFFu);
    }
}

// ------------------------------------------------------------------------------ batch kernel
// Frame-batched C2: B independent nq x nt problems in one launch (problem b: query rows
// [b nq, (b+1) nq), train rows [b nt, (b+1) nt), out rows [b nq, (b+1) nq)).  grid (ceil(nq / (64
// QL)), B) x 1024 threads: a lane holds QL queries in VGPRs (lane + 64 j), the 16 waves split the
// train rows (row r on wave r % 16), rows staged in LDS in chunks of BATCH_ROWS and read as
// wave-uniform broadcasts, so a pair costs the 19 VALU of the tile kernel and a row read from LDS
// serves QL queries.  The 16 waves' keys meet in LDS (the staging buffer, reused) and are merged
// in a fixed wave order: deterministic, and the same (first index, second with multiplicity) rule.
// SCALAR = 1: no LDS staging; each wave reads its rows with scalar loads (wave-uniform address,
// s_load_dwordx8 into SGPRs, v_xor with an SGPR operand), which frees the LDS return path that
// the broadcast reads share between the CU's four SIMDs.
constexpr int BATCH_ROWS = 2048;  // 64 KiB of LDS: two workgroups per CU
template <int QL, int SCALAR>
__global__ __launch_bounds__(1024) void k_top2_batch(const uint4 *__restrict__ query, int nq,
                                                     const uint4 *__restrict__ train, int nt,
                                                     int32_t *__restrict__ out)
{
    __shared__ uint4 s_rows[SCALAR ? 16 * 64 * QL / 2 : 2 * BATCH_ROWS];
    const int t = threadIdx.x, lane = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const size_t b = blockIdx.y;
    const uint4 *qf = query + 2 * b * (size_t)nq;
    const uint4 *tf = train + 2 * b * (size_t)nt;
    int32_t *of = out + 3 * b * (size_t)nq;
    const int q0 = blockIdx.x * 64 * QL;
    uint32_t qd[QL][8], k1[QL], k2[QL];
#pragma unroll
    for (int j = 0; j < QL; j++) {
        const int qq = min(q0 + 64 * j + lane, nq - 1);
        const uint4 a = qf[2 * qq], c = qf[2 * qq + 1];
        qd[j][0] = a.x; qd[j][1] = a.y; qd[j][2] = a.z; qd[j][3] = a.w;
        qd[j][4] = c.x; qd[j][5] = c.y; qd[j][6] = c.z; qd[j][7] = c.w;
        k1[j] = k2[j] = KEY_EMPTY;
    }
    if (SCALAR) {
        const uint32_t *tw = (const uint32_t *)tf;
        int r = w;
        for (; r + 48 < nt; r += 64) {
#pragma unroll
            for (int u = 0; u < 4; u++)
#pragma unroll
                for (int j = 0; j < QL; j++)
                    key_push(k1[j], k2[j], (hamming8(qd[j], tw + (size_t)(r + 16 * u) * 8) << KEY_SHIFT) |
                                               (uint32_t)(r + 16 * u));
        }
        for (; r < nt; r += 16)
#pragma unroll
            for (int j = 0; j < QL; j++)
                key_push(k1[j], k2[j], (hamming8(qd[j], tw + (size_t)r * 8) << KEY_SHIFT) | (uint32_t)r);
    }
    for (int c0 = 0; !SCALAR && c0 < nt; c0 += BATCH_ROWS) {
        const int n = min(BATCH_ROWS, nt - c0);
        if (c0 > 0) __syncthreads();  // previous chunk fully consumed
        const uint4 *src = tf + 2 * (size_t)c0;
        for (int i = t; i < 2 * n; i += 1024) s_rows[i] = src[i];
        __syncthreads();
        int r = w;
        for (; r + 48 < n; r += 64) {
            uint32_t tr[4][8];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint4 a = s_rows[2 * (r + 16 * u)], c = s_rows[2 * (r + 16 * u) + 1];
                tr[u][0] = a.x; tr[u][1] = a.y; tr[u][2] = a.z; tr[u][3] = a.w;
                tr[u][4] = c.x; tr[u][5] = c.y; tr[u][6] = c.z; tr[u][7] = c.w;
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
#pragma unroll
                for (int j = 0; j < QL; j++)
                    key_push(k1[j], k2[j], (hamming8(qd[j], tr[u]) << KEY_SHIFT) | (uint32_t)(c0 + r + 16 * u));
        }
        for (; r < n; r += 16) {
            const uint4 a = s_rows[2 * r], c = s_rows[2 * r + 1];
            const uint32_t tr[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
            for (int j = 0; j < QL; j++) key_push(k1[j], k2[j], (hamming8(qd[j], tr) << KEY_SHIFT) | (uint32_t)(c0 + r));
        }
    }
    __syncthreads();  // the staging buffer becomes the merge buffer
    uint32_t *sk1 = (uint32_t *)s_rows, *sk2 = sk1 + 16 * 64 * QL;
#pragma unroll
    for (int j = 0; j < QL; j++) {
        sk1[(w * QL + j) * 64 + lane] = k1[j];
        sk2[(w * QL + j) * 64 + lane] = k2[j];
    }
    __syncthreads();
    if (t < 64 * QL) {
        const int j = t >> 6, q = q0 + t;
        uint32_t a1 = sk1[t], a2 = sk2[t];
#pragma unroll
        for (int o = 1; o < 16; o++) key_merge(a1, a2, sk1[(o * QL + j) * 64 + (t & 63)], sk2[(o * QL + j) * 64 + (t & 63)]);
        if (q < nq) {
            const uint2 p = key_to_part(a1, a2, 0u);
            write_result(of, q, p.y >> 16, p.x, p.y & 0xFFFFu);
        }
    }
}

// ----------------------------------------------------------------------------- stream kernel
// Completion counters of the stream kernels: 8 group counters and one top counter, each on its
// own 128-B line at the end of ctx->counters (the tile kernel uses the first nqb entries).
constexpr int STREAM_CNT_BASE = OSG_N_COUNTERS - 512;
constexpr int STREAM_GROUPS = 8;

// Arrival of one workgroup: group counter (blockIdx % 8), the last of a group bumps the top
// counter; returns true in the workgroup that completes the whole grid.  Relaxed agent-scope
// atomics after write-through partial stores drained with vmcnt(0): no L2 writeback fences.
// Fan-in per counter is G / 8 instead of G (one device-scope atomic costs ~12 ns serialised).
__device__ __forceinline__ bool stream_arrive(uint32_t *counters, int G)
{
    const int g = blockIdx.x % STREAM_GROUPS;
    const int members = G / STREAM_GROUPS + (g < G % STREAM_GROUPS ? 1 : 0);
    const int groups = min(G, STREAM_GROUPS);
    uint32_t *gc = counters + STREAM_CNT_BASE + 32 * g;
    uint32_t *top = counters + STREAM_CNT_BASE + 32 * STREAM_GROUPS;
    const uint32_t prev = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev != (uint32_t)(members - 1)) return false;
    __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t tprev = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tprev != (uint32_t)(groups - 1)) return false;
    __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// Stream kernel, lane-pair layout: lane = one 16-B half of a train row, so every load
// instruction of a wave reads 1 KiB contiguous (32 rows); the half distances of a row meet with
// one DPP add (quad_perm [1,0,3,2]).  Both lanes of a pair then hold the same keys, so the
// butterfly starts at offset 2.  Rows double-buffered in registers (U steps of 128 rows per
// workgroup in flight while the previous U are consumed).
template <int NQ>
__global__ __launch_bounds__(256) void k_top2_stream(const uint32_t *__restrict__ query, int nq,
                                                      const u32x4 *__restrict__ train, int nt,
                                                      int rows_per_block, int G,
                                                      uint2 *__restrict__ part,
                                                      uint32_t *__restrict__ counters,
                                                      int32_t *__restrict__ out)
{
    constexpr int U = 4;
    __shared__ uint32_t s_k1[4][NQ], s_k2[4][NQ];
    __shared__ uint32_t s_D1[4], s_I1[4], s_D2[4];
    __shared__ int s_last;
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6, h = t & 1;

    uint32_t qh[NQ][4];
#pragma unroll
    for (int j = 0; j < NQ; j++) {
        const int jj = j < nq ? j : nq - 1;
#pragma unroll
        for (int i = 0; i < 4; i++) qh[j][i] = query[jj * 8 + 4 * h + i];
    }
    uint32_t k1[NQ], k2[NQ];
#pragma unroll
    for (int j = 0; j < NQ; j++) k1[j] = k2[j] = KEY_EMPTY;

    const int r0 = blockIdx.x * rows_per_block;
    const int r1 = min(nt, r0 + rows_per_block);
    const int nr = r1 - r0;
    const u32x4 *base = train + 2 * (size_t)r0;
    auto consume = [&](const u32x4 &v, uint32_t rl) {
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            uint32_t p = __popc(qh[j][0] ^ v.x);
            p = bcnt_acc(qh[j][1] ^ v.y, p);
            p = bcnt_acc(qh[j][2] ^ v.z, p);
            p = bcnt_acc(qh[j][3] ^ v.w, p);
            const uint32_t d = p + (uint32_t)__builtin_amdgcn_mov_dpp((int)p, 0xB1, 0xF, 0xF, false);
            key_push(k1[j], k2[j], (d << KEY_SHIFT) | rl);
        }
    };
    // full batches: U steps of 128 rows (256 16-B elements) each
    const int nfull = nr / (128 * U);
    int b = 0;
    if (nfull > 0) {
        u32x4 cur[U];
#pragma unroll
        for (int u = 0; u < U; u++) cur[u] = __builtin_nontemporal_load(&base[256 * u + t]);
        for (; b + 1 < nfull; b++) {
            u32x4 nxt[U];
            const u32x4 *nb = base + 256 * U * (b + 1);
#pragma unroll
            for (int u = 0; u < U; u++) nxt[u] = __builtin_nontemporal_load(&nb[256 * u + t]);
#pragma unroll
            for (int u = 0; u < U; u++) consume(cur[u], (uint32_t)(128 * (U * b + u) + (t >> 1)));
#pragma unroll
            for (int u = 0; u < U; u++) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < U; u++) consume(cur[u], (uint32_t)(128 * (U * b + u) + (t >> 1)));
        b++;
    }
    // tail steps of 128 rows
    for (int rs = 128 * U * b; rs < nr; rs += 128) {
        const int rl = rs + (t >> 1);
        const u32x4 v = base[2 * min(rl, nr - 1) + h];
        if (rl < nr) consume(v, (uint32_t)rl);  // both lanes of a pair share rl: DPP partner active
    }
#pragma unroll
    for (int j = 0; j < NQ; j++) {
#pragma unroll
        for (int off = 2; off < 64; off <<= 1) {
            const uint32_t a1 = __shfl_xor(k1[j], off), a2 = __shfl_xor(k2[j], off);
            key_merge(k1[j], k2[j], a1, a2);
        }
        if (lane == 0) {
            s_k1[w][j] = k1[j];
            s_k2[w][j] = k2[j];
        }
    }
    __syncthreads();
    if (t < nq) {
        const int j = t;
        uint32_t a1 = s_k1[0][j], a2 = s_k2[0][j];
        for (int o = 1; o < 4; o++) key_merge(a1, a2, s_k1[o][j], s_k2[o][j]);
        const uint2 p = key_to_part(a1, a2, (uint32_t)r0);
        if (G == 1) {
            write_result(out, j, p.y >> 16, p.x, p.y & 0xFFFFu);
        } else {
            const unsigned long long v = ((unsigned long long)p.y << 32) | p.x;
            __hip_atomic_store((unsigned long long *)&part[(size_t)blockIdx.x * nq + j], v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (G == 1) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) s_last = stream_arrive(counters, G);
    __syncthreads();
    if (!s_last) return;
    for (int j = 0; j < nq; j++) {
        uint32_t D1 = D_EMPTY, I1 = 0xFFFFFFFFu, D2 = D_EMPTY;
        for (int bb = t; bb < G; bb += 256) {
            const unsigned long long v = __hip_atomic_load((unsigned long long *)&part[(size_t)bb * nq + j],
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            part_merge(D1, I1, D2, make_uint2((uint32_t)v, (uint32_t)(v >> 32)));
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint2 o = make_uint2(__shfl_xor(I1, off), (__shfl_xor(D1, off) << 16) | __shfl_xor(D2, off));
            part_merge(D1, I1, D2, o);
        }
        if (lane == 0) {
            s_D1[w] = D1;
            s_I1[w] = I1;
            s_D2[w] = D2;
        }
        __syncthreads();
        if (t == 0) {
            for (int o = 1; o < 4; o++) part_merge(D1, I1, D2, make_uint2(s_I1[o], (s_D1[o] << 16) | s_D2[o]));
            write_result(out, j, D1, I1, D2);
        }
        __syncthreads();
    }
}

// --------------------------------------------------------------------------- pairwise distance
__global__ __launch_bounds__(256) void k_pair_dist(const uint4 *__restrict__ a, const uint4 *__restrict__ b,
                                                   int n, int32_t *__restrict__ out)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint4 a0 = a[2 * i], a1 = a[2 * i + 1], b0 = b[2 * i], b1 = b[2 * i + 1];
    out[i] = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
             __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// tuning knobs (environment, read once per process; defaults from the r01 sweeps on MI355X)
int env_int(const char *name, int dflt)
{
    const char *v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}
struct top2_knobs {
    int variant, waves, target_wg, min_rows, dbg, stream_g, qs_wg, qt;
};
const top2_knobs &knobs(int cus)
{
    static const top2_knobs k = {env_int("OSG_TOP2_VARIANT", 2), env_int("OSG_TOP2_WAVES", 0),
                                 env_int("OSG_TOP2_WG", cus), env_int("OSG_TOP2_MIN_ROWS", 64),
                                 env_int("OSG_TOP2_DEBUG", 0), env_int("OSG_TOP2_STREAM_G", 2 * cus),
                                 env_int("OSG_TOP2_QS_WG", cus * 9 / 10), env_int("OSG_TOP2_QT", 1)};
    return k;
}

}  // namespace

// Device-pointer launcher shared by the C ABI and the matcher engine.
int osg_launch_top2(osg_ctx *ctx, const void *d_query, int32_t nq, const void *d_train, int32_t nt,
                    void *d_out)
{
    if (nq <= 0) return OSG_OK;
    OSG_REQUIRE(ctx, nt >= 0 && nt <= (1 << 24), "nt=%d out of range [0, 2^24]", nt);
    if (nt == 0) {
        // no candidates: (-1, 256, 256) for every query
        static const int32_t sentinel[3] = {-1, 256, 256};
        int32_t *h = (int32_t *)osg_pinned(ctx, sizeof(int32_t) * 3 * (size_t)nq);
        if (!h) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
        OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
        for (int i = 0; i < nq; i++) memcpy(h + 3 * i, sentinel, sizeof sentinel);
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(d_out, h, sizeof(int32_t) * 3 * (size_t)nq, hipMemcpyHostToDevice, ctx->stream));
        return OSG_OK;
    }
    const int cus = ctx->num_cus;
    if (nq <= 8 && nt >= 65536) {
        // streaming shape: a lane pair per train row
        int G = knobs(cus).stream_g;
        int rpb = (nt + G - 1) / G;
        rpb = ((rpb + 1023) / 1024) * 1024;
        G = (nt + rpb - 1) / rpb;
        uint2 *part = nullptr;
        OSG_ALLOC(ctx, part, SLOT_PART, sizeof(uint2) * (size_t)G * nq);
        const uint32_t *q = (const uint32_t *)d_query;
        int32_t *o = (int32_t *)d_out;
        const u32x4 *t2 = (const u32x4 *)d_train;
        uint32_t *cn = ctx->counters;
        if (nq == 1) hipLaunchKernelGGL(k_top2_stream<1>, dim3(G), dim3(256), 0, ctx->stream, q, nq, t2, nt, rpb, G, part, cn, o);
        else if (nq == 2) hipLaunchKernelGGL(k_top2_stream<2>, dim3(G), dim3(256), 0, ctx->stream, q, nq, t2, nt, rpb, G, part, cn, o);
        else if (nq <= 4) hipLaunchKernelGGL(k_top2_stream<4>, dim3(G), dim3(256), 0, ctx->stream, q, nq, t2, nt, rpb, G, part, cn, o);
        else hipLaunchKernelGGL(k_top2_stream<8>, dim3(G), dim3(256), 0, ctx->stream, q, nq, t2, nt, rpb, G, part, cn, o);
        OSG_HIP_CHECK(ctx, hipGetLastError());
        return OSG_OK;
    }
    const top2_knobs &kn = knobs(cus);
    // OSG_TOP2_VARIANT: 2 = auto (default), 3 = query-split only, 4 = LDS-staged tile only,
    // 1 = scalar-load tile + write-through merge, 0 = scalar-load tile + fenced merge.
    // Query-split shape: enough workgroups of QB queries to cover the CUs (OSG_TOP2_QS_WG), whole
    // train set per workgroup
    const bool qsplit = (kn.variant == 3 || (kn.variant == 2 && nq <= 32 * cus)) && nt <= (int)IDX_MASK;
    if (qsplit) {
        int qb = 64;
        while (qb > 1 && (nq + qb - 1) / qb < kn.qs_wg) qb >>= 1;
        const dim3 grid((nq + qb - 1) / qb), block(1024);
        const uint4 *q = (const uint4 *)d_query;
        const uint4 *t = (const uint4 *)d_train;
        int32_t *o = (int32_t *)d_out;
        const int qt = std::min(kn.qt, qb);
        if (qt > 1 || kn.dbg) {  // QT queries per thread (sweeps: OSG_TOP2_QT, OSG_TOP2_DEBUG)
            const int dbg = kn.dbg;
#define OSG_MQ(QB_, QT_)                                                                                       \
    if (qb == QB_ && qt == QT_) {                                                                             \
        hipLaunchKernelGGL((k_top2_qsplit_mq<QB_, QT_>), grid, block, 0, ctx->stream, q, nq, t, nt, o, dbg);   \
        OSG_HIP_CHECK(ctx, hipGetLastError());                                                                 \
        return OSG_OK;                                                                                         \
    }
            OSG_MQ(8, 1) OSG_MQ(8, 2) OSG_MQ(8, 4) OSG_MQ(8, 8)
            OSG_MQ(16, 1) OSG_MQ(16, 2) OSG_MQ(16, 4) OSG_MQ(16, 8)
            OSG_MQ(4, 1) OSG_MQ(4, 2) OSG_MQ(4, 4)
#undef OSG_MQ
        }
        switch (qb) {
        case 64: hipLaunchKernelGGL(k_top2_qsplit<64>, grid, block, 0, ctx->stream, q, nq, t, nt, o); break;
        case 32: hipLaunchKernelGGL(k_top2_qsplit<32>, grid, block, 0, ctx->stream, q, nq, t, nt, o); break;
        case 16: hipLaunchKernelGGL(k_top2_qsplit<16>, grid, block, 0, ctx->stream, q, nq, t, nt, o); break;
        case 8: hipLaunchKernelGGL(k_top2_qsplit<8>, grid, block, 0, ctx->stream, q, nq, t, nt, o); break;
        case 4: hipLaunchKernelGGL(k_top2_qsplit<4>, grid, block, 0, ctx->stream, q, nq, t, nt, o); break;
        case 2: hipLaunchKernelGGL(k_top2_qsplit<2>, grid, block, 0, ctx->stream, q, nq, t, nt, o); break;
        default: hipLaunchKernelGGL(k_top2_qsplit<1>, grid, block, 0, ctx->stream, q, nq, t, nt, o); break;
        }
        OSG_HIP_CHECK(ctx, hipGetLastError());
        return OSG_OK;
    }
    const int waves = kn.waves > 0 ? kn.waves : (nq <= 4096 ? 16 : 8);
    const int WAVES = (waves >= 16) ? 16 : (waves >= 8 ? 8 : 4);
    const int nqb = (nq + 63) / 64;
    OSG_REQUIRE(ctx, nqb <= STREAM_CNT_BASE, "too many queries (%d)", nq);
    const int variant = kn.variant;
    const int dbg = kn.dbg;
    const int target_wg = kn.target_wg;
    const int min_rows = kn.min_rows;
    int G = (target_wg + nqb - 1) / nqb;
    G = std::min(G, std::max(1, nt / min_rows));
    G = std::max(G, (nt + (int)IDX_MASK) / ((int)IDX_MASK + 1)); // chunk-local index fits 23 bits
    if (variant == 2 || variant == 4) G = std::max(G, (nt + TILE_MAX_ROWS - 1) / TILE_MAX_ROWS);
    G = std::max(1, std::min(G, TILE_MAX_G));
    int rpc = (nt + G - 1) / G;
    G = (nt + rpc - 1) / rpc;
    const bool use_stage = (variant == 2 || variant == 4) && rpc <= TILE_MAX_ROWS;
    uint2 *part = nullptr;
    if (G > 1) OSG_ALLOC(ctx, part, SLOT_PART, sizeof(uint2) * (size_t)G * nq);
    const dim3 grid(nqb, G), block(WAVES * 64);
    const uint4 *q = (const uint4 *)d_query;
    const uint32_t *t = (const uint32_t *)d_train;
    int32_t *o = (int32_t *)d_out;
#define OSG_TILE_LAUNCH(W)                                                                                     \
    if (use_stage)                                                                                             \
        hipLaunchKernelGGL((k_top2_tile<W, 1, 1>), grid, block, 0, ctx->stream, q, nq, t, nt, rpc, G, part,   \
                           ctx->counters, o, dbg);                                                            \
    else if (variant == 0)                                                                                     \
        hipLaunchKernelGGL((k_top2_tile<W, 0, 0>), grid, block, 0, ctx->stream, q, nq, t, nt, rpc, G, part,   \
                           ctx->counters, o, dbg);                                                            \
    else                                                                                                       \
        hipLaunchKernelGGL((k_top2_tile<W, 0, 1>), grid, block, 0, ctx->stream, q, nq, t, nt, rpc, G, part,   \
                           ctx->counters, o, dbg);
    if (WAVES == 16) { OSG_TILE_LAUNCH(16) }
    else if (WAVES == 8) { OSG_TILE_LAUNCH(8) }
    else { OSG_TILE_LAUNCH(4) }
#undef OSG_TILE_LAUNCH
    OSG_HIP_CHECK(ctx, hipGetLastError());
    return OSG_OK;
}

extern "C" {

int osg_hamming_top2_plan(osg_ctx *ctx, int32_t nq, int32_t nt, char *name, int32_t len)
{
    if (!ctx || !name || len <= 0) return OSG_E_INVALID;
    const int cus = ctx->num_cus;
    const top2_knobs &kn = knobs(cus);
    char buf[160];
    if (nq <= 0 || nt <= 0) {
        snprintf(buf, sizeof buf, "none");
    } else if (nq <= 8 && nt >= 65536) {
        int G = kn.stream_g, rpb = (nt + G - 1) / G;
        rpb = ((rpb + 1023) / 1024) * 1024;
        snprintf(buf, sizeof buf, "k_top2_stream<%d> grid=%d x 256", nq == 1 ? 1 : nq == 2 ? 2 : nq <= 4 ? 4 : 8,
                 (nt + rpb - 1) / rpb);
    } else if ((kn.variant == 3 || (kn.variant == 2 && nq <= 32 * cus)) && nt <= (int)IDX_MASK) {
        int qb = 64;
        while (qb > 1 && (nq + qb - 1) / qb < kn.qs_wg) qb >>= 1;
        snprintf(buf, sizeof buf, "k_top2_qsplit<%d> grid=%d x 1024", qb, (nq + qb - 1) / qb);
    } else {
        snprintf(buf, sizeof buf, "k_top2_tile (variant %d)", kn.variant);
    }
    snprintf(name, (size_t)len, "%s", buf);
    return OSG_OK;
}

int osg_hamming_top2_dev(osg_ctx *ctx, const void *d_query, int32_t nq, const void *d_train, int32_t nt,
                         void *d_out)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, nq >= 0 && (nq == 0 || (d_query && d_out)) && (nt == 0 || d_train), "null pointer");
    return osg_launch_top2(ctx, d_query, nq, d_train, nt, d_out);
}

int osg_hamming_top2_batch_dev(osg_ctx *ctx, const void *d_query, int32_t nq, const void *d_train, int32_t nt,
                               int32_t nb, void *d_out)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, nq >= 0 && nt >= 0 && nb >= 0, "negative size");
    if (nq == 0 || nb == 0) return OSG_OK;
    OSG_REQUIRE(ctx, d_query && d_out && (nt == 0 || d_train), "null pointer");
    OSG_REQUIRE(ctx, nt <= (int)IDX_MASK, "nt=%d exceeds 2^23 rows per problem", nt);
    OSG_REQUIRE(ctx, nb <= 65535, "nb=%d exceeds 65535 problems per launch", nb);
    if (nt == 0) {
        for (int b = 0; b < nb; b++) {
            const int rc = osg_launch_top2(ctx, (const char *)d_query + (size_t)b * nq * 32, nq, nullptr, 0,
                                           (char *)d_out + (size_t)b * nq * 12);
            if (rc < 0) return rc;
        }
        return OSG_OK;
    }
    // The I8-MFMA form (hamming_mfma.hip) whenever the key's 13-bit row field holds nt;
    // OSG_TOP2_BATCH_MFMA=0 pins the popcount form below (A/B runs, the QL / SCALAR variants).
    static const int mf = getenv("OSG_TOP2_BATCH_MFMA") ? atoi(getenv("OSG_TOP2_BATCH_MFMA")) : 1;
    if (mf && nt <= osg_top2_mfma_max_rows()) return osg_launch_top2_batch_mfma(ctx, d_query, nq, d_train, nt, nb, d_out);
    static const int ql_env = getenv("OSG_TOP2_BATCH_QL") ? atoi(getenv("OSG_TOP2_BATCH_QL")) : 2;
    static const int sc = getenv("OSG_TOP2_BATCH_SCALAR") ? atoi(getenv("OSG_TOP2_BATCH_SCALAR")) : 1;
    const int ql = (ql_env == 1 || ql_env == 4) ? ql_env : 2;
    const dim3 grid((nq + 64 * ql - 1) / (64 * ql), nb), block(1024);
    const uint4 *q = (const uint4 *)d_query, *t = (const uint4 *)d_train;
    int32_t *o = (int32_t *)d_out;
#define OSG_BATCH(QL_, SC_) hipLaunchKernelGGL((k_top2_batch<QL_, SC_>), grid, block, 0, ctx->stream, q, nq, t, nt, o)
    if (sc) {
        if (ql == 1) OSG_BATCH(1, 1);
        else if (ql == 4) OSG_BATCH(4, 1);
        else OSG_BATCH(2, 1);
    } else {
        if (ql == 1) OSG_BATCH(1, 0);
        else if (ql == 4) OSG_BATCH(4, 0);
        else OSG_BATCH(2, 0);
    }
#undef OSG_BATCH
    OSG_HIP_CHECK(ctx, hipGetLastError());
    return OSG_OK;
}

int osg_hamming_top2(osg_ctx *ctx, const uint8_t *query, int32_t nq, const uint8_t *train, int32_t nt,
                     int32_t *best_idx, int32_t *best_dist, int32_t *second_dist)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, nq >= 0 && nt >= 0, "negative size");
    if (nq == 0) return OSG_OK;
    OSG_REQUIRE(ctx, query && best_idx && best_dist && second_dist && (nt == 0 || train), "null pointer");
    void *dq, *dt, *dout;
    OSG_ALLOC(ctx, dq, SLOT_Q, (size_t)nq * 32);
    OSG_ALLOC(ctx, dt, SLOT_T, (size_t)std::max(nt, 1) * 32);
    OSG_ALLOC(ctx, dout, SLOT_OUT, (size_t)nq * 12);
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dq, query, (size_t)nq * 32, hipMemcpyHostToDevice, ctx->stream));
    if (nt > 0) OSG_HIP_CHECK(ctx, hipMemcpyAsync(dt, train, (size_t)nt * 32, hipMemcpyHostToDevice, ctx->stream));
    int rc = osg_launch_top2(ctx, dq, nq, dt, nt, dout);
    if (rc < 0) return rc;
    int32_t *h = (int32_t *)osg_pinned(ctx, (size_t)nq * 12);
    if (!h) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_download(ctx, h, dout, (size_t)nq * 12));
    OSG_RC(osg_wait(ctx));
    for (int i = 0; i < nq; i++) {
        best_idx[i] = h[3 * i];
        best_dist[i] = h[3 * i + 1];
        second_dist[i] = h[3 * i + 2];
    }
    return OSG_OK;
}

int osg_descriptor_distance_pairs(osg_ctx *ctx, const uint8_t *a, const uint8_t *b, int32_t n, int32_t *out)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, n >= 0, "negative size");
    if (n == 0) return OSG_OK;
    OSG_REQUIRE(ctx, a && b && out, "null pointer");
    void *da, *db, *dout;
    OSG_ALLOC(ctx, da, SLOT_Q, (size_t)n * 32);
    OSG_ALLOC(ctx, db, SLOT_T, (size_t)n * 32);
    OSG_ALLOC(ctx, dout, SLOT_OUT, (size_t)n * 4);
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(da, a, (size_t)n * 32, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(db, b, (size_t)n * 32, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_pair_dist, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, (const uint4 *)da,
                       (const uint4 *)db, n, (int32_t *)dout);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_RC(osg_download(ctx, out, dout, (size_t)n * 4));
    OSG_RC(osg_wait(ctx));
    return OSG_OK;
}

}  // extern "C"
