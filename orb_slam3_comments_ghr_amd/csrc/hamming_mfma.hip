// hamming_mfma.hip — frame-batched brute-force top-2 on the I8 matrix cores (gfx950).
//
// Same semantics as k_top2_batch (hamming.hip) and the reference's candidate loop
// (ref:src/ORBmatcher.cc:327-355 over DescriptorDistance, :2388-2408): per query the smallest
// distance with the first index among ties, the second smallest distance counted with
// multiplicity, and a distance of 256 never entering (index -1).
//
// Distance as a dot product.  Every descriptor bit becomes one signed byte: a query bit is +64
// when set and -64 when clear, a train bit -128 when set and 0 when clear.  Summed over the 256 bits
// (|q| = popcount of the query, |t| of the train row, a = |q & t|):
//     sum_k q_k t_k = -128 * 64 * (a - (|t| - a)) = 8192 * (|q| + |t| - 2 a - |q|) = 8192 * (H - |q|),
// exact in the i32 accumulator of v_mfma_i32_32x32x32_i8.  |q| is the same for every train row of a
// query, so with the train row's offset inside its 32-row tile as the MFMA's C input, the
// accumulator comes out as a ready packed key
//     key = (H - |q|) << 13 | row          (row < 8192; smaller key = smaller H, then lower row)
// and the top-2 update is 1.5 VALU ops per (query, row): two keys at a time, k1 = min3(k1, x, y),
// k2 = min(med3(k1, x, y), k2).
// The 19 VALU ops per pair of the popcount form (8 xor, 8 bcnt, shift-or, min, med3) become the
// MFMA plus those.  Keys stay relative to the current tile: after each 32-row tile the kept
// keys drop by 32 (the same shift for every key, so the order is kept), and the base is added
// back once at the end.
//
// Layout (C/D map of the 32x32 MFMAs on gfx950, dtype-independent): lane l holds column
// n = l & 31 and rows (i & 3) + 8 (i >> 2) + 4 (l >> 5) in accumulator element i.  Queries are the
// columns (B operand), train rows the rows (A operand), so a lane owns one query and 16 of the
// tile's rows; the two lane halves merge once at the end.  K-step s (32 bits) of lane half h
// carries descriptor bits 32 s + 16 h .. + 15 on both operands (tools/micro/mfma_i8.hip probes the
// operand maps: A and B place the same k in the same lane half and byte).
//
// Data movement: one workgroup = NW waves x QT query tiles of 32 queries of one problem.  Train
// rows are expanded (32 B -> 256 B of signed bytes) once per workgroup into LDS chunks of CR rows
// through a 256-entry byte -> 8-byte table in LDS, double-buffered: while the waves multiply chunk
// c, the packed rows of chunk c + 1 are already in registers, and are expanded into the other
// buffer after the chunk's MFMAs.  LDS rows are 256 B of signed bytes padded to 272 B (MF_RS): the
// 16 rows that one ds_read_b128 of a lane half reads at one granule column then start 16 B apart
// modulo the 256-B bank window and land on 16 distinct 16-B bank groups.
//
// Full chunks run as one branch-free block pipelined by hand (PIPE = 1): K-step s of tile t issues
// its MFMAs, refills the A register it consumed with tile t + 1's granule, and performs pair s of
// tile t - 1's top-2 update, with sched_barrier keeping that order.  Measured: 182.6 us per 256 x
// 2000^2 launch, 0.57 of the I8 dense peak; the same MFMA chains alone run at 0.72 of it
// (tools/micro/mfma_i8_rate.hip: the chip holds 18.6 ns per 32x32x32 MFMA per SIMD, not 13.3).
#include <algorithm>
#include <cstdlib>

#include "osg_internal.h"

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int MF_SHIFT = 13;                       // key = (H - |q|) << 13 | row
constexpr int MF_MAX_ROWS = 1 << MF_SHIFT;         // rows per problem on this path
constexpr int MF_PAD = 1 << 30;                    // rows past nt: above every real key
constexpr int MF_RS = 272;                         // LDS row stride: 256 B of signed bytes + 16 B pad

// The median written as max(min(a, b), min(max(a, b), c)), which the backend selects as one
// v_med3_i32.  Not inline asm: its operands are MFMA results, and the compiler's MFMA -> VALU
// read hazard handling does not see inside an asm statement (an asm med3 read stale accumulators
// in ~1 % of the second distances on the GPU).
__device__ __forceinline__ int med3_i32(int a, int b, int c)
{
    return max(min(a, b), min(max(a, b), c));
}

// 4 query bits -> 4 signed bytes: bit y -> byte y = +64 (0x40) set, -64 (0xC0) clear.
// n * 0x204081 & 0x01010101 moves bit y to bit 8 y (the four shifted copies do not overlap);
// 0x80 - that bit per byte keeps bit 7 iff the bit is clear.
__device__ __forceinline__ uint32_t spread_query(uint32_t nib)
{
    const uint32_t s = __umul24(nib, 0x204081u) & 0x01010101u;
    return ((0x80808080u - s) & 0x80808080u) | 0x40404040u;
}

__device__ __forceinline__ void key_push(int &k1, int &k2, int key)
{
    k2 = med3_i32(k1, key, k2);
    k1 = min(k1, key);
}

// Two keys at once: with k1 <= k2 and S = {k1, x, y}, the smallest of S u {k2} is min3(k1, x, y) and
// the second is min(med3(k1, x, y), k2) (k2 >= k1 cannot be the strict smallest): 3 VALU for two
// keys (v_min3_i32, v_med3_i32, v_min_i32) instead of 4.
__device__ __forceinline__ void key_push2(int &k1, int &k2, int x, int y)
{
    const int m = med3_i32(k1, x, y);
    k1 = min(min(k1, x), y);
    k2 = min(m, k2);
}

// key_push2 for the FP4 path, whose keys are the bit patterns of positive normal floats (MX_BIAS, MX_KEY0
// below): their float order is their integer order, so the median is taken as v_med3_f32 on the same bits.
// Written this way the compiler selects one v_med3_f32 and one v_min3_i32 per pair and merges the k2 chain
// into v_min3_i32 (22 VALU ops per 32-row tile against 30 for key_push2, whose med3 and min3 patterns share
// the min(k1, x) node so that half the k1 updates become two v_min_i32).  Not for the I8 path: its keys can
// be negative integers.
__device__ __forceinline__ void key_push2f(int &k1, int &k2, int x, int y)
{
    const int m = __float_as_int(__builtin_amdgcn_fmed3f(__int_as_float(k1), __int_as_float(x), __int_as_float(y)));
    k1 = min(min(x, y), k1);
    k2 = min(m, k2);
}

__device__ __forceinline__ void key_merge(int &k1, int &k2, int a1, int a2)
{
    const int hi = max(k1, a1);
    k1 = min(k1, a1);
    k2 = min(min(k2, a2), hi);
}

template <int NW, int QT, int CR, int PIPE>
__global__ __launch_bounds__(NW * 64) void k_top2_mfma(const uint32_t *__restrict__ query, int nq,
                                                        const uint32_t *__restrict__ train, int nt,
                                                        int nqb, int32_t *__restrict__ out)
{
    constexpr int NT = NW * 64;
    constexpr int BPT = CR * 32 / NT;        // packed bytes per thread per chunk
    constexpr int WPT = BPT / 4;             // packed words per thread
    constexpr int TPR = 32 / BPT;            // threads per row
    constexpr int NTILE = CR / 32;           // 32-row tiles per chunk
    static_assert(CR * 32 % NT == 0 && BPT % 4 == 0 && TPR >= 1, "chunk / workgroup shape");
    __shared__ __attribute__((aligned(16))) unsigned char s_buf[2 * CR * MF_RS];   // [2][CR rows][272 B]
    __shared__ uint2 s_lut[256];             // train byte -> 8 signed bytes (bit y -> byte y: -128 / 0)

    const int t = threadIdx.x, lane = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    // XCD-aware numbering: consecutive logical blocks (the nqb blocks of one problem, which share
    // its train rows) land on one XCD when the grid is a multiple of 8.
    const int G = gridDim.x, L = blockIdx.x;
    const int logical = (G % 8 == 0) ? (L % 8) * (G / 8) + L / 8 : L;
    const int b = logical / nqb, qb = logical % nqb;
    const uint32_t *qf = query + (size_t)b * nq * 8;
    const uint32_t *tf = train + (size_t)b * nt * 8;
    int32_t *of = out + (size_t)b * nq * 3;

    for (int e = t; e < 256; e += NT) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int y = 0; y < 4; y++) {
            lo |= ((e >> y) & 1u) << (8 * y + 7);
            hi |= ((e >> (y + 4)) & 1u) << (8 * y + 7);
        }
        s_lut[e] = make_uint2(lo, hi);
    }

    const int r = lane & 31, h = lane >> 5;
    const int qw0 = qb * (NW * QT * 32) + w * (QT * 32);   // first query of this wave
    const bool active = qw0 < nq;                            // wave-uniform

    // B fragments: the wave's queries, expanded once.  Each query keeps two running top-2 pairs
    // (accumulator elements 0-7 and 8-15: two independent dependency chains), merged at the end;
    // both start at the sentinel key (H = 256, row 0).
    i32x4 bq[QT][8];
    int ka1[QT], ka2[QT], kb1[QT], kb2[QT], pq[QT];
#pragma unroll
    for (int j = 0; j < QT; j++) {
        const int q = min(qw0 + 32 * j + r, nq - 1);
        const uint4 lo = *(const uint4 *)(qf + (size_t)q * 8), hi = *(const uint4 *)(qf + (size_t)q * 8 + 4);
        const uint32_t wd[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        int pc = 0;
#pragma unroll
        for (int s = 0; s < 8; s++) {
            pc += __popc(wd[s]);
            const uint32_t hw = h ? (wd[s] >> 16) : (wd[s] & 0xFFFFu);
#pragma unroll
            for (int d = 0; d < 4; d++) bq[j][s][d] = (int)spread_query((hw >> (4 * d)) & 0xFu);
        }
        pq[j] = pc;
        ka1[j] = ka2[j] = kb1[j] = kb2[j] = (256 - pc) << MF_SHIFT;
    }
    // C input: the accumulator element's row inside the tile
    i32x16 crow;
#pragma unroll
    for (int i = 0; i < 16; i++) crow[i] = (i & 3) + 8 * (i >> 2) + 4 * h;
    // this lane's A granule of K-step s in a tile: row r, granule 2 s + h, at lbase + 32 s
    const int lbase = r * MF_RS + h * 16;

    // expansion of one chunk's packed rows: this thread's WPT words of row erow
    const int erow = t / TPR, epart = t % TPR;
    auto load_chunk = [&](int c0, uint32_t (&pw)[WPT]) {
        const int row = c0 + erow;
        if (row < nt) {
            const uint32_t *src = tf + (size_t)row * 8 + epart * WPT;
#pragma unroll
            for (int i = 0; i < WPT; i += 2) {
                const uint2 v = *(const uint2 *)(src + i);
                pw[i] = v.x;
                pw[i + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int i = 0; i < WPT; i++) pw[i] = 0u;   // expands to zero bytes: D = C exactly
        }
    };
    auto store_chunk = [&](int buf, const uint32_t (&pw)[WPT]) {
        unsigned char *dst = s_buf + ((size_t)buf * CR + erow) * MF_RS;
#pragma unroll
        for (int i = 0; i < WPT; i++) {
#pragma unroll
            for (int hh = 0; hh < 2; hh++) {    // granule = halfword hh of word (epart WPT + i)
                const int g = 2 * (epart * WPT + i) + hh;
                const uint2 v0 = s_lut[(pw[i] >> (16 * hh)) & 0xFFu];
                const uint2 v1 = s_lut[(pw[i] >> (16 * hh + 8)) & 0xFFu];
                *(i32x4 *)(dst + 16 * g) = i32x4{(int)v0.x, (int)v0.y, (int)v1.x, (int)v1.y};
            }
        }
    };

    auto frag = [&](const unsigned char *tb, int s) -> i32x4 { return *(const i32x4 *)(tb + lbase + 32 * s); };
    auto mfma = [&](const i32x4 &a, const i32x4 &bb, const i32x16 &c) {
        return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bb, c, 0, 0, 0);
    };
    // top-2 update of the wave's queries with one tile's accumulators, then the tile-base shift
    auto epi = [&](const i32x16 (&acc)[QT]) {
#pragma unroll
        for (int j = 0; j < QT; j++) {
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                key_push2(ka1[j], ka2[j], acc[j][i], acc[j][i + 1]);
                key_push2(kb1[j], kb2[j], acc[j][i + 8], acc[j][i + 9]);
            }
            ka1[j] -= 32;
            ka2[j] -= 32;
            kb1[j] -= 32;
            kb2[j] -= 32;
        }
    };
    // one tile, unpipelined: 8 K-steps of MFMA, then the update (partial chunks, the last tile)
    auto tile = [&](const unsigned char *tb, const i32x16 &cin) {
        i32x4 a[8];
#pragma unroll
        for (int s = 0; s < 8; s++) a[s] = frag(tb, s);
        i32x16 acc[QT];
#pragma unroll
        for (int j = 0; j < QT; j++) acc[j] = mfma(a[0], bq[j][0], cin);
#pragma unroll
        for (int s = 1; s < 8; s++)
#pragma unroll
            for (int j = 0; j < QT; j++) acc[j] = mfma(a[s], bq[j][s], acc[j]);
        epi(acc);
    };

    const int nch = (nt + CR - 1) / CR;
    {
        uint32_t pw[WPT];
        load_chunk(0, pw);
        __syncthreads();   // the table
        store_chunk(0, pw);
    }
    __syncthreads();
    for (int c = 0; c < nch; c++) {
        const int c0 = c * CR;
        uint32_t pw[WPT];
        const bool more = c + 1 < nch;
        if (more) load_chunk(c0 + CR, pw);
        if (active) {
            const unsigned char *sb = s_buf + (size_t)(c & 1) * CR * MF_RS;
            // full tiles with the plain row offsets; the one partial tile of the problem (its last)
            // separately, with rows past nt lifted above every real key
            const int nfull = min(NTILE, (nt - c0) / 32);
            if (PIPE && nfull == NTILE) {
                // A whole chunk as one branch-free block, software-pipelined by hand: K-step s of
                // tile t issues its QT MFMAs, refills the A register it just consumed with tile
                // t + 1's granule (8 MFMAs of latency cover that LDS read), and performs element s of
                // each of the two running top-2 chains for tile t - 1's accumulators (4 QT VALU in
                // the MFMAs' shadow).  sched_barrier keeps each step's instructions in this order.
                i32x4 a[8];
                i32x16 accp[QT], acc[QT];
#pragma unroll
                for (int s = 0; s < 8; s++) a[s] = frag(sb, s);
#pragma unroll
                for (int s = 0; s < 8; s++) {
#pragma unroll
                    for (int j = 0; j < QT; j++) accp[j] = mfma(a[s], bq[j][s], s ? accp[j] : crow);
                    a[s] = frag(sb + 32 * MF_RS, s);
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int tt = 1; tt < NTILE; tt++) {
#pragma unroll
                    for (int s = 0; s < 8; s++) {
#pragma unroll
                        for (int j = 0; j < QT; j++) acc[j] = mfma(a[s], bq[j][s], s ? acc[j] : crow);
                        if (tt + 1 < NTILE) a[s] = frag(sb + (tt + 1) * 32 * MF_RS, s);
#pragma unroll
                        for (int j = 0; j < QT; j++) {
                            // pair s of the tile's 8 key pairs: chain A elements 0-7, chain B 8-15
                            if (s & 1)
                                key_push2(kb1[j], kb2[j], accp[j][8 + (s & 6)], accp[j][9 + (s & 6)]);
                            else
                                key_push2(ka1[j], ka2[j], accp[j][s & 6], accp[j][1 + (s & 6)]);
                            if (s == 7) {
                                ka1[j] -= 32;
                                ka2[j] -= 32;
                                kb1[j] -= 32;
                                kb2[j] -= 32;
                            }
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
#pragma unroll
                    for (int j = 0; j < QT; j++) accp[j] = acc[j];
                }
                epi(accp);
            } else {
#pragma unroll
                for (int tt = 0; tt < NTILE; tt++) {
                    if (tt >= nfull) break;
                    tile(sb + tt * 32 * MF_RS, crow);
                }
            }
            const int lim = nt - (c0 + nfull * 32);   // rows of a partial tile (< 32 when there is one)
            if (nfull < NTILE && lim > 0) {
                i32x16 cin;
#pragma unroll
                for (int i = 0; i < 16; i++) cin[i] = crow[i] + (crow[i] >= lim ? MF_PAD : 0);
                tile(sb + nfull * 32 * MF_RS, cin);
            }
        }
        if (more) store_chunk((c + 1) & 1, pw);
        __syncthreads();
    }
    if (!active) return;
    const int base = 32 * ((nt + 31) / 32);   // the keys are relative to one tile past the last
#pragma unroll
    for (int j = 0; j < QT; j++) {
        int k1 = ka1[j], k2 = ka2[j];
        key_merge(k1, k2, kb1[j], kb2[j]);
        const int a1 = __shfl_xor(k1, 32), a2 = __shfl_xor(k2, 32);
        key_merge(k1, k2, a1, a2);
        const int q = qw0 + 32 * j + r;
        if (h == 0 && q < nq) {
            const int t1 = k1 + base, t2 = k2 + base;
            const int d1 = (t1 >> MF_SHIFT) + pq[j], d2 = (t2 >> MF_SHIFT) + pq[j];
            of[3 * q + 0] = d1 < 256 ? (t1 & (MF_MAX_ROWS - 1)) : -1;
            of[3 * q + 1] = min(d1, 256);
            of[3 * q + 2] = min(d2, 256);
        }
    }
}

// ---- FP4 (e2m1) block-scaled form -------------------------------------------------------------
// The same keys from v_mfma_scale_f32_32x32x64_f8f6f4 with FP4 operands (cbsz = blgp = 4): a query
// bit is +1 (set) or -1 (clear), a train bit -2 (set) or 0 (clear), so
//     sum_k q_k t_k = -2 (a - (|t| - a)) = 2 (H - |q|),
// and the train operand's E8M0 block scale 2^12 makes it 8192 (H - |q|): the i8 path's key, exact in
// the f32 accumulator (every product and partial sum is an integer multiple of 4096 of magnitude below
// 2^22, plus the row < 2^13 from C), so the summation order inside the instruction cannot round.
// C carries the bias 2^23 + 2^21 (plus the row in the tile), so every key the instruction produces lies in
// [2^23, 2^24), the f32 binade whose ulp is 1: there the bit pattern is 0x4B000000 + (value - 2^23), an
// affine map of the integer key.  The epilogue therefore runs on the bit patterns with the i8 path's
// integer v_min3 / v_med3 / rebasing ops (as floats, fminf / fmaxf each cost a canonicalising v_max_f32
// and the median no single instruction: 14 VALU ops per MFMA instead of 7).
// K = 64 bits per instruction at the cycles of the i8 form's K = 32 (MI355X_MICROARCH.md "Matrix cores":
// FP4 runs at 4x the BF16 rate per clock, I8 at 2x): 4 MFMAs per 32-row tile instead of 8, and an
// expanded train row is 128 B (one nibble per bit) instead of 256.
// Operand map: lane l carries row (A) / column (B) l & 31 and the K nibbles 32 (l >> 5) + j, j = 0..31,
// nibble j at bit 4 (j & 7) of register j >> 3; K-step s of lane half h carries descriptor word 2 s + h on
// both sides.  A dot product is unchanged by any K permutation applied to both operands alike, so the
// exact-data probe (tools/micro/mfma_fp4_layout.hip, profiles/r05_mfma_fp4_layout.txt) passes for every
// consistent map it tried; what it pins is the e2m1 codes, the E8M0 scaling and the C / D map.
constexpr int MX_RS = 144;                  // LDS row stride: 128 B of nibbles + 16 B pad (16 distinct banks)
constexpr int MX_SCALE_TRAIN = 127 + 12;    // E8M0 2^12 on the train operand
constexpr int MX_SCALE_ONE = 127;           // E8M0 1.0
constexpr float MX_BIAS = 10485760.0f;      // 2^23 + 2^21: keys of [-2^21, 2^21 + 32) land in [2^23, 2^24)
constexpr int MX_KEY0 = 0x4B000000 + (1 << 21);   // bit pattern of MX_BIAS: bits = key + MX_KEY0
constexpr float MX_PAD = 1073741824.0f;     // rows past nt: above every real key (2^30)

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// 8 bits -> bit y at bit 4 y
__device__ __forceinline__ uint32_t spread_nib(uint32_t x)
{
    x &= 0xFFu;
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    return (x | (x << 3)) & 0x11111111u;
}

template <int NW, int QT, int CR, int PIPE>
__global__ __launch_bounds__(NW * 64) void k_top2_fp4(const uint32_t *__restrict__ query, int nq,
                                                       const uint32_t *__restrict__ train, int nt,
                                                       int nqb, int32_t *__restrict__ out)
{
    constexpr int NT = NW * 64;
    constexpr int BPT = CR * 32 / NT;        // packed bytes per thread per chunk
    constexpr int WPT = BPT / 4;             // packed words per thread
    constexpr int TPR = 32 / BPT;            // threads per row
    constexpr int NTILE = CR / 32;           // 32-row tiles per chunk
    static_assert(CR * 32 % NT == 0 && BPT % 4 == 0 && TPR >= 1, "chunk / workgroup shape");
    __shared__ __attribute__((aligned(16))) unsigned char s_buf[2 * CR * MX_RS];   // [2][CR rows][144 B]
    __shared__ uint32_t s_lut[256];          // train byte -> 8 nibbles (bit y -> nibble y: 0xC = -2 / 0)

    const int t = threadIdx.x, lane = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int G = gridDim.x, L = blockIdx.x;
    const int logical = (G % 8 == 0) ? (L % 8) * (G / 8) + L / 8 : L;
    const int b = logical / nqb, qb = logical % nqb;
    const uint32_t *qf = query + (size_t)b * nq * 8;
    const uint32_t *tf = train + (size_t)b * nt * 8;
    int32_t *of = out + (size_t)b * nq * 3;

    for (int e = t; e < 256; e += NT) s_lut[e] = spread_nib((uint32_t)e) * 0xCu;

    const int r = lane & 31, h = lane >> 5;
    const int qw0 = qb * (NW * QT * 32) + w * (QT * 32);
    const bool active = qw0 < nq;

    // B fragments (the wave's queries, K-step s = descriptor word 2 s + h) and two running top-2
    // pairs per query (accumulator elements 0-7 and 8-15)
    i32x8 bq[QT][4];
    int ka1[QT], ka2[QT], kb1[QT], kb2[QT];
    // PIPE == 3 (the default shape): one running top-2 pair per query (both accumulator halves into ka):
    // two fewer rebasing subtractions per tile and no merge of the halves, a longer dependent chain per
    // lane; 852 -> 841 VALU ops, +1.8 % on the headline step (profiles/r05_top2_fp4_onechain.jsonl).
    // The two-pair form stays as OSG_TOP2_MFMA_SHAPE=7.
    constexpr bool ONE = PIPE == 3 || PIPE == 4 || PIPE == 5;
    // PIPE == 5: PIPE 3, and a chunk with fewer full tiles (the last one) also runs the pipelined block,
    // leaving it after its last full tile, instead of one unpipelined tile() per full tile
    constexpr bool PART = PIPE == 5;
    int(&kc1)[QT] = ONE ? ka1 : kb1;
    int(&kc2)[QT] = ONE ? ka2 : kb2;
    int pq[QT];
#pragma unroll
    for (int j = 0; j < QT; j++) {
        const int q = min(qw0 + 32 * j + r, nq - 1);
        const uint4 lo = *(const uint4 *)(qf + (size_t)q * 8), hi = *(const uint4 *)(qf + (size_t)q * 8 + 4);
        const uint32_t wd[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        int pc = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) pc += __popc(wd[k]);
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const uint32_t word = wd[2 * s + h];
#pragma unroll
            for (int d = 0; d < 4; d++)
                bq[j][s][d] = (int)(0x22222222u | ((~spread_nib(word >> (8 * d)) & 0x11111111u) << 3));
#pragma unroll
            for (int d = 4; d < 8; d++) bq[j][s][d] = 0;
        }
        pq[j] = pc;
        ka1[j] = ka2[j] = kb1[j] = kb2[j] = ((256 - pc) << MF_SHIFT) + MX_KEY0;
    }
    f32x16 crow;
#pragma unroll
    for (int i = 0; i < 16; i++) crow[i] = MX_BIAS + (float)((i & 3) + 8 * (i >> 2) + 4 * h);
    const int lbase = r * MX_RS + h * 16;

    const int erow = t / TPR, epart = t % TPR;
    auto load_chunk = [&](int c0, uint32_t (&pw)[WPT]) {
        const int row = c0 + erow;
        if (row < nt) {
            const uint32_t *src = tf + (size_t)row * 8 + epart * WPT;
#pragma unroll
            for (int i = 0; i < WPT; i += 2) {
                const uint2 v = *(const uint2 *)(src + i);
                pw[i] = v.x;
                pw[i + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int i = 0; i < WPT; i++) pw[i] = 0u;   // expands to zero nibbles: D = C exactly
        }
    };
    auto store_chunk = [&](int buf, const uint32_t (&pw)[WPT]) {
        unsigned char *dst = s_buf + ((size_t)buf * CR + erow) * MX_RS;
#pragma unroll
        for (int i = 0; i < WPT; i++) {
            const uint32_t x = pw[i];
            *(i32x4 *)(dst + 16 * (epart * WPT + i)) =
                i32x4{(int)s_lut[x & 0xFFu], (int)s_lut[(x >> 8) & 0xFFu], (int)s_lut[(x >> 16) & 0xFFu],
                      (int)s_lut[x >> 24]};
        }
    };

    auto frag = [&](const unsigned char *tb, int s) -> i32x8 {
        const i32x4 v = *(const i32x4 *)(tb + lbase + 32 * s);
        return i32x8{v[0], v[1], v[2], v[3], 0, 0, 0, 0};
    };
    auto mfma = [&](const i32x8 &a, const i32x8 &bb, const f32x16 &c) {
        return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, bb, c, 4, 4, 0, MX_SCALE_TRAIN, 0, MX_SCALE_ONE);
    };
    auto epi = [&](const f32x16 (&acc)[QT]) {
#pragma unroll
        for (int j = 0; j < QT; j++) {
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                key_push2f(ka1[j], ka2[j], __float_as_int(acc[j][i]), __float_as_int(acc[j][i + 1]));
                key_push2f(kc1[j], kc2[j], __float_as_int(acc[j][i + 8]), __float_as_int(acc[j][i + 9]));
            }
            ka1[j] -= 32;
            ka2[j] -= 32;
            if (!ONE) {
                kb1[j] -= 32;
                kb2[j] -= 32;
            }
        }
    };
    auto tile = [&](const unsigned char *tb, const f32x16 &cin) {
        i32x8 a[4];
#pragma unroll
        for (int s = 0; s < 4; s++) a[s] = frag(tb, s);
        f32x16 acc[QT];
#pragma unroll
        for (int j = 0; j < QT; j++) acc[j] = mfma(a[0], bq[j][0], cin);
#pragma unroll
        for (int s = 1; s < 4; s++)
#pragma unroll
            for (int j = 0; j < QT; j++) acc[j] = mfma(a[s], bq[j][s], acc[j]);
        epi(acc);
    };

    const int nch = (nt + CR - 1) / CR;
    {
        uint32_t pw[WPT];
        load_chunk(0, pw);
        __syncthreads();   // the table
        store_chunk(0, pw);
    }
    __syncthreads();
    for (int c = 0; c < nch; c++) {
        const int c0 = c * CR;
        uint32_t pw[WPT];
        const bool more = c + 1 < nch;
        if (more) load_chunk(c0 + CR, pw);
        if (active) {
            const unsigned char *sb = s_buf + (size_t)(c & 1) * CR * MX_RS;
            const int nfull = min(NTILE, (nt - c0) / 32);
            if (PIPE && (nfull == NTILE || (PART && nfull >= 1))) {
                // K-step s of tile t issues its MFMAs, refills the A register it consumed with tile
                // t + 1's granule, and performs key pairs 2 s, 2 s + 1 of tile t - 1 (as k_top2_mfma)
                i32x8 a[4];
                f32x16 accp[QT], acc[QT];
#pragma unroll
                for (int s = 0; s < 4; s++) a[s] = frag(sb, s);
#pragma unroll
                for (int s = 0; s < 4; s++) {
#pragma unroll
                    for (int j = 0; j < QT; j++) accp[j] = mfma(a[s], bq[j][s], s ? accp[j] : crow);
                    a[s] = frag(sb + 32 * MX_RS, s);
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int tt = 1; tt < NTILE; tt++) {
                    if (PART && tt >= nfull) break;  // accp holds the last full tile (epi below)
#pragma unroll
                    for (int s = 0; s < 4; s++) {
#pragma unroll
                        for (int j = 0; j < QT; j++) acc[j] = mfma(a[s], bq[j][s], s ? acc[j] : crow);
                        if (tt + 1 < NTILE) a[s] = frag(sb + (tt + 1) * 32 * MX_RS, s);
                        if (PIPE == 4) {
                            // the skip test: once a query's running pair has settled, a tile rarely holds a key
                            // below its second key (a 32-row tile of random descriptors beats k2 in ~1 of 4
                            // wave tiles at 2000 rows).  At K-step 1 (tile tt - 1's last MFMA has completed)
                            // every lane takes the min of its 16 keys (8 VALU ops); only if some lane of the
                            // wave has a key below its k2 does the wave run the 24-op update.  Keys are unique
                            // (the row is in the key), so a tile whose minimum is above k2 changes neither k1
                            // nor k2: the result is the update's, bit for bit.
                            if (s == 1) {
                                bool need = false;
#pragma unroll
                                for (int j = 0; j < QT; j++) {
                                    int m = __float_as_int(accp[j][0]);
#pragma unroll
                                    for (int e = 1; e < 16; e += 2)
                                        m = min(min(m, __float_as_int(accp[j][e])),
                                                __float_as_int(accp[j][e + 1 < 16 ? e + 1 : e]));
                                    need |= m < ka2[j];
                                }
                                if (__builtin_amdgcn_ballot_w64(need) != 0) {
#pragma unroll
                                    for (int j = 0; j < QT; j++)
#pragma unroll
                                        for (int e = 0; e < 16; e += 2)
                                            key_push2f(ka1[j], ka2[j], __float_as_int(accp[j][e]),
                                                      __float_as_int(accp[j][e + 1]));
                                }
#pragma unroll
                                for (int j = 0; j < QT; j++) {
                                    ka1[j] -= 32;
                                    ka2[j] -= 32;
                                }
                            }
                            __builtin_amdgcn_sched_barrier(0);
                            continue;
                        }
#pragma unroll
                        for (int j = 0; j < QT; j++) {
                            if (PIPE == 2) {
                                // key pairs of tile tt - 1 from K-step 1 on: its last MFMA (issued just before
                                // this tile's first) has completed once this tile's second one issues, so the
                                // reads never wait on it (tools/micro/mfma_fp4_rate.hip: the update overlaps
                                // the chains when it reads no fresh MFMA result).  Pairs p = 0..7 (chain A
                                // pair p, then chain B pair p - 4) as 3 / 3 / 2 over steps 1..3.
#pragma unroll
                                for (int p = 0; p < 8; p++) {
                                    if (p / 3 + 1 != s) continue;
                                    const int e = (p & 3) * 2 + (p >> 2) * 8;
                                    if (p < 4) key_push2f(ka1[j], ka2[j], __float_as_int(accp[j][e]), __float_as_int(accp[j][e + 1]));
                                    else key_push2f(kb1[j], kb2[j], __float_as_int(accp[j][e]), __float_as_int(accp[j][e + 1]));
                                }
                            } else {
                                // pairs 2 s (chain A: elements 4 s, 4 s + 1 ... ) and 2 s + 1 (chain B)
                                key_push2f(ka1[j], ka2[j], __float_as_int(accp[j][2 * s]),
                                          __float_as_int(accp[j][2 * s + 1]));
                                key_push2f(kc1[j], kc2[j], __float_as_int(accp[j][8 + 2 * s]),
                                          __float_as_int(accp[j][9 + 2 * s]));
                            }
                            if (s == 3) {
                                ka1[j] -= 32;
                                ka2[j] -= 32;
                                if (!ONE) {
                                    kb1[j] -= 32;
                                    kb2[j] -= 32;
                                }
                            }
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
#pragma unroll
                    for (int j = 0; j < QT; j++) accp[j] = acc[j];
                }
                epi(accp);
            } else {
#pragma unroll
                for (int tt = 0; tt < NTILE; tt++) {
                    if (tt >= nfull) break;
                    tile(sb + tt * 32 * MX_RS, crow);
                }
            }
            const int lim = nt - (c0 + nfull * 32);
            if (nfull < NTILE && lim > 0) {
                f32x16 cin;
#pragma unroll
                for (int i = 0; i < 16; i++)
                    cin[i] = crow[i] + ((i & 3) + 8 * (i >> 2) + 4 * h >= lim ? MX_PAD : 0.f);
                tile(sb + nfull * 32 * MX_RS, cin);
            }
        }
        if (more) store_chunk((c + 1) & 1, pw);
        __syncthreads();
    }
    if (!active) return;
    const int base = 32 * ((nt + 31) / 32);
#pragma unroll
    for (int j = 0; j < QT; j++) {
        int k1 = ka1[j], k2 = ka2[j];
        if (!ONE) key_merge(k1, k2, kb1[j], kb2[j]);
        const int a1 = __shfl_xor(k1, 32), a2 = __shfl_xor(k2, 32);
        key_merge(k1, k2, a1, a2);
        const int q = qw0 + 32 * j + r;
        if (h == 0 && q < nq) {
            const int t1 = k1 - MX_KEY0 + base, t2 = k2 - MX_KEY0 + base;
            const int d1 = (t1 >> MF_SHIFT) + pq[j], d2 = (t2 >> MF_SHIFT) + pq[j];
            of[3 * q + 0] = d1 < 256 ? (t1 & (MF_MAX_ROWS - 1)) : -1;
            of[3 * q + 1] = min(d1, 256);
            of[3 * q + 2] = min(d2, 256);
        }
    }
}

// The PIPE 3 kernel, persistent (OSG_TOP2_MFMA_SHAPE=13, A/B): one workgroup per CU takes items (frame,
// query block) item = blockIdx.x, + gridDim.x, ... (the same XCD-aware item -> (frame, block) map), keeps the
// byte table, and loads the next item's first train chunk during the current item's last chunk, so the per
// item start (table, first chunk, its barrier) is not paid 16 times per CU.  The same products and key
// updates in the same order as k_top2_fp4<.., 3>: bit-exact.
template <int NW, int QT, int CR>
__global__ __launch_bounds__(NW * 64) void k_top2_fp4p(const uint32_t *__restrict__ query, int nq,
                                                        const uint32_t *__restrict__ train, int nt,
                                                        int nqb, int n_items, int32_t *__restrict__ out)
{
    constexpr int NT = NW * 64;
    constexpr int BPT = CR * 32 / NT;
    constexpr int WPT = BPT / 4;
    constexpr int TPR = 32 / BPT;
    constexpr int NTILE = CR / 32;
    static_assert(CR * 32 % NT == 0 && BPT % 4 == 0 && TPR >= 1, "chunk / workgroup shape");
    __shared__ __attribute__((aligned(16))) unsigned char s_buf[2 * CR * MX_RS];
    __shared__ uint32_t s_lut[256];

    const int t = threadIdx.x, lane = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int G = gridDim.x;
    auto logical_of = [&](int item) { return (n_items % 8 == 0) ? (item % 8) * (n_items / 8) + item / 8 : item; };
    int item = blockIdx.x;
    if (item >= n_items) return;  // the whole workgroup
    for (int e = t; e < 256; e += NT) s_lut[e] = spread_nib((uint32_t)e) * 0xCu;
    const int r = lane & 31, h = lane >> 5;
    const int lbase = r * MX_RS + h * 16;
    const int erow = t / TPR, epart = t % TPR;
    auto load_chunk = [&](const uint32_t *tfp, int c0, uint32_t (&pw)[WPT]) {
        const int row = c0 + erow;
        if (row < nt) {
            const uint32_t *src = tfp + (size_t)row * 8 + epart * WPT;
#pragma unroll
            for (int i = 0; i < WPT; i += 2) {
                const uint2 v = *(const uint2 *)(src + i);
                pw[i] = v.x;
                pw[i + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int i = 0; i < WPT; i++) pw[i] = 0u;
        }
    };
    auto store_chunk = [&](int buf, const uint32_t (&pw)[WPT]) {
        unsigned char *dst = s_buf + ((size_t)buf * CR + erow) * MX_RS;
#pragma unroll
        for (int i = 0; i < WPT; i++) {
            const uint32_t x = pw[i];
            *(i32x4 *)(dst + 16 * (epart * WPT + i)) =
                i32x4{(int)s_lut[x & 0xFFu], (int)s_lut[(x >> 8) & 0xFFu], (int)s_lut[(x >> 16) & 0xFFu],
                      (int)s_lut[x >> 24]};
        }
    };
    auto frag = [&](const unsigned char *tb, int s) -> i32x8 {
        const i32x4 v = *(const i32x4 *)(tb + lbase + 32 * s);
        return i32x8{v[0], v[1], v[2], v[3], 0, 0, 0, 0};
    };
    auto mfma = [&](const i32x8 &a, const i32x8 &bb, const f32x16 &c) {
        return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, bb, c, 4, 4, 0, MX_SCALE_TRAIN, 0, MX_SCALE_ONE);
    };
    const int nch = (nt + CR - 1) / CR;
    {
        uint32_t pw[WPT];
        load_chunk(train + (size_t)(logical_of(item) / nqb) * nt * 8, 0, pw);
        __syncthreads();  // the table
        store_chunk(0, pw);
    }
    __syncthreads();
    int bufbase = 0;  // the LDS buffer of the item's chunk 0
    for (; item < n_items; item += G) {
        const int logical = logical_of(item);
        const int b = logical / nqb, qb = logical % nqb;
        const uint32_t *qf = query + (size_t)b * nq * 8;
        const uint32_t *tf = train + (size_t)b * nt * 8;
        int32_t *of = out + (size_t)b * nq * 3;
        const int next = item + G;
        const uint32_t *tfn = next < n_items ? train + (size_t)(logical_of(next) / nqb) * nt * 8 : nullptr;
        const int qw0 = qb * (NW * QT * 32) + w * (QT * 32);
        const bool active = qw0 < nq;
        i32x8 bq[QT][4];
        int ka1[QT], ka2[QT], pq[QT];
#pragma unroll
        for (int j = 0; j < QT; j++) {
            const int q = min(qw0 + 32 * j + r, nq - 1);
            const uint4 lo = *(const uint4 *)(qf + (size_t)q * 8), hi = *(const uint4 *)(qf + (size_t)q * 8 + 4);
            const uint32_t wd[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            int pc = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) pc += __popc(wd[k]);
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const uint32_t word = wd[2 * s + h];
#pragma unroll
                for (int d = 0; d < 4; d++)
                    bq[j][s][d] = (int)(0x22222222u | ((~spread_nib(word >> (8 * d)) & 0x11111111u) << 3));
#pragma unroll
                for (int d = 4; d < 8; d++) bq[j][s][d] = 0;
            }
            pq[j] = pc;
            ka1[j] = ka2[j] = ((256 - pc) << MF_SHIFT) + MX_KEY0;
        }
        // formed per item after the query fragments (held across items it pushed the setup past 128 VGPRs)
        f32x16 crow;
#pragma unroll
        for (int i = 0; i < 16; i++) crow[i] = MX_BIAS + (float)((i & 3) + 8 * (i >> 2) + 4 * h);
        auto epi = [&](const f32x16 (&acc)[QT]) {
#pragma unroll
            for (int j = 0; j < QT; j++) {
#pragma unroll
                for (int i = 0; i < 8; i += 2) {
                    key_push2f(ka1[j], ka2[j], __float_as_int(acc[j][i]), __float_as_int(acc[j][i + 1]));
                    key_push2f(ka1[j], ka2[j], __float_as_int(acc[j][i + 8]), __float_as_int(acc[j][i + 9]));
                }
                ka1[j] -= 32;
                ka2[j] -= 32;
            }
        };
        auto tile = [&](const unsigned char *tb, const f32x16 &cin) {
            i32x8 a[4];
#pragma unroll
            for (int s = 0; s < 4; s++) a[s] = frag(tb, s);
            f32x16 acc[QT];
#pragma unroll
            for (int j = 0; j < QT; j++) acc[j] = mfma(a[0], bq[j][0], cin);
#pragma unroll
            for (int s = 1; s < 4; s++)
#pragma unroll
                for (int j = 0; j < QT; j++) acc[j] = mfma(a[s], bq[j][s], acc[j]);
            epi(acc);
        };
        for (int c = 0; c < nch; c++) {
            const int c0 = c * CR;
            uint32_t pw[WPT];
            const bool more_in = c + 1 < nch, more = more_in || tfn != nullptr;
            if (more_in) load_chunk(tf, c0 + CR, pw);
            else if (tfn) load_chunk(tfn, 0, pw);  // the next item's first chunk
            if (active) {
                const unsigned char *sb = s_buf + (size_t)((c + bufbase) & 1) * CR * MX_RS;
                const int nfull = min(NTILE, (nt - c0) / 32);
                if (nfull == NTILE) {
                    i32x8 a[4];
                    f32x16 accp[QT], acc[QT];
#pragma unroll
                    for (int s = 0; s < 4; s++) a[s] = frag(sb, s);
#pragma unroll
                    for (int s = 0; s < 4; s++) {
#pragma unroll
                        for (int j = 0; j < QT; j++) accp[j] = mfma(a[s], bq[j][s], s ? accp[j] : crow);
                        a[s] = frag(sb + 32 * MX_RS, s);
                        __builtin_amdgcn_sched_barrier(0);
                    }
#pragma unroll
                    for (int tt = 1; tt < NTILE; tt++) {
#pragma unroll
                        for (int s = 0; s < 4; s++) {
#pragma unroll
                            for (int j = 0; j < QT; j++) acc[j] = mfma(a[s], bq[j][s], s ? acc[j] : crow);
                            if (tt + 1 < NTILE) a[s] = frag(sb + (tt + 1) * 32 * MX_RS, s);
#pragma unroll
                            for (int j = 0; j < QT; j++) {
                                key_push2f(ka1[j], ka2[j], __float_as_int(accp[j][2 * s]),
                                           __float_as_int(accp[j][2 * s + 1]));
                                key_push2f(ka1[j], ka2[j], __float_as_int(accp[j][8 + 2 * s]),
                                           __float_as_int(accp[j][9 + 2 * s]));
                                if (s == 3) {
                                    ka1[j] -= 32;
                                    ka2[j] -= 32;
                                }
                            }
                            __builtin_amdgcn_sched_barrier(0);
                        }
#pragma unroll
                        for (int j = 0; j < QT; j++) accp[j] = acc[j];
                    }
                    epi(accp);
                } else {
#pragma unroll
                    for (int tt = 0; tt < NTILE; tt++) {
                        if (tt >= nfull) break;
                        tile(sb + tt * 32 * MX_RS, crow);
                    }
                }
                const int lim = nt - (c0 + nfull * 32);
                if (nfull < NTILE && lim > 0) {
                    f32x16 cin;
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        cin[i] = crow[i] + ((i & 3) + 8 * (i >> 2) + 4 * h >= lim ? MX_PAD : 0.f);
                    tile(sb + nfull * 32 * MX_RS, cin);
                }
            }
            if (more) store_chunk((c + 1 + bufbase) & 1, pw);
            __syncthreads();
        }
        bufbase = (bufbase + nch) & 1;
        if (active) {
            const int base = 32 * ((nt + 31) / 32);
#pragma unroll
            for (int j = 0; j < QT; j++) {
                int k1 = ka1[j], k2 = ka2[j];
                const int a1 = __shfl_xor(k1, 32), a2 = __shfl_xor(k2, 32);
                key_merge(k1, k2, a1, a2);
                const int q = qw0 + 32 * j + r;
                if (h == 0 && q < nq) {
                    const int t1 = k1 - MX_KEY0 + base, t2 = k2 - MX_KEY0 + base;
                    const int d1 = (t1 >> MF_SHIFT) + pq[j], d2 = (t2 >> MF_SHIFT) + pq[j];
                    of[3 * q + 0] = d1 < 256 ? (t1 & (MF_MAX_ROWS - 1)) : -1;
                    of[3 * q + 1] = min(d1, 256);
                    of[3 * q + 2] = min(d2, 256);
                }
            }
        }
    }
}

template <int NW, int QT, int CR>
int launch_fp4p(osg_ctx *ctx, const void *d_query, int nq, const void *d_train, int nt, int nb, void *d_out)
{
    const int nqb = (nq + NW * QT * 32 - 1) / (NW * QT * 32);
    const long long items = (long long)nqb * nb;
    OSG_REQUIRE(ctx, items <= 0x7FFFFFFF, "grid too large");
    static int ncu = 0;
    if (ncu == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            ncu = n;
        else
            ncu = 256;
    }
    const int g = (int)std::min<long long>(items, ncu);  // one 16-wave workgroup per CU
    hipLaunchKernelGGL((k_top2_fp4p<NW, QT, CR>), dim3((unsigned)std::max(g, 1)), dim3(NW * 64), 0, ctx->stream,
                       (const uint32_t *)d_query, nq, (const uint32_t *)d_train, nt, nqb, (int)items, (int32_t *)d_out);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    return OSG_OK;
}

template <int NW, int QT, int CR, int PIPE>
int launch_fp4(osg_ctx *ctx, const void *d_query, int nq, const void *d_train, int nt, int nb, void *d_out)
{
    const int nqb = (nq + NW * QT * 32 - 1) / (NW * QT * 32);
    const long long g = (long long)nqb * nb;
    OSG_REQUIRE(ctx, g <= 0x7FFFFFFF, "grid too large");
    hipLaunchKernelGGL((k_top2_fp4<NW, QT, CR, PIPE>), dim3((unsigned)g), dim3(NW * 64), 0, ctx->stream,
                       (const uint32_t *)d_query, nq, (const uint32_t *)d_train, nt, nqb, (int32_t *)d_out);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    return OSG_OK;
}

template <int NW, int QT, int CR, int PIPE>
int launch(osg_ctx *ctx, const void *d_query, int nq, const void *d_train, int nt, int nb, void *d_out)
{
    const int nqb = (nq + NW * QT * 32 - 1) / (NW * QT * 32);
    const long long g = (long long)nqb * nb;
    OSG_REQUIRE(ctx, g <= 0x7FFFFFFF, "grid too large");
    hipLaunchKernelGGL((k_top2_mfma<NW, QT, CR, PIPE>), dim3((unsigned)g), dim3(NW * 64), 0, ctx->stream,
                       (const uint32_t *)d_query, nq, (const uint32_t *)d_train, nt, nqb, (int32_t *)d_out);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    return OSG_OK;
}

}  // namespace

int osg_top2_mfma_max_rows() { return MF_MAX_ROWS; }

namespace {
// the launch knobs, read once per process: OSG_TOP2_MFMA_SHAPE picks the workgroup shape,
// OSG_TOP2_FP4=0 the I8 form (k_top2_mfma) instead of the FP4 block-scaled one (k_top2_fp4, same keys,
// the default since late r05: 8.3 against 6.0 M Mmatches/s, profiles/r05_top2_fp4_ab.jsonl)
int mfma_shape()
{
    static const int shape = getenv("OSG_TOP2_MFMA_SHAPE") ? atoi(getenv("OSG_TOP2_MFMA_SHAPE")) : 0;
    return shape;
}
bool mfma_fp4()
{
    static const bool fp4 = !(getenv("OSG_TOP2_FP4") && atoi(getenv("OSG_TOP2_FP4")) == 0);
    return fp4;
}
// {NW, QT, CR, PIPE} of the shape the switches below launch
void mfma_shape_of(bool fp4, int shape, int *d)
{
    static const int i8[5][4] = {{16, 1, 256, 1}, {8, 2, 256, 1}, {16, 1, 256, 0}, {8, 2, 256, 0}, {8, 1, 256, 1}};
    static const int f4[14][4] = {{16, 1, 256, 3}, {8, 2, 256, 1}, {16, 1, 256, 0}, {16, 1, 256, 3}, {8, 1, 256, 1},
                                  {16, 2, 256, 1}, {16, 1, 256, 2}, {16, 1, 256, 1}, {16, 1, 256, 4}, {8, 1, 256, 3},
                                  {16, 1, 512, 3}, {16, 1, 256, 5}, {16, 1, 512, 5}, {16, 1, 256, 6}};
    const int *s = fp4 ? f4[(shape >= 1 && shape <= 13 && shape != 3) ? shape : 0]
                       : i8[(shape >= 1 && shape <= 4) ? shape : 0];
    for (int i = 0; i < 4; i++) d[i] = s[i];
}
}  // namespace

int osg_hamming_top2_batch_plan(osg_ctx *ctx, int32_t nq, int32_t nt, int32_t nb, char *name, int32_t len)
{
    if (!ctx || !name || len <= 0) return OSG_E_INVALID;
    const bool mf = getenv("OSG_TOP2_BATCH_MFMA") == nullptr || atoi(getenv("OSG_TOP2_BATCH_MFMA")) != 0;
    if (nq <= 0 || nb <= 0 || nt <= 0 || !mf || nt > MF_MAX_ROWS) {
        snprintf(name, (size_t)len, "%s", nq <= 0 || nb <= 0 ? "none" : "k_top2_batch");
        return OSG_OK;
    }
    int d[4];
    mfma_shape_of(mfma_fp4(), mfma_shape(), d);
    const int per_wg = d[0] * d[1] * 32;
    snprintf(name, (size_t)len, "%s<%d,%d,%d,%d> grid=%lld x %d", mfma_fp4() ? "k_top2_fp4" : "k_top2_mfma", d[0], d[1],
             d[2], d[3], (long long)((nq + per_wg - 1) / per_wg) * nb, d[0] * 64);
    return OSG_OK;
}

// B problems of nq x nt on the MFMA path; requires 1 <= nt <= 8192 (the key's row field)
int osg_launch_top2_batch_mfma(osg_ctx *ctx, const void *d_query, int32_t nq, const void *d_train, int32_t nt,
                               int32_t nb, void *d_out)
{
    OSG_REQUIRE(ctx, nt >= 1 && nt <= MF_MAX_ROWS, "nt=%d outside the MFMA path's 1..%d rows", nt, MF_MAX_ROWS);
    const int shape = mfma_shape();
    if (mfma_fp4()) {
        switch (shape) {
        case 1: return launch_fp4<8, 2, 256, 1>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 2: return launch_fp4<16, 1, 256, 0>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 4: return launch_fp4<8, 1, 256, 1>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 5: return launch_fp4<16, 2, 256, 1>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 6: return launch_fp4<16, 1, 256, 2>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 7: return launch_fp4<16, 1, 256, 1>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 8: return launch_fp4<16, 1, 256, 4>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 9: return launch_fp4<8, 1, 256, 3>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 10: return launch_fp4<16, 1, 512, 3>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 11: return launch_fp4<16, 1, 256, 5>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 12: return launch_fp4<16, 1, 512, 5>(ctx, d_query, nq, d_train, nt, nb, d_out);
        case 13: return launch_fp4p<16, 1, 256>(ctx, d_query, nq, d_train, nt, nb, d_out);
        default: return launch_fp4<16, 1, 256, 3>(ctx, d_query, nq, d_train, nt, nb, d_out);
        }
    }
    switch (shape) {
    case 1: return launch<8, 2, 256, 1>(ctx, d_query, nq, d_train, nt, nb, d_out);
    case 2: return launch<16, 1, 256, 0>(ctx, d_query, nq, d_train, nt, nb, d_out);
    case 3: return launch<8, 2, 256, 0>(ctx, d_query, nq, d_train, nt, nb, d_out);
    case 4: return launch<8, 1, 256, 1>(ctx, d_query, nq, d_train, nt, nb, d_out);
    default: return launch<16, 1, 256, 1>(ctx, d_query, nq, d_train, nt, nb, d_out);
    }
}
