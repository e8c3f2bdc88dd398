// ba.hip — the g2o inner loop of Optimizer::LocalBundleAdjustment on gfx950.
//
// Reference: ref:src/Optimizer.cc:1877-2203 (graph → optimize(10) → classification), running
// g2o's LM (ref:Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-194) over a
// BlockSolver<6,3> with the points marginalised (ref:Thirdparty/g2o/g2o/core/block_solver.hpp:143-604).
//
// Structure (built once per call, host, like BlockSolver::buildStructure):
//   Hessian order: free poses with >= 1 edge, then points (vertex-id order); one Hpl block per
//   (free pose, point) pair; CSR of edges per point and per pose; for every pose pair (i <= j)
//   the list of (block_i, block_j) contributions in landmark order (the Schur outer loop order).
//
// Batches: B independent graphs run in lockstep, one launch of each kernel per LM trial for all of
// them (grid.y = graph; a graph that skips a kernel this step leaves at once).
// Per LM iteration (device):
//   k_errors      per edge: error, Huber rho -> per-workgroup chi2 partials        (HBM/latency)
//   k_linearize   per landmark: its edges' Jacobians -> Hll, b_l, the Hpl blocks   (FP64 VALU)
//   k_pose_red    per pose: Hpp, b_p from its edges' pose Jacobians, recomputed in place (a
//                 workgroup reduction; no per-edge contribution round trip through HBM), its edge
//                 inputs from pose-major records (k_hp_rec, once per call)
// Per LM trial:
//   (k_schur_point per landmark: Dinv = (Hll + lambda I)^-1, Dinv b_l; only with OSG_SCHUR_POINT=1:
//                 by default k_schur_rows and k_update form Dinv from Hll themselves)
//   k_schur_rows   per row segment (pose i, 200 of its blocks): BD = Hpl Dinv staged in LDS, the
//                 segment's chunks of S_ij = sum_p BD_ip Hpl_jp^T on FP64 MFMA (v_mfma_f64_4x4x4f64,
//                 one contribution per instruction; OSG_SCHUR_VALU=1: the VALU form) and its share
//                 of b_schur
//   k_schur_pairs  per pose pair: chunk partials summed in chunk order -> the dense reduced camera
//                 matrix Hpp + lambda I - S, and b_schur
//   k_chol_col x ceil(n/32), k_chol_back   left-looking blocked Cholesky (FP64 MFMA tile updates),
//                 forward solve fused, backward solve; past n = 384 (BundleAdjustment) right-looking:
//                 k_chol_col + k_chol_trail per column block, then k_chol_back_large
//   k_update      per point: x_l = Dinv (b_l - Hpl^T x_p), new estimates (poses: exp(x) * T)
//                 and the LM scale sum;  then k_errors on the new estimates
//   k_step_reduce the step's scalars per graph (chi2 of trial and current, scale, lambda, pivot flag)
// The host reads back 5 scalars per graph per trial and runs the accept / reject / lambda logic
// exactly as the reference; push/pop is a swap of the current / trial estimate buffers.
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <string>
#include <thread>
#include <vector>

#include "ba_common.h"
#include "match_common.h"

using namespace osgba;

namespace {

constexpr int EB = 256;      // edge-parallel kernels
constexpr int RT_STRIDE = 16;  // hp_Rt doubles per hessian pose: R (9), t (3), c = R^T t (3), pad

// LbaDev's arrays are generic pointers; the hot gathers read them as global (address space 1) so
// they issue global_load (counted by vmcnt alone) instead of flat loads, whose lgkmcnt share makes
// every wait on an LDS read also wait for the outstanding HBM loads
#define GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ inline const GLOBAL T *gbl(const T *p)
{
    return (const GLOBAL T *)p;
}
constexpr int RED_CHUNK = 1024;  // k_step_reduce stages the partials in LDS this many at a time

// Per-graph control of one lockstep step (host → device each step; k_lambda_init may set lambda).
enum : int { M_ERRC = 1, M_LIN = 2, M_INIT = 4, M_ACT = 8, M_FIN = 16 };
struct LbaCtl {
    int mode;       // M_* bits: current errors / linearize / lambda init / trial / classify
    int sel;        // 0: estimate A is current, 1: B
    double lambda;
};

struct LbaDev {
    // sizes
    int np, npt, ne, nhp, nhl, nblk, npairs, n_cams;
    int n_graphs, xcd_map;        // the batch (the same in every graph's entry): LBA_GRAPH's mapping
    // inputs
    const uint8_t *pose_fixed;
    const int32_t *e_pose, *e_point, *e_cam;
    const int8_t *e_kind;
    const double *e_obs;
    const float *e_isig2;
    const uint8_t *e_robust;      // per edge Huber attached, or null: every edge (LocalBundleAdjustment)
    float hub_mono, hub_stereo;   // Huber deltas as the reference's floats (thHuberMono/2D, thHuberStereo/3D)
    const osg_camera *cams;
    // structure
    const int32_t *pose_h;        // per pose: hessian index or -1
    const int32_t *hp_pose;       // per hessian pose: pose index
    const int32_t *point_h;       // per point: landmark index or -1
    const int32_t *hl_point;      // per landmark: point index
    const int32_t *lm_e_start, *lm_e;    // edges per landmark
    int lm_e_ident;                      // lm_e[q] == q for every q (edges given landmark by landmark, as
                                         // LocalBundleAdjustment inserts them): k_linearize skips the lookup
    const int32_t *lg_start;             // k_linearize's landmark groups: <= EB edges, or one landmark; on the
                                         // device {first landmark, its first edge} per group boundary, so a
                                         // workgroup's edge range is one load, not a load of a load
    const int32_t *lm_b_start;           // blocks per landmark (blocks are numbered landmark-major)
    const int32_t *blk_pose;             // per block: hessian pose index
    const int32_t *edge_blk;             // per edge: 4 block + 2 (block has several edges) + 1 (not its
                                         // first edge), or -1
    const int32_t *hp_e_start, *hp_e;    // edges per hessian pose
    int nhe;                             // hp_e entries
    int32_t *hp_rec;                     // per hp_e entry, 4 ints (k_hp_rec, once per call): edge, point,
                                         // camera | kind << 16 | robust << 24, inverse sigma^2 bits
    const int32_t *hp_b;                 // blocks per hessian pose (hp_b_start on the host)
    const int32_t *pair_b;               // per contribution (a, b): its second block b
    int nchunks;
    const int32_t *chunk_start;          // contribution range of each chunk (chunks never span pairs
                                         // or row segments)
    const int32_t *pair_chunk;           // per pair: first chunk (npairs + 1)
    const int32_t *pair_rank;            // per contribution: rank of its first block in pose i's list
    int n_rs;                            // row segments: RS consecutive blocks of one hessian pose
    const int32_t *rs_info;              // k_schur_rows, 8 per workgroup (launch order): row segment,
                                         // pose, first rank, hp_b_start[pose], blocks, chunk range
    const int32_t *hp_b_lm;              // per hp_b entry: the block's landmark
    const int32_t *rs_chunk_start, *rs_chunk;  // chunks per row segment
    const int32_t *rs_cdesc;             // per rs_chunk entry: {chunk, first contribution, count, partner
                                         // hessian pose j}
    const int32_t *hp_rs_start;          // row segments per hessian pose
    double *chunk_part;                  // 36 per chunk
    double *bs_part;                     // 6 per row segment: sum of Hpl Dinv b_l
    // launch extents of this graph (grids are sized for the largest graph of the batch)
    int ge, gl, gll, gu, nblk_red;       // gll: k_linearize's landmark groups
    double user_lambda;
    // state: estimate buffers A / B; ctl->sel says which one is current
    double *poseA, *poseB, *pointA, *pointB;
    const double *pose0, *point0;        // the graph's input estimates (packed input), copied to A by k_init_state
    LbaCtl *ctl;                         // per-step control, written by the host each step
    double *out;                         // per-step results (k_step_reduce)
    uint8_t *bad;                        // classification
    double *chi2o;                       // per edge chi2 of the last computed error (classification)
    double *err;                         // 3 per edge
    double *Hll, *bl, *Hpl, *Hpp, *bp;
    // per landmark: Hll (3 x 3), b_l (3) and, compact, its position (lmX) at strides ls_h / ls_b / ls_x: three
    // arrays (strides 9, 3, 3) by default; OSG_LBA_LREC=1 one 128-byte record per landmark (stride 16: Hll at
    // 0, b_l at 9, X at 12), one line per landmark for the Schur staging's scattered reads but strided for
    // the landmark-parallel kernels: k_schur_rows_c 5.99 against 5.95-6.04 ms, k_linearize 1.82 against
    // 1.70 and k_update_c 1.50 against 1.29 ms per 14 launches (A/B runs, the same values)
    int ls_h, ls_b, ls_x;
    // the compact per-block factor (the default; OSG_LBA_HPL=1 stores Hpl whole): 6 doubles per block,
    // the symmetric M' = sum over the block's edges of J_point^T rho' W J_point (see z_rows), in Hpl's storage
    int compact;
    double *hp_Rt;                       // per hessian pose: R (row-major 9), t (3), c = R^T t (3) of the
                                         // current estimate (k_pose_red, every linearisation)
    double *lmX;                         // per landmark: its current position (k_linearize, compact form):
                                         // one dependent load level less for the Schur staging
    double *Dinv, *db;                   // k_schur_point's outputs (OSG_SCHUR_POINT=1 only)
    int dinv_inline;                     // 1: k_schur_rows / k_update form Dinv from Hll themselves
    double *Hs, *bs, *x;
    double *Linv;                        // inverses of the 32x32 diagonal blocks of L, row-major per block row
    int npart;                           // partial slots per kind (>= ge, gu, gll + nhp)
    double *part;                        // [0, P): chi of the trial, [P, 2P): scale, [2P, 3P): max diag,
                                         // [3P, 4P): chi of the current estimate (P = npart)
    // envelope of the reduced camera system by 32-row blocks (BundleAdjustment past CMAX): row block t
    // has nothing left of column block blk_first[t], in A and in its Cholesky factor (fill-in stays
    // inside the profile); blk_last[j] = the last row block t with blk_first[t] <= j
    const int32_t *blk_first, *blk_last;
    // per column block j (past CMAX): the row blocks t > j inside the envelope (blk_first[t] <= j),
    // ascending, as CSR: the rows k_chol_col / k_chol_trail touch.  A loop closure makes the last rows
    // reach column 0, so these lists are the band rows plus those few, not every row below j.
    const int32_t *col_rows_start, *col_rows;
    // pose pairs (i <= j) k_schur_pairs writes past CMAX: those whose 6 x 6 block reaches a lower tile
    // inside the envelope (the factorisation reads nothing else); null: every pair (n <= CMAX)
    const int32_t *live_pairs;
    int n_live;
    const int32_t *live_chunk;           // per live pair: its chunk range [first, end) (past CMAX)
    // past CMAX, Hs holds only the envelope's lower 32 x 32 tiles: row block t keeps column blocks
    // blk_first[t] .. t, contiguous after env_off[t] tiles, each tile row-major; null: dense n x n
    const int32_t *env_off;
    int chol_fused;                      // 0: column launches, 1: k_chol_dense, 2: k_chol_env (+ its own back solve)
    int *flag;                           // [0] cholesky ok
    unsigned long long *tstamp;          // phase timestamps (OSG_LBA_PROFILE=2), else null
};

__device__ inline double edge_w(const LbaDev &D, int e) { return (double)D.e_isig2[e]; }
constexpr int CB_ROWS = 32;  // the envelope tile edge (= CB, the factorisation's block)
// Hs element (R, C): dense row-major up to CMAX, else its place in the envelope tile store (which
// must hold it: hs_stored)
__device__ inline size_t hs_at(const LbaDev &D, int n, int R, int C)
{
    if (!D.env_off) return (size_t)R * n + C;
    const int t = R >> 5, u = C >> 5;
    return ((size_t)(D.env_off[t] + u - D.blk_first[t]) << 10) + (size_t)((R & 31) << 5) + (size_t)(C & 31);
}
// Row block t of Hs (rows 32 t .. 32 t + 31): element (32 t + r, C) at hs_el(blk, r, C).  The kernels
// that stay in one row block take this once instead of an envelope lookup per element.
struct HsBlk {
    long long base;
    int rs, ts;  // row stride, tile stride (dense: n, 32; envelope: 32, 1024)
};
__device__ inline HsBlk hs_blk(const LbaDev &D, int n, int t)
{
    if (!D.env_off) return HsBlk{(long long)CB_ROWS * t * n, n, CB_ROWS};
    return HsBlk{(long long)(D.env_off[t] - D.blk_first[t]) << 10, CB_ROWS, CB_ROWS * CB_ROWS};
}
__device__ inline size_t hs_el(const HsBlk &h, int r, int C)
{
    return (size_t)(h.base + (long long)r * h.rs + (long long)(C >> 5) * h.ts + (C & 31));
}
__device__ inline bool hs_stored(const LbaDev &D, int R, int C)
{
    if (!D.env_off) return true;
    const int t = R >> 5, u = C >> 5;
    return u <= t && u >= D.blk_first[t];
}
__device__ inline const double *cur_pose(const LbaDev &D) { return D.ctl->sel ? D.poseB : D.poseA; }
__device__ inline const double *cur_point(const LbaDev &D) { return D.ctl->sel ? D.pointB : D.pointA; }
__device__ inline double *new_pose(const LbaDev &D) { return D.ctl->sel ? D.poseA : D.poseB; }
__device__ inline double *new_point(const LbaDev &D) { return D.ctl->sel ? D.pointA : D.pointB; }
// One problem per workgroup row; a workgroup whose graph skips this kernel leaves at once.
// With OSG_LBA_XCD=1, batches of >= 8 graphs run XCD-aware: grid (8 gx, ceil(B / 8)); workgroup (x, y) of the launch
// goes to XCD x % 8 (dispatch is round-robin over the 8 XCDs in linear order and 8 gx is a multiple
// of 8), so graph (x % 8) + 8 y runs on one XCD and its Hpl / Dinv / edge arrays stay in that XCD's
// L2, while the chip works on 8 graphs at a time (their working set fits the MALL).  Measured slower
// than the default grid (gx, B), which spreads each graph over the whole chip.
#define LBA_GRAPH(MODEBITS)                                                                      \
    const bool xcd_map_ = Ds[0].xcd_map;                                                         \
    const int by = xcd_map_ ? (int)(blockIdx.x & 7) + 8 * (int)blockIdx.y : (int)blockIdx.y;     \
    const int bx = xcd_map_ ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;                          \
    (void)bx;                                                                                    \
    if (by >= Ds[0].n_graphs) return;                                                            \
    const LbaDev &D = Ds[by];                                                                    \
    if (!(D.ctl->mode & (MODEBITS))) return

// The edge's Huber kernel; an edge without one (BundleAdjustment with bRobust = false,
// ref:src/Optimizer.cc:3000-3007) gets an infinite delta, so rho = (e2, 1, 0) as g2o's unrobustified
// chi2 / quadratic form
__device__ inline void edge_delta_f(const LbaDev &D, bool robust, int kind, double &delta, float &dsqr)
{
    if (!robust) {
        delta = __builtin_inf();
        dsqr = __builtin_inff();
        return;
    }
    const float d = (kind == OSG_EDGE_STEREO) ? D.hub_stereo : D.hub_mono;
    delta = (double)d;
    dsqr = (float)((double)d * (double)d);
}
__device__ inline void edge_delta(const LbaDev &D, int e, int kind, double &delta, float &dsqr)
{
    if (D.e_robust && !D.e_robust[e]) {
        delta = __builtin_inf();
        dsqr = __builtin_inff();
        return;
    }
    const float d = (kind == OSG_EDGE_STEREO) ? D.hub_stereo : D.hub_mono;
    delta = (double)d;
    dsqr = (float)((double)d * (double)d);
}

__device__ inline double block_sum_d(double v, double *s)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_sum(v);
    if (lane == 0) s[w] = v;
    __syncthreads();
    double t = 0;
    for (int i = 0; i < nw; i++) t += s[i];
    __syncthreads();
    return t;
}

// per edge error + robust chi2 -> partial sums per workgroup (deterministic order)
// which = 0: the trial estimate -> part[0, ge); which = 1: the current estimate -> part[3 npart, ..)
__global__ __launch_bounds__(EB) void k_errors(const LbaDev *__restrict__ Ds, int which)
{
    LBA_GRAPH(which ? M_ERRC : M_ACT);
    if (bx >= D.ge) return;
    const double *poses = which ? cur_pose(D) : new_pose(D);
    const double *points = which ? cur_point(D) : new_point(D);
    const int part_off = which ? 3 * D.npart : 0;
    __shared__ double s[EB / 64];
    const int e = bx * EB + threadIdx.x;
    double rho0 = 0.0;
    if (e < D.ne) {
        const int k = D.e_kind[e];
        const SE3 T = se3_from7(poses + 7 * (size_t)D.e_pose[e]);
        const double *X = points + 3 * (size_t)D.e_point[e];
        double ev[3];
        edge_error(k, true, D.cams[D.e_cam[e]], T, X, D.e_obs + 3 * (size_t)e, ev);
        D.err[3 * e] = ev[0];
        D.err[3 * e + 1] = ev[1];
        D.err[3 * e + 2] = ev[2];
        const int dim = (k == OSG_EDGE_STEREO) ? 3 : 2;
        const double c = chi2_of(ev, dim, edge_w(D, e));
        double delta, r1;
        float dsqr;
        edge_delta(D, e, k, delta, dsqr);
        huber(c, delta, dsqr, rho0, r1);
    }
    const double t = block_sum_d(rho0, s);
    if (threadIdx.x == 0) D.part[part_off + bx] = t;
}

// ---- the compact per-block factor ------------------------------------------
// Every edge of the path has J_pose = P S(Xc) and J_point = P R, with P = d(error)/d(Xc), Xc = R X + t the
// point in the pose (body) frame and S(Xc) = [-[Xc]x | I] (se3deriv): EdgeSE3ProjectXYZ, ...ToBody (P
// through Trl) and EdgeStereoSE3ProjectXYZ alike (ref:src/OptimizableTypes.cpp:107-141, 231-265,
// ref:Thirdparty/g2o/g2o/types/types_six_dof_expmap.cpp:318-372).  So a block's
//     Hpl = sum_e J_pose^T rho' W J_point = S(Xc)^T M R,   M = sum_e P^T rho' W P,
// and with M' = R^T M R = sum_e J_point^T rho' W J_point (the block's own Hll terms, 3 x 3 symmetric)
// and c = R^T t ([R v]x = R [v]x R^T, so [Xc]x R = R [X + c]x):
//     Hpl = D(R) Z,   D(R) = diag(R, R),   Z = [[X + c]x M' ; M']          (6 x 3)
// A block keeps M' (6 doubles, 48 B, against Hpl's 18); X is its landmark's position, R, t, c its pose's.
// The Schur product S_ij = sum Hpl_a Dinv Hpl_b^T = D(R_i) [sum (Z_a Dinv) Z_b^T] D(R_j)^T, and
// Z_b^T = [-M'_b [X]x - M'_b [c_j]x | M'_b], so the chunks sum
//     [B | A] = sum_p (Z_a Dinv)_p [-M'_p [X_p]x | M'_p]         (k_schur_rows_c: per contribution the
//                                                                  partner's M' and the landmark's X)
// and k_schur_pairs forms S_ij = D(R_i) [B - A [c_j]x | A] D(R_j)^T once per pose pair.  The rounding
// differs from the whole-Hpl form's (BA parity is a tolerance).
//
// rows of Z = [[v]x M' ; M'] for v = X + c (the tile operand uses c = 0): column k of [v]x M' is
// v x (column k of M');  m = (m00, m01, m02, m11, m12, m22)
__device__ __forceinline__ void z_rows(const double *m, double x, double y, double z, double Z[6][3])
{
    const double M[3][3] = {{m[0], m[1], m[2]}, {m[1], m[3], m[4]}, {m[2], m[4], m[5]}};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        Z[0][k] = y * M[2][k] - z * M[1][k];
        Z[1][k] = z * M[0][k] - x * M[2][k];
        Z[2][k] = x * M[1][k] - y * M[0][k];
        Z[3][k] = M[0][k];
        Z[4][k] = M[1][k];
        Z[5][k] = M[2][k];
    }
}

// Linearisation (ref:Thirdparty/g2o/g2o/core/base_binary_edge.hpp:55-120, robust branch), edge-parallel
// with the landmark-major sums of a per-landmark loop.  Workgroup g takes the landmarks
// [lg_start[g], lg_start[g + 1]) — at most EB edges, or one landmark with more — and their edges in
// lm_e order (landmark-major, edge order inside a landmark), EB at a time:
//   * thread t computes one edge's Jacobians and robust weight, stages its Hll (upper 6) and b_l
//     terms in LDS, and writes its Hpl block when the block has no other edge;
//   * then thread t owns landmark lg_start[g] + t and adds its edges' terms in edge order — the sums
//     of a per-landmark reduction over lm_e — and the Hpl terms of a block with several edges (a
//     two-camera rig's left and right observations), first edge stored, the others added.
// The workgroup's max |diag Hll| goes to the computeLambdaInit partials.  The edges' pose parts
// {Hpp upper 21, b_p 6} are not stored: k_pose_red recomputes them pose-major (27 doubles per edge
// written and read back cost more HBM time than the recomputed Jacobian costs VALU time).
// WPE: the minimum waves per SIMD the register allocation must allow (1: the compiler's choice, 146
// VGPRs = 3 waves; 4: 128 VGPRs with a few spills, OSG_LIN_WPE=4)
// COMPACT (the default): a block's M' (its Hll terms, 6) instead of its Hpl (18)
template <bool MULTI, int WPE = 1, bool COMPACT = false>
__global__ __launch_bounds__(EB) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_linearize(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_LIN);
    if (bx >= max(D.gll, 1)) return;
    constexpr int HN = COMPACT ? 6 : 18;          // doubles per block
    __shared__ double s_t[9][EB];                 // per edge: Hll upper 6 | b_l 3
    __shared__ double s_h[MULTI ? HN : 1][EB];    // per edge of a several-edge block: its Hpl / M terms
    __shared__ double s_m[EB / 64];
    double md = 0.0;
    if (D.nhl > 0) {
        typedef int i2 __attribute__((ext_vector_type(2)));
        const i2 g0 = *(const GLOBAL i2 *)(gbl(D.lg_start) + 2 * bx), g1 = *(const GLOBAL i2 *)(gbl(D.lg_start) + 2 * bx + 2);
        const int l0 = g0.x, l1 = g1.x, q0 = g0.y, q1 = g1.y;
        const int ol = l0 + (int)threadIdx.x;  // the landmark this thread sums
        const bool owner = ol < l1;
        const int oq0 = owner ? D.lm_e_start[ol] : 0, oq1 = owner ? D.lm_e_start[ol + 1] : 0;
        const double *poses = cur_pose(D), *points = cur_point(D);
        double H6[6] = {0, 0, 0, 0, 0, 0}, bl3[3] = {0, 0, 0};
        for (int c0 = q0; c0 < q1; c0 += EB) {
            const int q = c0 + (int)threadIdx.x;
            if (q < q1) {
                // the identity map saves the edge loads one dependent level
                int e = q;
                if (!D.lm_e_ident) e = D.lm_e[q];
                const int k = D.e_kind[e];
                const SE3 T = se3_from7(poses + 7 * (size_t)D.e_pose[e]);
                double Jp[3][6], Jx[3][3];
                edge_jacobians(k, true, D.cams[D.e_cam[e]], T, points + 3 * (size_t)D.e_point[e], Jp, Jx);
                const int dim = (k == OSG_EDGE_STEREO) ? 3 : 2;
                const double w = edge_w(D, e);
                const double ev[3] = {D.err[3 * e], D.err[3 * e + 1], D.err[3 * e + 2]};
                double delta, r0, rho1;
                float dsqr;
                edge_delta(D, e, k, delta, dsqr);
                huber(chi2_of(ev, dim, w), delta, dsqr, r0, rho1);
                const double ww = rho1 * w;
                double om[3];
                for (int d = 0; d < 3; d++) om[d] = (d < dim) ? -(w * ev[d]) * rho1 : 0.0;
                if (dim == 2) {
                    for (int j = 0; j < 6; j++) Jp[2][j] = 0.0;
                    for (int j = 0; j < 3; j++) Jx[2][j] = 0.0;
                }
                // the edge's Hll terms (upper 6): also the compact form's M' of a one-edge block
                double hl6[6];
                {
                    int c = 0;
                    for (int a = 0; a < 3; a++)
                        for (int bb = a; bb < 3; bb++)
                            hl6[c++] = Jx[0][a] * ww * Jx[0][bb] + Jx[1][a] * ww * Jx[1][bb] + Jx[2][a] * ww * Jx[2][bb];
                }
                const int code = D.edge_blk[e];
                if (code >= 0) {  // free pose: Hpl (the pose part is recomputed by k_pose_red)
                    const bool multi = MULTI && (code & 2);
                    double *hp = D.Hpl + HN * (size_t)(code >> 2);
                    if constexpr (COMPACT) {
#pragma unroll
                        for (int c = 0; c < 6; c++) {
                            if (multi) s_h[MULTI ? c : 0][threadIdx.x] = hl6[c];
                            else hp[c] = hl6[c];
                        }
                    } else {
                        for (int a = 0; a < 6; a++)
                            for (int bb = 0; bb < 3; bb++) {
                                const double v = Jp[0][a] * ww * Jx[0][bb] + Jp[1][a] * ww * Jx[1][bb] + Jp[2][a] * ww * Jx[2][bb];
                                if (multi) s_h[MULTI ? 3 * a + bb : 0][threadIdx.x] = v;
                                else hp[3 * a + bb] = v;
                            }
                    }
                }
                for (int c = 0; c < 6; c++) s_t[c][threadIdx.x] = hl6[c];
                for (int a = 0; a < 3; a++)
                    s_t[6 + a][threadIdx.x] = Jx[0][a] * om[0] + Jx[1][a] * om[1] + Jx[2][a] * om[2];
            }
            __syncthreads();
            if (owner) {
                const int a0 = max(oq0, c0), a1 = min(oq1, c0 + EB);
                for (int qq = a0; qq < a1; qq++) {
                    const int t = qq - c0;
                    for (int c = 0; c < 6; c++) H6[c] += s_t[c][t];
                    for (int a = 0; a < 3; a++) bl3[a] += s_t[6 + a][t];
                    if (MULTI) {
                        const int code = D.edge_blk[D.lm_e_ident ? qq : D.lm_e[qq]];
                        if (code >= 0 && (code & 2)) {
                            double *hp = D.Hpl + HN * (size_t)(code >> 2);
                            const bool first = !(code & 1);
                            for (int i = 0; i < HN; i++) hp[i] = first ? s_h[MULTI ? i : 0][t] : hp[i] + s_h[MULTI ? i : 0][t];
                        }
                    }
                }
            }
            __syncthreads();
        }
        if (COMPACT && owner) {
            const int p = D.hl_point[ol];
            for (int k = 0; k < 3; k++) D.lmX[D.ls_x * (size_t)ol + k] = points[3 * (size_t)p + k];
        }
        if (owner) {
            const double H[9] = {H6[0], H6[1], H6[2], H6[1], H6[3], H6[4], H6[2], H6[4], H6[5]};
            for (int i = 0; i < 9; i++) D.Hll[D.ls_h * (size_t)ol + i] = H[i];
            for (int i = 0; i < 3; i++) D.bl[D.ls_b * (size_t)ol + i] = bl3[i];
            md = fmax(fabs(H[0]), fmax(fabs(H[4]), fabs(H[8])));
        }
    }
    // max |diag| per workgroup for computeLambdaInit
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int off = 32; off >= 1; off >>= 1) md = fmax(md, __shfl_xor(md, off));
    if (lane == 0) s_m[w] = md;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = 0;
        for (int i = 0; i < EB / 64; i++) m = fmax(m, s_m[i]);
        D.part[2 * D.npart + bx] = m;
    }
}

// The input estimates into estimate buffer A, every graph of the batch in one launch (instead of two
// copy-engine blits per graph: 128 dispatches of ~5 us each for a 64-window batch, r05a trace)
__global__ __launch_bounds__(EB) void k_init_state(const LbaDev *__restrict__ Ds)
{
    const bool xcd_map_ = Ds[0].xcd_map;
    const int by = xcd_map_ ? (int)(blockIdx.x & 7) + 8 * (int)blockIdx.y : (int)blockIdx.y;
    const int bx = xcd_map_ ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    if (by >= Ds[0].n_graphs) return;
    const LbaDev &D = Ds[by];
    const size_t i = (size_t)bx * EB + threadIdx.x, np7 = 7 * (size_t)D.np, npt3 = 3 * (size_t)D.npt;
    if (i < np7) D.poseA[i] = D.pose0[i];
    if (i < npt3) D.pointA[i] = D.point0[i];
}

// The static inputs k_pose_red reads per edge, gathered once per call into pose-major records: one
// 16-byte load per edge instead of five scattered loads (the edge arrays are in landmark order)
__global__ __launch_bounds__(EB) void k_hp_rec(const LbaDev *__restrict__ Ds)
{
    // launched before the first step's control upload: no mode check
    const bool xcd_map_ = Ds[0].xcd_map;
    const int by = xcd_map_ ? (int)(blockIdx.x & 7) + 8 * (int)blockIdx.y : (int)blockIdx.y;
    const int bx = xcd_map_ ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    if (by >= Ds[0].n_graphs) return;
    const LbaDev &D = Ds[by];
    const int q = bx * EB + threadIdx.x;
    if (q >= D.nhe) return;
    const int e = D.hp_e[q];
    const int robust = D.e_robust ? (D.e_robust[e] != 0) : 1;
    const int meta = (D.e_cam[e] & 0xffff) | ((D.e_kind[e] & 0xff) << 16) | (robust << 24);
    typedef int i4 __attribute__((ext_vector_type(4)));
    *(i4 *)(D.hp_rec + 4 * (size_t)q) = i4{e, D.e_point[e], meta, __float_as_int(D.e_isig2[e])};
}

// per free pose (one workgroup): Hpp (6x6) and b_p from its edges.  REC: the edge inputs from the
// pose-major records (default); false: gathered through hp_e (OSG_POSE_RED_GATHER=1, A/B runs)
template <bool REC>
__global__ __launch_bounds__(EB) __attribute__((amdgpu_waves_per_eu(3, 8))) void k_pose_red(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_LIN);
    const int i = bx;
    if (i >= D.nhp) return;
    const int diag_off = 2 * D.npart + D.gll;
    __shared__ double s[EB / 64][27];
    double acc[27];
    for (int k = 0; k < 27; k++) acc[k] = 0.0;
    // every edge of the pose: its pose Jacobian and robust weight recomputed from the estimate and
    // the error k_errors stored (the same expressions k_linearize evaluates per edge, so the sums are
    // those of a stored-Jacobian reduction, without writing / reading EC doubles per edge)
    const SE3 T = se3_from7(cur_pose(D) + 7 * (size_t)D.hp_pose[i]);
    const double *points = cur_point(D);
    typedef int i4 __attribute__((ext_vector_type(4)));
    // REC: the thread's next record is loaded one edge ahead, so an edge waits for its point and error
    // (which the record indexes) but not for the record itself
    const int q_end = D.hp_e_start[i + 1];
    i4 rnext = i4{0, 0, 0, 0};
    if (REC && D.hp_e_start[i] + (int)threadIdx.x < q_end)
        rnext = *(const GLOBAL i4 *)(gbl(D.hp_rec) + 4 * (size_t)(D.hp_e_start[i] + threadIdx.x));
    for (int q = D.hp_e_start[i] + threadIdx.x; q < q_end; q += EB) {
        int e, k, cam, pt;
        bool robust;
        double w;
        if (REC) {
            const i4 r = rnext;
            if (q + EB < q_end) rnext = *(const GLOBAL i4 *)(gbl(D.hp_rec) + 4 * (size_t)(q + EB));
            e = r.x;
            pt = r.y;
            cam = r.z & 0xffff;
            k = (int)(int8_t)((r.z >> 16) & 0xff);
            robust = (r.z >> 24) & 1;
            w = (double)__int_as_float(r.w);
        } else {
            e = D.hp_e[q];
            k = D.e_kind[e];
            cam = D.e_cam[e];
            pt = D.e_point[e];
            robust = !(D.e_robust && !D.e_robust[e]);
            w = edge_w(D, e);
        }
        double Jp[3][6], Jx[3][3];
        edge_jacobians(k, true, D.cams[cam], T, points + 3 * (size_t)pt, Jp, Jx);
        const int dim = (k == OSG_EDGE_STEREO) ? 3 : 2;
        const double ev[3] = {D.err[3 * e], D.err[3 * e + 1], D.err[3 * e + 2]};
        double delta, r0, rho1;
        float dsqr;
        edge_delta_f(D, robust, k, delta, dsqr);
        huber(chi2_of(ev, dim, w), delta, dsqr, r0, rho1);
        const double ww = rho1 * w;
        double om[3];
        for (int d = 0; d < 3; d++) om[d] = (d < dim) ? -(w * ev[d]) * rho1 : 0.0;
        if (dim == 2)
            for (int j = 0; j < 6; j++) Jp[2][j] = 0.0;
        int c = 0;
        for (int a = 0; a < 6; a++)
            for (int bb = a; bb < 6; bb++)
                acc[c++] += Jp[0][a] * ww * Jp[0][bb] + Jp[1][a] * ww * Jp[1][bb] + Jp[2][a] * ww * Jp[2][bb];
        for (int a = 0; a < 6; a++) acc[c++] += Jp[0][a] * om[0] + Jp[1][a] * om[1] + Jp[2][a] * om[2];
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int k = 0; k < 27; k++) acc[k] = wave_sum(acc[k]);
    if (lane == 0)
        for (int k = 0; k < 27; k++) s[w][k] = acc[k];
    __syncthreads();
    if (threadIdx.x < 27) {
        double t = 0;
        for (int ww = 0; ww < EB / 64; ww++) t += s[ww][threadIdx.x];
        s[0][threadIdx.x] = t;  // only wave 0's slot is reused after all reads below
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double H[36];
        int c = 0;
        double md = 0;
        for (int a = 0; a < 6; a++)
            for (int b = a; b < 6; b++) {
                H[a * 6 + b] = s[0][c];
                H[b * 6 + a] = s[0][c];
                c++;
            }
        for (int k = 0; k < 36; k++) D.Hpp[36 * (size_t)i + k] = H[k];
        if (D.hp_Rt) {  // the pose's R, t and c = R^T t for the compact factor's readers
            double Rm[3][3];
            quat_to_R(T.q, Rm);
            double *o = D.hp_Rt + RT_STRIDE * (size_t)i;
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++) o[3 * r + c] = Rm[r][c];
            for (int r = 0; r < 3; r++) o[9 + r] = T.t[r];
            for (int c = 0; c < 3; c++) o[12 + c] = Rm[0][c] * T.t[0] + Rm[1][c] * T.t[1] + Rm[2][c] * T.t[2];
            o[15] = 0.0;
        }
        for (int a = 0; a < 6; a++) {
            D.bp[6 * (size_t)i + a] = s[0][21 + a];
            md = fmax(md, fabs(H[a * 7]));
        }
        D.part[diag_off + i] = md;
    }
}

__device__ inline void inv3(const double *m, double *o)
{  // Eigen compute_inverse<Matrix3>: cofactors, determinant along column 0
#define M_(i, j) m[(i)*3 + (j)]
#define COF(i, j) (M_(((i) + 1) % 3, ((j) + 1) % 3) * M_(((i) + 2) % 3, ((j) + 2) % 3) - M_(((i) + 1) % 3, ((j) + 2) % 3) * M_(((i) + 2) % 3, ((j) + 1) % 3))
    const double c00 = COF(0, 0), c10 = COF(1, 0), c20 = COF(2, 0);
    const double det = c00 * M_(0, 0) + c10 * M_(1, 0) + c20 * M_(2, 0);
    const double invdet = 1.0 / det;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) o[i * 3 + j] = COF(j, i) * invdet;
#undef COF
#undef M_
}

// computeLambdaInit (ref:Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:178-194): tau
// times the largest |diagonal| of H, unless the user set an initial lambda
__global__ void k_lambda_init(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_INIT);
    if (threadIdx.x != 0) return;
    if (D.user_lambda > 0) {
        D.ctl->lambda = D.user_lambda;
        return;
    }
    double md = 0;
    for (int i = 0; i < D.gll + D.nhp; i++) md = fmax(md, D.part[2 * D.npart + i]);
    D.ctl->lambda = 1e-5 * md;
}

// Dinv_l = (Hll_l + lambda I)^-1 and, with db, Dinv_l b_l (ref:Thirdparty/g2o/g2o/core/block_solver.hpp:
// 381-395).  Formed where it is used (the BD staging of k_schur_rows, and k_update) instead of
// written by a kernel of its own and read back: Hll is as many bytes as Dinv, so each reader's
// traffic is unchanged, and k_schur_point's launch and its 107 MB per 64 C4 windows are gone.
__device__ inline void landmark_dinv(const LbaDev &D, int l, double lambda, double *Di, double *db)
{
    double Dm[9];
    for (int i = 0; i < 9; i++) Dm[i] = D.Hll[D.ls_h * (size_t)l + i];
    Dm[0] += lambda;
    Dm[4] += lambda;
    Dm[8] += lambda;
    inv3(Dm, Di);
    if (db) {
        const double *b = D.bl + D.ls_b * (size_t)l;
        for (int r = 0; r < 3; r++) db[r] = Di[3 * r] * b[0] + Di[3 * r + 1] * b[1] + Di[3 * r + 2] * b[2];
    }
}

// the separate per-landmark pass (OSG_SCHUR_POINT=1, A/B runs): bit-identical
__global__ __launch_bounds__(EB) void k_schur_point(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    const double lambda = D.ctl->lambda;
    const int l = bx * EB + threadIdx.x;
    if (l >= D.nhl) return;
    double Di[9], db[3];
    landmark_dinv(D, l, lambda, Di, db);
    for (int i = 0; i < 9; i++) D.Dinv[9 * (size_t)l + i] = Di[i];
    for (int r = 0; r < 3; r++) D.db[3 * (size_t)l + r] = db[r];
}

// Schur accumulation S_ij = sum_p BD_ip Hpl_jp^T (BD = Hpl Dinv) over the (block_i, block_j)
// contributions of every pose pair (i <= j), in landmark order — the order of g2o's Schur loop
// (ref:Thirdparty/g2o/g2o/core/block_solver.hpp:381-432).  Row-staged: one workgroup per row segment
// (hessian pose i, RS consecutive blocks of pose i in block order).  It forms BD_a = Hpl_a Dinv_l for
// its blocks into LDS once — with the segment's share of b_schur, sum of Hpl_a (Dinv b_l) — and its
// waves take the segment's chunks (<= SCH contributions of one pair (i, j >= i) whose first block is
// in the segment): BD_a from LDS, Hpl_b from HBM.  A block's BD is formed once per trial instead of
// written to HBM and gathered again per contribution (the contribution count is sum_l k_l(k_l+1)/2
// against the block count sum_l k_l).
//   The product runs on FP64 MFMA by default (layout below, at the chunk loop).  The VALU form
// (OSG_SCHUR_VALU=1, kept for A/B measurements: DESIGN.md §3.4) uses lane = (group g = lane >> 2,
// quarter q = lane & 3); group g takes contributions g, g + 16, ... of the chunk; quarter q owns
// rows 3 (q >> 1) .. + 2 and columns 3 (q & 1) .. + 2 of the 6x6 product (9 + 9 doubles loaded for
// 27 FMAs), the 16 groups summed by a fixed xor butterfly.  Both are deterministic; k_schur_pairs
// then sums a pair's chunks in chunk order.
constexpr int SCH = 64;
constexpr int RS = 200;  // blocks per row segment: 200 x 18 doubles = 28 KiB of LDS
constexpr int RT = 512;  // threads per row-segment workgroup
template <bool VALU, bool DIRECT = false>
__global__ __launch_bounds__(RT, 6) void k_schur_rows(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    if (bx >= D.n_rs) return;
    typedef int i4 __attribute__((ext_vector_type(4)));
    // the segment's indices in one 32-byte load (one dependent level instead of four)
    const i4 inf0 = ((const GLOBAL i4 *)gbl(D.rs_info))[2 * bx];
    const i4 inf1 = ((const GLOBAL i4 *)gbl(D.rs_info))[2 * bx + 1];
    const int rs = __builtin_amdgcn_readfirstlane(inf0.x);
    const int rb = __builtin_amdgcn_readfirstlane(inf0.z), hb0 = __builtin_amdgcn_readfirstlane(inf0.w);
    const int nr = __builtin_amdgcn_readfirstlane(inf1.x);
    const double lam = D.ctl->lambda;
    __shared__ double s_bd[RS * 18 + 2];  // + a zero: the MFMA's K-padding lanes read it
    __shared__ double s_cf[RT / 64][6];
    if (threadIdx.x == 0) s_bd[RS * 18] = 0.0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // FP64 MFMA (v_mfma_f64_4x4x4f64: four independent 4x4x4 blocks per wave instruction).  A
    // chunk's S_ij = sum_p BD_p Hpl_p^T is the GEMM (6 x 3P)(3P x 6); one instruction takes one
    // contribution (K = its 3 landmark dimensions, padded to 4) for the whole 6x6 product: block
    // beta = (rb, cb) covers rows 4 rb .. 4 rb + 3 and columns 4 cb .. 4 cb + 3 (rows / columns 6, 7
    // padded).  Operand layout on gfx950 (tools/micro/mfma_f64.hip, profiles/r02_mfma_f64.txt):
    //   A(beta, row i, k) in lane 16 k + 4 beta + i,  B(beta, k, col j) in lane 16 k + 4 beta + j,
    //   D(beta, row i, col j) in lane 16 i + 4 beta + j.
    // Contributions accumulate in chunk order (= landmark order) through two alternating
    // accumulators, summed once at the end: deterministic.
    const int kk = lane >> 4, beta = (lane >> 2) & 3, ri = lane & 3;
    const int arow = 4 * (beta >> 1) + ri, bcol = 4 * (beta & 1) + ri;
    // Padding without arithmetic: the K-padding lanes (k = 3) of A read the zero after s_bd, so the
    // fourth product of every output is exactly 0; the padded rows (A) and columns (B) 6, 7 read
    // row / column 5 again and only reach the padded outputs, which are never stored.  B's k = 3
    // lanes read a real (finite) element, multiplied by that zero.
    const int a_m = kk < 3 ? 18 : 0;  // A's address: a_m * rank + aoff
    const int aoff = kk < 3 ? 3 * min(arow, 5) + kk : RS * 18;
    const int boff = 3 * min(bcol, 5) + min(kk, 2);
    const int orow = 4 * (beta >> 1) + kk, ocol = 4 * (beta & 1) + ri;  // D: i = lane >> 4
    const GLOBAL double *__restrict__ Hv = gbl(D.Hpl);
    // Hpl_j blocks are staged per wave through LDS, 16 contributions at a time: 144 16-byte granules
    // read by 64 lanes with 3 dwordx4 loads (one gather instruction per 5 contributions instead of
    // one per contribution), the next group's loads in flight while this group's MFMAs run
    constexpr int GC = 16;
    __shared__ __attribute__((aligned(16))) double s_hb[RT / 64][GC * 18];
    double *hb = s_hb[wv];
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const int t1 = __builtin_amdgcn_readfirstlane(inf1.z);
    int t = __builtin_amdgcn_readfirstlane(inf1.y) + wv;
    const GLOBAL i4 *__restrict__ cd = (const GLOBAL i4 *)gbl(D.rs_cdesc);
    // chunk descriptor {chunk, first contribution, count (<= SCH = 64)} of rs_chunk entry tt
    auto desc = [&](int tt) -> i4 {
        i4 d = tt < t1 ? cd[tt] : i4{0, 0, 0, 0};
        // wave-uniform: scalar registers
        return i4{__builtin_amdgcn_readfirstlane(d.x), __builtin_amdgcn_readfirstlane(d.y),
                  __builtin_amdgcn_readfirstlane(d.z), 0};
    };
    // lane q: rank (in the segment) of contribution q's first block, and its second block
    auto contrib = [&](const i4 &d, int &mr, int &mb) {
        mr = lane < d.z ? gbl(D.pair_rank)[d.y + lane] - rb : 0;
        mb = lane < d.z ? gbl(D.pair_b)[d.y + lane] : 0;
    };
    // granules of group u0 (contributions u0 .. u0 + cnt - 1) into registers
    auto load_group = [&](int u0, int cnt, int mb, u4 (&R)[3]) {
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const int idx = lane + 64 * r;
            const int c = idx / 9, gq = idx - 9 * c;
            const int bj = __shfl(mb, (u0 + c) & 63);
            if (idx < GC * 9 && c < cnt) R[r] = *(const GLOBAL u4 *)(Hv + 18 * (size_t)bj + 2 * gq);
        }
    };
    i4 dc = {0, 0, 0, 0}, dn = {0, 0, 0, 0};
    int my_rank = 0, my_b = 0, n_rank = 0, n_b = 0;
    u4 R[3];
    if (!VALU) {
        dc = desc(t);
        dn = desc(t + RT / 64);
        contrib(dc, my_rank, my_b);
        contrib(dn, n_rank, n_b);
    }
    double cf[6] = {0, 0, 0, 0, 0, 0};
    // two threads per block (rows 3h .. 3h + 2 each): half the staging registers per thread
    {
        const int h = threadIdx.x & 1;  // RT is even: a thread keeps its half
        double c3[3] = {0, 0, 0};
        for (int r2 = threadIdx.x; r2 < 2 * nr; r2 += RT) {
            const int r = r2 >> 1;
            const int a = gbl(D.hp_b)[hb0 + rb + r];
            const int l = gbl(D.hp_b_lm)[hb0 + rb + r];
            double Di[9], db[3], B[9];
            if (D.dinv_inline) {
                landmark_dinv(D, l, lam, Di, db);
            } else {
                for (int k = 0; k < 9; k++) Di[k] = gbl(D.Dinv)[9 * (size_t)l + k];
                for (int k = 0; k < 3; k++) db[k] = gbl(D.db)[3 * (size_t)l + k];
            }
            for (int k = 0; k < 9; k++) B[k] = gbl(D.Hpl)[18 * (size_t)a + 9 * h + k];
            double *BD = s_bd + 18 * r + 9 * h;
            for (int rr = 0; rr < 3; rr++) {
                for (int c = 0; c < 3; c++)
                    BD[3 * rr + c] = B[3 * rr] * Di[c] + B[3 * rr + 1] * Di[3 + c] + B[3 * rr + 2] * Di[6 + c];
                c3[rr] += B[3 * rr] * db[0] + B[3 * rr + 1] * db[1] + B[3 * rr + 2] * db[2];
            }
        }
        for (int k = 0; k < 6; k++) cf[k] = (k / 3 == h) ? c3[k % 3] : 0.0;
    }
    for (int k = 0; k < 6; k++) cf[k] = wave_sum(cf[k]);
    if (lane == 0)
        for (int k = 0; k < 6; k++) s_cf[wv][k] = cf[k];
    __syncthreads();
    if (threadIdx.x < 6) {
        double t = 0.0;
        for (int w = 0; w < RT / 64; w++) t += s_cf[w][threadIdx.x];
        D.bs_part[6 * (size_t)rs + threadIdx.x] = t;
    }
    if (VALU) {
        const int g = lane >> 2, q = lane & 3;
        const int r0 = 3 * (q >> 1), c0 = 3 * (q & 1);
        const double *__restrict__ Hv = D.Hpl;
        for (int t = D.rs_chunk_start[rs] + wv; t < D.rs_chunk_start[rs + 1]; t += RT / 64) {
            const int ch = D.rs_chunk[t];
            const int q0 = D.chunk_start[ch], q1 = D.chunk_start[ch + 1];
            double acc[9];
#pragma unroll
            for (int k = 0; k < 9; k++) acc[k] = 0.0;
            for (int qq = q0 + g; qq < q1; qq += 16) {
                const int rank = D.pair_rank[qq] - rb;
                const int b = D.pair_b[qq];
                const double *BD = s_bd + 18 * rank + 3 * r0;  // rows r0..r0+2 of BD_i (6x3)
                const double *Bj = Hv + 18 * (size_t)b + 3 * c0;  // rows c0..c0+2 of Hpl_j (6x3)
                double av[9], bv[9];
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    av[k] = BD[k];
                    bv[k] = Bj[k];
                }
#pragma unroll
                for (int r = 0; r < 3; r++)
#pragma unroll
                    for (int c = 0; c < 3; c++)
                        acc[3 * r + c] += av[3 * r] * bv[3 * c] + av[3 * r + 1] * bv[3 * c + 1] + av[3 * r + 2] * bv[3 * c + 2];
            }
#pragma unroll
            for (int off = 4; off < 64; off <<= 1)
#pragma unroll
                for (int k = 0; k < 9; k++) acc[k] += __shfl_xor(acc[k], off);
            if (g == 0) {
                double *out = D.chunk_part + 36 * (size_t)ch;
#pragma unroll
                for (int r = 0; r < 3; r++)
#pragma unroll
                    for (int c = 0; c < 3; c++) out[6 * (r0 + r) + c0 + c] = acc[3 * r + c];
            }
        }
        return;
    }
    if (DIRECT) {
        // OSG_SCHUR_DIRECT=1: every lane loads its own element of Hpl_j straight from global memory
        // (no LDS staging, no wave barrier), 16 contributions' loads issued before their MFMAs; the
        // same operands in the same order as below, so the same sums
        for (; t < t1; t += RT / 64) {
            const i4 d2 = desc(t + 2 * (RT / 64));
            const int nq = dc.z;
            double acc0 = 0.0, acc1 = 0.0;
            int v = 0;
            for (; v + GC <= nq; v += GC) {
                double bv[GC];
#pragma unroll
                for (int w = 0; w < GC; w++) {
                    const int bj = __builtin_amdgcn_readlane(my_b, v + w);
                    bv[w] = Hv[18 * (size_t)bj + boff];
                }
#pragma unroll
                for (int w = 0; w < GC; w += 2) {
                    const int r0 = __builtin_amdgcn_readlane(my_rank, v + w);
                    const int r1 = __builtin_amdgcn_readlane(my_rank, v + w + 1);
                    acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * r0 + aoff], bv[w], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * r1 + aoff], bv[w + 1], acc1, 0, 0, 0);
                }
            }
            for (; v < nq; v++) {  // the tail one at a time, even / odd contributions as above
                const int bj = __builtin_amdgcn_readlane(my_b, v), rk = __builtin_amdgcn_readlane(my_rank, v);
                const double b1 = Hv[18 * (size_t)bj + boff];
                if (v & 1) acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * rk + aoff], b1, acc1, 0, 0, 0);
                else acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * rk + aoff], b1, acc0, 0, 0, 0);
            }
            if (orow < 6 && ocol < 6) D.chunk_part[36 * (size_t)dc.x + 6 * orow + ocol] = acc0 + acc1;
            dc = dn;
            my_rank = n_rank;
            my_b = n_b;
            dn = d2;
            contrib(dn, n_rank, n_b);
        }
        return;
    }
    // The descriptors and contributions (rank, block) of the wave's first two chunks were issued
    // before the BD staging above, so their latency overlaps it.  In the loop the descriptor two
    // chunks ahead is issued at the top and its contributions at the bottom: no dependent load chain
    // is waited on between chunks.
    load_group(0, dc.z, my_b, R);
    for (; t < t1; t += RT / 64) {
        const i4 d2 = desc(t + 2 * (RT / 64));
        const int nq = dc.z;
        double acc0 = 0.0, acc1 = 0.0;
        for (int u = 0; u < nq; u += GC) {
            const int cnt = min(GC, nq - u);
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const int idx = lane + 64 * r;
                if (idx < GC * 9 && idx < 9 * cnt) *(u4 *)(hb + 2 * idx) = R[r];
            }
            __builtin_amdgcn_wave_barrier();
            // next group: the rest of this chunk, else the first group of the next chunk
            if (u + GC < nq) load_group(u + GC, nq - u - GC, my_b, R);
            else load_group(0, dn.z, n_b, R);
            if (cnt == GC) {
                // a full group: straight-line, so the LDS reads of later contributions issue while
                // earlier MFMAs run (the guarded form below waits on each pair's reads)
#pragma unroll
                for (int v = 0; v < GC; v += 2) {
                    const int r0 = __builtin_amdgcn_readlane(my_rank, u + v);
                    const int r1 = __builtin_amdgcn_readlane(my_rank, u + v + 1);
                    acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * r0 + aoff], hb[18 * v + boff], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * r1 + aoff], hb[18 * (v + 1) + boff], acc1, 0, 0,
                                                              0);
                }
            } else {
#pragma unroll
                for (int v = 0; v < GC; v += 2) {
                    if (v < cnt) {
                        const int rank = __builtin_amdgcn_readlane(my_rank, u + v);
                        acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * rank + aoff], hb[18 * v + boff], acc0, 0, 0,
                                                                  0);
                    }
                    if (v + 1 < cnt) {
                        const int rank = __builtin_amdgcn_readlane(my_rank, u + v + 1);
                        acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * rank + aoff], hb[18 * (v + 1) + boff], acc1,
                                                                  0, 0, 0);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (orow < 6 && ocol < 6) D.chunk_part[36 * (size_t)dc.x + 6 * orow + ocol] = acc0 + acc1;
        dc = dn;
        my_rank = n_rank;
        my_b = n_b;
        dn = d2;
        contrib(dn, n_rank, n_b);
    }
}

// The Schur product on the compact per-block factor (the default; see z_rows).  The same row segments,
// chunks, MFMA layout, group pipeline and accumulation order as k_schur_rows<false>; what changes is what
// a contribution reads (the partner block's M', 48 B, instead of its Hpl, 144 B) and that the products
// are summed in the world frame, k_schur_pairs rotating each pose pair's sum once.
//   * BD staging: BD' = Z_a Dinv with Z_a = [[X + c_i]x M'_a ; M'_a] (pose i's c, the landmark's X from
//     lmX, landmark order), and the segment's share of b_schur as sum Z_a Dinv b_l (rotated later too);
//     X is kept in LDS per rank for the chunks.
//   * Chunks, per group of GC contributions: lane 3 c + k (c < GC) loads column k of contribution c's M'
//     (three 8-byte loads inside one 48-byte block, shared lines across the contribution's three lanes;
//     one group ahead, as the whole-Hpl form's granules) and, at the group, writes column k of
//     [[X]x M' ; M'] (X from LDS, 6 FMA, no pose) into the wave's LDS tile: the transposed operand
//     [-M'[X]x | M'] of the product.  A chunk's partial is [B | A] of the comment above z_rows.
// PF = 2 (the default): the gathers two groups ahead, a group pair at a time (see the loop); PF = 1
// (OSG_SCHUR_PF=1) one group ahead
// WPE: the waves per SIMD the register allocation must allow (6: 80 VGPRs; 5: 92)
#ifdef OSG_SR_PROF
// profiling builds only (make SR_PROF=1): per workgroup of graph 0, wall-clock ticks (100 MHz) at the start,
// after the BD staging and at each wave's end, the segment's chunk count and blocks, the XCC / CU it ran on
constexpr int SR_PROF_N = 1024;
__device__ unsigned long long g_sr_prof[SR_PROF_N][13];
#define SR_PROF_AT(slot) \
    if (by == 0 && bx < SR_PROF_N && (threadIdx.x & 63) == 0) g_sr_prof[bx][slot] = wall_clock64()
#else
#define SR_PROF_AT(slot)
#endif
// HOIST (OSG_SCHUR_HOIST=1, A/B): the first group's gathers are issued between the staging's index loads and
// its block loads, so their latency overlaps the staging instead of following it (15 VGPRs spilled in the
// staging for it; without it the kernel allocates 80 VGPRs with none)
template <int PF = 1, int WPE = 6, bool HOIST = false>
__global__ __launch_bounds__(RT, WPE) void k_schur_rows_c(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    if (bx >= D.n_rs) return;
    if (threadIdx.x == 0) SR_PROF_AT(0);
    typedef int i4 __attribute__((ext_vector_type(4)));
    const i4 inf0 = ((const GLOBAL i4 *)gbl(D.rs_info))[2 * bx];
    const i4 inf1 = ((const GLOBAL i4 *)gbl(D.rs_info))[2 * bx + 1];
    const int rs = __builtin_amdgcn_readfirstlane(inf0.x), pi = __builtin_amdgcn_readfirstlane(inf0.y);
    const int rb = __builtin_amdgcn_readfirstlane(inf0.z), hb0 = __builtin_amdgcn_readfirstlane(inf0.w);
    const int nr = __builtin_amdgcn_readfirstlane(inf1.x);
    const double lam = D.ctl->lambda;
    constexpr int GC = 16;
    __shared__ double s_bd[RS * 18 + 2];  // + a zero: the MFMA's K-padding lanes read it
    __shared__ double s_xw[RS * 3];       // per rank: its landmark's current position
    __shared__ double s_cf[RT / 64][6];
    __shared__ __attribute__((aligned(16))) double s_hb[RT / 64][GC * 18];
    if (threadIdx.x == 0) s_bd[RS * 18] = 0.0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int kk = lane >> 4, beta = (lane >> 2) & 3, ri = lane & 3;
    const int arow = 4 * (beta >> 1) + ri, bcol = 4 * (beta & 1) + ri;
    const int a_m = kk < 3 ? 18 : 0;
    const int aoff = kk < 3 ? 3 * min(arow, 5) + kk : RS * 18;
    const int boff = 3 * min(bcol, 5) + min(kk, 2);
    const int orow = 4 * (beta >> 1) + kk, ocol = 4 * (beta & 1) + ri;
    const GLOBAL double *__restrict__ Mv = gbl(D.Hpl);
    double *hb = s_hb[wv];
    const int t1 = __builtin_amdgcn_readfirstlane(inf1.z);
    int t = __builtin_amdgcn_readfirstlane(inf1.y) + wv;
    const GLOBAL i4 *__restrict__ cd = (const GLOBAL i4 *)gbl(D.rs_cdesc);
    auto desc = [&](int tt) -> i4 {
        i4 d = tt < t1 ? cd[tt] : i4{0, 0, 0, 0};
        return i4{__builtin_amdgcn_readfirstlane(d.x), __builtin_amdgcn_readfirstlane(d.y),
                  __builtin_amdgcn_readfirstlane(d.z), 0};
    };
    auto contrib = [&](const i4 &d, int &mr, int &mb) {
        mr = lane < d.z ? gbl(D.pair_rank)[d.y + lane] - rb : 0;
        mb = lane < d.z ? gbl(D.pair_b)[d.y + lane] : 0;
    };
    // the column roles: lane 3 rc + rk, rc < GC; column rk of the symmetric M' = (m00 m01 m02 m11 m12 m22)
    const int rc = lane / 3, rk = lane - 3 * rc;
    const bool rl = rc < GC;
    const int mo0 = rk, mo1 = rk == 0 ? 1 : (rk == 1 ? 3 : 4), mo2 = rk == 0 ? 2 : (rk == 1 ? 4 : 5);
    auto load_col = [&](int u0, int cnt, int mb, double (&Mc)[3]) {
        const int bj = __shfl(mb, (u0 + rc) & 63);
        if (rl && rc < cnt) {
            const GLOBAL double *src = Mv + 6 * (size_t)bj;
            Mc[0] = src[mo0];
            Mc[1] = src[mo1];
            Mc[2] = src[mo2];
        }
    };
    i4 dc = desc(t), dn = desc(t + RT / 64);
    // PF == 4: the wave's chunks t + 8 k, one descriptor per lane (k < 64), loaded before the staging, so no
    // chunk waits for its descriptor (desc() of the chunk two ahead waited at the top of every iteration)
    const int nchw = t < t1 ? (t1 - t + RT / 64 - 1) / (RT / 64) : 0;
    i4 dl = i4{0, 0, 0, 0};
    if (PF == 4 && lane < nchw) dl = cd[t + (RT / 64) * lane];
    int my_rank = 0, my_b = 0, n_rank = 0, n_b = 0;
    contrib(dc, my_rank, my_b);
    contrib(dn, n_rank, n_b);
    double cf[6] = {0, 0, 0, 0, 0, 0};
    double M0[3] = {0, 0, 0}, M1[3] = {0, 0, 0};  // PF >= 2: the gathers of the wave's first group pair
    static_assert(2 * RS <= RT, "one block per thread pair in the staging");
    {
        const double *ci = D.hp_Rt + RT_STRIDE * (size_t)pi + 12;  // pose i's c = R^T t
        const double c0 = ci[0], c1 = ci[1], c2 = ci[2];
        const int h = threadIdx.x & 1;  // two threads per block: rows 3h .. 3h + 2
        double c3[3] = {0, 0, 0};
        const bool st = (int)threadIdx.x < 2 * nr;
        const int r = threadIdx.x >> 1;
        const int a = st ? gbl(D.hp_b)[hb0 + rb + r] : 0;
        const int l = st ? gbl(D.hp_b_lm)[hb0 + rb + r] : 0;
        if (HOIST) load_col(0, dc.z, my_b, M0);
        if (st) {
            // this thread's half of Z_a first (rows 3h .. 3h + 2: [X + c_i]x M' for h = 0, M' for h = 1), so
            // that M' is dead before Dinv is formed (the whole Z beside Dinv spilled)
            double Zh[3][3];
            const double X0 = gbl(D.lmX)[D.ls_x * (size_t)l], X1 = gbl(D.lmX)[D.ls_x * (size_t)l + 1],
                         X2 = gbl(D.lmX)[D.ls_x * (size_t)l + 2];
            {
                const GLOBAL double *mp = Mv + 6 * (size_t)a;
                const double m00 = mp[0], m01 = mp[1], m02 = mp[2], m11 = mp[3], m12 = mp[4], m22 = mp[5];
                const double M[3][3] = {{m00, m01, m02}, {m01, m11, m12}, {m02, m12, m22}};
                const double x = X0 + c0, y = X1 + c1, z = X2 + c2;
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    Zh[0][k] = h ? M[0][k] : y * M[2][k] - z * M[1][k];
                    Zh[1][k] = h ? M[1][k] : z * M[0][k] - x * M[2][k];
                    Zh[2][k] = h ? M[2][k] : x * M[1][k] - y * M[0][k];
                }
            }
            if (h == 0) {  // X is dead from here on
                s_xw[3 * r] = X0;
                s_xw[3 * r + 1] = X1;
                s_xw[3 * r + 2] = X2;
            }
            double Di[9], db[3];
            if (D.dinv_inline) {
                landmark_dinv(D, l, lam, Di, db);
            } else {
                for (int k = 0; k < 9; k++) Di[k] = gbl(D.Dinv)[9 * (size_t)l + k];
                for (int k = 0; k < 3; k++) db[k] = gbl(D.db)[3 * (size_t)l + k];
            }
            double *BD = s_bd + 18 * r + 9 * h;
            for (int rr = 0; rr < 3; rr++) {
                const double *B = Zh[rr];
                for (int c = 0; c < 3; c++)
                    BD[3 * rr + c] = B[0] * Di[c] + B[1] * Di[3 + c] + B[2] * Di[6 + c];
                c3[rr] += B[0] * db[0] + B[1] * db[1] + B[2] * db[2];
            }
        }
        for (int k = 0; k < 6; k++) cf[k] = (k / 3 == h) ? c3[k % 3] : 0.0;
    }
    for (int k = 0; k < 6; k++) cf[k] = wave_sum(cf[k]);
    if (lane == 0)
        for (int k = 0; k < 6; k++) s_cf[wv][k] = cf[k];
    __syncthreads();
    if (threadIdx.x == 0) SR_PROF_AT(1);
    if (threadIdx.x < 6) {
        double tt = 0.0;
        for (int w = 0; w < RT / 64; w++) tt += s_cf[w][threadIdx.x];
        D.bs_part[6 * (size_t)rs + threadIdx.x] = tt;
    }
    double Mc[3] = {0, 0, 0};
    // one group of GC contributions: its operand rows into the tile, then its MFMAs
    auto run_group = [&](int u, int cnt, const double (&Mg)[3], double &acc0, double &acc1) {
        {
            const int rank = __shfl(my_rank, (u + rc) & 63);
            const double x = s_xw[3 * rank], y = s_xw[3 * rank + 1], z = s_xw[3 * rank + 2];
            if (rl && rc < cnt) {
                double *dst = hb + 18 * rc + rk;
                dst[0] = y * Mg[2] - z * Mg[1];
                dst[3] = z * Mg[0] - x * Mg[2];
                dst[6] = x * Mg[1] - y * Mg[0];
                dst[9] = Mg[0];
                dst[12] = Mg[1];
                dst[15] = Mg[2];
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (cnt == GC) {
#pragma unroll
            for (int v = 0; v < GC; v += 2) {
                const int r0 = __builtin_amdgcn_readlane(my_rank, u + v);
                const int r1 = __builtin_amdgcn_readlane(my_rank, u + v + 1);
                acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * r0 + aoff], hb[18 * v + boff], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * r1 + aoff], hb[18 * (v + 1) + boff], acc1, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int v = 0; v < GC; v += 2) {
                if (v < cnt) {
                    const int rank = __builtin_amdgcn_readlane(my_rank, u + v);
                    acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * rank + aoff], hb[18 * v + boff], acc0, 0, 0, 0);
                }
                if (v + 1 < cnt) {
                    const int rank = __builtin_amdgcn_readlane(my_rank, u + v + 1);
                    acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * rank + aoff], hb[18 * (v + 1) + boff], acc1, 0,
                                                              0, 0);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    };
    if (PF >= 2) {
        // group pairs (u, u + GC) of a chunk: the next pair's gathers (the rest of this chunk, else the
        // next chunk's first pair) are issued before this pair's first group, so 2 GC contributions'
        // loads are in flight while a pair runs; the same products in the same order
        if (!HOIST) load_col(0, dc.z, my_b, M0);
        load_col(GC, dc.z - GC, my_b, M1);
        // PF == 3: a chunk is mostly one group, so the chain descriptor -> (rank, block) -> M' spans
        // iterations: descriptors are loaded four chunks ahead (raw, in VGPRs) and made uniform three
        // ahead, and a chunk's (rank, block) loads then never wait on a descriptor of the same iteration
        auto desc_raw = [&](int tt) -> i4 { return tt < t1 ? cd[tt] : i4{0, 0, 0, 0}; };
        auto uni = [&](const i4 &d) -> i4 {
            return i4{__builtin_amdgcn_readfirstlane(d.x), __builtin_amdgcn_readfirstlane(d.y),
                      __builtin_amdgcn_readfirstlane(d.z), 0};
        };
        if (PF == 4) {
            // the descriptors come from dl by readlane; the (rank, block) loads of chunk k + 2 are issued at
            // the top of chunk k and hold raw values until its end (the "- rb" right after a load made it wait
            // at once), so every load has a whole chunk to land
            auto dsc = [&](int k) -> i4 {
                if (k >= nchw) return i4{0, 0, 0, 0};
                if (k < 64)
                    return i4{__builtin_amdgcn_readlane(dl.x, k), __builtin_amdgcn_readlane(dl.y, k),
                              __builtin_amdgcn_readlane(dl.z, k), 0};
                return desc(t + (RT / 64) * k);  // past 64 chunks of one wave (rare): a direct load
            };
            // loads without branches: a load under a lane guard is skipped by a branch when no lane needs
            // it, and across such branches the compiler cannot count the loads in flight, so it waits for
            // all of them (vmcnt(0)); a clamped index keeps every load in the straight line
            auto contrib_raw = [&](const i4 &d, int &mr, int &mb) {
                const int qi = d.y + min(lane, max(d.z - 1, 0));
                const int vr = gbl(D.pair_rank)[qi], vb = gbl(D.pair_b)[qi];
                mr = lane < d.z ? vr : rb;
                mb = lane < d.z ? vb : 0;
            };
            auto load_col_u = [&](int u0, int cnt, int mb, double (&Mc)[3]) {
                const int bs = __shfl(mb, (u0 + rc) & 63);  // every lane takes part: bpermute reads
                const int bj = (rl && rc < cnt) ? bs : 0;     // nothing from lanes outside EXEC
                const GLOBAL double *src = Mv + 6 * (size_t)bj;
                Mc[0] = src[mo0];
                Mc[1] = src[mo1];
                Mc[2] = src[mo2];
            };
            int nrr = n_rank + rb;  // chunk k + 1's raw rank (n_rank came through contrib)
            // one chunk: dcur's contributions in (my_rank, my_b); the next chunk's in (nrr, n_b)
            auto chunk = [&](int k, int &la, int &lb) {
                const i4 dcur = dsc(k), dnext = dsc(k + 1), dnn = dsc(k + 2);
                contrib_raw(dnn, la, lb);
                const int nq = dcur.z;
                double acc0 = 0.0, acc1 = 0.0;
                for (int u = 0; u < nq; u += 2 * GC) {
                    double N0[3], N1[3];
                    const bool inner = u + 2 * GC < nq;
                    const int u2 = inner ? u + 2 * GC : 0, c2 = inner ? nq - u - 2 * GC : dnext.z;
                    const int mbn = inner ? my_b : n_b;
                    load_col_u(u2, c2, mbn, N0);
                    load_col_u(u2 + GC, c2 - GC, mbn, N1);
                    run_group(u, min(GC, nq - u), M0, acc0, acc1);
                    if (u + GC < nq) run_group(u + GC, min(GC, nq - u - GC), M1, acc0, acc1);
#pragma unroll
                    for (int q = 0; q < 3; q++) {
                        M0[q] = N0[q];
                        M1[q] = N1[q];
                    }
                }
                if (orow < 6 && ocol < 6) D.chunk_part[36 * (size_t)dcur.x + 6 * orow + ocol] = acc0 + acc1;
                my_rank = nrr - rb;
                my_b = n_b;
            };
            for (int k = 0; k < nchw; k++) {
                int la = rb, lb = 0;
                chunk(k, la, lb);  // chunk k + 2's loads into (la, lb) at its top
                nrr = la;          // ... the next chunk's "next"
                n_b = lb;
            }
#ifdef OSG_SR_PROF
            SR_PROF_AT(2 + wv);
#endif
            return;
        }
        i4 dn2 = PF == 3 ? desc(t + 2 * (RT / 64)) : i4{0, 0, 0, 0};
        i4 raw1 = PF == 3 ? desc_raw(t + 3 * (RT / 64)) : i4{0, 0, 0, 0};
        for (; t < t1; t += RT / 64) {
            const i4 d2 = PF == 3 ? i4{0, 0, 0, 0} : desc(t + 2 * (RT / 64));
            const i4 raw0 = PF == 3 ? desc_raw(t + 4 * (RT / 64)) : i4{0, 0, 0, 0};
            const int nq = dc.z;
            double acc0 = 0.0, acc1 = 0.0;
            for (int u = 0; u < nq; u += 2 * GC) {
                // the next pair's gathers land in N0 / N1 and move into M0 / M1 after this pair's groups: a
                // copy at the top (the loop-carried registers reused by the new loads) waited for the last
                // pair's gathers before the next ones were even issued
                double N0[3] = {0, 0, 0}, N1[3] = {0, 0, 0};
                if (u + 2 * GC < nq) {
                    load_col(u + 2 * GC, nq - u - 2 * GC, my_b, N0);
                    load_col(u + 3 * GC, nq - u - 3 * GC, my_b, N1);
                } else {
                    load_col(0, dn.z, n_b, N0);
                    load_col(GC, dn.z - GC, n_b, N1);
                }
                run_group(u, min(GC, nq - u), M0, acc0, acc1);
                if (u + GC < nq) run_group(u + GC, min(GC, nq - u - GC), M1, acc0, acc1);
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    M0[k] = N0[k];
                    M1[k] = N1[k];
                }
            }
            if (orow < 6 && ocol < 6) D.chunk_part[36 * (size_t)dc.x + 6 * orow + ocol] = acc0 + acc1;
            dc = dn;
            my_rank = n_rank;
            my_b = n_b;
            if (PF == 3) {
                dn = dn2;
                dn2 = uni(raw1);
                raw1 = raw0;
            } else {
                dn = d2;
            }
            contrib(dn, n_rank, n_b);
        }
#ifdef OSG_SR_PROF
        SR_PROF_AT(2 + wv);
        if (by == 0 && bx < SR_PROF_N && threadIdx.x == 0) {
            g_sr_prof[bx][10] = (unsigned long long)(t1 - __builtin_amdgcn_readfirstlane(inf1.y));
            g_sr_prof[bx][11] = (unsigned long long)nr;
            // XCC_ID (hardware register 20, bits 0..3) and HW_ID (4) bits 8..15 (CU, SH, SE)
            g_sr_prof[bx][12] = (unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) |
                                ((unsigned long long)__builtin_amdgcn_s_getreg((7 << 11) | (8 << 6) | 4) << 32);
        }
#endif
        return;
    }
    load_col(0, dc.z, my_b, Mc);
    for (; t < t1; t += RT / 64) {
        const i4 d2 = desc(t + 2 * (RT / 64));
        const int nq = dc.z;
        double acc0 = 0.0, acc1 = 0.0;
        for (int u = 0; u < nq; u += GC) {
            const int cnt = min(GC, nq - u);
            {
                // column rk of contribution u + rc's operand rows [[X]x M' ; M'] into the tile
                const int rank = __shfl(my_rank, (u + rc) & 63);
                const double x = s_xw[3 * rank], y = s_xw[3 * rank + 1], z = s_xw[3 * rank + 2];
                if (rl && rc < cnt) {
                    double *dst = hb + 18 * rc + rk;
                    dst[0] = y * Mc[2] - z * Mc[1];
                    dst[3] = z * Mc[0] - x * Mc[2];
                    dst[6] = x * Mc[1] - y * Mc[0];
                    dst[9] = Mc[0];
                    dst[12] = Mc[1];
                    dst[15] = Mc[2];
                }
            }
            __builtin_amdgcn_wave_barrier();
            // next group: the rest of this chunk, else the first group of the next chunk
            if (u + GC < nq) load_col(u + GC, nq - u - GC, my_b, Mc);
            else load_col(0, dn.z, n_b, Mc);
            if (cnt == GC) {
#pragma unroll
                for (int v = 0; v < GC; v += 2) {
                    const int r0 = __builtin_amdgcn_readlane(my_rank, u + v);
                    const int r1 = __builtin_amdgcn_readlane(my_rank, u + v + 1);
                    acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * r0 + aoff], hb[18 * v + boff], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * r1 + aoff], hb[18 * (v + 1) + boff], acc1, 0, 0,
                                                              0);
                }
            } else {
#pragma unroll
                for (int v = 0; v < GC; v += 2) {
                    if (v < cnt) {
                        const int rank = __builtin_amdgcn_readlane(my_rank, u + v);
                        acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * rank + aoff], hb[18 * v + boff], acc0, 0, 0,
                                                                  0);
                    }
                    if (v + 1 < cnt) {
                        const int rank = __builtin_amdgcn_readlane(my_rank, u + v + 1);
                        acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(s_bd[a_m * rank + aoff], hb[18 * (v + 1) + boff], acc1,
                                                                  0, 0, 0);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (orow < 6 && ocol < 6) D.chunk_part[36 * (size_t)dc.x + 6 * orow + ocol] = acc0 + acc1;
        dc = dn;
        my_rank = n_rank;
        my_b = n_b;
        dn = d2;
        contrib(dn, n_rank, n_b);
    }
}

// The same product with the partner blocks staged (OSG_SCHUR_STAGE=1).  A row segment's contributions
// (a, b) pair each of its blocks a (landmark l) with the blocks b >= a of l, and a landmark's blocks
// are consecutive (numbered landmark-major, sorted by pose): the partners of rank r are the span
// [a_r, end of l).  The workgroup copies every span of the segment into LDS once (contiguous global
// reads, issued together), forms BD from the staged Hpl_a, and its 16 waves then run the chunk loop
// on LDS operands only.  Slots past the LDS capacity (a segment whose landmarks are observed by
// unusually many poses) read Hpl_b from global memory.  Same products, same accumulation order as
// k_schur_rows<false>: the results are bit-identical.
constexpr int RT2 = 1024;               // 16 waves: one workgroup per CU (its LDS)
constexpr int SPAN_CAP = 880;           // staged blocks: 880 x 144 B = 124 KiB
__global__ __launch_bounds__(RT2, 1) void k_schur_rows_st(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    if (bx >= D.n_rs) return;
    typedef int i4 __attribute__((ext_vector_type(4)));
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const i4 inf0 = ((const GLOBAL i4 *)gbl(D.rs_info))[2 * bx];
    const i4 inf1 = ((const GLOBAL i4 *)gbl(D.rs_info))[2 * bx + 1];
    const int rs = __builtin_amdgcn_readfirstlane(inf0.x);
    const int rb = __builtin_amdgcn_readfirstlane(inf0.z), hb0 = __builtin_amdgcn_readfirstlane(inf0.w);
    const int nr = __builtin_amdgcn_readfirstlane(inf1.x);
    __shared__ __attribute__((aligned(16))) double s_span[SPAN_CAP * 18];
    __shared__ double s_bd[RS * 18 + 2];
    __shared__ int s_pre[RS + 1], s_a[RS];
    __shared__ double s_cf[RT2 / 64][6];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const GLOBAL double *__restrict__ Hv = gbl(D.Hpl);
    // 1. spans: first block and length per rank, exclusive prefix (wave 0: 4 ranks per lane)
    if (wv == 0) {
        int len[4], a4[4], tot = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int r = 4 * lane + u;
            len[u] = 0;
            a4[u] = 0;
            if (r < nr) {
                a4[u] = gbl(D.hp_b)[hb0 + rb + r];
                const int l = gbl(D.hp_b_lm)[hb0 + rb + r];
                len[u] = gbl(D.lm_b_start)[l + 1] - a4[u];
            }
            tot += len[u];
        }
        int inc = tot;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int v = __shfl_up(inc, off);
            if (lane >= off) inc += v;
        }
        int run = inc - tot;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int r = 4 * lane + u;
            if (r < nr) {
                s_pre[r] = run;
                s_a[r] = a4[u];
            }
            run += len[u];
        }
        if (lane == 63) s_pre[nr] = inc;
        if (threadIdx.x == 0) s_bd[RS * 18] = 0.0;
    }
    __syncthreads();
    // 2. stage the spans: wave w copies ranks w, w + 16, ...; a span is len x 9 16-byte granules,
    // contiguous in global memory
    for (int r = wv; r < nr; r += RT2 / 64) {
        const int p0 = s_pre[r], n9 = 9 * (s_pre[r + 1] - p0), a = s_a[r];
        for (int g = lane; g < n9; g += 64) {
            const int slot = p0 + g / 9;
            if (slot < SPAN_CAP)
                *(u4 *)(s_span + 18 * (size_t)slot + 2 * (g % 9)) = *(const GLOBAL u4 *)(Hv + 18 * (size_t)a + 2 * g);
        }
    }
    __syncthreads();
    // 3. BD = Hpl_a Dinv_l into LDS with the segment's share of b_schur (as k_schur_rows)
    double cf[6] = {0, 0, 0, 0, 0, 0};
    {
        const int h = threadIdx.x & 1;
        double c3[3] = {0, 0, 0};
        for (int r2 = threadIdx.x; r2 < 2 * nr; r2 += RT2) {
            const int r = r2 >> 1;
            const int l = gbl(D.hp_b_lm)[hb0 + rb + r];
            const int p0 = s_pre[r];
            double Di[9], db[3], B[9];
            if (D.dinv_inline) {
                landmark_dinv(D, l, D.ctl->lambda, Di, db);
            } else {
                for (int k = 0; k < 9; k++) Di[k] = gbl(D.Dinv)[9 * (size_t)l + k];
                for (int k = 0; k < 3; k++) db[k] = gbl(D.db)[3 * (size_t)l + k];
            }
            if (p0 < SPAN_CAP)
                for (int k = 0; k < 9; k++) B[k] = s_span[18 * (size_t)p0 + 9 * h + k];
            else
                for (int k = 0; k < 9; k++) B[k] = Hv[18 * (size_t)s_a[r] + 9 * h + k];
            double *BD = s_bd + 18 * r + 9 * h;
            for (int rr = 0; rr < 3; rr++) {
                for (int c = 0; c < 3; c++)
                    BD[3 * rr + c] = B[3 * rr] * Di[c] + B[3 * rr + 1] * Di[3 + c] + B[3 * rr + 2] * Di[6 + c];
                c3[rr] += B[3 * rr] * db[0] + B[3 * rr + 1] * db[1] + B[3 * rr + 2] * db[2];
            }
        }
        for (int k = 0; k < 6; k++) cf[k] = (k / 3 == h) ? c3[k % 3] : 0.0;
    }
    // the butterfly in the same lane order as k_schur_rows (RT = 512: waves 0..7 summed), then the
    // 16 waves in order
    for (int k = 0; k < 6; k++) cf[k] = wave_sum(cf[k]);
    if (lane == 0)
        for (int k = 0; k < 6; k++) s_cf[wv][k] = cf[k];
    __syncthreads();
    if (threadIdx.x < 6) {
        double t = 0.0;
        for (int w = 0; w < RT2 / 64; w++) t += s_cf[w][threadIdx.x];
        D.bs_part[6 * (size_t)rs + threadIdx.x] = t;
    }
    // 4. the chunks: per lane q (< count) the contribution's rank and its partner's slot
    const int kk = lane >> 4, beta = (lane >> 2) & 3, ri = lane & 3;
    const int arow = 4 * (beta >> 1) + ri, bcol = 4 * (beta & 1) + ri;
    const int a_m = kk < 3 ? 18 : 0;
    const int aoff = kk < 3 ? 3 * min(arow, 5) + kk : RS * 18;
    const int boff = 3 * min(bcol, 5) + min(kk, 2);
    const int orow = 4 * (beta >> 1) + kk, ocol = 4 * (beta & 1) + ri;
    const int t1 = __builtin_amdgcn_readfirstlane(inf1.z);
    const GLOBAL i4 *__restrict__ cd = (const GLOBAL i4 *)gbl(D.rs_cdesc);
    for (int t = __builtin_amdgcn_readfirstlane(inf1.y) + wv; t < t1; t += RT2 / 64) {
        const i4 d = cd[t];
        const int ch = __builtin_amdgcn_readfirstlane(d.x), q0 = __builtin_amdgcn_readfirstlane(d.y);
        const int nq = __builtin_amdgcn_readfirstlane(d.z);
        int rank = 0, slot = 0, bblk = 0;
        if (lane < nq) {
            rank = gbl(D.pair_rank)[q0 + lane] - rb;
            bblk = gbl(D.pair_b)[q0 + lane];
            slot = s_pre[rank] + bblk - s_a[rank];
        }
        double acc0 = 0.0, acc1 = 0.0;
        for (int v = 0; v < nq; v++) {
            const int rk = __builtin_amdgcn_readlane(rank, v), sl = __builtin_amdgcn_readlane(slot, v);
            const double av = s_bd[a_m * rk + aoff];
            const double bv = sl < SPAN_CAP ? s_span[18 * sl + boff]
                                            : Hv[18 * (size_t)__builtin_amdgcn_readlane(bblk, v) + boff];
            if (v & 1) acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(av, bv, acc1, 0, 0, 0);
            else acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(av, bv, acc0, 0, 0, 0);
        }
        if (orow < 6 && ocol < 6) D.chunk_part[36 * (size_t)ch + 6 * orow + ocol] = acc0 + acc1;
    }
}

__global__ __launch_bounds__(256) void k_schur_pairs(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    const double lambda = D.ctl->lambda;
    const int slot = (bx * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (slot >= (D.live_pairs ? D.n_live : D.npairs)) return;
    if (slot == 0 && lane == 0) D.flag[0] = 1;  // the Cholesky of this trial clears it on failure
    const int wave = D.live_pairs ? D.live_pairs[slot] : slot;  // the pair's index (i-major, j >= i)
    // pair index -> (i, j): start(i) = i nhp - i (i - 1) / 2 <= wave < start(i + 1), from the root of
    // the quadratic, then corrected by one either way for rounding
    const long long m = D.nhp;
    int i = (int)(((2.0 * m + 1.0) - sqrt((2.0 * m + 1.0) * (2.0 * m + 1.0) - 8.0 * (double)wave)) * 0.5);
    auto start = [&](long long a) { return a * m - a * (a - 1) / 2; };
    i = max(0, min(i, (int)m - 1));
    while (i > 0 && start(i) > wave) i--;
    while (i + 1 < m && start(i + 1) <= wave) i++;
    const int j = i + (int)(wave - start(i));
    const int n = 6 * D.nhp;
    if (D.compact) {
        // the compact factor's chunks summed [B | A] in the world frame (see z_rows): the pair's sum T,
        // then S_ij = D(R_i) [B - A [c_j]x | A] D(R_j)^T; b_schur's share likewise D(R_i) v.  A wave is a chain
        // of memory round trips, so the lane's rotation operands (and Hpp on the diagonal) are loaded before
        // the sums, and the sums load four partials at a time (added in the same order)
        __shared__ double s_T[4][48];
        double *T = s_T[threadIdx.x >> 6];
        const GLOBAL double *Ri = gbl(D.hp_Rt) + RT_STRIDE * (size_t)i, *Rj = gbl(D.hp_Rt) + RT_STRIDE * (size_t)j;
        const int r = lane / 6, c = lane % 6, k6 = lane - 36;
        const bool prow = lane < 36, brow = !prow && i == j && lane < 42;
        double ri[3] = {0, 0, 0}, rj[3] = {0, 0, 0}, cj[3] = {0, 0, 0}, hpp = 0.0;
        if (prow) {
            for (int q = 0; q < 3; q++) {
                ri[q] = Ri[3 * (r % 3) + q];
                rj[q] = Rj[3 * (c % 3) + q];
                cj[q] = Rj[12 + q];
            }
            if (i == j) hpp = gbl(D.Hpp)[36 * (size_t)i + lane];
        } else if (brow) {
            for (int q = 0; q < 3; q++) ri[q] = Ri[3 * (k6 % 3) + q];
        }
        // sum_{t in [t0, t1)} src[stride t], in t order, four loads in flight
        auto ordered_sum = [](const GLOBAL double *src, size_t stride, int t0, int t1) {
            double acc = 0.0;
            int t = t0;
            for (; t + 4 <= t1; t += 4) {
                const double v0 = src[stride * t], v1 = src[stride * (t + 1)], v2 = src[stride * (t + 2)],
                             v3 = src[stride * (t + 3)];
                acc += v0;
                acc += v1;
                acc += v2;
                acc += v3;
            }
            const int rem = t1 - t;
            const double w0 = rem > 0 ? src[stride * t] : 0.0, w1 = rem > 1 ? src[stride * (t + 1)] : 0.0,
                         w2 = rem > 2 ? src[stride * (t + 2)] : 0.0;
            if (rem > 0) acc += w0;
            if (rem > 1) acc += w1;
            if (rem > 2) acc += w2;
            return acc;
        };
        if (prow) {
            const int ch0 = D.live_chunk ? D.live_chunk[2 * slot] : D.pair_chunk[wave];
            const int ch1 = D.live_chunk ? D.live_chunk[2 * slot + 1] : D.pair_chunk[wave + 1];
            T[lane] = ordered_sum(gbl(D.chunk_part) + lane, 36, ch0, ch1);
        } else if (brow) {
            T[lane] = ordered_sum(gbl(D.bs_part) + k6, 6, D.hp_rs_start[i], D.hp_rs_start[i + 1]);
        }
        __builtin_amdgcn_wave_barrier();
        __shared__ double s_U[4][36];
        double *Uw = s_U[threadIdx.x >> 6];
        if (prow) {
            const int mb = 3 * (c / 3);
            // T' = [B - A [c_j]x | A] (element (r, c) of it), then U = T' D(R_j)^T, S = D(R_i) U
            double tp = T[lane];
            if (c < 3) {
                const double a0 = T[6 * r + 3], a1 = T[6 * r + 4], a2 = T[6 * r + 5];
                tp -= c == 0 ? a1 * cj[2] - a2 * cj[1] : (c == 1 ? a2 * cj[0] - a0 * cj[2] : a0 * cj[1] - a1 * cj[0]);
            }
            __builtin_amdgcn_wave_barrier();
            T[lane] = tp;
            __builtin_amdgcn_wave_barrier();
            Uw[lane] = T[6 * r + mb] * rj[0] + T[6 * r + mb + 1] * rj[1] + T[6 * r + mb + 2] * rj[2];
            __builtin_amdgcn_wave_barrier();
            const int kb = 3 * (r / 3);
            const double sv = ri[0] * Uw[6 * kb + c] + ri[1] * Uw[6 * (kb + 1) + c] + ri[2] * Uw[6 * (kb + 2) + c];
            double v = -sv;
            if (i == j) {
                v += hpp;
                if (r == c) v += lambda;
            }
            if (hs_stored(D, 6 * i + r, 6 * j + c)) D.Hs[hs_at(D, n, 6 * i + r, 6 * j + c)] = v;
            if (i != j && hs_stored(D, 6 * j + c, 6 * i + r)) D.Hs[hs_at(D, n, 6 * j + c, 6 * i + r)] = v;
        } else if (brow) {
            const int kb = 36 + 3 * (k6 / 3);
            const double rv = ri[0] * T[kb] + ri[1] * T[kb + 1] + ri[2] * T[kb + 2];
            D.bs[6 * i + k6] = D.bp[6 * (size_t)i + k6] - rv;
        }
        return;
    }
    if (lane < 36) {
        const int r = lane / 6, c = lane % 6;
        double acc = 0.0;
        const int ch0 = D.live_chunk ? D.live_chunk[2 * slot] : D.pair_chunk[wave];
        const int ch1 = D.live_chunk ? D.live_chunk[2 * slot + 1] : D.pair_chunk[wave + 1];
        for (int ch = ch0; ch < ch1; ch++) acc += D.chunk_part[36 * (size_t)ch + lane];
        double v = -acc;
        if (i == j) {
            v += D.Hpp[36 * (size_t)i + lane];
            if (r == c) v += lambda;
        }
        if (hs_stored(D, 6 * i + r, 6 * j + c)) D.Hs[hs_at(D, n, 6 * i + r, 6 * j + c)] = v;
        if (i != j && hs_stored(D, 6 * j + c, 6 * i + r)) D.Hs[hs_at(D, n, 6 * j + c, 6 * i + r)] = v;
    } else if (i == j && lane < 42) {  // b_schur_i = b_p,i - its row segments' sums, in segment order
        const int k = lane - 36;
        double t = 0.0;
        for (int rs = D.hp_rs_start[i]; rs < D.hp_rs_start[i + 1]; rs++) t += D.bs_part[6 * (size_t)rs + k];
        D.bs[6 * i + k] = D.bp[6 * (size_t)i + k] - t;
    }
}

// ---------------------------------------------------------------------------------------------
// Reduced camera system: blocked left-looking Cholesky (L L^T, lower, in place in Hs) over column
// blocks of CB = 32, one launch per column block (k_chol_col: FP64-MFMA update of the block's
// tiles from all previous columns, LDS factorisation of the diagonal tile, its inverse, L21 as
// X L^-T, forward substitution fused), then k_chol_back.  The MFMA tile updates are the dense
// Schur GEMM of the path.  A non-positive pivot clears flag[0] (g2o's solvers then reject the step).
constexpr int CB = 32;
constexpr int CMAX = 384;  // max reduced dimension (64 free poses)
typedef double d4 __attribute__((ext_vector_type(4)));

// Left-looking tile updates of column block j on FP64 MFMA (v_mfma_f64_16x16x4f64):
//   sT = A_jj - sum_{m < K} L_jm L_jm^T      (the diagonal tile)
//   sX = A_tj - sum_{m < K} L_tm L_jm^T      (row block t, when R0 >= 0)
//   s_rp[w][r] = partial of sum_{m < K} L_jm[r][m] y_m   (when y != null: forward substitution)
// K (= 32 j) is split over the 4 waves; each wave issues every load of its K-slice before its
// first MFMA (one memory latency per launch instead of one per 16-wide step), computes all 4
// quadrants of each tile, and the 4 partial tiles are summed through LDS.  MFMA operand layout:
// lane l holds row (l & 15) and k-group (l >> 4); per 16-wide step a lane loads the 4
// consecutive elements m0 + 4 (l >> 4) .. + 3 and MFMA i consumes element i, so each step covers
// m0 .. m0 + 15 once.  The L_j rows serve as both operands of the diagonal tile.  Rows past n
// read as zero; tile entries past n become the identity (keeps the padded factorisation finite).
constexpr int LU_STEPS = CMAX / 64;  // 16-wide steps per wave at most

__device__ __forceinline__ void tile_left_update2(const LbaDev &D, const double *__restrict__ A, int n, int C0, int R0, int K,
                                                  const double *__restrict__ y,
                                                  double (*sT)[CB + 1], double (*sX)[CB + 1],
                                                  double (*sP)[CB][CB + 1], double (*s_rp)[CB])
{
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const bool two = R0 >= 0;
    // originals first: their latency overlaps the GEMM
    double aT[4], aX[4];
    const HsBlk bT = hs_blk(D, n, C0 >> 5), bX = hs_blk(D, n, two ? R0 >> 5 : C0 >> 5);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int e = threadIdx.x + 256 * q, r = e >> 5, c = e & 31;
        aT[q] = (C0 + r < n && C0 + c < n) ? A[hs_el(bT, r, C0 + c)] : 0.0;
        aX[q] = (two && R0 + r < n && C0 + c < n) ? A[hs_el(bX, r, C0 + c)] : 0.0;
    }
    const int g4 = 4 * (l >> 4);
    const int rj0 = C0 + (l & 15), rj1 = C0 + 16 + (l & 15);
    const int rt0 = R0 + (l & 15), rt1 = R0 + 16 + (l & 15);
    const bool vj0 = rj0 < n, vj1 = rj1 < n, vt0 = two && rt0 < n, vt1 = two && rt1 < n;
    const double *pj0 = A + (size_t)(vj0 ? rj0 : 0) * n + g4, *pj1 = A + (size_t)(vj1 ? rj1 : 0) * n + g4;
    const double *pt0 = A + (size_t)(vt0 ? rt0 : 0) * n + g4, *pt1 = A + (size_t)(vt1 ? rt1 : 0) * n + g4;
    d4 accT[2][2], accX[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) accT[a][b] = accX[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    double rp0 = 0.0, rp1 = 0.0;
    // K in chunks of CMAX columns (one chunk up to the LocalBA size; BundleAdjustment's larger
    // systems loop), each chunk split over the 4 waves
    for (int kb = 0; kb < K; kb += CMAX) {
    const int Kc = min(CMAX, K - kb);
    const int kq = ((Kc + 63) / 64) * 16;  // per-wave slice, multiple of 16
    const int mb = kb + w * kq, me = min(kb + Kc, mb + kq);
    double2 j0[LU_STEPS][2], j1[LU_STEPS][2], t0[LU_STEPS][2], t1[LU_STEPS][2], yy[LU_STEPS][2];
    const int nst = max(0, (me - mb) / 16);  // wave-uniform step count of this slice
#pragma unroll
    for (int s = 0; s < LU_STEPS; s++) {
        if (s >= nst) break;
        const int m = mb + 16 * s;
        j0[s][0] = *(const double2 *)(pj0 + m); j0[s][1] = *(const double2 *)(pj0 + m + 2);
        j1[s][0] = *(const double2 *)(pj1 + m); j1[s][1] = *(const double2 *)(pj1 + m + 2);
        if (two) {
            t0[s][0] = *(const double2 *)(pt0 + m); t0[s][1] = *(const double2 *)(pt0 + m + 2);
            t1[s][0] = *(const double2 *)(pt1 + m); t1[s][1] = *(const double2 *)(pt1 + m + 2);
        }
        if (y) {
            yy[s][0] = *(const double2 *)(y + g4 + m); yy[s][1] = *(const double2 *)(y + g4 + m + 2);
        }
    }
#pragma unroll
    for (int s = 0; s < LU_STEPS; s++) {
        if (s < nst) {
            double ja[2][4], ta[2][4];
            const bool z0 = !vj0, z1 = !vj1, y0 = !vt0, y1 = !vt1;
            ja[0][0] = z0 ? 0.0 : j0[s][0].x; ja[0][1] = z0 ? 0.0 : j0[s][0].y;
            ja[0][2] = z0 ? 0.0 : j0[s][1].x; ja[0][3] = z0 ? 0.0 : j0[s][1].y;
            ja[1][0] = z1 ? 0.0 : j1[s][0].x; ja[1][1] = z1 ? 0.0 : j1[s][0].y;
            ja[1][2] = z1 ? 0.0 : j1[s][1].x; ja[1][3] = z1 ? 0.0 : j1[s][1].y;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                accT[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(ja[0][i], ja[0][i], accT[0][0], 0, 0, 0);
                accT[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(ja[1][i], ja[0][i], accT[1][0], 0, 0, 0);
                accT[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(ja[1][i], ja[1][i], accT[1][1], 0, 0, 0);
            }
            if (y) {
                const double yv[4] = {yy[s][0].x, yy[s][0].y, yy[s][1].x, yy[s][1].y};
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    rp0 += ja[0][i] * yv[i];
                    rp1 += ja[1][i] * yv[i];
                }
            }
            if (two) {
                ta[0][0] = y0 ? 0.0 : t0[s][0].x; ta[0][1] = y0 ? 0.0 : t0[s][0].y;
                ta[0][2] = y0 ? 0.0 : t0[s][1].x; ta[0][3] = y0 ? 0.0 : t0[s][1].y;
                ta[1][0] = y1 ? 0.0 : t1[s][0].x; ta[1][1] = y1 ? 0.0 : t1[s][0].y;
                ta[1][2] = y1 ? 0.0 : t1[s][1].x; ta[1][3] = y1 ? 0.0 : t1[s][1].y;
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int a = 0; a < 2; a++)
#pragma unroll
                        for (int b = 0; b < 2; b++)
                            accX[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(ta[a][i], ja[b][i], accX[a][b], 0, 0, 0);
            }
        }
    }
    }  // K chunks
    if (y) {  // sum the 4 k-groups of a row (lanes l, l ^ 16, l ^ 32, l ^ 48)
        rp0 += __shfl_xor(rp0, 16);
        rp0 += __shfl_xor(rp0, 32);
        rp1 += __shfl_xor(rp1, 16);
        rp1 += __shfl_xor(rp1, 32);
        if (l < 16) {
            s_rp[w][l] = rp0;
            s_rp[w][16 + l] = rp1;
        }
    }
    // diagonal tile: lower quadrants only (the upper one mirrors (1,0))
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) {
            if (b > a) continue;
#pragma unroll
            for (int q = 0; q < 4; q++) sP[w][16 * a + (l >> 4) + 4 * q][16 * b + (l & 15)] = accT[a][b][q];
        }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int e = threadIdx.x + 256 * q, r = e >> 5, c = e & 31;
        const double sum = (c <= r) ? ((sP[0][r][c] + sP[1][r][c]) + sP[2][r][c]) + sP[3][r][c] : 0.0;
        sT[r][c] = (C0 + r < n && C0 + c < n) ? aT[q] - sum : (r == c ? 1.0 : 0.0);
    }
    if (!two) return;
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int q = 0; q < 4; q++) sP[w][16 * a + (l >> 4) + 4 * q][16 * b + (l & 15)] = accX[a][b][q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int e = threadIdx.x + 256 * q, r = e >> 5, c = e & 31;
        const double sum = ((sP[0][r][c] + sP[1][r][c]) + sP[2][r][c]) + sP[3][r][c];
        sX[r][c] = (R0 + r < n && C0 + c < n) ? aX[q] - sum : 0.0;
    }
}

// 1 / d to full double precision: v_rcp_f64 and two Newton steps
__device__ __forceinline__ double rcp_nr(double d)
{
    double r = __builtin_amdgcn_rcp(d);
    r = fma(r, fma(-d, r, 1.0), r);
    r = fma(r, fma(-d, r, 1.0), r);
    return r;
}

// Column block j (rows/cols k0 = 32 j ..), left-looking: every previous column block is final.
//  1. T = A_jj - sum_{m < k0} L_jm L_jm^T (every workgroup) and, in workgroup t > 0,
//     X = A_tj - sum_{m < k0} L_tm L_jm^T (tile_left_update2, FP64 MFMA); workgroup 0 also
//     reduces b_j - sum_{m < k0} L_jm y_m from the same operand registers.
//  2. T = Lt D Lt^T by elimination in LDS, one barrier per column; the same row operations
//     applied to the identity give M = Lt^-1, so L_jj^-1 = D^-1/2 M without a triangular solve.
//  3. workgroup 0: L_jj^-1 -> Linv, y_j = L_jj^-1 rhs -> x;  workgroup t > 0: L_tj = X L_jj^-T
//     (MFMA) written over A_tj.  A_jj itself is never written (nothing downstream needs L_jj).
// The LDS of one column step (k_chol_col)
struct CholLds {
    double sP[4][CB][CB + 1];  // per-wave partial tiles
    double sG[CB][CB + 1];     // T under elimination
    double sM[CB][CB + 1];     // Lt^-1, then L_jj^-1
    double sX[CB][CB + 1];     // X (row blocks below)
    double s_rsq[CB];          // D^-1/2
    double s_d[CB];            // pivots
    double s_rp[4][CB];
    double s_rhs[CB];
};

// Step 2: T (in sG) = Lt D Lt^T by elimination in LDS, one barrier per two columns; the same row
// operations applied to the identity in sM give M = Lt^-1, then L_jj^-1 = D^-1/2 M.  Returns the
// pivots' positivity.
//   Elimination two columns per barrier (2x2 pivot block c, c + 1, redundantly in every thread):
//   d0 = g_cc, l10 = g_c+1,c / d0, d1 = g_c+1,c+1 - g_c+1,c l10, g'_i,c+1 = g_i,c+1 - g_ic l10
//   G: g_i,jj -= g_ic g_jj,c / d0 + g'_i,c+1 g'_jj,c+1 / d1        (c + 1 < jj <= i)
//   M: m_i,m  -= g_ic / d0 m_c,m + g'_i,c+1 / d1 (m_c+1,m - l10 m_c,m)  (i > c + 1, m <= c + 1)
//      m_c+1,m -= l10 m_c,m (m <= c): written one step later (other threads read row c + 1 now;
//      nothing reads it in the next step).  Pivots go to s_d (the diagonal of G is read now).
// An odd nb pairs its last column with padding column nb (identity: l10 = 0, d1 = 1).
// GUARD: a workgroup of more than 256 threads (k_chol_dense), of which threads 0..255 eliminate and
// every thread takes the barriers.
template <bool GUARD = false, class LDS>
__device__ __forceinline__ int chol_factor_diag(LDS &L, int nb)
{
    const int tid = threadIdx.x;
    const bool act = !GUARD || tid < 256;
    const int jj = tid & 31, ib = (tid >> 5) & 7;
    int ok = 1;
    double defer_val = 0.0;
    int defer_at = -1;  // index into sM of the deferred row-(c+1) value
    for (int c = 0; c < nb; c += 2) {
        if (!act) {
            __syncthreads();
            continue;
        }
        if (defer_at >= 0) (&L.sM[0][0])[defer_at] = defer_val;
        defer_at = -1;
        const double d0 = L.sG[c][c], e = L.sG[c + 1][c], d1r = L.sG[c + 1][c + 1];
        const double gj0 = L.sG[jj][c], gj1 = L.sG[jj][c + 1];
        const double mc = L.sM[c][jj], mc1 = L.sM[c + 1][jj];
        double *const base = (jj > c + 1) ? &L.sG[0][0] : &L.sM[0][0];
        double gi0[4], gi1[4], cur[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int i = ib + 8 * q;
            gi0[q] = L.sG[i][c];
            gi1[q] = L.sG[i][c + 1];
            cur[q] = base[i * (CB + 1) + jj];
        }
        const double r0 = rcp_nr(d0 > 0.0 ? d0 : 1.0);
        const double l10 = e * r0;
        const double d1 = d1r - e * l10;
        ok &= (d0 > 0.0) & (d1 > 0.0);
        const double r1 = rcp_nr(d1 > 0.0 ? d1 : 1.0);
        if (tid == 0) {
            L.s_d[c] = d0;
            L.s_d[c + 1] = d1;
        }
        const double gj1p = gj1 - gj0 * l10;
        const double mc1p = mc1 - l10 * mc;
        const bool gcol = jj > c + 1;
        const double a0 = gcol ? gj0 * r0 : mc * r0;     // coefficient of g_ic
        const double a1 = gcol ? gj1p * r1 : mc1p * r1;  // coefficient of g'_i,c+1
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int i = ib + 8 * q;
            const double gi1p = gi1[q] - gi0[q] * l10;
            const double v = cur[q] - gi0[q] * a0 - gi1p * a1;
            if (i < nb && i > c + 1 && jj <= i) base[i * (CB + 1) + jj] = v;
            if (i == c + 1 && i < nb && jj <= c) {
                defer_val = mc1p;
                defer_at = i * (CB + 1) + jj;
            }
        }
        __syncthreads();
    }
    if (act && defer_at >= 0) (&L.sM[0][0])[defer_at] = defer_val;
    __syncthreads();
    if (tid < CB) {
        const double d = L.s_d[tid];
        L.s_rsq[tid] = (tid < nb && d > 0.0) ? 1.0 / sqrt(d) : 1.0;
    }
    __syncthreads();
    // L_jj^-1 = D^-1/2 M (lower)
    for (int e = tid; e < CB * CB; e += blockDim.x) {
        const int i = e >> 5, m = e & 31;
        L.sM[i][m] = (m <= i) ? L.sM[i][m] * L.s_rsq[i] : 0.0;
    }
    __syncthreads();
    return ok;
}

// chol_factor_diag four columns per barrier (OSG_CHOL_ELIM=4): the 4 x 4 pivot block P = LP DP LP^T is
// factored redundantly in every thread (four reciprocals in sequence), a row's block entries B_i become
// Y_i = B_i LP^-T by forward substitution, and then
//   G: g_i,jj -= sum_p Y_ip Y_jj,p / d_p                           (c + 3 < jj <= i)
//   M: m_i,m  -= sum_p Y_ip / d_p M'_p,m,  M'_blk = LP^-1 M_blk     (i > c + 3, m <= c + 3)
// with the block rows M'_blk written one step later (other threads read M_blk now).  Eight barriers
// instead of sixteen for a 32-column tile; the same factor to rounding.
template <bool GUARD = false, class LDS>
__device__ __forceinline__ int chol_factor_diag4(LDS &L, int nb)
{
    const int tid = threadIdx.x;
    const bool act = !GUARD || tid < 256;
    const int jj = tid & 31, ib = (tid >> 5) & 7;
    int ok = 1;
    double defer_val = 0.0;
    int defer_at = -1;  // index into sM of the deferred block-row value
    for (int c = 0; c < nb; c += 4) {
        if (!act) {
            __syncthreads();
            continue;
        }
        if (defer_at >= 0) (&L.sM[0][0])[defer_at] = defer_val;
        defer_at = -1;
        const double P00 = L.sG[c][c], P10 = L.sG[c + 1][c], P20 = L.sG[c + 2][c], P30 = L.sG[c + 3][c];
        const double P11 = L.sG[c + 1][c + 1], P21 = L.sG[c + 2][c + 1], P31 = L.sG[c + 3][c + 1];
        const double P22 = L.sG[c + 2][c + 2], P32 = L.sG[c + 3][c + 2], P33 = L.sG[c + 3][c + 3];
        const bool gcol = jj > c + 3;
        double bj[4], gi[4][4], cur[4];
        if (gcol) {
#pragma unroll
            for (int p = 0; p < 4; p++) bj[p] = L.sG[jj][c + p];
        } else {
#pragma unroll
            for (int p = 0; p < 4; p++) bj[p] = L.sM[c + p][jj];
        }
        double *const base = gcol ? &L.sG[0][0] : &L.sM[0][0];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int i = ib + 8 * q;
#pragma unroll
            for (int p = 0; p < 4; p++) gi[q][p] = L.sG[i][c + p];
            cur[q] = base[i * (CB + 1) + jj];
        }
        // LP DP LP^T of the pivot block
        const double d0 = P00, r0 = rcp_nr(d0 > 0.0 ? d0 : 1.0);
        const double l10 = P10 * r0, l20 = P20 * r0, l30 = P30 * r0;
        const double d1 = P11 - P10 * l10, r1 = rcp_nr(d1 > 0.0 ? d1 : 1.0);
        const double t21 = P21 - P20 * l10, t31 = P31 - P30 * l10;
        const double l21 = t21 * r1, l31 = t31 * r1;
        const double d2 = P22 - P20 * l20 - t21 * l21, r2 = rcp_nr(d2 > 0.0 ? d2 : 1.0);
        const double t32 = P32 - P30 * l20 - t31 * l21;
        const double l32 = t32 * r2;
        const double d3 = P33 - P30 * l30 - t31 * l31 - t32 * l32, r3 = rcp_nr(d3 > 0.0 ? d3 : 1.0);
        ok &= (d0 > 0.0) & (d1 > 0.0) & (d2 > 0.0) & (d3 > 0.0);
        if (tid == 0) {
            L.s_d[c] = d0;
            L.s_d[c + 1] = d1;
            L.s_d[c + 2] = d2;
            L.s_d[c + 3] = d3;
        }
        // this column's coefficients: Y_jj / d (G) or M'_blk / d (M), both by forward substitution with LP
        const double y0 = bj[0], y1 = bj[1] - y0 * l10, y2 = bj[2] - y0 * l20 - y1 * l21;
        const double y3 = bj[3] - y0 * l30 - y1 * l31 - y2 * l32;
        const double a0 = y0 * r0, a1 = y1 * r1, a2 = y2 * r2, a3 = y3 * r3;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int i = ib + 8 * q;
            const double Y0 = gi[q][0], Y1 = gi[q][1] - Y0 * l10, Y2 = gi[q][2] - Y0 * l20 - Y1 * l21;
            const double Y3 = gi[q][3] - Y0 * l30 - Y1 * l31 - Y2 * l32;
            const double v = cur[q] - Y0 * a0 - Y1 * a1 - Y2 * a2 - Y3 * a3;
            if (i < nb && i > c + 3 && (!gcol || jj <= i)) base[i * (CB + 1) + jj] = v;
            if (!gcol && i >= c && i <= c + 3 && i < nb) {  // block row i of M' (deferred)
                const int pi = i - c;
                defer_val = pi == 0 ? y0 : (pi == 1 ? y1 : (pi == 2 ? y2 : y3));
                defer_at = i * (CB + 1) + jj;
            }
        }
        __syncthreads();
    }
    if (act && defer_at >= 0) (&L.sM[0][0])[defer_at] = defer_val;
    __syncthreads();
    if (tid < CB) {
        const double d = L.s_d[tid];
        L.s_rsq[tid] = (tid < nb && d > 0.0) ? 1.0 / sqrt(d) : 1.0;
    }
    __syncthreads();
    // L_jj^-1 = D^-1/2 M (lower)
    for (int e = tid; e < CB * CB; e += blockDim.x) {
        const int i = e >> 5, m = e & 31;
        L.sM[i][m] = (m <= i) ? L.sM[i][m] * L.s_rsq[i] : 0.0;
    }
    __syncthreads();
    return ok;
}

// Step 3 of the diagonal role: L_jj^-1 -> Linv, y_j = L_jj^-1 (b_j - sum_m L_jm y_m) -> x
__device__ __forceinline__ void chol_diag_out(const LbaDev &D, CholLds &L, int k0, int nb, int n, double bj, int ok)
{
    const int tid = threadIdx.x;
    if (tid == 0 && !ok) D.flag[0] = 0;
    for (int e = tid; e < CB * CB; e += 256) {
        const int r = e >> 5, c = e & 31;
        if (k0 + r < n) D.Linv[(size_t)(k0 + r) * CB + c] = L.sM[r][c];
    }
    if (tid < CB)
        L.s_rhs[tid] = (tid < nb) ? bj - (((L.s_rp[0][tid] + L.s_rp[1][tid]) + L.s_rp[2][tid]) + L.s_rp[3][tid]) : 0.0;
    __syncthreads();
    // y_i = sum_{m <= i} Linv[i][m] rhs_m, 8 threads per row
    const int i = tid >> 3, p = tid & 7;
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 4; q++) acc += L.sM[i][p + 8 * q] * L.s_rhs[p + 8 * q];
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    if (p == 0 && i < nb) D.x[k0 + i] = acc;
}

// Step 3 of a row-block role: L_tj = X L_jj^-T on MFMA, quadrant (qr, qc) per wave, A = X rows,
// B[k][c] = Linv[c][k], written over A_tj
__device__ __forceinline__ void chol_offdiag_out(const LbaDev &D, CholLds &L, int k0, int R0, int nb, int n)
{
    const int tid = threadIdx.x;
    const int w = tid >> 6, l = tid & 63;
    const int qr = (w >> 1) * 16, qc = (w & 1) * 16;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < CB / 4; ks++) {
        const int k = 4 * ks + (l >> 4);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(L.sX[qr + (l & 15)][k], L.sM[qc + (l & 15)][k], acc, 0, 0, 0);
    }
    const int c = qc + (l & 15);
    double *Aw = D.Hs;
    const HsBlk bR = hs_blk(D, n, R0 >> 5);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int r = qr + (l >> 4) + 4 * q;
        if (R0 + r < n && c < nb) Aw[hs_el(bR, r, k0 + c)] = acc[q];
    }
}

// Column block j (rows/cols k0 = 32 j ..), left-looking: every previous column block is final.
//  1. T = A_jj - sum_{m < k0} L_jm L_jm^T (every workgroup) and, in workgroup t > 0,
//     X = A_tj - sum_{m < k0} L_tm L_jm^T (tile_left_update2, FP64 MFMA); workgroup 0 also
//     reduces b_j - sum_{m < k0} L_jm y_m from the same operand registers.
//  2. chol_factor_diag: T = Lt D Lt^T, L_jj^-1 = D^-1/2 Lt^-1 without a triangular solve.
//  3. workgroup 0: chol_diag_out;  workgroup t > 0: chol_offdiag_out.  A_jj itself is never
//     written (nothing downstream needs L_jj).
template <int ELIM>
__global__ __launch_bounds__(256) void k_chol_col(const LbaDev *__restrict__ Ds, int j)
{
    LBA_GRAPH(M_ACT);
    if (j >= D.nblk_red || bx >= D.nblk_red - j) return;
    if (D.chol_fused) return;  // factored by k_chol_dense / k_chol_env
    // past CMAX workgroup 0 is the diagonal block and workgroup b >= 1 the b-th envelope row of the
    // column (col_rows): a row block outside the envelope has an all-zero tile here, and its L_tj
    // stays zero
    const bool big = 6 * D.nhp > CMAX;
    if (big && bx > 0 && bx > D.col_rows_start[j + 1] - D.col_rows_start[j]) return;
    __shared__ CholLds L;
    const int n = 6 * D.nhp;
    const double *A = D.Hs;
    const int k0 = j * CB;
    const int nb = min(CB, n - k0);
    const int t = (big && bx > 0) ? D.col_rows[D.col_rows_start[j] + bx - 1] - j : bx;  // row block j + t
    const int tid = threadIdx.x;
    const int R0 = k0 + t * CB;
    unsigned long long *ts = (D.tstamp && t < 2 && tid == 0 && j < 32) ? D.tstamp + 8 * (2 * j + t) : nullptr;
    if (ts) ts[0] = wall_clock64();

    const double bj = (t == 0 && tid < nb) ? D.bs[k0 + tid] : 0.0;
    for (int e = tid; e < CB * (CB + 1); e += 256) (&L.sM[0][0])[e] = 0.0;
    // past CMAX the system is factored right-looking: k_chol_trail has already applied every earlier
    // column block to these tiles and to b, so nothing is left to subtract (K = 0)
    tile_left_update2(D, A, n, k0, t > 0 ? R0 : -1, n > CMAX ? 0 : k0, t == 0 ? D.x : nullptr, L.sG, L.sX, L.sP, L.s_rp);
    if (tid < CB) L.sM[tid][tid] = 1.0;
    __syncthreads();
    if (ts) ts[1] = wall_clock64();
    const int ok = ELIM == 4 ? chol_factor_diag4(L, nb) : chol_factor_diag(L, nb);
    if (ts) ts[2] = wall_clock64();
    if (t == 0) chol_diag_out(D, L, k0, nb, n, bj, ok);
    else chol_offdiag_out(D, L, k0, R0, nb, n);
    if (ts) ts[3] = ts[4] = wall_clock64();
}

// The whole left-looking factorisation of a dense reduced system (n <= CMAX: LocalBundleAdjustment)
// in one 1024-thread workgroup per graph, instead of one k_chol_col launch per column block: the
// column steps' latency chains (operand loads, the elimination's barriers) then follow each other
// without a launch boundary, and the diagonal tile is eliminated once per column instead of once per
// row-block workgroup.  Per column block j (k0 = 32 j, row blocks j .. nblk - 1 held in LDS):
//   1. tasks over the 16 waves: 16 x 16 quadrants X_t = A_tj - sum_{m < k0} L_tm L_jm^T (FP64 MFMA
//      over the whole K; the diagonal tile's lower quadrants only), and b_j - sum_m L_jm y_m;
//   2. chol_factor_diag on threads 0..255: L_jj^-1 = D^-1/2 Lt^-1;
//   3. Linv and y_j out, then L_tj = X_t L_jj^-T per quadrant (FP64 MFMA) over A_tj.
// The outputs are k_chol_col's (L below the diagonal in Hs, Linv, y in x), so k_chol_back follows
// unchanged.  Its sums are ordered differently from k_chol_col's (one MFMA chain per quadrant
// instead of four K slices), so the two agree to rounding (OSG_CHOL_DENSE=0 selects the column
// launches, tests/test_ba_gpu.py compares them).
constexpr int CD_T = 1024;  // k_chol_env's workgroup; k_chol_dense takes its own as a template argument
template <int CD_T, int RING, int ELIM>
__global__ __launch_bounds__(CD_T) void k_chol_dense(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    const int n = 6 * D.nhp;
    if (n == 0 || n > CMAX || D.chol_fused != 1) return;
    __shared__ double s_x[CMAX / CB][CB][CB + 1];
    __shared__ double s_m[CB][CB + 1];
    __shared__ double s_rsq[CB], s_d[CB], s_rhs[CB];
    __shared__ double s_pq[CD_T / 64][16][17];   // K-slice partial quadrants (the last columns)
    __shared__ double s_prp[CD_T / 64][16];      // ... and their b_j partials
    struct Lds {
        double (&sG)[CB][CB + 1];
        double (&sM)[CB][CB + 1];
        double *s_rsq, *s_d;
    } L{s_x[0], s_m, s_rsq, s_d};
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    double *A = D.Hs;
    const int nblk = (n + CB - 1) / CB;
    const int g4 = 4 * (l >> 4);
    for (int j = 0; j < nblk; j++) {
        const int k0 = j * CB, nb = min(CB, n - k0), ntile = nblk - j;
        // the diagonal tile's lower quadrants (tasks 0..2) and the row blocks' quadrants; when they are few
        // (the last columns, K largest), each quadrant's K is split over ks waves whose partial sums are
        // added in slice order through LDS
        // OSG_LBA_PROFILE=2: column phases of graph 0 (update | elimination | outputs), k_chol_col's slots
        unsigned long long *ts = (D.tstamp && tid == 0 && j < 32) ? D.tstamp + 8 * (2 * j) : nullptr;
        if (ts) ts[0] = wall_clock64();
        const int ntask = 3 + 4 * (ntile - 1);
        const int ks = ntask * 4 <= CD_T / 64 ? 4 : (ntask * 2 <= CD_T / 64 ? 2 : 1);
        const int nst = k0 / 16, sps = (nst + ks - 1) / ks;  // 16-column steps in all, per slice
        for (int e = tid; e < CB * (CB + 1); e += CD_T) (&s_m[0][0])[e] = 0.0;
        auto decode = [&](int task, int &t, int &a, int &b) {
            if (task < 3) {
                t = 0;
                a = task > 0 ? 1 : 0;
                b = task == 2 ? 1 : 0;
            } else {
                t = 1 + (task - 3) / 4;
                a = ((task - 3) >> 1) & 1;
                b = (task - 3) & 1;
            }
        };
        for (int item = w; item < ntask * ks; item += CD_T / 64) {
            const int task = item / ks, sl = item - task * ks;
            int t, a, b;
            decode(task, t, a, b);
            const int R0 = k0 + t * CB + 16 * a, C0 = k0 + 16 * b;  // quadrant rows, columns
            const int ra = R0 + (l & 15), rb = C0 + (l & 15);
            const bool va = ra < n, vb = rb < n;
            const double *pa = A + (size_t)(va ? ra : 0) * n + g4, *pb = A + (size_t)(vb ? rb : 0) * n + g4;
            // the diagonal quadrants (0, 0) and (1, 1) also reduce b_j - sum_m L_jm y_m for their rows from
            // the same A operands (rows of block j)
            const bool rhs = t == 0 && a == b;
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            double rp = 0.0;
            // a ring of RING 16-column steps in flight: the operand loads run RING - 1 steps ahead of the MFMAs
            const int s0 = sl * sps, s1 = min(nst, s0 + sps);
            double2 ring[RING][4], yring[RING][2];
            auto load = [&](int st, double2 (&o)[4], double2 (&yo)[2]) {
                const int m = 16 * st;
                o[0] = *(const double2 *)(pa + m);
                o[1] = *(const double2 *)(pa + m + 2);
                o[2] = *(const double2 *)(pb + m);
                o[3] = *(const double2 *)(pb + m + 2);
                if (rhs) {
                    yo[0] = *(const double2 *)(D.x + g4 + m);
                    yo[1] = *(const double2 *)(D.x + g4 + m + 2);
                }
            };
#pragma unroll
            for (int u = 0; u < RING; u++)
                if (s0 + u < s1) load(s0 + u, ring[u], yring[u]);
            for (int st = s0; st < s1; st += RING) {
#pragma unroll
                for (int u = 0; u < RING; u++) {
                    if (st + u >= s1) break;
                    const double2 *c4 = ring[u];
                    const double av[4] = {va ? c4[0].x : 0.0, va ? c4[0].y : 0.0, va ? c4[1].x : 0.0, va ? c4[1].y : 0.0};
                    const double bv[4] = {vb ? c4[2].x : 0.0, vb ? c4[2].y : 0.0, vb ? c4[3].x : 0.0, vb ? c4[3].y : 0.0};
#pragma unroll
                    for (int i = 0; i < 4; i++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[i], acc, 0, 0, 0);
                    if (rhs) {
                        const double yv[4] = {yring[u][0].x, yring[u][0].y, yring[u][1].x, yring[u][1].y};
#pragma unroll
                        for (int i = 0; i < 4; i++) rp += av[i] * yv[i];
                    }
                    if (st + u + RING < s1) load(st + u + RING, ring[u], yring[u]);
                }
            }
            if (rhs) {  // the 4 k-groups of a row: lanes l, l ^ 16, l ^ 32, l ^ 48
                rp += __shfl_xor(rp, 16);
                rp += __shfl_xor(rp, 32);
            }
            if (ks > 1) {  // partial sums, added below in slice order
#pragma unroll
                for (int q = 0; q < 4; q++) s_pq[item][(l >> 4) + 4 * q][l & 15] = acc[q];
                if (rhs && l < 16) s_prp[item][l] = rp;
                continue;
            }
            if (rhs) {
                const int r = 16 * a + (l & 15);
                if (l < 16) s_rhs[r] = (k0 + r < n) ? D.bs[k0 + r] - rp : 0.0;
            }
            const int c = 16 * b + (l & 15);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = 16 * a + (l >> 4) + 4 * q;
                const int gr = k0 + t * CB + r, gc = k0 + c;
                double v;
                if (gr < n && gc < n) v = A[(size_t)gr * n + gc] - acc[q];
                else v = (t == 0 && r == c) ? 1.0 : 0.0;   // identity padding of the diagonal tile
                s_x[t][r][c] = v;
                if (t == 0 && a == 1 && b == 0) s_x[0][c][r] = 0.0;  // upper quadrant: read, never used
            }
        }
        if (ks > 1) {
            __syncthreads();
            for (int e = tid; e < ntask * 256; e += CD_T) {
                const int task = e >> 8, r16 = (e >> 4) & 15, c16 = e & 15;
                int t, a, b;
                decode(task, t, a, b);
                double sum = s_pq[task * ks][r16][c16];
                for (int sl = 1; sl < ks; sl++) sum += s_pq[task * ks + sl][r16][c16];
                const int r = 16 * a + r16, c = 16 * b + c16, gr = k0 + t * CB + r, gc = k0 + c;
                double v;
                if (gr < n && gc < n) v = A[(size_t)gr * n + gc] - sum;
                else v = (t == 0 && r == c) ? 1.0 : 0.0;
                s_x[t][r][c] = v;
                if (t == 0 && a == 1 && b == 0) s_x[0][c][r] = 0.0;
            }
            if (tid < CB) {  // rows 0..15: task 0, rows 16..31: task 2
                const int task = tid < 16 ? 0 : 2, r16 = tid & 15;
                double sum = s_prp[task * ks][r16];
                for (int sl = 1; sl < ks; sl++) sum += s_prp[task * ks + sl][r16];
                s_rhs[tid] = (k0 + tid < n) ? D.bs[k0 + tid] - sum : 0.0;
            }
        }
        __syncthreads();
        if (tid < CB) s_m[tid][tid] = 1.0;
        __syncthreads();
        if (ts) ts[1] = wall_clock64();
        const int ok = ELIM == 4 ? chol_factor_diag4<true>(L, nb) : chol_factor_diag<true>(L, nb);
        if (ts) ts[2] = wall_clock64();
        if (tid == 0 && !ok) D.flag[0] = 0;
        for (int e = tid; e < CB * CB; e += CD_T) {
            const int r = e >> 5, c = e & 31;
            if (k0 + r < n) D.Linv[(size_t)(k0 + r) * CB + c] = s_m[r][c];
        }
        if (tid < 256) {  // y_j = L_jj^-1 rhs, 8 threads per row
            const int i = tid >> 3, p = tid & 7;
            double acc = 0.0;
#pragma unroll
            for (int q = 0; q < 4; q++) acc += s_m[i][p + 8 * q] * s_rhs[p + 8 * q];
            acc += __shfl_xor(acc, 1);
            acc += __shfl_xor(acc, 2);
            acc += __shfl_xor(acc, 4);
            if (p == 0 && i < nb) D.x[k0 + i] = acc;
        }
        // L_tj = X_t L_jj^-T, quadrant (qr, qc) per task
        for (int task = w; task < 4 * (ntile - 1); task += CD_T / 64) {
            const int t = 1 + task / 4, qr = 16 * ((task >> 1) & 1), qc = 16 * (task & 1);
            d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int ks = 0; ks < CB / 4; ks++) {
                const int k = 4 * ks + (l >> 4);
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(s_x[t][qr + (l & 15)][k], s_m[qc + (l & 15)][k], acc, 0, 0, 0);
            }
            const int c = qc + (l & 15), R0 = k0 + t * CB;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = qr + (l >> 4) + 4 * q;
                if (R0 + r < n && c < nb) A[(size_t)(R0 + r) * n + k0 + c] = acc[q];
            }
        }
        __syncthreads();  // L_tj, Linv and y_j of this column before the next column reads them
        if (ts) ts[3] = wall_clock64();
    }
}

// The right-looking envelope factorisation (past CMAX: BundleAdjustment) and its backward solve in one
// 1024-thread workgroup per graph, for systems whose column blocks have at most ENV_T - 1 envelope rows
// below the diagonal (a banded map: 7 for the 1500-KF open map, 13 closed into a loop) and n <= ENV_NX.
// It replaces k_chol_col + k_chol_trail per column block (two launches of a few workgroups each) and
// the backward solve's launches with one workgroup whose column steps follow each other in LDS:
//   1. stage the diagonal tile and the column's envelope tiles (already trailing-updated) in LDS;
//   2. chol_factor_diag; Linv and y_j out (y_j also kept in LDS);
//   3. L_tj = X_t L_jj^-T per quadrant (FP64 MFMA), written over A_tj and kept in LDS;
//   4. the trailing update A_tu -= L_tj L_uj^T of every envelope pair (t >= u) and b_t -= L_tj y_j.
// The same products in the same order as k_chol_col (K = 0 past CMAX) and k_chol_trail, so the factor is
// theirs bit for bit; the backward solve is k_chol_back_large's, with x in the tiles' LDS.
constexpr int ENV_T = 16;                       // staged tiles: the diagonal + up to 15 envelope rows
constexpr int ENV_NX = ENV_T * CB * (CB + 1);   // x of the backward solve in the same LDS (16 896)
template <int ELIM>
__global__ __launch_bounds__(CD_T) void k_chol_env(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    if (D.chol_fused != 2) return;
    const int n = 6 * D.nhp;
    __shared__ double s_x[ENV_T][CB][CB + 1];
    __shared__ double s_m[CB][CB + 1];
    __shared__ double s_part[CB][CB + 1];
    __shared__ double s_rsq[CB], s_d[CB], s_rhs[CB], s_y[CB];
    __shared__ int s_rb[ENV_T];
    struct Lds {
        double (&sG)[CB][CB + 1];
        double (&sM)[CB][CB + 1];
        double *s_rsq, *s_d;
    } L{s_x[0], s_m, s_rsq, s_d};
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    double *A = D.Hs;
    const int nblk = D.nblk_red;
    for (int j = 0; j < nblk; j++) {
        const int k0 = j * CB, nb = min(CB, n - k0);
        const int r0 = D.col_rows_start[j], m = D.col_rows_start[j + 1] - r0;
        if (tid <= m) s_rb[tid] = tid == 0 ? j : D.col_rows[r0 + tid - 1];
        for (int e = tid; e < CB * (CB + 1); e += CD_T) (&s_m[0][0])[e] = 0.0;
        if (tid < CB) s_rhs[tid] = tid < nb ? D.bs[k0 + tid] - 0.0 : 0.0;
        __syncthreads();
        // 1. the tiles as k_chol_trail left them (K = 0: nothing left to subtract)
        for (int e = tid; e < (m + 1) * CB * CB; e += CD_T) {
            const int t = e >> 10, r = (e >> 5) & 31, c = e & 31, rb = s_rb[t], R = rb * CB + r;
            double v;
            if (t == 0) v = (R < n && k0 + c < n) ? (c <= r ? A[hs_el(hs_blk(D, n, rb), r, k0 + c)] : 0.0) : (r == c ? 1.0 : 0.0);
            else v = (R < n && k0 + c < n) ? A[hs_el(hs_blk(D, n, rb), r, k0 + c)] : 0.0;
            s_x[t][r][c] = v;
        }
        __syncthreads();
        if (tid < CB) s_m[tid][tid] = 1.0;
        __syncthreads();
        // 2.
        const int ok = ELIM == 4 ? chol_factor_diag4<true>(L, nb) : chol_factor_diag<true>(L, nb);
        if (tid == 0 && !ok) D.flag[0] = 0;
        for (int e = tid; e < CB * CB; e += CD_T) {
            const int r = e >> 5, c = e & 31;
            if (k0 + r < n) D.Linv[(size_t)(k0 + r) * CB + c] = s_m[r][c];
        }
        if (tid < 256) {  // y_j = L_jj^-1 rhs, 8 threads per row (chol_diag_out's sums)
            const int i = tid >> 3, p = tid & 7;
            double acc = 0.0;
#pragma unroll
            for (int q = 0; q < 4; q++) acc += s_m[i][p + 8 * q] * s_rhs[p + 8 * q];
            acc += __shfl_xor(acc, 1);
            acc += __shfl_xor(acc, 2);
            acc += __shfl_xor(acc, 4);
            if (p == 0 && i < nb) D.x[k0 + i] = acc;
            if (p == 0) s_y[i] = i < nb ? acc : 0.0;
        }
        // 3. L_tj = X_t L_jj^-T (chol_offdiag_out's products), at most 4 quadrants per wave
        d4 lt[(4 * (ENV_T - 1) + CD_T / 64 - 1) / (CD_T / 64)];
#pragma unroll
        for (int k = 0; k < (int)(sizeof(lt) / sizeof(lt[0])); k++) {
            const int task = w + (CD_T / 64) * k;
            if (task >= 4 * m) break;
            const int t = 1 + task / 4, qr = 16 * ((task >> 1) & 1), qc = 16 * (task & 1);
            d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int ks = 0; ks < CB / 4; ks++) {
                const int kk = 4 * ks + (l >> 4);
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(s_x[t][qr + (l & 15)][kk], s_m[qc + (l & 15)][kk], acc, 0, 0, 0);
            }
            lt[k] = acc;
            const int c = qc + (l & 15), rb = s_rb[t];
            const HsBlk bR = hs_blk(D, n, rb);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = qr + (l >> 4) + 4 * q;
                if (rb * CB + r < n && c < nb) A[hs_el(bR, r, k0 + c)] = acc[q];
            }
        }
        __syncthreads();  // every read of the X tiles is done
#pragma unroll
        for (int k = 0; k < (int)(sizeof(lt) / sizeof(lt[0])); k++) {
            const int task = w + (CD_T / 64) * k;
            if (task >= 4 * m) break;
            const int t = 1 + task / 4, qr = 16 * ((task >> 1) & 1), qc = 16 * (task & 1);
            const int c = qc + (l & 15), rb = s_rb[t];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = qr + (l >> 4) + 4 * q;
                s_x[t][r][c] = (rb * CB + r < n && c < nb) ? lt[k][q] : 0.0;  // k_chol_trail's staged L tile
            }
        }
        __syncthreads();
        // 4. trailing update of every envelope pair (a >= b) and the right-hand side
        const int npr = m * (m + 1) / 2;
        for (int task = w; task < 4 * npr; task += CD_T / 64) {
            const int pr = task >> 2;
            int a = (int)((sqrt(8.0 * pr + 1.0) - 1.0) * 0.5);  // pr = a (a + 1) / 2 + b, b <= a
            while (a * (a + 1) / 2 > pr) a--;
            while ((a + 1) * (a + 2) / 2 <= pr) a++;
            const int b = pr - a * (a + 1) / 2;
            const int ta = 1 + a, tb = 1 + b, qr = 16 * ((task >> 1) & 1), qc = 16 * (task & 1);
            d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int ks = 0; ks < CB / 4; ks++) {
                const int kk = 4 * ks + (l >> 4);
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(s_x[ta][qr + (l & 15)][kk], s_x[tb][qc + (l & 15)][kk], acc, 0, 0, 0);
            }
            const int R0 = s_rb[ta] * CB, C0 = s_rb[tb] * CB, c = qc + (l & 15);
            const HsBlk bt = hs_blk(D, n, s_rb[ta]);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = qr + (l >> 4) + 4 * q;
                if (R0 + r < n && C0 + c < n) A[hs_el(bt, r, C0 + c)] -= acc[q];
            }
        }
        if (tid < m * CB) {  // b_t -= L_tj y_j (k_chol_trail's diagonal-pair sums)
            const int t = 1 + (tid >> 5), r = tid & 31, R = s_rb[t] * CB + r;
            double sacc = 0.0;
#pragma unroll 8
            for (int k = 0; k < CB; k++) sacc += s_x[t][r][k] * s_y[k];
            if (R < n) D.bs[R] -= sacc;
        }
        __syncthreads();  // the updated tiles and b before the next column stages them
    }
    // backward solve L^T x = y (k_chol_back_large's blocks and sums), x over the tiles' LDS
    double *xv = &s_x[0][0][0];
    for (int i = tid; i < n; i += CD_T) xv[i] = 0.0;
    const int c = tid & 31, g = tid >> 5;
    for (int bi = nblk - 1; bi >= 0; bi--) {
        const int k0 = bi * CB, nb = min(CB, n - k0);
        (&s_m[0][0])[tid] = D.Linv[(size_t)min(k0 + (tid >> 5), n - 1) * CB + (tid & 31)];  // s_li[r * CB + c]
        __syncthreads();
        double acc = 0.0;
        if (c < nb) {
            for (int q = D.col_rows_start[bi]; q < D.col_rows_start[bi + 1]; q++) {
                const int rb = D.col_rows[q], row = rb * CB + g;
                if (row < n) acc += A[hs_el(hs_blk(D, n, rb), g, k0 + c)] * xv[row];
            }
        }
        s_part[c][g] = acc;
        __syncthreads();
        if (tid < CB) {
            double sp = 0.0;
#pragma unroll
            for (int gg = 0; gg < 32; gg++) sp += s_part[tid][gg];
            s_rhs[tid] = (tid < nb) ? D.x[k0 + tid] - sp : 0.0;
        }
        __syncthreads();
        if (tid < nb) {
            double xs = 0.0;
#pragma unroll
            for (int r = 0; r < CB; r++) xs += (&s_m[0][0])[r * CB + tid] * s_rhs[r];
            xv[k0 + tid] = xs;
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += CD_T) D.x[i] = xv[i];
}

// Backward substitution L^T x = y (y in x after the column launches), one 1024-thread
// workgroup, blocked by 32 from the last block: rhs_k = y_k - sum_{rows below} L[row][k]^T x_row
// (all threads, LDS partials), then x_k = L_kk^-T rhs_k (32 threads).  Linv and y are staged in
// LDS once; the L rows of the next block are loaded while the current block is being solved.
constexpr int BK_ROWS = CMAX / 32;  // rows per thread per block at most

// Workgroup barrier for LDS traffic only: __syncthreads() also waits for every outstanding global
// load (vmcnt(0)), which would drain the prefetch of the next block's rows each block.
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__global__ __launch_bounds__(1024) void k_chol_back(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    if (D.nhp == 0 || 6 * D.nhp > CMAX) return;
    __shared__ double s_x[CMAX];
    __shared__ double s_y[CMAX];
    __shared__ double s_li[CMAX * CB];
    __shared__ double s_part[32][33];
    __shared__ double s_rhs[CB];
    const int n = 6 * D.nhp;
    const double *A = D.Hs;
    const int tid = threadIdx.x;
    // staging: every load issued before the first LDS store (a load -> store loop would pay one
    // memory latency per iteration)
    {
        constexpr int NL = CMAX * CB / 1024;
        double v[NL];
#pragma unroll
        for (int k = 0; k < NL; k++) v[k] = D.Linv[min(tid + 1024 * k, n * CB - 1)];
        const double yv = D.x[min(tid, n - 1)];
#pragma unroll
        for (int k = 0; k < NL; k++)
            if (tid + 1024 * k < n * CB) s_li[tid + 1024 * k] = v[k];
        if (tid < n) {
            s_x[tid] = 0.0;
            s_y[tid] = yv;
        }
    }
    const int nblk = (n + CB - 1) / CB;
    const int c = tid & 31, g = tid >> 5;  // 32 groups of rows
    double cur[BK_ROWS];
    // unconditional (clamped) loads: branch-free, so the prefetch keeps counted waits
    auto load_block = [&](int bi, double (&v)[BK_ROWS]) {
        const int k0 = bi * CB, nb = min(CB, n - k0);
        const int cc = k0 + min(c, nb - 1);
#pragma unroll
        for (int i = 0; i < BK_ROWS; i++) {
            const int row = min(k0 + nb + g + 32 * i, n - 1);
            v[i] = A[(size_t)row * n + cc];
        }
    };
    // one block: rows below from v (loaded one block earlier), the next block's rows into w
    unsigned long long *ts = (D.tstamp && tid == 0) ? D.tstamp + 8 * 2 * 32 : nullptr;  // after k_chol_col's
    if (ts) ts[0] = wall_clock64();
    auto solve_block = [&](int bi, const double (&v)[BK_ROWS], double (&w)[BK_ROWS]) {
        if (ts) ts[1 + bi] = wall_clock64();
        const int k0 = bi * CB;
        const int nb = min(CB, n - k0);
        load_block(max(bi - 1, 0), w);  // unconditional; stays in flight: only LDS barriers below
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < BK_ROWS; i++) {
            const int row = k0 + nb + g + 32 * i;
            const bool ok = row < n && c < nb;
            acc += (ok ? v[i] : 0.0) * s_x[ok ? row : 0];
        }
        s_part[c][g] = acc;
        lds_barrier();
        if (tid < CB) {
            double s = 0.0;
#pragma unroll
            for (int gg = 0; gg < 32; gg++) s += s_part[tid][gg];
            s_rhs[tid] = (tid < nb) ? s_y[k0 + tid] - s : 0.0;  // zero-padded past nb
        }
        lds_barrier();
        if (tid < nb) {
            // Linv is zero above its diagonal and s_rhs past nb: no predicates, so the 32 LDS
            // reads pipeline instead of one branch + wait each
            double xv = 0.0;
#pragma unroll
            for (int r = 0; r < CB; r++) xv += s_li[min(k0 + r, n - 1) * CB + tid] * s_rhs[r];
            s_x[k0 + tid] = xv;
        }
        lds_barrier();
    };
    double alt[BK_ROWS];
    load_block(nblk - 1, cur);
    __syncthreads();
    if (ts) ts[41] = wall_clock64();
    // ping-pong between cur and alt (a register copy would wait for the prefetch to land)
    for (int bi = nblk - 1; bi >= 0; bi -= 2) {
        solve_block(bi, cur, alt);
        if (bi - 1 >= 0) solve_block(bi - 1, alt, cur);
    }
    if (ts) ts[40] = wall_clock64();
    for (int i = tid; i < n; i += 1024) D.x[i] = s_x[i];
}

// Right-looking trailing update for reduced systems past CMAX (BundleAdjustment): after column
// block j is factored, every lower tile (t, u), j < u <= t, takes A_tu -= L_tj L_uj^T (FP64 MFMA, one
// workgroup per tile, both L tiles staged in LDS), and the diagonal-tile workgroups update the
// forward-substitution right-hand side b_t -= L_tj y_j.  The column launches then read their tiles as
// they stand (K = 0): the O(n^3) work is spread over (nblk - j)^2 / 2 workgroups per step instead of
// one K-long GEMM per row block (which left one CU per row block MFMA-bound at large n).
// PRE (the default; OSG_TRAIL_PRE=0 for the previous order, bit-identical): the thread's four target
// entries A_tu (and a diagonal tile's b_t / y_j) are loaded with the L tiles, before the MFMA, instead of
// after it: one memory round trip per workgroup instead of two in a row.
template <bool PRE>
__global__ __launch_bounds__(256) void k_chol_trail(const LbaDev *__restrict__ Ds, int j)
{
    LBA_GRAPH(M_ACT);
    const int n = 6 * D.nhp;
    if (n <= CMAX || D.chol_fused) return;
    if (j >= D.nblk_red) return;
    // the envelope rows of column j (L_tj nonzero): tile (t, u) for every pair of them, u <= t
    const int r0 = D.col_rows_start[j], m = D.col_rows_start[j + 1] - r0;
    if (m <= 0 || bx >= m * (m + 1) / 2) return;
    int a = (int)((sqrt(8.0 * bx + 1.0) - 1.0) * 0.5);  // bx = a (a + 1) / 2 + b, b <= a
    while (a * (a + 1) / 2 > bx) a--;
    while ((a + 1) * (a + 2) / 2 <= bx) a++;
    const int b = bx - a * (a + 1) / 2;
    const int tb = D.col_rows[r0 + a], ub = D.col_rows[r0 + b];
    const int t = tb - j - 1, u = ub - j - 1;  // as offsets below block j
    const int R0 = tb * CB, C0 = ub * CB, K0 = j * CB;
    __shared__ double sLt[CB][CB + 1], sLu[CB][CB + 1];
    const int tid = threadIdx.x;
    const HsBlk bt = hs_blk(D, n, tb), bu = hs_blk(D, n, ub);
    const int w = tid >> 6, l = tid & 63;
    const int qr = (w >> 1) * 16, qc = (w & 1) * 16;
    double old[4], bsv = 0.0, yv[CB];
    if (PRE) {
        const int c = qc + (l & 15);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int r = qr + (l >> 4) + 4 * q;
            old[q] = (R0 + r < n && C0 + c < n) ? D.Hs[hs_el(bt, r, C0 + c)] : 0.0;
        }
        if (t == u && tid < CB && R0 + tid < n) {
            bsv = D.bs[R0 + tid];
#pragma unroll
            for (int k = 0; k < CB; k++) yv[k] = D.x[K0 + k];
        }
    }
    for (int e = tid; e < CB * CB; e += 256) {
        const int r = e >> 5, c = e & 31;
        sLt[r][c] = (R0 + r < n) ? D.Hs[hs_el(bt, r, K0 + c)] : 0.0;
        sLu[r][c] = (C0 + r < n) ? D.Hs[hs_el(bu, r, K0 + c)] : 0.0;
    }
    __syncthreads();
    d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < CB / 4; ks++) {
        const int k = 4 * ks + (l >> 4);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sLt[qr + (l & 15)][k], sLu[qc + (l & 15)][k], acc, 0, 0, 0);
    }
    const int c = qc + (l & 15);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int r = qr + (l >> 4) + 4 * q;
        if (R0 + r < n && C0 + c < n) {
            if (PRE) D.Hs[hs_el(bt, r, C0 + c)] = old[q] - acc[q];
            else D.Hs[hs_el(bt, r, C0 + c)] -= acc[q];
        }
    }
    if (t == u && tid < CB && R0 + tid < n) {  // block j is full (m > 0): y_j is 32 entries
        double s = 0.0;
        if (PRE) {
#pragma unroll
            for (int k = 0; k < CB; k++) s += sLt[tid][k] * yv[k];
            D.bs[R0 + tid] = bsv - s;
        } else {
#pragma unroll 8
            for (int k = 0; k < CB; k++) s += sLt[tid][k] * D.x[K0 + k];
            D.bs[R0 + tid] -= s;
        }
    }
}

// Backward substitution for reduced systems past CMAX (BundleAdjustment): the same blocks and
// summation order as k_chol_back, with x held in LDS (n <= CMAX_LARGE) and each block's 32 x 32
// L_kk^-1 tile read from Linv when the block is reached instead of staged up front.
constexpr int CMAX_LARGE = 6144;  // 1024 free poses

// PRE (the default; OSG_BACKL_PRE=0 for the previous order, bit-identical): block bi - 1's Linv entry is
// loaded while block bi is solved, so a block does not start with a global round trip.
template <bool PRE>
__global__ __launch_bounds__(1024) void k_chol_back_large(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    const int n = 6 * D.nhp;
    if (n <= CMAX || n > CMAX_LARGE || D.chol_fused) return;
    __shared__ double s_x[CMAX_LARGE];
    __shared__ double s_y[CMAX_LARGE];
    __shared__ double s_li[CB * CB];
    __shared__ double s_part[32][33];
    __shared__ double s_rhs[CB];
    const double *A = D.Hs;
    const int tid = threadIdx.x;
    for (int i = tid; i < n; i += 1024) {
        s_x[i] = 0.0;
        s_y[i] = D.x[i];
    }
    const int nblk = (n + CB - 1) / CB;
    const int c = tid & 31, g = tid >> 5;
    double li_next = PRE ? D.Linv[(size_t)min((nblk - 1) * CB + (tid >> 5), n - 1) * CB + (tid & 31)] : 0.0;
    for (int bi = nblk - 1; bi >= 0; bi--) {
        const int k0 = bi * CB, nb = min(CB, n - k0);
        if (PRE) {
            s_li[tid] = li_next;
            if (bi > 0) li_next = D.Linv[(size_t)min(k0 - CB + (tid >> 5), n - 1) * CB + (tid & 31)];
        } else {
            s_li[tid] = D.Linv[(size_t)min(k0 + (tid >> 5), n - 1) * CB + (tid & 31)];
        }
        __syncthreads();
        // the rows below the block inside the envelope only (column block bi's envelope rows, ascending):
        // every other L entry of this column is zero, and is not stored (k_schur_pairs writes only the
        // pairs the factorisation reads).  Group g takes row g of each of those row blocks.
        double acc = 0.0;
        if (c < nb) {
            for (int q = D.col_rows_start[bi]; q < D.col_rows_start[bi + 1]; q++) {
                const int rb = D.col_rows[q], row = rb * CB + g;
                if (row < n) acc += A[hs_el(hs_blk(D, n, rb), g, k0 + c)] * s_x[row];
            }
        }
        s_part[c][g] = acc;
        __syncthreads();
        if (tid < CB) {
            double s = 0.0;
#pragma unroll
            for (int gg = 0; gg < 32; gg++) s += s_part[tid][gg];
            s_rhs[tid] = (tid < nb) ? s_y[k0 + tid] - s : 0.0;
        }
        __syncthreads();
        if (tid < nb) {
            double xv = 0.0;
#pragma unroll
            for (int r = 0; r < CB; r++) xv += s_li[r * CB + tid] * s_rhs[r];
            s_x[k0 + tid] = xv;
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += 1024) D.x[i] = s_x[i];
}

// Backward substitution past CMAX_LARGE (maps of more than 1024 free KeyFrames), right-looking by
// block, one launch per block from the last: every workgroup forms x_bi = L_bi,bi^-T y'_bi (y' =
// y less the contributions of the blocks already solved; 32 x 32 from Linv, redundantly per
// workgroup) and subtracts L_bi,u^T x_bi from y'_u for its share of the columns u left of the block,
// inside the envelope.  y' lives in x, the solution goes to bs (free after the forward
// substitution) and k_back_copy moves it to x.  The work is the envelope's O(n bw), spread over the
// chip, instead of one workgroup streaming the whole triangle through LDS.
constexpr int BSC = 256;  // columns per workgroup of k_back_step
// PRE (the default; OSG_BACK_PRE=0 for the previous order, bit-identical): the thread's 32 L entries and the
// 32 x 32 Linv column are loaded before y'_bi, which the previous step wrote, so a step waits out one memory
// round trip instead of three in a row (y', then Linv, then L); the sums are the same, in the same order.
template <bool PRE>
__global__ __launch_bounds__(BSC) void k_back_step(const LbaDev *__restrict__ Ds, int step)
{
    LBA_GRAPH(M_ACT);
    const int n = 6 * D.nhp;
    if (n <= CMAX_LARGE || D.chol_fused) return;
    const int bi = D.nblk_red - 1 - step;
    if (bi < 0) return;
    const int k0 = bi * CB, nb = min(CB, n - k0);
    const int c0 = D.blk_first[bi] * CB;  // first column of the row panel inside the envelope
    if (bx > 0 && c0 + (bx - 1) * BSC >= k0) return;
    __shared__ double s_rhs[CB], s_x[CB];
    const int tid = threadIdx.x;
    const double *A = D.Hs;
    const int u = c0 + (bx - 1) * BSC + tid;
    double a[CB], li[CB];
    if (PRE) {
        if (bx > 0 && u < k0) {
            const HsBlk bb = hs_blk(D, n, bi);
#pragma unroll
            for (int r = 0; r < CB; r++) a[r] = r < nb ? A[hs_el(bb, r, u)] : 0.0;
        }
        if (tid < CB)
#pragma unroll
            for (int r = 0; r < CB; r++) li[r] = D.Linv[(size_t)min(k0 + r, n - 1) * CB + tid];
    }
    if (tid < CB) s_rhs[tid] = tid < nb ? D.x[k0 + tid] : 0.0;
    __syncthreads();
    if (tid < CB) {
        double xv = 0.0;
        if (PRE) {
#pragma unroll
            for (int r = 0; r < CB; r++) xv += li[r] * s_rhs[r];
        } else {
#pragma unroll
            for (int r = 0; r < CB; r++) xv += D.Linv[(size_t)min(k0 + r, n - 1) * CB + tid] * s_rhs[r];
        }
        s_x[tid] = tid < nb ? xv : 0.0;
        if (bx == 0 && tid < nb) D.bs[k0 + tid] = xv;
    }
    __syncthreads();
    if (bx == 0) return;  // workgroup 0 solved the block; 1.. update the columns
    if (u >= k0) return;
    double acc = 0.0;
    if (PRE) {
#pragma unroll
        for (int r = 0; r < CB; r++)
            if (r < nb) acc += a[r] * s_x[r];
    } else {
        const HsBlk bb = hs_blk(D, n, bi);
#pragma unroll 8
        for (int r = 0; r < nb; r++) acc += A[hs_el(bb, r, u)] * s_x[r];
    }
    D.x[u] -= acc;
}
__global__ __launch_bounds__(EB) void k_back_copy(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    const int n = 6 * D.nhp;
    if (n <= CMAX_LARGE || D.chol_fused) return;
    const int i = bx * EB + threadIdx.x;
    if (i < n) D.x[i] = D.bs[i];
}

// landmark back-substitution + new estimates + LM scale partials.  Each thread walks its landmark's
// Hpl blocks (16-byte loads, many in flight per thread).  STAGE (OSG_UPDATE_STAGE=1, A/B runs,
// bit-identical): the workgroup's Hpl blocks (its EB landmarks' blocks are consecutive) come through
// LDS in UB-block pieces read with coalesced 16-byte loads; measured slower (2.34 against 2.08 ms per
// 14 launches of 64 C4 windows, profiles/r04_lba_dinv_ab.txt): the pieces serialise load, barrier
// and compute, where the per-thread walks keep more loads in flight.
// COOP (the default; OSG_UPDATE_COOP=0 for the walks, bit-identical): one thread per block, EB consecutive blocks of the
// workgroup's landmarks at a time (coalesced 144-byte blocks, no LDS copy of them): each thread forms its
// block's Hplᵀ(−x_p) in registers and leaves the 3 values in LDS, then each landmark's thread adds its
// blocks' values in block order, the per-thread walk's sums.
constexpr int UB = 256;  // blocks per staged piece: 36 KiB of LDS
template <bool STAGE, bool COOP = false>
__global__ __launch_bounds__(EB) void k_update(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    if (bx >= D.gu) return;
    const double lambda = D.ctl->lambda;
    const double *pose_cur = cur_pose(D), *point_cur = cur_point(D);
    double *pose_new = new_pose(D), *point_new = new_point(D);
    __shared__ double s[EB / 64];
    const int t = bx * EB + threadIdx.x;
    const int sp = 6 * D.nhp;
    double sc = 0.0;
    double cl[3] = {0, 0, 0};
    if (t < D.nhl) {
        cl[0] = D.bl[D.ls_b * (size_t)t];
        cl[1] = D.bl[D.ls_b * (size_t)t + 1];
        cl[2] = D.bl[D.ls_b * (size_t)t + 2];
    }
    if (STAGE) {
        __shared__ double s_b[UB * 18];
        typedef int i4 __attribute__((ext_vector_type(4)));
        const int l0 = bx * EB;
        const int g0 = l0 < D.nhl ? D.lm_b_start[l0] : 0;
        const int g1 = l0 < D.nhl ? D.lm_b_start[min(l0 + EB, D.nhl)] : 0;
        const int mb0 = t < D.nhl ? D.lm_b_start[t] : 0, mb1 = t < D.nhl ? D.lm_b_start[t + 1] : 0;
        for (int p0 = g0; p0 < g1; p0 += UB) {  // workgroup-uniform
            const int nb = min(UB, g1 - p0);
            const i4 *src = (const i4 *)(D.Hpl + 18 * (size_t)p0);
            for (int k = threadIdx.x; k < 9 * nb; k += EB) ((i4 *)s_b)[k] = src[k];
            __syncthreads();
            const int a1 = min(mb1, p0 + nb);
            for (int blk = max(mb0, p0); blk < a1; blk++) {
                const int i1 = D.blk_pose[blk];
                const double *B = s_b + 18 * (blk - p0);
                for (int c = 0; c < 3; c++) {
                    double s_ = 0;
                    for (int r = 0; r < 6; r++) s_ += B[3 * r + c] * (-D.x[6 * i1 + r]);
                    cl[c] += s_;
                }
            }
            __syncthreads();
        }
    }
    if (COOP) {
        __shared__ double s_v[3][EB];
        const int l0 = bx * EB;
        const int g0 = l0 < D.nhl ? D.lm_b_start[l0] : 0;
        const int g1 = l0 < D.nhl ? D.lm_b_start[min(l0 + EB, D.nhl)] : 0;
        const int mb0 = t < D.nhl ? D.lm_b_start[t] : 0, mb1 = t < D.nhl ? D.lm_b_start[t + 1] : 0;
        for (int p0 = g0; p0 < g1; p0 += EB) {  // workgroup-uniform
            const int blk = p0 + (int)threadIdx.x;
            if (blk < g1) {
                const int i1 = D.blk_pose[blk];
                const double *B = D.Hpl + 18 * (size_t)blk;
                for (int c = 0; c < 3; c++) {
                    double s_ = 0;
                    for (int r = 0; r < 6; r++) s_ += B[3 * r + c] * (-D.x[6 * i1 + r]);
                    s_v[c][threadIdx.x] = s_;
                }
            }
            __syncthreads();
            const int a1 = min(mb1, p0 + EB);
            for (int b2 = max(mb0, p0); b2 < a1; b2++)
                for (int c = 0; c < 3; c++) cl[c] += s_v[c][b2 - p0];
            __syncthreads();
        }
    }
    if (t < D.nhl) {
        const int l = t;
        if (!STAGE && !COOP)
            for (int blk = D.lm_b_start[l]; blk < D.lm_b_start[l + 1]; blk++) {
                const int i1 = D.blk_pose[blk];
                const double *B = D.Hpl + 18 * (size_t)blk;
                for (int c = 0; c < 3; c++) {
                    double s_ = 0;
                    for (int r = 0; r < 6; r++) s_ += B[3 * r + c] * (-D.x[6 * i1 + r]);
                    cl[c] += s_;
                }
            }
        // Dinv into registers from either source (a pointer to a local-or-global array put it in scratch)
        double Di[9];
        if (D.dinv_inline) landmark_dinv(D, l, lambda, Di, nullptr);
        else
            for (int k = 0; k < 9; k++) Di[k] = D.Dinv[9 * (size_t)l + k];
        const int p = D.hl_point[l];
        for (int r = 0; r < 3; r++) {
            const double xl = Di[3 * r] * cl[0] + Di[3 * r + 1] * cl[1] + Di[3 * r + 2] * cl[2];
            D.x[sp + 3 * l + r] = xl;
            point_new[3 * (size_t)p + r] = point_cur[3 * (size_t)p + r] + xl;
            sc += xl * (lambda * xl + D.bl[D.ls_b * (size_t)l + r]);
        }
    }
    if (t < D.np) {  // poses: exp(x) * T for free active poses, copy otherwise
        const int hi = D.pose_h[t];
        if (hi >= 0) {
            SE3 T = se3_from7(pose_cur + 7 * (size_t)t);
            double upd[6];
            for (int k = 0; k < 6; k++) {
                upd[k] = D.x[6 * hi + k];
                sc += upd[k] * (lambda * upd[k] + D.bp[6 * (size_t)hi + k]);
            }
            se3_oplus(T, upd);
            se3_to7(T, pose_new + 7 * (size_t)t);
        } else {
            for (int k = 0; k < 7; k++) pose_new[7 * (size_t)t + k] = pose_cur[7 * (size_t)t + k];
        }
    }
    // points without a landmark index (no edges) keep their estimate
    if (t < D.npt && D.point_h[t] < 0)
        for (int k = 0; k < 3; k++) point_new[3 * (size_t)t + k] = point_cur[3 * (size_t)t + k];
    const double tot = block_sum_d(sc, s);
    if (threadIdx.x == 0) D.part[D.npart + bx] = tot;
}

// k_update on the compact per-block factor (the default): the COOP form's one thread per block, forming
// Hpl^T x_p from the block's M', its pose's R and c and its landmark's position (z_rows' algebra); each
// workgroup's landmark positions and each piece's block -> landmark map come through LDS from the
// landmarks' threads.  The per-landmark sums keep the COOP order.
__global__ __launch_bounds__(EB) void k_update_c(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT);
    if (bx >= D.gu) return;
    const double lambda = D.ctl->lambda;
    const double *pose_cur = cur_pose(D), *point_cur = cur_point(D);
    double *pose_new = new_pose(D), *point_new = new_point(D);
    __shared__ double s[EB / 64];
    __shared__ double s_v[3][EB];
    __shared__ double s_xw[3][EB];
    __shared__ int s_lm[EB];
    const int t = bx * EB + threadIdx.x;
    const int sp = 6 * D.nhp;
    double sc = 0.0;
    double cl[3] = {0, 0, 0};
    const int l0 = bx * EB;
    const int g0 = l0 < D.nhl ? D.lm_b_start[l0] : 0;
    const int g1 = l0 < D.nhl ? D.lm_b_start[min(l0 + EB, D.nhl)] : 0;
    const int mb0 = t < D.nhl ? D.lm_b_start[t] : 0, mb1 = t < D.nhl ? D.lm_b_start[t + 1] : 0;
    int p = -1;
    if (t < D.nhl) {
        cl[0] = D.bl[D.ls_b * (size_t)t];
        cl[1] = D.bl[D.ls_b * (size_t)t + 1];
        cl[2] = D.bl[D.ls_b * (size_t)t + 2];
        p = D.hl_point[t];
        for (int k = 0; k < 3; k++) s_xw[k][threadIdx.x] = point_cur[3 * (size_t)p + k];
    }
    // the thread's block of the next piece (its pose and M') is loaded one piece ahead, so a piece waits
    // for its pose's R, c and x_p only
    int i1n = 0;
    double mn[6] = {0, 0, 0, 0, 0, 0};
    auto fetch = [&](int p) {
        const int blk = p + (int)threadIdx.x;
        if (blk < g1) {
            i1n = gbl(D.blk_pose)[blk];
            for (int k = 0; k < 6; k++) mn[k] = gbl(D.Hpl)[6 * (size_t)blk + k];
        }
    };
    if (g0 < g1) fetch(g0);
    for (int p0 = g0; p0 < g1; p0 += EB) {  // workgroup-uniform
        const int i1 = i1n;
        double m[6];
        for (int k = 0; k < 6; k++) m[k] = mn[k];
        if (p0 + EB < g1) fetch(p0 + EB);
        // the piece's block -> landmark (local index) map, from the landmarks' threads
        for (int b2 = max(mb0, p0); b2 < min(mb1, p0 + EB); b2++) s_lm[b2 - p0] = threadIdx.x;
        __syncthreads();
        const int blk = p0 + (int)threadIdx.x;
        if (blk < g1) {
            // Hpl^T x_p = Z^T D(R)^T x_p = M' (y2 - (X + c) x y1), y = (R^T x_p[0:3], R^T x_p[3:6]) (z_rows)
            const int ll = s_lm[threadIdx.x];
            const double *R = D.hp_Rt + RT_STRIDE * (size_t)i1;
            double Rv[15], xp[6];
            for (int k = 0; k < 15; k++) Rv[k] = R[k];
            for (int r = 0; r < 6; r++) xp[r] = D.x[6 * i1 + r];
            const double w0 = s_xw[0][ll] + Rv[12], w1 = s_xw[1][ll] + Rv[13], w2 = s_xw[2][ll] + Rv[14];
            double y1[3], y2[3];
            for (int c = 0; c < 3; c++) {
                y1[c] = Rv[c] * xp[0] + Rv[3 + c] * xp[1] + Rv[6 + c] * xp[2];
                y2[c] = Rv[c] * xp[3] + Rv[3 + c] * xp[4] + Rv[6 + c] * xp[5];
            }
            const double u0 = y2[0] - (w1 * y1[2] - w2 * y1[1]);
            const double u1 = y2[1] - (w2 * y1[0] - w0 * y1[2]);
            const double u2 = y2[2] - (w0 * y1[1] - w1 * y1[0]);
            s_v[0][threadIdx.x] = -(m[0] * u0 + m[1] * u1 + m[2] * u2);
            s_v[1][threadIdx.x] = -(m[1] * u0 + m[3] * u1 + m[4] * u2);
            s_v[2][threadIdx.x] = -(m[2] * u0 + m[4] * u1 + m[5] * u2);
        }
        __syncthreads();
        const int a1 = min(mb1, p0 + EB);
        for (int b2 = max(mb0, p0); b2 < a1; b2++)
            for (int c = 0; c < 3; c++) cl[c] += s_v[c][b2 - p0];
        __syncthreads();
    }
    if (t < D.nhl) {
        const int l = t;
        // Dinv into registers from either source (a pointer to a local-or-global array put it in scratch)
        double Di[9];
        if (D.dinv_inline) landmark_dinv(D, l, lambda, Di, nullptr);
        else
            for (int k = 0; k < 9; k++) Di[k] = D.Dinv[9 * (size_t)l + k];
        for (int r = 0; r < 3; r++) {
            const double xl = Di[3 * r] * cl[0] + Di[3 * r + 1] * cl[1] + Di[3 * r + 2] * cl[2];
            D.x[sp + 3 * l + r] = xl;
            point_new[3 * (size_t)p + r] = point_cur[3 * (size_t)p + r] + xl;
            sc += xl * (lambda * xl + D.bl[D.ls_b * (size_t)l + r]);
        }
    }
    if (t < D.np) {  // poses: exp(x) * T for free active poses, copy otherwise
        const int hi = D.pose_h[t];
        if (hi >= 0) {
            SE3 T = se3_from7(pose_cur + 7 * (size_t)t);
            double upd[6];
            for (int k = 0; k < 6; k++) {
                upd[k] = D.x[6 * hi + k];
                sc += upd[k] * (lambda * upd[k] + D.bp[6 * (size_t)hi + k]);
            }
            se3_oplus(T, upd);
            se3_to7(T, pose_new + 7 * (size_t)t);
        } else {
            for (int k = 0; k < 7; k++) pose_new[7 * (size_t)t + k] = pose_cur[7 * (size_t)t + k];
        }
    }
    if (t < D.npt && D.point_h[t] < 0)
        for (int k = 0; k < 3; k++) point_new[3 * (size_t)t + k] = point_cur[3 * (size_t)t + k];
    const double tot = block_sum_d(sc, s);
    if (threadIdx.x == 0) D.part[D.npart + bx] = tot;
}

__global__ __launch_bounds__(EB) void k_classify(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_FIN);
    const double *poses = cur_pose(D), *points = cur_point(D);
    uint8_t *bad = D.bad;
    const int e = bx * EB + threadIdx.x;
    if (e >= D.ne) return;
    const int k = D.e_kind[e];
    const int dim = (k == OSG_EDGE_STEREO) ? 3 : 2;
    const double ev[3] = {D.err[3 * e], D.err[3 * e + 1], D.err[3 * e + 2]};
    const double th = (k == OSG_EDGE_STEREO) ? 7.815 : 5.991;
    const SE3 T = se3_from7(poses + 7 * (size_t)D.e_pose[e]);
    const bool pos = edge_depth_positive(k, D.cams[D.e_cam[e]], T, points + 3 * (size_t)D.e_point[e]);
    const double c2 = chi2_of(ev, dim, edge_w(D, e));
    bad[e] = (c2 > th || !pos) ? 1 : 0;
    D.chi2o[e] = c2;
}

// The step's scalars per graph, summed in the host's former order (sequential from index 0):
// out = {chi of the trial, LM scale, Cholesky ok, lambda used, chi of the current estimate}.
// The partials are first staged in LDS by all threads (one memory latency), then summed in order.
__global__ __launch_bounds__(256) void k_step_reduce(const LbaDev *__restrict__ Ds)
{
    LBA_GRAPH(M_ACT | M_ERRC);
    __shared__ double s_chi[RED_CHUNK], s_sc[RED_CHUNK], s_cur[RED_CHUNK];
    const int mode = D.ctl->mode;
    const bool act = (mode & M_ACT) != 0, errc = (mode & M_ERRC) != 0;
    const int P = D.npart;
    double chi = 0, sc = 0, chic = 0;
    for (int base = 0; base < max(D.ge, D.gu); base += RED_CHUNK) {
        const int ne = min(RED_CHUNK, max(D.ge - base, 0)), nu = min(RED_CHUNK, max(D.gu - base, 0));
        for (int i = threadIdx.x; i < ne; i += 256) {
            s_chi[i] = act ? D.part[base + i] : 0.0;
            s_cur[i] = errc ? D.part[3 * P + base + i] : 0.0;
        }
        for (int i = threadIdx.x; i < nu; i += 256) s_sc[i] = act ? D.part[P + base + i] : 0.0;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = 0; i < ne; i++) chi += s_chi[i];
            for (int i = 0; i < nu; i++) sc += s_sc[i];
            for (int i = 0; i < ne; i++) chic += s_cur[i];
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    D.out[0] = chi;
    D.out[1] = sc;
    D.out[2] = (D.nhp > 0 && act) ? (double)D.flag[0] : 1.0;
    D.out[3] = D.ctl->lambda;
    D.out[4] = chic;
}

template <typename T>
T *carve(char *base, size_t &off, size_t count)
{
    off = (off + 255) & ~size_t(255);
    T *p = (T *)(base + off);
    off += sizeof(T) * std::max<size_t>(count, 1);
    return p;
}

// ---------------------------------------------------------------------------------------------
// Host side.  One graph = one LbaHost: the BlockSolver structure (built once, like
// BlockSolver::buildStructure) and g2o's LM state.  A batch runs B graphs in lockstep: every step
// is one LM trial of every graph still running (one launch of each kernel for all of them, grid.y
// = graph), then ONE download of 5 scalars per graph, and the host applies the reference's
// accept / reject / lambda rules per graph.  A graph starting an iteration also linearises (and
// recomputes the current estimate's errors, or initialises lambda) in the same step.
struct LbaHost {
    const osg_ba_graph *G = nullptr;
    osg_ba_result *R = nullptr;
    int np = 0, npt = 0, ne = 0, nhp = 0, nhl = 0, nblk = 0, npairs = 0, nchunks = 0;
    int ge = 0, gl = 0, gll = 0, gu = 0, nblk_red = 0, npart = 64;
    bool multi = false;  // a block with several edges (k_linearize<true>)
    std::vector<int32_t> blk_first, blk_last;  // envelope of the reduced system by row block (see LbaDev)
    std::vector<int32_t> col_rows_start, col_rows, live_pairs;  // envelope rows per column block, live pairs
    std::vector<int32_t> live_chunk, env_off;  // per live pair its chunk range; envelope tiles before each row block
    int max_col_rows = 0;
    bool trivial = false;  // nothing to optimise: the estimates are returned unchanged
    int lm_e_ident = 0;
    std::vector<int32_t> pose_h, hp_pose, point_h, hl_point, lm_e_start, lm_e, lg_start, lg_lq, lm_b_start, blk_pose, edge_blk, blk_lm,
        hp_e_start, hp_e, hp_b_start, hp_b, pair_start, pair_b, chunk_start, pair_chunk,
        pair_rank, rs_pose, rs_rank0, rs_chunk_start, rs_chunk, hp_rs_start, rs_order, rs_cdesc, rs_info, hp_b_lm;
    int n_rs = 0;
    double t_struct = 0;
    // LM state (ref:Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-194 and
    // sparse_optimizer.cpp optimize())
    double lambda = 0, ni = 2, currentChi = 0, iniChi = 0, rho = 0;
    int nBad = 0, iters = 0, trials = 0, qmax = 0, it = 0, sel = 0;
    bool errors_current = true, new_iter = true, done = false;
    size_t o_in = 0, o_st = 0;  // offsets of this graph's inputs / state

    // new call: scalars back to their initial values; the vectors keep their capacity (a batch of
    // windows frees and re-faults hundreds of MB otherwise)
    void reset()
    {
        G = nullptr;
        R = nullptr;
        np = npt = ne = nhp = nhl = nblk = npairs = nchunks = n_rs = 0;
        ge = gl = gll = gu = nblk_red = 0;
        multi = false;
        npart = 64;
        blk_first.clear();
        blk_last.clear();
        col_rows_start.clear();
        col_rows.clear();
        live_pairs.clear();
        live_chunk.clear();
        env_off.clear();
        max_col_rows = 0;
        trivial = false;
        hp_pose.clear();
        hl_point.clear();
        blk_pose.clear();
        chunk_start.clear();
        rs_pose.clear();
        rs_order.clear();
        rs_cdesc.clear();
        rs_info.clear();
        hp_b_lm.clear();
        rs_rank0.clear();
        rs_chunk.clear();
        t_struct = 0;
        lambda = 0;
        ni = 2;
        currentChi = iniChi = rho = 0;
        nBad = iters = trials = qmax = it = sel = 0;
        errors_current = true;
        new_iter = true;
        done = false;
    }
};

struct LbaCache {
    std::vector<LbaHost> H;
    std::vector<hipEvent_t> kev;  // osg_lba_kernel_times marks
    std::vector<int> kcls;
    ~LbaCache()
    {
        for (hipEvent_t e : kev) (void)hipEventDestroy(e);
    }
};
enum { KT_ERR, KT_LIN, KT_POSE, KT_LINIT, KT_SPOINT, KT_SROWS, KT_SPAIRS, KT_CHOL, KT_BACK, KT_UPD, KT_RED, KT_CLASS, KT_END };
static_assert(KT_END == OSG_LBA_NK, "osg_lba_kernel_times slots");

// Stable counting sort of the indices [0, n) by key(i) in [0, K) (negative: left out) on up to
// `threads` host workers: contiguous index ranges, per-range histograms, offsets in (key, range)
// order, so every key's indices keep their order.  start gets K + 1 offsets, out the indices.
template <class KeyF>
void counting_sort_par(int n, int K, KeyF key, std::vector<int32_t> &start, std::vector<int32_t> &out, int threads)
{
    const int T = std::max(1, std::min(threads, (n + 4095) / 4096));
    std::vector<int32_t> hist((size_t)T * K, 0);
    auto range = [&](int t, int &i0, int &i1) {
        i0 = (int)((int64_t)n * t / T);
        i1 = (int)((int64_t)n * (t + 1) / T);
    };
    osg_parallel_for(T, T, [&](int t) {
        int i0, i1;
        range(t, i0, i1);
        int32_t *h = hist.data() + (size_t)t * K;
        for (int i = i0; i < i1; i++) {
            const int k = key(i);
            if (k >= 0) h[k]++;
        }
    });
    start.assign(K + 1, 0);
    int32_t run = 0;
    for (int k = 0; k < K; k++) {
        start[k] = run;
        for (int t = 0; t < T; t++) {
            const int32_t c = hist[(size_t)t * K + k];
            hist[(size_t)t * K + k] = run;
            run += c;
        }
    }
    start[K] = run;
    out.assign(std::max(run, 1), 0);
    osg_parallel_for(T, T, [&](int t) {
        int i0, i1;
        range(t, i0, i1);
        int32_t *h = hist.data() + (size_t)t * K;
        for (int i = i0; i < i1; i++) {
            const int k = key(i);
            if (k >= 0) out[h[k]++] = i;
        }
    });
}

// phase clocks of the structure build (tools/micro/lba_host_time.hip defines OSG_LBA_STRUCT_PROF)
#ifdef OSG_LBA_STRUCT_PROF
thread_local double g_struct_cp[16];
#define STRUCT_CP(k) g_struct_cp[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0).count()
#else
#define STRUCT_CP(k)
#endif
int build_structure(osg_ctx *ctx, const osg_ba_graph *G, LbaHost &H)
{
    const auto tp0 = std::chrono::steady_clock::now();
    const int np = G->n_poses, npt = G->n_points, ne = G->n_edges;
    H.np = np;
    H.npt = npt;
    H.ne = ne;
    std::vector<int32_t> pose_cnt(np, 0), point_cnt(npt, 0);
    for (int e = 0; e < ne; e++) {
        pose_cnt[G->e_pose[e]]++;
        point_cnt[G->e_point[e]]++;
    }
    H.pose_h.assign(np, -1);
    H.point_h.assign(npt, -1);
    for (int i = 0; i < np; i++)
        if (!G->pose_fixed[i] && pose_cnt[i] > 0) {
            H.pose_h[i] = (int)H.hp_pose.size();
            H.hp_pose.push_back(i);
        }
    for (int i = 0; i < npt; i++)
        if (point_cnt[i] > 0) {
            H.point_h[i] = (int)H.hl_point.size();
            H.hl_point.push_back(i);
        }
    const int nhp = (int)H.hp_pose.size(), nhl = (int)H.hl_point.size();
    H.nhp = nhp;
    H.nhl = nhl;
    if (nhp + nhl == 0) {
        H.trivial = true;
        return OSG_OK;
    }
    // the pose-pair index (i <= j) is an int32_t; past CMAX the reduced system lives on its envelope
    if ((size_t)nhp * ((size_t)nhp + 1) / 2 >= (size_t(1) << 31))
        return osg_set_error(ctx, OSG_E_INVALID, "%d free poses: the pose-pair index would exceed 2^31", nhp);
    STRUCT_CP(1);
    const std::vector<int32_t> &pose_h = H.pose_h, &point_h = H.point_h;
    // edges per landmark (stable in edge order)
    H.lm_e_start.assign(nhl + 1, 0);
    H.lm_e.assign(ne, 0);
    for (int e = 0; e < ne; e++) H.lm_e_start[point_h[G->e_point[e]] + 1]++;
    for (int l = 0; l < nhl; l++) H.lm_e_start[l + 1] += H.lm_e_start[l];
    {
        std::vector<int32_t> fill(H.lm_e_start.begin(), H.lm_e_start.end() - 1);
        for (int e = 0; e < ne; e++) H.lm_e[fill[point_h[G->e_point[e]]]++] = e;
        // OSG_LBA_LMIDENT=0: always through lm_e (A/B runs, the same values)
        static const bool ident_ok = !(getenv("OSG_LBA_LMIDENT") && atoi(getenv("OSG_LBA_LMIDENT")) == 0);
        H.lm_e_ident = ident_ok ? 1 : 0;
        for (int q = 0; q < ne && H.lm_e_ident; q++) H.lm_e_ident = H.lm_e[q] == q;
        // k_linearize's landmark groups: consecutive landmarks with at most EB edges together, a
        // landmark with more alone
        H.lg_start.assign(1, 0);
        for (int l = 0; l < nhl;) {
            int l1 = l + 1;
            while (l1 < nhl && H.lm_e_start[l1 + 1] - H.lm_e_start[l] <= EB) l1++;
            H.lg_start.push_back(l1);
            l = l1;
        }
        if (nhl == 0) H.lg_start.push_back(0);
        H.lg_lq.resize(2 * H.lg_start.size());
        for (size_t g = 0; g < H.lg_start.size(); g++) {
            H.lg_lq[2 * g] = H.lg_start[g];
            H.lg_lq[2 * g + 1] = H.lm_e_start[H.lg_start[g]];
        }
    }
    STRUCT_CP(2);
    // a map (one large graph per call) builds its structure on host workers; a window (many per batch,
    // each on its own worker) keeps the sequential passes.  Both give the same arrays.
    // (OSG_LBA_MAP_MODE=1 takes the map path for any graph: the host-runtime tests compare the two)
    const bool map_mode = nhp >= 512 || (getenv("OSG_LBA_MAP_MODE") && atoi(getenv("OSG_LBA_MAP_MODE")) == 1);
    if (map_mode) {
        // blocks per landmark: unique free poses sorted by hessian index, counted then filled per
        // landmark range; the per-edge block code as below, settled landmark by landmark (a block's
        // edges all belong to its landmark and lm_e lists them in edge order)
        const int NR = std::max(1, std::min(256, nhl / 256));
        auto lrange = [&](int r, int &l0, int &l1) {
            l0 = (int)((int64_t)nhl * r / NR);
            l1 = (int)((int64_t)nhl * (r + 1) / NR);
        };
        auto distinct = [&](int l, std::vector<int32_t> &stamp, std::vector<int32_t> &tmp) {
            tmp.clear();
            for (int q = H.lm_e_start[l]; q < H.lm_e_start[l + 1]; q++) {
                const int ph = pose_h[G->e_pose[H.lm_e[q]]];
                if (ph >= 0 && stamp[ph] != l) {
                    stamp[ph] = l;
                    tmp.push_back(ph);
                }
            }
        };
        H.lm_b_start.assign(nhl + 1, 0);
        osg_parallel_for(NR, 16, [&](int r) {
            thread_local std::vector<int32_t> stamp, tmp;
            stamp.assign(nhp, -1);
            int l0, l1;
            lrange(r, l0, l1);
            for (int l = l0; l < l1; l++) {
                distinct(l, stamp, tmp);
                H.lm_b_start[l + 1] = (int)tmp.size();
            }
        });
        for (int l = 0; l < nhl; l++) H.lm_b_start[l + 1] += H.lm_b_start[l];
        const int nb = H.lm_b_start[nhl];
        H.blk_pose.assign(nb, 0);
        H.blk_lm.assign(nb, 0);
        H.edge_blk.assign(ne, -1);
        std::atomic<bool> multi(false);
        osg_parallel_for(NR, 16, [&](int r) {
            thread_local std::vector<int32_t> stamp, tmp, cnt;
            thread_local std::vector<uint8_t> seen;
            stamp.assign(nhp, -1);
            bool m = false;
            int l0, l1;
            lrange(r, l0, l1);
            for (int l = l0; l < l1; l++) {
                distinct(l, stamp, tmp);
                std::sort(tmp.begin(), tmp.end());
                const int base = H.lm_b_start[l], k = (int)tmp.size();
                cnt.assign(k, 0);
                seen.assign(k, 0);
                for (int u = 0; u < k; u++) {
                    H.blk_pose[base + u] = tmp[u];
                    H.blk_lm[base + u] = l;
                }
                auto slot = [&](int ph) { return (int)(std::lower_bound(tmp.begin(), tmp.end(), ph) - tmp.begin()); };
                for (int q = H.lm_e_start[l]; q < H.lm_e_start[l + 1]; q++) {
                    const int ph = pose_h[G->e_pose[H.lm_e[q]]];
                    if (ph >= 0) cnt[slot(ph)]++;
                }
                for (int q = H.lm_e_start[l]; q < H.lm_e_start[l + 1]; q++) {
                    const int e = H.lm_e[q];
                    const int ph = pose_h[G->e_pose[e]];
                    if (ph < 0) continue;
                    const int u = slot(ph);
                    H.edge_blk[e] = 4 * (base + u) + (cnt[u] > 1 ? 2 : 0) + (seen[u] ? 1 : 0);
                    seen[u] = 1;
                    m |= cnt[u] > 1;
                }
            }
            if (m) multi = true;
        });
        H.multi = multi.load();
    } else {
        // blocks per landmark: unique free poses sorted by hessian index
        H.lm_b_start.assign(nhl + 1, 0);
        H.edge_blk.assign(ne, -1);
        H.blk_pose.reserve(ne);
        std::vector<int32_t> tmp;
        for (int l = 0; l < nhl; l++) {
            tmp.clear();
            for (int q = H.lm_e_start[l]; q < H.lm_e_start[l + 1]; q++) {
                const int ph = pose_h[G->e_pose[H.lm_e[q]]];
                if (ph >= 0) tmp.push_back(ph);
            }
            std::sort(tmp.begin(), tmp.end());
            tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
            const int base = (int)H.blk_pose.size();
            for (int ph : tmp) H.blk_pose.push_back(ph);
            H.lm_b_start[l + 1] = (int)H.blk_pose.size();
            for (int q = H.lm_e_start[l]; q < H.lm_e_start[l + 1]; q++) {
                const int e = H.lm_e[q];
                const int ph = pose_h[G->e_pose[e]];
                if (ph < 0) continue;
                for (int k = 0; k < (int)tmp.size(); k++)
                    if (tmp[k] == ph) {
                        H.edge_blk[e] = base + k;
                        break;
                    }
            }
        }
        const int nb = (int)H.blk_pose.size();
        H.blk_lm.assign(nb, 0);
        for (int l = 0; l < nhl; l++)
            for (int b = H.lm_b_start[l]; b < H.lm_b_start[l + 1]; b++) H.blk_lm[b] = l;
        // per edge 4 block + 2 (the block has several edges) + 1 (not the block's first edge in edge
        // order): k_linearize writes a lone edge's Hpl block directly, and stores the first edge's terms
        // of a shared block and adds the others' (a per-block reduction in edge order)
        std::vector<int32_t> cnt(nb, 0);
        for (int e = 0; e < ne; e++)
            if (H.edge_blk[e] >= 0) cnt[H.edge_blk[e]]++;
        std::vector<uint8_t> seen(nb, 0);
        for (int e = 0; e < ne; e++)
            if (H.edge_blk[e] >= 0) {
                const int b = H.edge_blk[e];
                H.edge_blk[e] = 4 * b + (cnt[b] > 1 ? 2 : 0) + (seen[b] ? 1 : 0);
                seen[b] = 1;
                H.multi |= cnt[b] > 1;
            }
    }
    STRUCT_CP(3);
    const int nblk = (int)H.blk_pose.size();
    H.nblk = nblk;
    STRUCT_CP(4);
    // edges / blocks per hessian pose
    if (map_mode) {
        counting_sort_par(ne, nhp, [&](int e) { return pose_h[G->e_pose[e]]; }, H.hp_e_start, H.hp_e, 16);
        H.hp_e.resize(H.hp_e_start[nhp]);
        counting_sort_par(nblk, nhp, [&](int b) { return H.blk_pose[b]; }, H.hp_b_start, H.hp_b, 16);
        H.hp_b.resize(nblk);
    } else {
    H.hp_e_start.assign(nhp + 1, 0);
    H.hp_b_start.assign(nhp + 1, 0);
    H.hp_b.assign(nblk, 0);
    for (int e = 0; e < ne; e++)
        if (pose_h[G->e_pose[e]] >= 0) H.hp_e_start[pose_h[G->e_pose[e]] + 1]++;
    for (int i = 0; i < nhp; i++) H.hp_e_start[i + 1] += H.hp_e_start[i];
    H.hp_e.assign(H.hp_e_start[nhp], 0);
    {
        std::vector<int32_t> fill(H.hp_e_start.begin(), H.hp_e_start.end() - 1);
        for (int e = 0; e < ne; e++)
            if (pose_h[G->e_pose[e]] >= 0) H.hp_e[fill[pose_h[G->e_pose[e]]]++] = e;
    }
    for (int b = 0; b < nblk; b++) H.hp_b_start[H.blk_pose[b] + 1]++;
    for (int i = 0; i < nhp; i++) H.hp_b_start[i + 1] += H.hp_b_start[i];
    {
        std::vector<int32_t> fill(H.hp_b_start.begin(), H.hp_b_start.end() - 1);
        for (int b = 0; b < nblk; b++) H.hp_b[fill[H.blk_pose[b]]++] = b;
    }
    }
    STRUCT_CP(5);
    // pose pairs (i <= j), dense index pid(i, j) = i nhp - i (i - 1) / 2 + j - i; the contributions
    // (a, b) of a pair in landmark order, of which the device reads b and the rank of a in pose i's
    // block list.  A window (tens of poses, many per batch on host threads) walks the landmarks in
    // order.  A map (one large graph per call) goes row by row on host workers: pose i's block list
    // is in landmark order and each of its blocks a pairs with the blocks b >= a of its landmark
    // (poses j >= i), so row i counts and then fills its own pairs (consecutive in pid) in landmark
    // order.  Both give the same arrays.
    const int npairs = nhp * (nhp + 1) / 2;
    H.npairs = npairs;
    auto rowbase = [nhp](int i) { return (size_t)i * nhp - (size_t)i * (i - 1) / 2 - i; };  // pid(i, j) - j
    const int row_threads = map_mode ? 16 : 1;
    H.pair_start.assign(npairs + 1, 0);
    std::vector<int32_t> hpb_end, blk_rank;  // per hp_b entry: one past its landmark's last block
    if (row_threads > 1) {
        hpb_end.resize(std::max(nblk, 1));
        osg_parallel_for(64, row_threads, [&](int t) {
            const size_t q0 = H.hp_b.size() * t / 64, q1 = H.hp_b.size() * (t + 1) / 64;
            for (size_t q = q0; q < q1; q++) hpb_end[q] = H.lm_b_start[H.blk_lm[H.hp_b[q]] + 1];
        });
        osg_parallel_for(nhp, row_threads, [&](int i) {
            int32_t *ps = H.pair_start.data() + 1 + rowbase(i);  // [j]
            for (int q = H.hp_b_start[i]; q < H.hp_b_start[i + 1]; q++)
                for (int b = H.hp_b[q], e = hpb_end[q]; b < e; b++) ps[H.blk_pose[b]]++;
        });
    } else {
        blk_rank.resize(std::max(nblk, 1));
        for (int i = 0; i < nhp; i++)
            for (int q = H.hp_b_start[i]; q < H.hp_b_start[i + 1]; q++) blk_rank[H.hp_b[q]] = q - H.hp_b_start[i];
        for (int l = 0; l < nhl; l++)
            for (int a = H.lm_b_start[l]; a < H.lm_b_start[l + 1]; a++) {
                int32_t *ps = H.pair_start.data() + 1 + rowbase(H.blk_pose[a]);
                for (int b = a; b < H.lm_b_start[l + 1]; b++) ps[H.blk_pose[b]]++;
            }
    }
    for (int k = 0; k < npairs; k++) H.pair_start[k + 1] += H.pair_start[k];
    const size_t ncontrib = (size_t)H.pair_start[npairs];
    H.pair_b.assign(std::max<size_t>(ncontrib, 1), 0);
    H.pair_rank.assign(std::max<size_t>(ncontrib, 1), 0);
    if (row_threads > 1) {
        osg_parallel_for(nhp, row_threads, [&](int i) {
            thread_local std::vector<int32_t> fill;
            fill.resize(nhp);
            const size_t rb = rowbase(i);
            const int hb0 = H.hp_b_start[i], hb1 = H.hp_b_start[i + 1];
            int jmax = i;  // the row's pairs reach no further than its blocks' poses
            for (int q = hb0; q < hb1; q++) jmax = std::max(jmax, (int)H.blk_pose[hpb_end[q] - 1]);
            for (int j = i; j <= jmax; j++) fill[j] = H.pair_start[rb + j];
            for (int q = hb0; q < hb1; q++)
                for (int b = H.hp_b[q], e = hpb_end[q]; b < e; b++) {
                    const int k = fill[H.blk_pose[b]]++;
                    H.pair_b[k] = b;
                    H.pair_rank[k] = q - hb0;
                }
        });
    } else {
        std::vector<int32_t> fill(H.pair_start.begin(), H.pair_start.end() - 1);
        for (int l = 0; l < nhl; l++)
            for (int a = H.lm_b_start[l]; a < H.lm_b_start[l + 1]; a++) {
                int32_t *fa = fill.data() + rowbase(H.blk_pose[a]);
                for (int b = a; b < H.lm_b_start[l + 1]; b++) {
                    const int k = fa[H.blk_pose[b]]++;
                    H.pair_b[k] = b;
                    H.pair_rank[k] = blk_rank[a];
                }
            }
    }
    STRUCT_CP(6);
    // envelope of the reduced system (used past CMAX): a pose row's first nonzero pose column is the
    // smallest pose it shares a landmark with; row block t starts at the smallest over its rows
    {
        std::vector<int32_t> minJ(nhp);
        for (int i = 0; i < nhp; i++) minJ[i] = i;
        for (int l = 0; l < nhl; l++) {
            int pm = INT32_MAX;
            for (int a = H.lm_b_start[l]; a < H.lm_b_start[l + 1]; a++) pm = std::min(pm, (int)H.blk_pose[a]);
            for (int a = H.lm_b_start[l]; a < H.lm_b_start[l + 1]; a++)
                minJ[H.blk_pose[a]] = std::min(minJ[H.blk_pose[a]], pm);
        }
        const int n = 6 * nhp, nb = (n + CB - 1) / CB;
        H.blk_first.assign(nb, 0);
        H.blk_last.assign(nb, 0);
        for (int t = 0; t < nb; t++) {
            int f = t;
            for (int r = CB * t; r < std::min(n, CB * t + CB); r++) f = std::min(f, 6 * minJ[r / 6] / CB);
            H.blk_first[t] = f;
        }
        for (int j = 0; j < nb; j++) H.blk_last[j] = j;
        for (int t = 0; t < nb; t++)
            for (int j = H.blk_first[t]; j <= t; j++) H.blk_last[j] = std::max(H.blk_last[j], t);
        if (n > CMAX) {
            H.col_rows_start.assign(nb + 1, 0);
            for (int t = 0; t < nb; t++)
                for (int j = H.blk_first[t]; j < t; j++) H.col_rows_start[j + 1]++;
            for (int j = 0; j < nb; j++) H.col_rows_start[j + 1] += H.col_rows_start[j];
            H.col_rows.assign(std::max(H.col_rows_start[nb], 1), 0);
            std::vector<int32_t> fill(H.col_rows_start.begin(), H.col_rows_start.end() - 1);
            for (int t = 0; t < nb; t++)  // t ascending: each list comes out sorted
                for (int j = H.blk_first[t]; j < t; j++) H.col_rows[fill[j]++] = t;
            for (int j = 0; j < nb; j++)
                H.max_col_rows = std::max(H.max_col_rows, H.col_rows_start[j + 1] - H.col_rows_start[j]);
            // the envelope tile store (hs_at): row block t keeps tiles blk_first[t] .. t
            H.env_off.assign(nb + 1, 0);
            for (int t = 0; t < nb; t++) H.env_off[t + 1] = H.env_off[t] + (t - H.blk_first[t] + 1);
            // live pairs: (i <= j) with some entry (row in pose j, column in pose i) in a lower
            // envelope tile: row block of 6 j + r, column block of 6 i + c, blk_first[row blk] <= col blk
            std::vector<int32_t> fj(nhp);  // the smallest envelope start over pose j's two row blocks
            for (int j = 0; j < nhp; j++) fj[j] = std::min(H.blk_first[(6 * j) / CB], H.blk_first[(6 * j + 5) / CB]);
            for (int i = 0, k = 0; i < nhp; i++) {
                const int cb1 = (6 * i + 5) / CB;  // the block's last column block
                for (int j = i; j < nhp; j++, k++)
                    if (fj[j] <= cb1) H.live_pairs.push_back(k);
            }
        }
    }
    STRUCT_CP(7);
    // row segments of RS ranks
    H.hp_rs_start.assign(nhp + 1, 0);
    for (int i = 0; i < nhp; i++) {
        const int nb = H.hp_b_start[i + 1] - H.hp_b_start[i];
        H.hp_rs_start[i + 1] = H.hp_rs_start[i] + std::max(1, (nb + RS - 1) / RS);
        for (int r = 0; r < std::max(1, (nb + RS - 1) / RS); r++) {
            H.rs_pose.push_back(i);
            H.rs_rank0.push_back(r * RS);
        }
    }
    H.n_rs = H.hp_rs_start[nhp];
    // launch order of the row segments: by the landmark at the middle of the segment (pose order on
    // ties) when OSG_SCHUR_ORDER=1, so the segments in flight together read the Hpl blocks of one
    // landmark range; identity otherwise.  Only which workgroup takes a segment changes: every sum
    // keeps its order, the results are bit-identical.
    H.rs_order.resize(H.n_rs);
    for (int r = 0; r < H.n_rs; r++) H.rs_order[r] = r;
    static const bool schur_order = getenv("OSG_SCHUR_ORDER") && atoi(getenv("OSG_SCHUR_ORDER")) == 1;
    if (schur_order) {
        std::vector<int32_t> key(H.n_rs);
        for (int r = 0; r < H.n_rs; r++) {
            const int i = H.rs_pose[r], hb0 = H.hp_b_start[i], nb = H.hp_b_start[i + 1] - hb0;
            const int mid = std::min(nb - 1, H.rs_rank0[r] + std::min(RS, nb - H.rs_rank0[r]) / 2);
            key[r] = nb > 0 ? H.blk_lm[H.hp_b[hb0 + mid]] : 0;
        }
        std::stable_sort(H.rs_order.begin(), H.rs_order.end(), [&](int a, int b) { return key[a] < key[b]; });
    }
    STRUCT_CP(8);
    // chunks of <= SCH contributions, never spanning two pairs or two row segments; listed per row
    // segment (pair order, then contribution order).  A row's chunks belong to its own segments, so
    // the rows are numbered from per-row counts and filled independently (host workers for a map).
    // A pair's ranks ascend (landmark order): a chunk ends at SCH contributions or at the first rank
    // of the next segment.
    auto row_chunks = [&](int i, auto &&emit) {
        const size_t rb = rowbase(i);
        for (int j = i; j < nhp; j++) {
            const int k = (int)(rb + j), q1 = H.pair_start[k + 1];
            emit(k, -1, 0);  // the pair's first chunk
            for (int q = H.pair_start[k]; q < q1;) {
                const int seg = H.pair_rank[q] / RS, seg_end = (seg + 1) * RS;
                const int e1 = std::min(q1, q + SCH);
                int e = q + 1;
                while (e < e1 && H.pair_rank[e] < seg_end) e++;
                emit(k, q, seg);
                q = e;
            }
        }
    };
    std::vector<int32_t> chunk_rs;
    if (row_threads == 1) {  // a window: one pass in pair order
        H.pair_chunk.assign(npairs + 1, 0);
        H.chunk_start.clear();
        for (int i = 0; i < nhp; i++)
            row_chunks(i, [&](int k, int q, int seg) {
                if (q < 0) {
                    H.pair_chunk[k] = (int)H.chunk_start.size();
                    return;
                }
                H.chunk_start.push_back(q);
                chunk_rs.push_back(H.hp_rs_start[i] + seg);
            });
        H.nchunks = (int)H.chunk_start.size();
        H.pair_chunk[npairs] = H.nchunks;
        H.chunk_start.push_back(H.pair_start[npairs]);
        H.rs_chunk_start.assign(H.n_rs + 1, 0);
        for (int c = 0; c < H.nchunks; c++) H.rs_chunk_start[chunk_rs[c] + 1]++;
        for (int r = 0; r < H.n_rs; r++) H.rs_chunk_start[r + 1] += H.rs_chunk_start[r];
        H.rs_chunk.assign(std::max(H.nchunks, 1), 0);
        std::vector<int32_t> fill(H.rs_chunk_start.begin(), H.rs_chunk_start.end() - 1);
        for (int c = 0; c < H.nchunks; c++) H.rs_chunk[fill[chunk_rs[c]]++] = c;
    } else {  // a map: rows numbered from per-row counts, filled on host workers
    std::vector<int32_t> row_c0(nhp + 1, 0);
    osg_parallel_for(nhp, row_threads, [&](int i) {
        int n = 0;
        row_chunks(i, [&](int, int q, int) { n += q >= 0; });
        row_c0[i + 1] = n;
    });
    for (int i = 0; i < nhp; i++) row_c0[i + 1] += row_c0[i];
    H.nchunks = row_c0[nhp];
    H.pair_chunk.assign(npairs + 1, 0);
    H.chunk_start.assign(H.nchunks + 1, 0);
    chunk_rs.resize(std::max(H.nchunks, 1));
    H.rs_chunk_start.assign(H.n_rs + 1, 0);
    osg_parallel_for(nhp, row_threads, [&](int i) {
        int c = row_c0[i];
        row_chunks(i, [&](int k, int q, int seg) {
            if (q < 0) {
                H.pair_chunk[k] = c;
                return;
            }
            H.chunk_start[c] = q;
            chunk_rs[c] = H.hp_rs_start[i] + seg;
            H.rs_chunk_start[chunk_rs[c] + 1]++;  // the row's own segments
            c++;
        });
    });
    H.pair_chunk[npairs] = H.nchunks;
    H.chunk_start[H.nchunks] = H.pair_start[npairs];
    for (int r = 0; r < H.n_rs; r++) H.rs_chunk_start[r + 1] += H.rs_chunk_start[r];
    H.rs_chunk.assign(std::max(H.nchunks, 1), 0);
    osg_parallel_for(nhp, row_threads, [&](int i) {
        thread_local std::vector<int32_t> fill;
        const int r0 = H.hp_rs_start[i], r1 = H.hp_rs_start[i + 1];
        fill.assign(H.rs_chunk_start.begin() + r0, H.rs_chunk_start.begin() + r1);
        for (int c = row_c0[i]; c < row_c0[i + 1]; c++) H.rs_chunk[fill[chunk_rs[c] - r0]++] = c;
    });
    }
    if (!H.env_off.empty()) {  // past CMAX k_schur_pairs walks the live pairs only
        H.live_chunk.resize(2 * std::max<size_t>(H.live_pairs.size(), 1));
        for (size_t s = 0; s < H.live_pairs.size(); s++) {
            H.live_chunk[2 * s] = H.pair_chunk[H.live_pairs[s]];
            H.live_chunk[2 * s + 1] = H.pair_chunk[H.live_pairs[s] + 1];
        }
    }
    STRUCT_CP(9);
    H.rs_info.assign(8 * (size_t)std::max(H.n_rs, 1), 0);
    for (int w = 0; w < H.n_rs; w++) {
        const int r = H.rs_order[w], i = H.rs_pose[r], hb0 = H.hp_b_start[i];
        int32_t *f = &H.rs_info[8 * (size_t)w];
        f[0] = r;
        f[1] = i;
        f[2] = H.rs_rank0[r];
        f[3] = hb0;
        f[4] = std::min(RS, H.hp_b_start[i + 1] - hb0 - H.rs_rank0[r]);
        f[5] = H.rs_chunk_start[r];
        f[6] = H.rs_chunk_start[r + 1];
    }
    H.hp_b_lm.assign(std::max<size_t>(H.hp_b.size(), 1), 0);
    for (size_t q = 0; q < H.hp_b.size(); q++) H.hp_b_lm[q] = H.blk_lm[H.hp_b[q]];
    H.rs_cdesc.assign(4 * (size_t)std::max(H.nchunks, 1), 0);
    for (int t = 0; t < H.nchunks; t++) {
        const int c = H.rs_chunk[t];
        H.rs_cdesc[4 * (size_t)t] = c;
        H.rs_cdesc[4 * (size_t)t + 1] = H.chunk_start[c];
        H.rs_cdesc[4 * (size_t)t + 2] = H.chunk_start[c + 1] - H.chunk_start[c];
        H.rs_cdesc[4 * (size_t)t + 3] = H.blk_pose[H.pair_b[H.chunk_start[c]]];  // the partner pose j
    }
    STRUCT_CP(10);
    H.ge = (ne + EB - 1) / EB;
    H.gl = (nhl + EB - 1) / EB;
    H.gll = (int)H.lg_start.size() - 1;
    H.gu = (std::max(std::max(nhl, np), npt) + EB - 1) / EB;
    H.nblk_red = (6 * nhp + CB - 1) / CB;
    H.npart = (std::max(std::max(H.ge, H.gu), std::max(H.gll + nhp, 1)) + 63) & ~63;
    H.t_struct = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0).count();
    return OSG_OK;
}

int check_graph(osg_ctx *ctx, const osg_ba_graph *G, const osg_ba_result *R)
{
    OSG_REQUIRE(ctx, G && R, "null argument");
    const int np = G->n_poses, npt = G->n_points, ne = G->n_edges;
    OSG_REQUIRE(ctx, np >= 0 && npt >= 0 && ne >= 0 && G->n_cams >= 0, "sizes");
    OSG_REQUIRE(ctx, R->pose && R->point && (ne == 0 || R->edge_bad), "result buffers");
    for (int e = 0; e < ne; e++) {
        if (G->e_pose[e] < 0 || G->e_pose[e] >= np || G->e_point[e] < 0 || G->e_point[e] >= npt ||
            G->e_cam[e] < 0 || G->e_cam[e] >= G->n_cams)
            return osg_set_error(ctx, OSG_E_INVALID, "edge %d references out of range", e);
    }
    return OSG_OK;
}

// device state of one graph (sizes only when base == nullptr)
void carve_state(char *base, size_t &off, const LbaHost &H, LbaDev *D, bool prof_ts, bool compact)
{
    const int np = H.np, npt = H.npt, ne = H.ne, nhl = H.nhl, nhp = H.nhp, nblk = H.nblk;
    const int sp = 6 * nhp;
    double *pA = carve<double>(base, off, 7 * (size_t)np);
    double *pB = carve<double>(base, off, 7 * (size_t)np);
    double *qA = carve<double>(base, off, 3 * (size_t)npt);
    double *qB = carve<double>(base, off, 3 * (size_t)npt);
    double *err = carve<double>(base, off, 3 * (size_t)ne);
    static const bool lrec = getenv("OSG_LBA_LREC") && atoi(getenv("OSG_LBA_LREC")) == 1;
    double *Hll = carve<double>(base, off, (lrec ? 16 : 9) * (size_t)nhl);
    double *bl = lrec ? Hll + 9 : carve<double>(base, off, 3 * (size_t)nhl);
    double *Hpl = carve<double>(base, off, (compact ? 6 : 18) * (size_t)nblk);  // the compact M, or Hpl
    double *hp_Rt = carve<double>(base, off, RT_STRIDE * (size_t)nhp);
    double *lmX = lrec ? Hll + 12 : carve<double>(base, off, compact ? 3 * (size_t)nhl : 1);
    double *Hpp = carve<double>(base, off, 36 * (size_t)nhp);
    double *bp = carve<double>(base, off, 6 * (size_t)nhp);
    double *Dinv = carve<double>(base, off, 9 * (size_t)nhl);
    double *bs_part = carve<double>(base, off, 6 * (size_t)std::max(H.n_rs, 1));
    // dense up to CMAX; past it the envelope's tiles only (the dense n^2 capped maps at 7 723 free KeyFrames)
    double *Hs = carve<double>(base, off, H.env_off.empty() ? (size_t)sp * sp : (size_t)H.env_off.back() * CB * CB);
    double *bs = carve<double>(base, off, (size_t)sp);
    double *x = carve<double>(base, off, (size_t)sp + 3 * (size_t)nhl);
    double *part = carve<double>(base, off, 4 * (size_t)H.npart + 64);
    double *chunk_part = carve<double>(base, off, 36 * (size_t)std::max(H.nchunks, 1));
    double *db = carve<double>(base, off, 3 * (size_t)nhl);
    double *Linv = carve<double>(base, off, (size_t)sp * CB);
    int *flag = carve<int>(base, off, 16);
    unsigned long long *ts = prof_ts ? carve<unsigned long long>(base, off, 8 * 2 * 64 + 64) : nullptr;
    double *chi2o = carve<double>(base, off, (size_t)std::max(ne, 1));
    uint8_t *bad = carve<uint8_t>(base, off, ne);
    int32_t *hp_rec = carve<int32_t>(base, off, 4 * std::max<size_t>(H.hp_e.size(), 1));
    if (!D) return;
    D->hp_rec = hp_rec;
    D->poseA = pA;
    D->poseB = pB;
    D->pointA = qA;
    D->pointB = qB;
    D->err = err;
    D->Hll = Hll;
    D->bl = bl;
    D->ls_h = lrec ? 16 : 9;
    D->ls_b = lrec ? 16 : 3;
    D->ls_x = lrec ? 16 : 3;
    D->Hpl = Hpl;
    D->hp_Rt = hp_Rt;
    D->lmX = lmX;
    D->compact = compact ? 1 : 0;
    D->Hpp = Hpp;
    D->bp = bp;
    D->Dinv = Dinv;
    D->bs_part = bs_part;
    D->Hs = Hs;
    D->bs = bs;
    D->x = x;
    D->part = part;
    D->chunk_part = chunk_part;
    D->db = db;
    D->Linv = Linv;
    D->flag = flag;
    D->tstamp = ts;
    D->bad = bad;
    D->chi2o = chi2o;
}

int lba_batch(osg_ctx *ctx, const osg_ba_graph *graphs, osg_ba_result *results, int B, const volatile uint8_t *stop)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, B >= 0 && (B == 0 || (graphs && results)), "batch arguments");
    static const int prof_level = getenv("OSG_LBA_PROFILE") ? atoi(getenv("OSG_LBA_PROFILE")) : 0;
    const bool prof = prof_level > 0, prof_ts = prof_level >= 2 && B == 1;
    // OSG_SCHUR_VALU=1: the VALU Schur product (A/B measurements); default FP64 MFMA
    static const bool schur_valu = getenv("OSG_SCHUR_VALU") && atoi(getenv("OSG_SCHUR_VALU")) != 0;
    // OSG_SCHUR_STAGE=1: partner spans staged in LDS (k_schur_rows_st), bit-identical
    static const bool schur_stage = getenv("OSG_SCHUR_STAGE") && atoi(getenv("OSG_SCHUR_STAGE")) != 0;
    // OSG_SCHUR_DIRECT=1: Hpl_j operands loaded per lane from global memory (k_schur_rows<false, true>)
    static const bool schur_direct = getenv("OSG_SCHUR_DIRECT") && atoi(getenv("OSG_SCHUR_DIRECT")) != 0;
    // OSG_POSE_RED_GATHER=1: k_pose_red gathers its edge inputs through hp_e (A/B runs), bit-identical
    static const bool pose_red_gather = getenv("OSG_POSE_RED_GATHER") && atoi(getenv("OSG_POSE_RED_GATHER")) != 0;
    // OSG_UPDATE_STAGE=1: k_update reads Hpl through LDS pieces (A/B runs), bit-identical
    // OSG_SCHUR_POINT=1: Dinv and Dinv b_l from a kernel of their own (A/B runs), bit-identical
    static const bool schur_point = getenv("OSG_SCHUR_POINT") && atoi(getenv("OSG_SCHUR_POINT")) != 0;
    // OSG_LIN_WPE=4: k_linearize compiled for 4 waves per SIMD (A/B runs), bit-identical
    static const bool lin_wpe4 = getenv("OSG_LIN_WPE") && atoi(getenv("OSG_LIN_WPE")) == 4;
    static const bool update_stage = getenv("OSG_UPDATE_STAGE") && atoi(getenv("OSG_UPDATE_STAGE")) != 0;
    // k_update with one thread per Hpl block (the default since the end of r05: 150 -> 143 us per 64-window
    // step, profiles/r05_update_coop_ab.txt); OSG_UPDATE_COOP=0 restores the per-thread walks, bit-identical
    static const bool update_coop = !(getenv("OSG_UPDATE_COOP") && atoi(getenv("OSG_UPDATE_COOP")) == 0);
    // OSG_CHOL_DENSE=0: the per-column k_chol_col (+ k_chol_trail) launches for every system (A/B runs)
    // instead of the one-workgroup factorisations k_chol_dense and k_chol_env
    static const bool chol_dense = !(getenv("OSG_CHOL_DENSE") && atoi(getenv("OSG_CHOL_DENSE")) == 0);
    // OSG_CHOL_ENV=1: k_chol_env for narrow-envelope maps (A/B runs; measured slower than the column launches:
    // one workgroup serialises each column's trailing update, which k_chol_trail spreads over the chip)
    static const bool chol_env = getenv("OSG_CHOL_ENV") && atoi(getenv("OSG_CHOL_ENV")) == 1;
    // OSG_CHOL_DENSE_NT=512: k_chol_dense with 8 waves (256 VGPRs, a 3-step operand ring) instead of 16 (A/B)
    static const int chol_dense_nt = getenv("OSG_CHOL_DENSE_NT") ? atoi(getenv("OSG_CHOL_DENSE_NT")) : 1024;
    // the column launches' (and k_chol_env's) diagonal tiles eliminated four columns per barrier
    // (chol_factor_diag4: 7.3-8.0 against 9.0 us per tile, global_ba_map +6 %); OSG_CHOL_ELIM=2 for the
    // two-column form.  k_chol_dense keeps two: in its 1024-thread workgroup the four-column form spills
    // (20-26 us per tile, gpurun_out/elim4).
    static const int chol_elim = getenv("OSG_CHOL_ELIM") ? atoi(getenv("OSG_CHOL_ELIM")) : 4;
    // the compact per-block factor (k_linearize<.., true>, k_schur_rows_c, k_update_c) unless OSG_LBA_HPL=1
    // stores Hpl whole; the Hpl-reading A/B variants above run on the whole-Hpl form
    static const bool hpl_full = (getenv("OSG_LBA_HPL") && atoi(getenv("OSG_LBA_HPL")) == 1) || schur_valu ||
                                 schur_stage || schur_direct || update_stage || !update_coop;
    const bool compact = !hpl_full;
    // k_schur_rows_c with its gathers two groups ahead (the default since late r06: 6.40 against 6.47 ms per
    // 14 launches, gpurun_out/r06k); OSG_SCHUR_PF=1 one group ahead (A/B runs; the same sums)
    // OSG_SCHUR_PF=3: also the chunk descriptors four chunks ahead (A/B)
    static const int schur_pf = getenv("OSG_SCHUR_PF") ? std::min(4, std::max(1, atoi(getenv("OSG_SCHUR_PF")))) : 2;
    // OSG_SCHUR_WPE=5: k_schur_rows_c allocated for 5 waves per SIMD (92 VGPRs, no spills) instead of 6 (A/B)
    static const bool schur_wpe5 = getenv("OSG_SCHUR_WPE") && atoi(getenv("OSG_SCHUR_WPE")) == 5;
    // OSG_SCHUR_HOIST=1: k_schur_rows_c's first gathers issued inside the staging (A/B)
    static const bool schur_hoist = getenv("OSG_SCHUR_HOIST") && atoi(getenv("OSG_SCHUR_HOIST")) == 1;
    const auto tp0 = std::chrono::steady_clock::now();
    auto ms_since = [&](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    for (int b = 0; b < B; b++) {
        const int rc = check_graph(ctx, &graphs[b], &results[b]);
        if (rc < 0) return B > 1 ? osg_set_error(ctx, rc, "graph %d: %s", b, std::string(ctx->last_error).c_str()) : rc;
        osg_ba_result *R = &results[b];
        const osg_ba_graph *G = &graphs[b];
        R->iterations = 0;
        R->trials = 0;
        R->aborted = 0;
        R->chi2_initial = R->chi2_final = 0.0;
        std::memcpy(R->pose, G->pose, sizeof(double) * 7 * G->n_poses);
        std::memcpy(R->point, G->point, sizeof(double) * 3 * G->n_points);
        if (G->n_edges > 0) std::memset(R->edge_bad, 0, G->n_edges);
        if (R->edge_chi2)
            for (int e = 0; e < G->n_edges; e++) R->edge_chi2[e] = 0.0;
    }
    if (stop && *stop) {  // ref:src/Optimizer.cc:2112-2114
        for (int b = 0; b < B; b++) results[b].aborted = 1;
        return 0;
    }
    // ---- structures (host threads for a batch; each graph is independent)
    if (!ctx->lba_cache) ctx->lba_cache = std::make_shared<LbaCache>();
    LbaCache &cache = *static_cast<LbaCache *>(ctx->lba_cache.get());
    std::vector<LbaHost> &H = cache.H;
    if ((int)H.size() < B) H.resize(B);
    for (int b = 0; b < B; b++) H[b].reset();
    std::vector<int> rcs(B, OSG_OK);
    osg_parallel_for(B, 16, [&](int b) {
        H[b].G = &graphs[b];
        H[b].R = &results[b];
        if (graphs[b].n_edges == 0) {
            H[b].trivial = true;
            return;
        }
        rcs[b] = build_structure(ctx, &graphs[b], H[b]);
    });
    {
        for (int b = 0; b < B; b++)
            if (rcs[b] < 0)
                return B > 1 ? osg_set_error(ctx, rcs[b], "graph %d: structure", b) : rcs[b];
    }
    std::vector<int> act;  // graphs with something to optimise
    for (int b = 0; b < B; b++)
        if (!H[b].trivial) act.push_back(b);
    const int NA = (int)act.size();
    if (NA == 0) return 0;
    const double t_struct = ms_since(tp0);
    // ---- device layout: one packed input block, one state block, the LbaDev / control arrays
    osg_packer pk;
    struct InOff {
        size_t fixed, epose, epoint, ecam, ekind, eobs, eisig, cams, poseh, hppose, pointh, hlpoint, lmes, lme, lgs, lmbs,
            blkpose, eblk, hpes, hpe, hpb, pairb, chs, pch, pose0, point0, erob,
            prank, rscs, rsc, hprs, bfirst, blast, rsinfo, hpblm, rscd, crs, cr, live, envo;
    };
    std::vector<InOff> io(NA);
    for (int a = 0; a < NA; a++) {
        const LbaHost &h = H[act[a]];
        const osg_ba_graph *G = h.G;
        const int np = h.np, npt = h.npt, ne = h.ne, nhp = h.nhp, nhl = h.nhl, nblk = h.nblk;
        InOff &o = io[a];
        o.fixed = pk.add(G->pose_fixed, np);
        o.epose = pk.add(G->e_pose, 4 * (size_t)ne);
        o.epoint = pk.add(G->e_point, 4 * (size_t)ne);
        o.ecam = pk.add(G->e_cam, 4 * (size_t)ne);
        o.ekind = pk.add(G->e_kind, ne);
        o.eobs = pk.add(G->e_obs, 24 * (size_t)ne);
        o.eisig = pk.add(G->e_inv_sigma2, 4 * (size_t)ne);
        o.cams = pk.add(G->cams, sizeof(osg_camera) * G->n_cams);
        o.erob = G->e_robust ? pk.add(G->e_robust, ne) : SIZE_MAX;
        o.poseh = pk.add(h.pose_h.data(), 4 * (size_t)np);
        o.hppose = pk.add(h.hp_pose.data(), 4 * (size_t)nhp);
        o.pointh = pk.add(h.point_h.data(), 4 * (size_t)npt);
        o.hlpoint = pk.add(h.hl_point.data(), 4 * (size_t)nhl);
        o.lmes = pk.add(h.lm_e_start.data(), 4 * (size_t)(nhl + 1));
        o.lme = pk.add(h.lm_e.data(), 4 * (size_t)ne);
        o.lgs = pk.add(h.lg_lq.data(), 4 * h.lg_lq.size());
        o.lmbs = pk.add(h.lm_b_start.data(), 4 * (size_t)(nhl + 1));
        o.blkpose = pk.add(h.blk_pose.data(), 4 * (size_t)nblk);
        o.eblk = pk.add(h.edge_blk.data(), 4 * (size_t)ne);
        o.hpes = pk.add(h.hp_e_start.data(), 4 * (size_t)(nhp + 1));
        o.hpe = pk.add(h.hp_e.data(), 4 * h.hp_e.size());
        o.hpb = pk.add(h.hp_b.data(), 4 * (size_t)nblk);
        o.pairb = pk.add(h.pair_b.data(), 4 * h.pair_b.size());
        o.chs = pk.add(h.chunk_start.data(), 4 * h.chunk_start.size());
        // past CMAX only the live pairs' chunk ranges (the pair-indexed table is nhp^2 / 2 entries)
        o.pch = h.env_off.empty() ? pk.add(h.pair_chunk.data(), 4 * h.pair_chunk.size())
                                  : pk.add(h.live_chunk.data(), 4 * h.live_chunk.size());
        o.envo = h.env_off.empty() ? SIZE_MAX : pk.add(h.env_off.data(), 4 * h.env_off.size());
        o.prank = pk.add(h.pair_rank.data(), 4 * h.pair_rank.size());
        o.bfirst = pk.add(h.blk_first.data(), 4 * std::max<size_t>(h.blk_first.size(), 1));
        o.blast = pk.add(h.blk_last.data(), 4 * std::max<size_t>(h.blk_last.size(), 1));
        o.crs = h.col_rows_start.empty() ? SIZE_MAX : pk.add(h.col_rows_start.data(), 4 * h.col_rows_start.size());
        o.cr = h.col_rows_start.empty() ? SIZE_MAX : pk.add(h.col_rows.data(), 4 * h.col_rows.size());
        o.live = h.col_rows_start.empty() ? SIZE_MAX : pk.add(h.live_pairs.data(), 4 * std::max<size_t>(h.live_pairs.size(), 1));
        o.rsinfo = pk.add(h.rs_info.data(), 4 * h.rs_info.size());
        o.hpblm = pk.add(h.hp_b_lm.data(), 4 * h.hp_b_lm.size());
        o.rscs = pk.add(h.rs_chunk_start.data(), 4 * h.rs_chunk_start.size());
        o.rsc = pk.add(h.rs_chunk.data(), 4 * h.rs_chunk.size());
        o.rscd = pk.add(h.rs_cdesc.data(), 4 * h.rs_cdesc.size());
        o.hprs = pk.add(h.hp_rs_start.data(), 4 * h.hp_rs_start.size());
        o.pose0 = pk.add(G->pose, 56 * (size_t)np);
        o.point0 = pk.add(G->point, 24 * (size_t)npt);
    }
    // state sizes
    std::vector<size_t> st_off(NA + 1, 0);
    for (int a = 0; a < NA; a++) {
        size_t sz = 0;
        carve_state(nullptr, sz, H[act[a]], nullptr, prof_ts, compact);
        st_off[a + 1] = st_off[a] + ((sz + 255) & ~size_t(255)) + 256;
    }
    const size_t in_pad = (pk.total + 255) & ~size_t(255);
    const size_t dev_bytes = sizeof(LbaDev) * (size_t)NA;
    const size_t ctl_bytes = sizeof(LbaCtl) * (size_t)NA;
    const size_t out_bytes = sizeof(double) * 8 * (size_t)NA;
    char *pin = (char *)osg_pinned(ctx, in_pad + dev_bytes + ctl_bytes + out_bytes + 1024);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    pk.fill_parallel(pin, 16);
    LbaDev *h_dev = (LbaDev *)(pin + in_pad);
    LbaCtl *h_ctl = (LbaCtl *)((char *)h_dev + dev_bytes);
    double *h_out = (double *)((char *)h_ctl + ctl_bytes);
    char *din = nullptr, *dst = nullptr, *dsm = nullptr;
    OSG_ALLOC(ctx, din, SLOT_BA2, pk.total + 256);
    OSG_ALLOC(ctx, dst, SLOT_BA3, st_off[NA]);
    OSG_ALLOC(ctx, dsm, SLOT_BA4, dev_bytes + ctl_bytes + out_bytes + 256);
    LbaDev *d_dev = (LbaDev *)dsm;
    LbaCtl *d_ctl = (LbaCtl *)(dsm + dev_bytes);
    double *d_out = (double *)(dsm + dev_bytes + ctl_bytes);
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(din, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    int mx_gll = 1;
    bool any_multi = false;
    int mx_nhe = 0;
    size_t mx_init = 0;  // k_init_state's extent: the largest 7 np / 3 npt of the batch
    int mx_ge = 0, mx_gl = 1, mx_gu = 0, mx_nblk = 0, mx_nhp = 0, mx_chunks = 0, mx_pairs = 0, mx_red = 0, mx_rs = 0;
    // XCD-aware graph placement (LBA_GRAPH) for batches of >= 8 graphs: OSG_LBA_XCD=1.  Off by
    // default: measured slower (64 C4 windows: k_schur_rows 10.4 vs 8.9 ms, k_linearize 5.4 vs 4.4 ms
    // per 14-step batch; profiles/r02_lba_xcd.txt)
    static const bool xcd_env = getenv("OSG_LBA_XCD") && atoi(getenv("OSG_LBA_XCD")) == 1;
    const bool xcd = xcd_env && NA >= 8;
    bool large = false;  // some graph's reduced system is past CMAX
    bool any_dense = false;  // some graph is factored by k_chol_dense (n <= CMAX, at least one free pose)
    bool any_env = false;    // ... by k_chol_env (past CMAX, a narrow envelope)
    bool any_col = false;    // ... by column launches (the others)
    bool huge_col = false;   // ... and past CMAX_LARGE (k_back_step)
    for (int a = 0; a < NA; a++) {
        const LbaHost &h = H[act[a]];
        const InOff &o = io[a];
        LbaDev &D = h_dev[a];
        D = LbaDev{};
        D.np = h.np;
        D.npt = h.npt;
        D.ne = h.ne;
        D.nhp = h.nhp;
        D.nhl = h.nhl;
        D.nblk = h.nblk;
        D.npairs = h.npairs;
        D.n_cams = h.G->n_cams;
        D.n_graphs = NA;
        D.xcd_map = xcd ? 1 : 0;
        D.pose_fixed = osg_dptr<uint8_t>(din, o.fixed);
        D.e_pose = osg_dptr<int32_t>(din, o.epose);
        D.e_point = osg_dptr<int32_t>(din, o.epoint);
        D.e_cam = osg_dptr<int32_t>(din, o.ecam);
        D.e_kind = osg_dptr<int8_t>(din, o.ekind);
        D.e_obs = osg_dptr<double>(din, o.eobs);
        D.e_isig2 = osg_dptr<float>(din, o.eisig);
        D.cams = osg_dptr<osg_camera>(din, o.cams);
        D.e_robust = o.erob == SIZE_MAX ? nullptr : osg_dptr<uint8_t>(din, o.erob);
        D.hub_mono = h.G->huber_mono > 0.f ? h.G->huber_mono : (float)std::sqrt(5.991);   // thHuberMono
        D.hub_stereo = h.G->huber_stereo > 0.f ? h.G->huber_stereo : (float)std::sqrt(7.815);
        large |= 6 * h.nhp > CMAX;
        if (chol_dense && h.nhp > 0 && 6 * h.nhp <= CMAX) D.chol_fused = 1;
        else if (chol_env && 6 * h.nhp > CMAX && 6 * h.nhp <= ENV_NX && h.max_col_rows <= ENV_T - 1) D.chol_fused = 2;
        any_dense |= D.chol_fused == 1;
        any_env |= D.chol_fused == 2;
        any_col |= h.nhp > 0 && D.chol_fused == 0;
        huge_col |= 6 * h.nhp > CMAX_LARGE && D.chol_fused == 0;
        D.pose_h = osg_dptr<int32_t>(din, o.poseh);
        D.hp_pose = osg_dptr<int32_t>(din, o.hppose);
        D.point_h = osg_dptr<int32_t>(din, o.pointh);
        D.hl_point = osg_dptr<int32_t>(din, o.hlpoint);
        D.lm_e_start = osg_dptr<int32_t>(din, o.lmes);
        D.lm_e = osg_dptr<int32_t>(din, o.lme);
        D.lm_e_ident = h.lm_e_ident;
        D.lg_start = osg_dptr<int32_t>(din, o.lgs);
        D.lm_b_start = osg_dptr<int32_t>(din, o.lmbs);
        D.blk_pose = osg_dptr<int32_t>(din, o.blkpose);
        D.edge_blk = osg_dptr<int32_t>(din, o.eblk);
        D.hp_e_start = osg_dptr<int32_t>(din, o.hpes);
        D.hp_e = osg_dptr<int32_t>(din, o.hpe);
        D.nhe = (int)h.hp_e.size();
        D.hp_b = osg_dptr<int32_t>(din, o.hpb);
        D.pair_b = osg_dptr<int32_t>(din, o.pairb);
        D.nchunks = h.nchunks;
        D.chunk_start = osg_dptr<int32_t>(din, o.chs);
        D.pair_chunk = h.env_off.empty() ? osg_dptr<int32_t>(din, o.pch) : nullptr;
        D.live_chunk = h.env_off.empty() ? nullptr : osg_dptr<int32_t>(din, o.pch);
        D.env_off = o.envo == SIZE_MAX ? nullptr : osg_dptr<int32_t>(din, o.envo);
        D.pair_rank = osg_dptr<int32_t>(din, o.prank);
        D.blk_first = osg_dptr<int32_t>(din, o.bfirst);
        D.blk_last = osg_dptr<int32_t>(din, o.blast);
        D.col_rows_start = o.crs == SIZE_MAX ? nullptr : osg_dptr<int32_t>(din, o.crs);
        D.col_rows = o.cr == SIZE_MAX ? nullptr : osg_dptr<int32_t>(din, o.cr);
        D.live_pairs = o.live == SIZE_MAX ? nullptr : osg_dptr<int32_t>(din, o.live);
        D.n_live = (int)h.live_pairs.size();
        D.npart = h.npart;
        D.n_rs = h.n_rs;
        D.rs_info = osg_dptr<int32_t>(din, o.rsinfo);
        D.hp_b_lm = osg_dptr<int32_t>(din, o.hpblm);
        D.rs_chunk_start = osg_dptr<int32_t>(din, o.rscs);
        D.rs_cdesc = osg_dptr<int32_t>(din, o.rscd);
        D.rs_chunk = osg_dptr<int32_t>(din, o.rsc);
        D.hp_rs_start = osg_dptr<int32_t>(din, o.hprs);
        D.ge = h.ge;
        D.gl = h.gl;
        D.gll = h.gll;
        D.gu = h.gu;
        D.nblk_red = h.nblk_red;
        D.user_lambda = h.G->user_lambda_init;
        D.dinv_inline = schur_point ? 0 : 1;
        size_t off = 0;
        carve_state(dst + st_off[a], off, h, &D, prof_ts, compact);
        D.ctl = d_ctl + a;
        D.out = d_out + 8 * a;
        D.pose0 = osg_dptr<double>(din, o.pose0);
        D.point0 = osg_dptr<double>(din, o.point0);
        mx_init = std::max(mx_init, std::max(7 * (size_t)h.np, 3 * (size_t)h.npt));
        mx_ge = std::max(mx_ge, h.ge);
        mx_gl = std::max(mx_gl, h.gl);
        mx_gll = std::max(mx_gll, h.gll);
        any_multi |= h.multi;
        mx_gu = std::max(mx_gu, h.gu);
        mx_nblk = std::max(mx_nblk, h.nblk);
        mx_nhp = std::max(mx_nhp, h.nhp);
        mx_nhe = std::max(mx_nhe, (int)h.hp_e.size());
        mx_chunks = std::max(mx_chunks, h.nchunks);
        mx_rs = std::max(mx_rs, h.n_rs);
        mx_pairs = std::max(mx_pairs, h.col_rows_start.empty() ? h.npairs : (int)h.live_pairs.size());
        mx_red = std::max(mx_red, h.nblk_red);
    }
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(d_dev, h_dev, dev_bytes, hipMemcpyHostToDevice, ctx->stream));
    {
        const int gi = (int)std::max<size_t>((mx_init + EB - 1) / EB, 1);
        hipLaunchKernelGGL(k_init_state, xcd ? dim3(8 * gi, (NA + 7) / 8) : dim3(gi, NA), dim3(EB), 0, ctx->stream, d_dev);
    }
    if (mx_nhe > 0 && !pose_red_gather) {
        const dim3 g = xcd ? dim3(8 * ((mx_nhe + EB - 1) / EB), (NA + 7) / 8) : dim3((mx_nhe + EB - 1) / EB, NA);
        hipLaunchKernelGGL(k_hp_rec, g, dim3(EB), 0, ctx->stream, d_dev);
    }
    const double t_upload = ms_since(tp0) - t_struct;
    const auto tp1 = std::chrono::steady_clock::now();

    // osg_lba_kernel_times: an event before each launch group and one after the last; after the
    // step's sync, the time between two marks goes to the group that starts at the first
    int nmark = 0;
    auto mark = [&](int cls) -> int {
        if (!ctx->lba_ktime) return OSG_OK;
        if (nmark == (int)cache.kev.size()) {
            hipEvent_t e;
            OSG_HIP_CHECK(ctx, hipEventCreate(&e));
            cache.kev.push_back(e);
            cache.kcls.push_back(0);
        }
        OSG_HIP_CHECK(ctx, hipEventRecord(cache.kev[nmark], ctx->stream));
        cache.kcls[nmark++] = cls;
        return OSG_OK;
    };
    auto collect = [&]() -> int {  // after a stream sync
        for (int m = 0; m + 1 < nmark; m++) {
            float ms = 0.f;
            OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, cache.kev[m], cache.kev[m + 1]));
            ctx->lba_kms[cache.kcls[m]] += ms;
            ctx->lba_kn[cache.kcls[m]]++;
        }
        nmark = 0;
        return OSG_OK;
    };
#define LBA_MARK(cls)                  \
    do {                               \
        const int _rc = mark(cls);     \
        if (_rc < 0) return _rc;       \
    } while (0)

    // one lockstep step: every kernel once for all graphs, then 5 scalars per graph back
    auto run_step = [&]() -> int {
        // the per-step control through a copy kernel in the stream's own queue (osg_upload), not the
        // copy engine: the first kernel of the step then does not wait for an SDMA completion signal
        OSG_RC(osg_upload(ctx, d_ctl, h_ctl, ctl_bytes));
        const dim3 yb = xcd ? dim3(8, (NA + 7) / 8) : dim3(1, NA);
        auto gx = [&](int n) { return xcd ? dim3(8 * std::max(n, 1), (NA + 7) / 8) : dim3(std::max(n, 1), NA); };
        LBA_MARK(KT_ERR);
        hipLaunchKernelGGL(k_errors, gx(mx_ge), dim3(EB), 0, ctx->stream, d_dev, 1);
        LBA_MARK(KT_LIN);
        if (compact) {
            if (any_multi) hipLaunchKernelGGL((k_linearize<true, 1, true>), gx(mx_gll), dim3(EB), 0, ctx->stream, d_dev);
            else if (lin_wpe4) hipLaunchKernelGGL((k_linearize<false, 4, true>), gx(mx_gll), dim3(EB), 0, ctx->stream, d_dev);
            else hipLaunchKernelGGL((k_linearize<false, 1, true>), gx(mx_gll), dim3(EB), 0, ctx->stream, d_dev);
        } else if (any_multi) hipLaunchKernelGGL(k_linearize<true>, gx(mx_gll), dim3(EB), 0, ctx->stream, d_dev);
        else if (lin_wpe4) hipLaunchKernelGGL((k_linearize<false, 4>), gx(mx_gll), dim3(EB), 0, ctx->stream, d_dev);
        else hipLaunchKernelGGL(k_linearize<false>, gx(mx_gll), dim3(EB), 0, ctx->stream, d_dev);
        LBA_MARK(KT_POSE);
        if (mx_nhp > 0) {
            if (pose_red_gather) hipLaunchKernelGGL(k_pose_red<false>, gx(mx_nhp), dim3(EB), 0, ctx->stream, d_dev);
            else hipLaunchKernelGGL(k_pose_red<true>, gx(mx_nhp), dim3(EB), 0, ctx->stream, d_dev);
        }
        LBA_MARK(KT_LINIT);
        hipLaunchKernelGGL(k_lambda_init, yb, dim3(64), 0, ctx->stream, d_dev);
        LBA_MARK(KT_SPOINT);
        if (schur_point) hipLaunchKernelGGL(k_schur_point, gx(mx_gl), dim3(EB), 0, ctx->stream, d_dev);
        if (mx_nhp > 0) {
            LBA_MARK(KT_SROWS);
            if (compact) {
                auto sr = schur_pf == 4 ? k_schur_rows_c<4, 6>
                          : schur_pf == 3 ? (schur_wpe5 ? k_schur_rows_c<3, 5> : k_schur_rows_c<3, 6>)
                          : schur_pf == 2 ? (schur_wpe5 ? k_schur_rows_c<2, 5>
                                                        : (schur_hoist ? k_schur_rows_c<2, 6, true> : k_schur_rows_c<2, 6>))
                                          : k_schur_rows_c<1, 6>;
                hipLaunchKernelGGL(sr, gx(mx_rs), dim3(RT), 0, ctx->stream, d_dev);
            }
            else if (schur_valu) hipLaunchKernelGGL(k_schur_rows<true>, gx(mx_rs), dim3(RT), 0, ctx->stream, d_dev);
            else if (schur_stage) hipLaunchKernelGGL(k_schur_rows_st, gx(mx_rs), dim3(RT2), 0, ctx->stream, d_dev);
            else if (schur_direct)
                hipLaunchKernelGGL((k_schur_rows<false, true>), gx(mx_rs), dim3(RT), 0, ctx->stream, d_dev);
            else hipLaunchKernelGGL(k_schur_rows<false>, gx(mx_rs), dim3(RT), 0, ctx->stream, d_dev);
            LBA_MARK(KT_SPAIRS);
            hipLaunchKernelGGL(k_schur_pairs, gx((int)(((size_t)mx_pairs * 64 + 255) / 256)), dim3(256), 0, ctx->stream, d_dev);
            LBA_MARK(KT_CHOL);
            // dense systems (n <= CMAX) in one k_chol_dense workgroup per graph, narrow envelopes in one
            // k_chol_env workgroup (with its backward solve), the others by column launches
            if (any_dense) {
                if (chol_dense_nt == 512) hipLaunchKernelGGL((k_chol_dense<512, 3, 2>), yb, dim3(512), 0, ctx->stream, d_dev);
                else hipLaunchKernelGGL((k_chol_dense<1024, 2, 2>), yb, dim3(1024), 0, ctx->stream, d_dev);
            }
            if (any_env) {
                if (chol_elim == 4) hipLaunchKernelGGL(k_chol_env<4>, yb, dim3(CD_T), 0, ctx->stream, d_dev);
                else hipLaunchKernelGGL(k_chol_env<2>, yb, dim3(CD_T), 0, ctx->stream, d_dev);
            }
            const char *tp = getenv("OSG_TRAIL_PRE");  // tests pin the variant (read per call)
            const bool trail_pre = !(tp && atoi(tp) == 0);
            if (any_col) for (int jb = 0; jb < mx_red; jb++) {  // row blocks at and below the diagonal block
                // past CMAX only the envelope's rows: grids sized by the largest reach of any graph
                int rows = 0, m = 0;
                for (int a = 0; a < NA; a++) {
                    const LbaHost &h = H[act[a]];
                    if (jb >= h.nblk_red) continue;
                    const bool big = 6 * h.nhp > CMAX;
                    if (h_dev[a].chol_fused) continue;
                    const int nr = big ? h.col_rows_start[jb + 1] - h.col_rows_start[jb] : 0;
                    rows = std::max(rows, big ? 1 + nr : h.nblk_red - jb);
                    if (big) m = std::max(m, nr);
                }
                if (rows == 0) continue;
                if (chol_elim == 4) hipLaunchKernelGGL(k_chol_col<4>, gx(rows), dim3(256), 0, ctx->stream, d_dev, jb);
                else hipLaunchKernelGGL(k_chol_col<2>, gx(rows), dim3(256), 0, ctx->stream, d_dev, jb);
                if (large && m > 0) {
                    if (trail_pre)
                        hipLaunchKernelGGL(k_chol_trail<true>, gx(m * (m + 1) / 2), dim3(256), 0, ctx->stream, d_dev, jb);
                    else
                        hipLaunchKernelGGL(k_chol_trail<false>, gx(m * (m + 1) / 2), dim3(256), 0, ctx->stream, d_dev, jb);
                }
            }
            LBA_MARK(KT_BACK);
            hipLaunchKernelGGL(k_chol_back, yb, dim3(1024), 0, ctx->stream, d_dev);
            if (any_col) {
                const char *lp = getenv("OSG_BACKL_PRE");  // tests pin the variant (read per call)
                if (!(lp && atoi(lp) == 0)) hipLaunchKernelGGL(k_chol_back_large<true>, yb, dim3(1024), 0, ctx->stream, d_dev);
                else hipLaunchKernelGGL(k_chol_back_large<false>, yb, dim3(1024), 0, ctx->stream, d_dev);
            }
            if (huge_col) {
                const char *bp = getenv("OSG_BACK_PRE");  // tests pin the variant (read per call)
                const bool back_pre = !(bp && atoi(bp) == 0);
                for (int step = 0; step < mx_red; step++) {
                    int cols = 0;
                    for (int a = 0; a < NA; a++) {
                        const LbaHost &h = H[act[a]];
                        const int bi = h.nblk_red - 1 - step;
                        if (6 * h.nhp > CMAX_LARGE && bi >= 0) cols = std::max(cols, CB * (bi - h.blk_first[bi]));
                    }
                    if (back_pre)
                        hipLaunchKernelGGL(k_back_step<true>, gx(1 + (cols + BSC - 1) / BSC), dim3(BSC), 0, ctx->stream, d_dev, step);
                    else
                        hipLaunchKernelGGL(k_back_step<false>, gx(1 + (cols + BSC - 1) / BSC), dim3(BSC), 0, ctx->stream, d_dev, step);
                }
                hipLaunchKernelGGL(k_back_copy, gx((6 * mx_nhp + EB - 1) / EB), dim3(EB), 0, ctx->stream, d_dev);
            }
        }
        LBA_MARK(KT_UPD);
        if (compact) hipLaunchKernelGGL(k_update_c, gx(mx_gu), dim3(EB), 0, ctx->stream, d_dev);
        else if (update_stage) hipLaunchKernelGGL(k_update<true>, gx(mx_gu), dim3(EB), 0, ctx->stream, d_dev);
        else if (update_coop) hipLaunchKernelGGL((k_update<false, true>), gx(mx_gu), dim3(EB), 0, ctx->stream, d_dev);
        else hipLaunchKernelGGL(k_update<false>, gx(mx_gu), dim3(EB), 0, ctx->stream, d_dev);
        LBA_MARK(KT_ERR);
        hipLaunchKernelGGL(k_errors, gx(mx_ge), dim3(EB), 0, ctx->stream, d_dev, 0);
        LBA_MARK(KT_RED);
        hipLaunchKernelGGL(k_step_reduce, yb, dim3(256), 0, ctx->stream, d_dev);
        LBA_MARK(KT_END);
        OSG_HIP_CHECK(ctx, hipGetLastError());
        OSG_RC(osg_download(ctx, h_out, d_out, out_bytes));
        OSG_RC(osg_wait(ctx));
        return collect();
    };

    // initial chi2 (activeRobustChi2 before optimising): a step with only M_ERRC
    for (int a = 0; a < NA; a++) h_ctl[a] = LbaCtl{M_ERRC, 0, 0.0};
    {
        const int rc = run_step();
        if (rc < 0) return rc;
    }
    for (int a = 0; a < NA; a++) {
        LbaHost &h = H[act[a]];
        h.currentChi = h_out[8 * a + 4];
        h.R->chi2_initial = h.currentChi;
        h.errors_current = true;
    }
    int steps = 0;
    bool ts_printed = false;
    for (;;) {
        const bool stopped = stop && *stop;
        int n_run = 0;
        for (int a = 0; a < NA; a++) {
            LbaHost &h = H[act[a]];
            LbaCtl &c = h_ctl[a];
            c = LbaCtl{0, h.sel, h.lambda};
            if (h.done) continue;
            if (h.new_iter) {
                // sparse_optimizer.cpp optimize(): for (i < iterations && !terminate() && ok)
                if (h.it >= h.G->iterations || stopped) {
                    h.done = true;
                    continue;
                }
                c.mode = M_LIN | M_ACT | (h.errors_current ? 0 : M_ERRC) | (h.it == 0 ? M_INIT : 0);
            } else {
                c.mode = M_ACT;  // another trial (the loop condition was evaluated after the last one)
            }
            n_run++;
        }
        if (n_run == 0) break;
        {
            const int rc = run_step();
            if (rc < 0) return rc;
        }
        steps++;
#ifdef OSG_SR_PROF
        // profiling builds: graph 0's k_schur_rows_c timeline of the third step to $OSG_SR_PROF_OUT (raw u64)
        if (steps == 3 && getenv("OSG_SR_PROF_OUT")) {
            std::vector<unsigned long long> hp((size_t)SR_PROF_N * 13);
            OSG_HIP_CHECK(ctx, hipMemcpyFromSymbol(hp.data(), HIP_SYMBOL(g_sr_prof), hp.size() * sizeof(unsigned long long)));
            if (FILE *f = fopen(getenv("OSG_SR_PROF_OUT"), "wb")) {
                fwrite(hp.data(), sizeof(unsigned long long), hp.size(), f);
                fclose(f);
            }
        }
#endif
        if (prof_ts && !ts_printed && H[act[0]].nhp > 0) {
            ts_printed = true;
            const LbaDev &D0 = h_dev[0];
            const int nbr = H[act[0]].nblk_red;
            std::vector<unsigned long long> hts(8 * 2 * nbr);
            OSG_HIP_CHECK(ctx, hipMemcpy(hts.data(), D0.tstamp, sizeof(unsigned long long) * hts.size(), hipMemcpyDeviceToHost));
            std::vector<unsigned long long> hb(64);
            OSG_HIP_CHECK(ctx, hipMemcpy(hb.data(), D0.tstamp + 8 * 2 * 32, sizeof(unsigned long long) * 64, hipMemcpyDeviceToHost));
            fprintf(stderr, "[osg back] staging %.2f us;", (hb[41] - hb[0]) * 0.01);
            for (int bb = nbr - 1; bb >= 0; bb--) fprintf(stderr, " b%d@%.2f", bb, (hb[1 + bb] - hb[0]) * 0.01);
            fprintf(stderr, " end@%.2f\n", (hb[40] - hb[0]) * 0.01);
            for (int jb = 0; jb < nbr; jb++)
                for (int tt = 0; tt < 2 && tt < nbr - jb; tt++) {
                    const unsigned long long *q = &hts[8 * (2 * jb + tt)];
                    fprintf(stderr, "[osg chol] j=%d wg=%d gemm %.2f factor+inverse %.2f tail %.2f us\n", jb, tt,
                            (q[1] - q[0]) * 0.01, (q[2] - q[1]) * 0.01, (q[3] - q[2]) * 0.01);
                }
        }
        // optimization_algorithm_levenberg.cpp:61-176, per graph
        for (int a = 0; a < NA; a++) {
            LbaHost &h = H[act[a]];
            const int mode = h_ctl[a].mode;
            if (!(mode & M_ACT)) continue;
            const double *o = h_out + 8 * a;
            if (mode & M_ERRC) h.currentChi = o[4];
            if (h.new_iter) {
                h.iniChi = h.currentChi;
                if (mode & M_INIT) {
                    h.lambda = o[3];
                    h.ni = 2;
                    h.nBad = 0;
                }
                h.qmax = 0;
                h.new_iter = false;
            }
            h.trials++;
            double tempChi = o[0];
            if (o[2] == 0.0) tempChi = DBL_MAX;
            double rho = h.currentChi - tempChi;
            const double scale = o[1] + 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - osgx::cube_rn(2 * rho - 1);  // pow(., 3), correctly rounded
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                h.lambda *= scaleFactor;
                h.ni = 2;
                h.currentChi = tempChi;
                h.sel ^= 1;  // the trial estimate becomes current
                h.errors_current = true;
            } else {
                h.lambda *= h.ni;
                h.ni *= 2;
                h.errors_current = false;  // err[] holds the rejected estimate's errors
            }
            h.rho = rho;
            h.qmax++;
            const bool again = rho < 0 && h.qmax < 10 && !(stop && *stop);
            if (again) continue;
            // iteration done
            h.iters++;
            h.it++;
            h.new_iter = true;
            if (h.qmax == 10 || rho == 0) {
                h.done = true;
            } else {
                if ((h.iniChi - h.currentChi) * 1e3 < h.iniChi) h.nBad++;
                else h.nBad = 0;
                if (h.nBad >= 3) h.done = true;
            }
        }
    }
    const double t_lm = ms_since(tp1);
    const auto tp2 = std::chrono::steady_clock::now();
    // classification with the last computed errors (current estimate's, or the rejected trial's,
    // exactly as the reference's computeActiveErrors order leaves them); estimates out
    for (int a = 0; a < NA; a++) h_ctl[a] = LbaCtl{M_FIN, H[act[a]].sel, 0.0};
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(d_ctl, h_ctl, ctl_bytes, hipMemcpyHostToDevice, ctx->stream));
    LBA_MARK(KT_CLASS);
    hipLaunchKernelGGL(k_classify, xcd ? dim3(8 * std::max(mx_ge, 1), (NA + 7) / 8) : dim3(std::max(mx_ge, 1), NA),
                       dim3(EB), 0, ctx->stream, d_dev);
    LBA_MARK(KT_END);
#undef LBA_MARK
    OSG_HIP_CHECK(ctx, hipGetLastError());
    int total_iters = 0;
    for (int a = 0; a < NA; a++) {
        LbaHost &h = H[act[a]];
        const LbaDev &D = h_dev[a];
        osg_ba_result *R = h.R;
        R->iterations = h.iters;
        R->trials = h.trials;
        R->aborted = (stop && *stop) ? 1 : 0;
        R->chi2_final = h.currentChi;
        total_iters += h.iters;
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(R->pose, h.sel ? D.poseB : D.poseA, 56 * (size_t)h.np, hipMemcpyDeviceToHost,
                                          ctx->stream));
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(R->point, h.sel ? D.pointB : D.pointA, 24 * (size_t)h.npt,
                                          hipMemcpyDeviceToHost, ctx->stream));
        OSG_HIP_CHECK(ctx, hipMemcpyAsync(R->edge_bad, D.bad, h.ne, hipMemcpyDeviceToHost, ctx->stream));
        if (R->edge_chi2 && h.ne > 0)
            OSG_HIP_CHECK(ctx, hipMemcpyAsync(R->edge_chi2, D.chi2o, 8 * (size_t)h.ne, hipMemcpyDeviceToHost, ctx->stream));
    }
    OSG_RC(osg_wait(ctx));
    {
        const int rc = collect();
        if (rc < 0) return rc;
    }
    if (prof)
        fprintf(stderr, "[osg lba] %d graphs: structure %.3f ms (graph 0: %.3f ms), pack+upload %.3f ms, LM %.3f ms "
                        "(%d lockstep steps), classify+download %.3f ms, total %.3f ms\n",
                NA, t_struct, H[act[0]].t_struct, t_upload, t_lm, steps, ms_since(tp2), ms_since(tp0));
    return B == 1 ? results[0].iterations : total_iters;
}

}  // namespace

extern "C" int osg_local_bundle_adjustment(osg_ctx *ctx, const osg_ba_graph *G, osg_ba_result *R,
                                           const volatile uint8_t *stop)
{
    return lba_batch(ctx, G, R, 1, stop);
}

extern "C" int osg_bundle_adjustment(osg_ctx *ctx, const osg_ba_graph *G, osg_ba_result *R, const volatile uint8_t *stop)
{  // Optimizer::BundleAdjustment: the same LM over the whole map (the caller's Huber fields)
    return lba_batch(ctx, G, R, 1, stop);
}

extern "C" int osg_lba_kernel_times(osg_ctx *ctx, int32_t enable, double *ms, int64_t *steps)
{
    if (!ctx) return OSG_E_INVALID;
    for (int k = 0; k < OSG_LBA_NK; k++) {
        if (ms) ms[k] = ctx->lba_kms[k];
        if (steps) steps[k] = ctx->lba_kn[k];
    }
    if (enable && !ctx->lba_ktime)
        for (int k = 0; k < OSG_LBA_NK; k++) {
            ctx->lba_kms[k] = 0;
            ctx->lba_kn[k] = 0;
        }
    ctx->lba_ktime = enable != 0;
    return OSG_OK;
}

extern "C" int osg_local_bundle_adjustment_batch(osg_ctx *ctx, const osg_ba_graph *graphs, int32_t n_graphs,
                                                 osg_ba_result *results, const volatile uint8_t *stop)
{
    return lba_batch(ctx, graphs, results, n_graphs, stop);
}
