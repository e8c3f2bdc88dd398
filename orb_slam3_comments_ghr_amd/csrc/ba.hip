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
// Per LM iteration (device):
//   k_errors      per edge: error, Huber rho -> per-workgroup chi2 partials        (HBM/latency)
//   k_linearize   per edge: Jacobians -> the edge's Hpp/b_p/Hll/b_l/Hpl terms      (FP64 VALU)
//   k_point_red   per point: sums Hll, b_l and its Hpl blocks                      (segmented, no atomics)
//   k_pose_red    per pose: Hpp, b_p from its edges (workgroup reduction)
// Per LM trial (lambda known on the host):
//   k_schur_point per point: Dinv = (Hll + lambda I)^-1, BDinv = Hpl Dinv, coef = Hpl Dinv b_l
//   k_schur_pairs per pose pair (i <= j), one wave: S_ij = sum_p BDinv_ip Hpl_jp^T ; writes the
//                 dense reduced camera matrix Hpp + lambda I - S and b_schur
//   k_chol_*      blocked Cholesky of the reduced system (n = 6 x free poses): panel kernel,
//                 FP64-MFMA trailing SYRK, blocked triangular solves
//   k_update      per point: x_l = Dinv (b_l - Hpl^T x_p), new estimates (poses: exp(x) * T)
//                 and the LM scale sum;  then k_errors on the new estimates -> tempChi
// The host reads back 3 scalars per trial and runs the accept / reject / lambda logic exactly as
// the reference; push/pop is a swap of the current / trial estimate buffers.
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <vector>

#include "ba_common.h"
#include "match_common.h"

using namespace osgba;

namespace {

constexpr int EB = 256;      // edge-parallel kernels
constexpr int NPART = 1024;  // max chi2 / scale partials

struct LbaDev {
    // sizes
    int np, npt, ne, nhp, nhl, nblk, npairs, n_cams;
    // inputs
    const uint8_t *pose_fixed;
    const int32_t *e_pose, *e_point, *e_cam;
    const int8_t *e_kind;
    const double *e_obs;
    const float *e_isig2;
    const osg_camera *cams;
    // structure
    const int32_t *pose_h;        // per pose: hessian index or -1
    const int32_t *hp_pose;       // per hessian pose: pose index
    const int32_t *point_h;       // per point: landmark index or -1
    const int32_t *hl_point;      // per landmark: point index
    const int32_t *lm_e_start, *lm_e;    // edges per landmark
    const int32_t *lm_b_start;           // blocks per landmark (blocks are numbered landmark-major)
    const int32_t *blk_pose;             // per block: hessian pose index
    const int32_t *edge_blk;             // per edge: block or -1
    const int32_t *blk_lm;               // per block: landmark
    const int32_t *blk_e_start, *blk_e;  // edges per block (edge order)
    const int32_t *hp_e_start, *hp_e;    // edges per hessian pose
    const int32_t *hp_b_start, *hp_b;    // blocks per hessian pose
    const int32_t *pair_start;           // dense (i <= j) pairs
    const int32_t *pair_ab;              // 2 ints per contribution
    int nchunks;
    const int32_t *chunk_start;          // contribution range of each chunk (chunks never span pairs)
    const int32_t *pair_chunk;           // per pair: first chunk (npairs + 1)
    double *chunk_part;                  // 36 per chunk
    // state
    const double *pose_cur, *point_cur;
    double *pose_new, *point_new;
    double *err;                         // 3 per edge
    double *J;                           // EC per edge: quadratic-form contributions
    double *Hll, *bl, *Hpl, *Hpp, *bp;
    double *Dinv, *db, *BDinv, *coef;
    double *Hs, *bs, *x;
    double *Lkk;                         // factored 32x32 diagonal blocks, row-major per block row
    double *part;                        // [0..NPART): chi partials, [NPART..2NPART): scale, [2NPART..]: max diag
    int *flag;                           // [0] cholesky ok
};

__device__ inline double edge_w(const LbaDev &D, int e) { return (double)D.e_isig2[e]; }

__device__ inline void kind_delta(int kind, double &delta, float &dsqr)
{
    const float dm = (float)sqrt(5.991), ds = (float)sqrt(7.815);
    const float d = (kind == OSG_EDGE_STEREO) ? ds : dm;
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
__global__ __launch_bounds__(EB) void k_errors(LbaDev D, const double *__restrict__ poses,
                                               const double *__restrict__ points, int part_off)
{
    __shared__ double s[EB / 64];
    const int e = blockIdx.x * EB + threadIdx.x;
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
        kind_delta(k, delta, dsqr);
        huber(c, delta, dsqr, rho0, r1);
    }
    const double t = block_sum_d(rho0, s);
    if (threadIdx.x == 0) D.part[part_off + blockIdx.x] = t;
}

// per edge: Jacobians and the edge's quadratic-form contributions (ref:Thirdparty/g2o/g2o/core/
// base_binary_edge.hpp:55-120, robust branch): C[e] = {Hpp 21 (upper), b_p 6, Hll 6 (upper),
// b_l 3, Hpl 18 (6x3)} = 54 doubles; the reductions below only sum them.
constexpr int EC = 54;
__global__ __launch_bounds__(EB) void k_linearize(LbaDev D)
{
    const int e = blockIdx.x * EB + threadIdx.x;
    if (e >= D.ne) return;
    const int k = D.e_kind[e];
    const SE3 T = se3_from7(D.pose_cur + 7 * (size_t)D.e_pose[e]);
    const double *X = D.point_cur + 3 * (size_t)D.e_point[e];
    double Jp[3][6], Jx[3][3];
    edge_jacobians(k, true, D.cams[D.e_cam[e]], T, X, Jp, Jx);
    const int dim = (k == OSG_EDGE_STEREO) ? 3 : 2;
    const double w = edge_w(D, e);
    const double ev[3] = {D.err[3 * e], D.err[3 * e + 1], D.err[3 * e + 2]};
    double delta, r0, rho1;
    float dsqr;
    kind_delta(k, delta, dsqr);
    huber(chi2_of(ev, dim, w), delta, dsqr, r0, rho1);
    const double ww = rho1 * w;
    double om[3];
    for (int d = 0; d < 3; d++) om[d] = (d < dim) ? -(w * ev[d]) * rho1 : 0.0;
    if (dim == 2) {
        for (int j = 0; j < 6; j++) Jp[2][j] = 0.0;
        for (int j = 0; j < 3; j++) Jx[2][j] = 0.0;
    }
    double *o = D.J + EC * (size_t)e;
    int c = 0;
    for (int a = 0; a < 6; a++)
        for (int bb = a; bb < 6; bb++)
            o[c++] = Jp[0][a] * ww * Jp[0][bb] + Jp[1][a] * ww * Jp[1][bb] + Jp[2][a] * ww * Jp[2][bb];
    for (int a = 0; a < 6; a++) o[c++] = Jp[0][a] * om[0] + Jp[1][a] * om[1] + Jp[2][a] * om[2];
    for (int a = 0; a < 3; a++)
        for (int bb = a; bb < 3; bb++)
            o[c++] = Jx[0][a] * ww * Jx[0][bb] + Jx[1][a] * ww * Jx[1][bb] + Jx[2][a] * ww * Jx[2][bb];
    for (int a = 0; a < 3; a++) o[c++] = Jx[0][a] * om[0] + Jx[1][a] * om[1] + Jx[2][a] * om[2];
    for (int a = 0; a < 6; a++)
        for (int bb = 0; bb < 3; bb++)
            o[c++] = Jp[0][a] * ww * Jx[0][bb] + Jp[1][a] * ww * Jx[1][bb] + Jp[2][a] * ww * Jx[2][bb];
}

// per block: Hpl = sum of its edges' contributions (usually one edge; mono + body of one
// keyframe share a block)
__global__ __launch_bounds__(EB) void k_block_red(LbaDev D)
{
    const int blk = blockIdx.x * EB + threadIdx.x;
    if (blk >= D.nblk) return;
    double h[18];
    for (int i = 0; i < 18; i++) h[i] = 0.0;
    for (int q = D.blk_e_start[blk]; q < D.blk_e_start[blk + 1]; q++) {
        const double *C = D.J + EC * (size_t)D.blk_e[q];
        for (int i = 0; i < 18; i++) h[i] += C[36 + i];
    }
    for (int i = 0; i < 18; i++) D.Hpl[18 * (size_t)blk + i] = h[i];
}

// per landmark: Hll (3x3) and b_l (sums of edge contributions)
__global__ __launch_bounds__(EB) void k_point_red(LbaDev D)
{
    __shared__ double s[EB / 64];
    const int l = blockIdx.x * EB + threadIdx.x;
    double md = 0.0;
    if (l < D.nhl) {
        double H6[6] = {0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
        for (int q = D.lm_e_start[l]; q < D.lm_e_start[l + 1]; q++) {
            const int e = D.lm_e[q];
            const double *C = D.J + EC * (size_t)e;
            for (int i = 0; i < 6; i++) H6[i] += C[27 + i];
            for (int i = 0; i < 3; i++) b[i] += C[33 + i];
        }
        const double H[9] = {H6[0], H6[1], H6[2], H6[1], H6[3], H6[4], H6[2], H6[4], H6[5]};
        for (int i = 0; i < 9; i++) D.Hll[9 * (size_t)l + i] = H[i];
        for (int i = 0; i < 3; i++) D.bl[3 * (size_t)l + i] = b[i];
        md = fmax(fabs(H[0]), fmax(fabs(H[4]), fabs(H[8])));
    }
    // max |diag| per workgroup for computeLambdaInit
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int off = 32; off >= 1; off >>= 1) md = fmax(md, __shfl_xor(md, off));
    if (lane == 0) s[w] = md;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = 0;
        for (int i = 0; i < EB / 64; i++) m = fmax(m, s[i]);
        D.part[2 * NPART + blockIdx.x] = m;
    }
}

// per free pose (one workgroup): Hpp (6x6) and b_p from its edges
__global__ __launch_bounds__(EB) void k_pose_red(LbaDev D, int diag_off)
{
    __shared__ double s[EB / 64][27];
    const int i = blockIdx.x;
    double acc[27];
    for (int k = 0; k < 27; k++) acc[k] = 0.0;
    for (int q = D.hp_e_start[i] + threadIdx.x; q < D.hp_e_start[i + 1]; q += EB) {
        const int e = D.hp_e[q];
        const double *C = D.J + EC * (size_t)e;
        for (int k = 0; k < 27; k++) acc[k] += C[k];
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

__global__ __launch_bounds__(EB) void k_schur_point(LbaDev D, double lambda)
{
    const int l = blockIdx.x * EB + threadIdx.x;
    if (l >= D.nhl) return;
    double Dm[9];
    for (int i = 0; i < 9; i++) Dm[i] = D.Hll[9 * (size_t)l + i];
    Dm[0] += lambda;
    Dm[4] += lambda;
    Dm[8] += lambda;
    double Di[9];
    inv3(Dm, Di);
    for (int i = 0; i < 9; i++) D.Dinv[9 * (size_t)l + i] = Di[i];
    const double *b = D.bl + 3 * (size_t)l;
    for (int r = 0; r < 3; r++) D.db[3 * (size_t)l + r] = Di[3 * r] * b[0] + Di[3 * r + 1] * b[1] + Di[3 * r + 2] * b[2];
}

// per block: BDinv = Hpl Dinv, coef = Hpl Dinv b_l
__global__ __launch_bounds__(EB) void k_schur_block(LbaDev D)
{
    const int blk = blockIdx.x * EB + threadIdx.x;
    if (blk >= D.nblk) return;
    const int l = D.blk_lm[blk];
    double Di[9], db[3], B[18];
    for (int i = 0; i < 9; i++) Di[i] = D.Dinv[9 * (size_t)l + i];
    for (int i = 0; i < 3; i++) db[i] = D.db[3 * (size_t)l + i];
    for (int i = 0; i < 18; i++) B[i] = D.Hpl[18 * (size_t)blk + i];
    double *BD = D.BDinv + 18 * (size_t)blk;
    double *cf = D.coef + 6 * (size_t)blk;
    for (int r = 0; r < 6; r++) {
        for (int c = 0; c < 3; c++) BD[3 * r + c] = B[3 * r] * Di[c] + B[3 * r + 1] * Di[3 + c] + B[3 * r + 2] * Di[6 + c];
        cf[r] = B[3 * r] * db[0] + B[3 * r + 1] * db[1] + B[3 * r + 2] * db[2];
    }
}

// Schur accumulation S_ij = sum_p BDinv_ip Hpl_jp^T over the (block_i, block_j) contributions of
// every pose pair (i <= j), in landmark order — the order of g2o's Schur loop
// (ref:Thirdparty/g2o/g2o/core/block_solver.hpp:381-432).  Diagonal pairs carry ~10x the
// contributions of off-diagonal ones, so the lists are cut into chunks of <= SCH contributions:
//   k_schur_chunks  one wave per chunk, lane (r, c) < 36 owns S[r][c] (no cross-lane reduction),
//                   8 contributions' loads in flight per step -> chunk partial;
//   k_schur_pairs   one wave per pair: sums its chunk partials in chunk order (deterministic),
//                   writes Hs = Hpp + lambda I - S (both triangles) and b_schur.
constexpr int SCH = 32;
__global__ __launch_bounds__(256) void k_schur_chunks(LbaDev D)
{
    const int ch = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (ch >= D.nchunks) return;
    const int r = (lane < 36) ? lane / 6 : 0, c = (lane < 36) ? lane % 6 : 0;
    const double *__restrict__ BDv = D.BDinv;
    const double *__restrict__ Hv = D.Hpl;
    const int *__restrict__ ab = D.pair_ab;
    const int q0 = D.chunk_start[ch], q1 = D.chunk_start[ch + 1];
    double acc = 0.0;
    int q = q0;
    for (; q + 7 < q1; q += 8) {
        int a[8], b[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            a[u] = ab[2 * (q + u)];
            b[u] = ab[2 * (q + u) + 1];
        }
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const double *BD = BDv + 18 * (size_t)a[u] + 3 * r;
            const double *Bj = Hv + 18 * (size_t)b[u] + 3 * c;
            t[u] = BD[0] * Bj[0] + BD[1] * Bj[1] + BD[2] * Bj[2];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) acc += t[u];
    }
    for (; q < q1; q++) {
        const int a = ab[2 * q], b = ab[2 * q + 1];
        const double *BD = BDv + 18 * (size_t)a + 3 * r;
        const double *Bj = Hv + 18 * (size_t)b + 3 * c;
        acc += BD[0] * Bj[0] + BD[1] * Bj[1] + BD[2] * Bj[2];
    }
    if (lane < 36) D.chunk_part[36 * (size_t)ch + lane] = acc;
}

__global__ __launch_bounds__(256) void k_schur_pairs(LbaDev D, double lambda)
{
    const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wave >= D.npairs) return;
    int i = 0, rem = wave;
    while (rem >= D.nhp - i) {
        rem -= D.nhp - i;
        i++;
    }
    const int j = i + rem;
    if (wave == 0 && lane == 0) D.flag[0] = 1;  // the Cholesky of this trial clears it on failure
    const int n = 6 * D.nhp;
    if (lane < 36) {
        const int r = lane / 6, c = lane % 6;
        double acc = 0.0;
        for (int ch = D.pair_chunk[wave]; ch < D.pair_chunk[wave + 1]; ch++) acc += D.chunk_part[36 * (size_t)ch + lane];
        double v = -acc;
        if (i == j) {
            v += D.Hpp[36 * (size_t)i + lane];
            if (r == c) v += lambda;
        }
        D.Hs[(size_t)(6 * i + r) * n + 6 * j + c] = v;
        if (i != j) D.Hs[(size_t)(6 * j + c) * n + 6 * i + r] = v;
    }
}

// b_schur_i = b_p,i - sum over pose i's blocks of Hpl Dinv b_l: one workgroup per pose
__global__ __launch_bounds__(256) void k_bschur(LbaDev D)
{
    __shared__ double s[4][6];
    const int i = blockIdx.x;
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int q = D.hp_b_start[i] + threadIdx.x; q < D.hp_b_start[i + 1]; q += 256) {
        const double *cf = D.coef + 6 * (size_t)D.hp_b[q];
        for (int k = 0; k < 6; k++) acc[k] += cf[k];
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int k = 0; k < 6; k++) acc[k] = wave_sum(acc[k]);
    if (lane == 0)
        for (int k = 0; k < 6; k++) s[w][k] = acc[k];
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        D.bs[6 * i + k] = D.bp[6 * (size_t)i + k] - (((s[0][k] + s[1][k]) + s[2][k]) + s[3][k]);
    }
}

__device__ inline double readlane_d(double v, int lane)
{  // wave-uniform lane index: two v_readlane_b32 instead of a ds_bpermute round trip
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// ---------------------------------------------------------------------------------------------
// Reduced camera system: blocked right-looking Cholesky (LL^T, lower, in place in Hs) over
// panels of CB = 32 columns with the forward substitution fused, then a blocked backward solve.
// Per panel:
//   k_chol_panel  one wave per 32-row block: diagonal block factored in registers (readlane),
//                 rows below solved against it, b updated;
//   k_chol_syrk   trailing update A22 -= L21 L21^T on 32x32 lower tiles, one workgroup per tile,
//                 one wave per 16x16 quadrant on FP64 MFMA (v_mfma_f64_16x16x4_f64, K = 32 as
//                 8 MFMAs) — the only MFMA use on the path (the dense Schur GEMM).
// The factorisation reports failure on a non-positive pivot (g2o's solvers then reject the step).
constexpr int CB = 32;
constexpr int CMAX = 384;  // max reduced dimension (64 free poses)
typedef double d4 __attribute__((ext_vector_type(4)));

// Panel step k0, one 64-thread workgroup per 32-row block at or below the diagonal block.  Every
// workgroup factors the 32x32 diagonal block itself (lane = row, registers, v_readlane
// broadcasts, no barriers) and solves y_k = L_kk^-1 b_k; workgroup 0 stores L_kk and y_k,
// workgroup t > 0 turns its 32 rows into L21 rows (x L_kk^T = a) and updates b for them
// (b_row -= L_row . y_k).  Workgroup 0 writes L_kk to Lkk and y_k to x (forward substitution fused).
__global__ __launch_bounds__(64) void k_chol_panel(LbaDev D, int k0)
{
    const int n = 6 * D.nhp;
    double *A = D.Hs;
    double *bs = D.bs;
    const int nb = min(CB, n - k0);
    const int r = threadIdx.x;  // lane
    double a[CB];
#pragma unroll
    for (int c = 0; c < CB; c++) a[c] = (r < nb && c < nb && c <= r) ? A[(size_t)(k0 + r) * n + k0 + c] : 0.0;
    double yv = (r < nb) ? bs[k0 + r] : 0.0;
    int ok = 1;
#pragma unroll
    for (int c = 0; c < CB; c++) {
        if (c < nb) {
            const double d = readlane_d(a[c], c);
            ok &= d > 0.0;
            const double piv = sqrt(fmax(d, 1e-300));
            if (r == c) a[c] = piv;
            else if (r > c) a[c] /= piv;
            const double lrc = a[c];
#pragma unroll
            for (int cc = c + 1; cc < CB; cc++) {
                const double lcc = readlane_d(a[c], cc);  // L[cc][c]
                if (cc < nb && r >= cc) a[cc] -= lrc * lcc;
            }
            // forward substitution of b inside the block
            const double yc = readlane_d(yv, c) / piv;
            if (r == c) yv = yc;
            else if (r > c && r < nb) yv -= lrc * yc;
        }
    }
    if (blockIdx.x == 0) {
        if (r == 0 && !ok) D.flag[0] = 0;
        // the diagonal block of Hs and b_k stay untouched: the other workgroups of this launch read them
        if (r < nb) {
#pragma unroll
            for (int c = 0; c < CB; c++) D.Lkk[(size_t)(k0 + r) * CB + c] = a[c];
            D.x[k0 + r] = yv;
        }
        return;
    }
    // rows of block t: x L_kk^T = a_row  ->  x_c = (a_c - sum_{k<c} x_k L[c][k]) / L[c][c]
    const int row = k0 + blockIdx.x * CB + r;
    const bool has = r < CB && row < n;
    double x[CB];
#pragma unroll
    for (int c = 0; c < CB; c++) x[c] = (has && c < nb) ? A[(size_t)row * n + k0 + c] : 0.0;
#pragma unroll
    for (int c = 0; c < CB; c++) {
        if (c < nb) {
            double v = x[c];
#pragma unroll
            for (int k = 0; k < c; k++) v -= x[k] * readlane_d(a[k], c);  // L[c][k] lives in lane c
            x[c] = v / readlane_d(a[c], c);
        }
    }
    double dot = 0.0;
#pragma unroll
    for (int c = 0; c < CB; c++)
        if (c < nb) dot += x[c] * readlane_d(yv, c);
    if (has) {
#pragma unroll
        for (int c = 0; c < CB; c++)
            if (c < nb) A[(size_t)row * n + k0 + c] = x[c];
        bs[row] -= dot;
    }
}

// tile (ti, tj), ti >= tj, of the trailing matrix starting at t0 = k0 + CB
__global__ __launch_bounds__(256) void k_chol_syrk(LbaDev D, int k0)
{
    const int n = 6 * D.nhp;
    double *A = D.Hs;
    const int t0 = k0 + CB;
    // decode lower-triangular tile index
    int ti = 0, rem = blockIdx.x;
    while (rem > ti) {
        rem -= ti + 1;
        ti++;
    }
    const int tj = rem;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int R0 = t0 + ti * CB + (w >> 1) * 16;  // quadrant rows
    const int C0 = t0 + tj * CB + (w & 1) * 16;   // quadrant cols
    if (R0 >= n || C0 >= n) return;
    if (ti == tj && (w & 1) > (w >> 1)) return;   // strictly upper quadrant of a diagonal tile
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    const int ra = R0 + (l & 15), cb = C0 + (l & 15);
#pragma unroll
    for (int ks = 0; ks < CB / 4; ks++) {
        const int kk = k0 + ks * 4 + (l >> 4);
        const double a = (ra < n) ? A[(size_t)ra * n + kk] : 0.0;  // L[R0+i][k]
        const double b = (cb < n) ? A[(size_t)cb * n + kk] : 0.0;  // L[C0+j][k] (= B[k][j])
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    const int col = C0 + (l & 15);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int row = R0 + (l >> 4) + 4 * q;
        if (row < n && col < n && col <= row) A[(size_t)row * n + col] -= acc[q];
    }
}

// Backward substitution L^T x = y (y in x after the fused forward pass), one 1024-thread
// workgroup, blocked by 32: for block k (last to first) the right-hand side
// y_k - sum_{rows below} L[row][k-block]^T x_row is reduced by all threads (LDS), then one wave
// solves the 32x32 upper-triangular block with readlane broadcasts.
__global__ __launch_bounds__(1024) void k_chol_back(LbaDev D)
{
    __shared__ double s_x[CMAX];
    __shared__ double s_part[32][33];
    const int n = 6 * D.nhp;
    const double *A = D.Hs;
    const int tid = threadIdx.x;
    for (int i = tid; i < n; i += 1024) s_x[i] = 0.0;
    __syncthreads();
    const int nblk = (n + CB - 1) / CB;
    for (int bi = nblk - 1; bi >= 0; bi--) {
        const int k0 = bi * CB;
        const int nb = min(CB, n - k0);
        {
            const int c = tid & 31, g = tid >> 5;  // 32 groups of rows
            double acc = 0.0;
            if (c < nb)
                for (int row = k0 + nb + g; row < n; row += 32) acc += A[(size_t)row * n + k0 + c] * s_x[row];
            s_part[c][g] = acc;
        }
        __syncthreads();
        if (tid < 64) {
            const int r = tid;
            double rhs = 0.0;
            if (r < nb) {
                double t = 0.0;
                for (int g = 0; g < 32; g++) t += s_part[r][g];
                rhs = D.x[k0 + r] - t;  // y_k from the panel pass
            }
            double Lc[CB];
#pragma unroll
            for (int c = 0; c < CB; c++) Lc[c] = (r < nb && c < nb && c >= r) ? D.Lkk[(size_t)(k0 + c) * CB + r] : 0.0;
            double xv = rhs;
#pragma unroll
            for (int c = CB - 1; c >= 0; c--) {
                if (c < nb) {
                    const double xc = readlane_d(xv, c) / readlane_d(Lc[c], c);  // L[c][c] in lane c
                    if (r == c) xv = xc;
                    else if (r < c) xv -= Lc[c] * xc;  // L^T[r][c] = L[c][r]
                }
            }
            if (r < nb) s_x[k0 + r] = xv;
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += 1024) D.x[i] = s_x[i];
}

// landmark back-substitution + new estimates + LM scale partials
__global__ __launch_bounds__(EB) void k_update(LbaDev D, double lambda)
{
    __shared__ double s[EB / 64];
    const int t = blockIdx.x * EB + threadIdx.x;
    const int sp = 6 * D.nhp;
    double sc = 0.0;
    if (t < D.nhl) {
        const int l = t;
        double cl[3] = {D.bl[3 * (size_t)l], D.bl[3 * (size_t)l + 1], D.bl[3 * (size_t)l + 2]};
        for (int blk = D.lm_b_start[l]; blk < D.lm_b_start[l + 1]; blk++) {
            const int i1 = D.blk_pose[blk];
            const double *B = D.Hpl + 18 * (size_t)blk;
            for (int c = 0; c < 3; c++) {
                double s_ = 0;
                for (int r = 0; r < 6; r++) s_ += B[3 * r + c] * (-D.x[6 * i1 + r]);
                cl[c] += s_;
            }
        }
        const double *Di = D.Dinv + 9 * (size_t)l;
        const int p = D.hl_point[l];
        for (int r = 0; r < 3; r++) {
            const double xl = Di[3 * r] * cl[0] + Di[3 * r + 1] * cl[1] + Di[3 * r + 2] * cl[2];
            D.x[sp + 3 * l + r] = xl;
            D.point_new[3 * (size_t)p + r] = D.point_cur[3 * (size_t)p + r] + xl;
            sc += xl * (lambda * xl + D.bl[3 * (size_t)l + r]);
        }
    }
    if (t < D.np) {  // poses: exp(x) * T for free active poses, copy otherwise
        const int hi = D.pose_h[t];
        if (hi >= 0) {
            SE3 T = se3_from7(D.pose_cur + 7 * (size_t)t);
            double upd[6];
            for (int k = 0; k < 6; k++) {
                upd[k] = D.x[6 * hi + k];
                sc += upd[k] * (lambda * upd[k] + D.bp[6 * (size_t)hi + k]);
            }
            se3_oplus(T, upd);
            se3_to7(T, D.pose_new + 7 * (size_t)t);
        } else {
            for (int k = 0; k < 7; k++) D.pose_new[7 * (size_t)t + k] = D.pose_cur[7 * (size_t)t + k];
        }
    }
    // points without a landmark index (no edges) keep their estimate
    if (t < D.npt && D.point_h[t] < 0)
        for (int k = 0; k < 3; k++) D.point_new[3 * (size_t)t + k] = D.point_cur[3 * (size_t)t + k];
    const double tot = block_sum_d(sc, s);
    if (threadIdx.x == 0) D.part[NPART + blockIdx.x] = tot;
}

__global__ __launch_bounds__(EB) void k_classify(LbaDev D, const double *__restrict__ poses,
                                                 const double *__restrict__ points, uint8_t *__restrict__ bad)
{
    const int e = blockIdx.x * EB + threadIdx.x;
    if (e >= D.ne) return;
    const int k = D.e_kind[e];
    const int dim = (k == OSG_EDGE_STEREO) ? 3 : 2;
    const double ev[3] = {D.err[3 * e], D.err[3 * e + 1], D.err[3 * e + 2]};
    const double th = (k == OSG_EDGE_STEREO) ? 7.815 : 5.991;
    const SE3 T = se3_from7(poses + 7 * (size_t)D.e_pose[e]);
    const bool pos = edge_depth_positive(k, D.cams[D.e_cam[e]], T, points + 3 * (size_t)D.e_point[e]);
    bad[e] = (chi2_of(ev, dim, edge_w(D, e)) > th || !pos) ? 1 : 0;
}

template <typename T>
T *carve(char *base, size_t &off, size_t count)
{
    off = (off + 255) & ~size_t(255);
    T *p = (T *)(base + off);
    off += sizeof(T) * std::max<size_t>(count, 1);
    return p;
}

}  // namespace

extern "C" int osg_local_bundle_adjustment(osg_ctx *ctx, const osg_ba_graph *G, osg_ba_result *R,
                                           const volatile int *stop)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, G && R, "null argument");
    const int np = G->n_poses, npt = G->n_points, ne = G->n_edges;
    OSG_REQUIRE(ctx, np >= 0 && npt >= 0 && ne >= 0 && G->n_cams >= 0, "sizes");
    OSG_REQUIRE(ctx, R->pose && R->point && (ne == 0 || R->edge_bad), "result buffers");
    R->iterations = 0;
    R->trials = 0;
    R->aborted = 0;
    R->chi2_initial = R->chi2_final = 0.0;
    std::memcpy(R->pose, G->pose, sizeof(double) * 7 * np);
    std::memcpy(R->point, G->point, sizeof(double) * 3 * npt);
    if (ne > 0) std::memset(R->edge_bad, 0, ne);
    if (stop && *stop) {  // ref:src/Optimizer.cc:2112-2114
        R->aborted = 1;
        return 0;
    }
    if (ne == 0) return 0;
    for (int e = 0; e < ne; e++) {
        if (G->e_pose[e] < 0 || G->e_pose[e] >= np || G->e_point[e] < 0 || G->e_point[e] >= npt ||
            G->e_cam[e] < 0 || G->e_cam[e] >= G->n_cams)
            return osg_set_error(ctx, OSG_E_INVALID, "edge %d references out of range", e);
    }
    // ---------------------------------------------------------------- structure (host)
    static const bool prof = getenv("OSG_LBA_PROFILE") && atoi(getenv("OSG_LBA_PROFILE"));
    const auto tp0 = std::chrono::steady_clock::now();
    auto ms_since = [&](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    std::vector<int32_t> pose_cnt(np, 0), point_cnt(npt, 0);
    for (int e = 0; e < ne; e++) {
        pose_cnt[G->e_pose[e]]++;
        point_cnt[G->e_point[e]]++;
    }
    std::vector<int32_t> pose_h(np, -1), hp_pose, point_h(npt, -1), hl_point;
    for (int i = 0; i < np; i++)
        if (!G->pose_fixed[i] && pose_cnt[i] > 0) {
            pose_h[i] = (int)hp_pose.size();
            hp_pose.push_back(i);
        }
    for (int i = 0; i < npt; i++)
        if (point_cnt[i] > 0) {
            point_h[i] = (int)hl_point.size();
            hl_point.push_back(i);
        }
    const int nhp = (int)hp_pose.size(), nhl = (int)hl_point.size();
    if (nhp + nhl == 0) return 0;
    OSG_REQUIRE(ctx, 6 * nhp <= CMAX, "%d free poses exceed the dense reduced-system limit (%d)", nhp, CMAX / 6);
    // edges per landmark (stable in edge order)
    std::vector<int32_t> lm_e_start(nhl + 1, 0), lm_e(ne);
    for (int e = 0; e < ne; e++) lm_e_start[point_h[G->e_point[e]] + 1]++;
    for (int l = 0; l < nhl; l++) lm_e_start[l + 1] += lm_e_start[l];
    {
        std::vector<int32_t> fill(lm_e_start.begin(), lm_e_start.end() - 1);
        for (int e = 0; e < ne; e++) lm_e[fill[point_h[G->e_point[e]]]++] = e;
    }
    // blocks per landmark: unique free poses sorted by hessian index
    std::vector<int32_t> lm_b_start(nhl + 1, 0), blk_pose, edge_blk(ne, -1);
    blk_pose.reserve(ne);
    std::vector<int32_t> tmp;
    for (int l = 0; l < nhl; l++) {
        tmp.clear();
        for (int q = lm_e_start[l]; q < lm_e_start[l + 1]; q++) {
            const int ph = pose_h[G->e_pose[lm_e[q]]];
            if (ph >= 0) tmp.push_back(ph);
        }
        std::sort(tmp.begin(), tmp.end());
        tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
        const int base = (int)blk_pose.size();
        for (int ph : tmp) blk_pose.push_back(ph);
        lm_b_start[l + 1] = (int)blk_pose.size();
        for (int q = lm_e_start[l]; q < lm_e_start[l + 1]; q++) {
            const int e = lm_e[q];
            const int ph = pose_h[G->e_pose[e]];
            if (ph < 0) continue;
            for (int k = 0; k < (int)tmp.size(); k++)
                if (tmp[k] == ph) {
                    edge_blk[e] = base + k;
                    break;
                }
        }
    }
    const int nblk = (int)blk_pose.size();
    std::vector<int32_t> blk_lm(nblk), blk_e_start(nblk + 1, 0), blk_e;
    for (int l = 0; l < nhl; l++)
        for (int b = lm_b_start[l]; b < lm_b_start[l + 1]; b++) blk_lm[b] = l;
    for (int e = 0; e < ne; e++)
        if (edge_blk[e] >= 0) blk_e_start[edge_blk[e] + 1]++;
    for (int b = 0; b < nblk; b++) blk_e_start[b + 1] += blk_e_start[b];
    blk_e.resize(blk_e_start[nblk]);
    {
        std::vector<int32_t> fill(blk_e_start.begin(), blk_e_start.end() - 1);
        for (int e = 0; e < ne; e++)
            if (edge_blk[e] >= 0) blk_e[fill[edge_blk[e]]++] = e;
    }
    // edges / blocks per hessian pose
    std::vector<int32_t> hp_e_start(nhp + 1, 0), hp_e, hp_b_start(nhp + 1, 0), hp_b(nblk);
    for (int e = 0; e < ne; e++)
        if (pose_h[G->e_pose[e]] >= 0) hp_e_start[pose_h[G->e_pose[e]] + 1]++;
    for (int i = 0; i < nhp; i++) hp_e_start[i + 1] += hp_e_start[i];
    hp_e.resize(hp_e_start[nhp]);
    {
        std::vector<int32_t> fill(hp_e_start.begin(), hp_e_start.end() - 1);
        for (int e = 0; e < ne; e++)
            if (pose_h[G->e_pose[e]] >= 0) hp_e[fill[pose_h[G->e_pose[e]]]++] = e;
    }
    for (int b = 0; b < nblk; b++) hp_b_start[blk_pose[b] + 1]++;
    for (int i = 0; i < nhp; i++) hp_b_start[i + 1] += hp_b_start[i];
    {
        std::vector<int32_t> fill(hp_b_start.begin(), hp_b_start.end() - 1);
        for (int b = 0; b < nblk; b++) hp_b[fill[blk_pose[b]]++] = b;
    }
    // pose pairs (i <= j), dense index; contributions in landmark order
    const int npairs = nhp * (nhp + 1) / 2;
    auto pid = [nhp](int i, int j) { return i * nhp - i * (i - 1) / 2 + (j - i); };
    std::vector<int32_t> pair_start(npairs + 1, 0);
    for (int l = 0; l < nhl; l++)
        for (int a = lm_b_start[l]; a < lm_b_start[l + 1]; a++)
            for (int b = a; b < lm_b_start[l + 1]; b++) pair_start[pid(blk_pose[a], blk_pose[b]) + 1]++;
    for (int k = 0; k < npairs; k++) pair_start[k + 1] += pair_start[k];
    std::vector<int32_t> pair_ab(2 * (size_t)std::max(pair_start[npairs], 1));
    {
        std::vector<int32_t> fill(pair_start.begin(), pair_start.end() - 1);
        for (int l = 0; l < nhl; l++)
            for (int a = lm_b_start[l]; a < lm_b_start[l + 1]; a++)
                for (int b = a; b < lm_b_start[l + 1]; b++) {
                    const int k = fill[pid(blk_pose[a], blk_pose[b])]++;
                    pair_ab[2 * k] = a;
                    pair_ab[2 * k + 1] = b;
                }
    }
    const double t_struct = ms_since(tp0);
    // chunks of <= SCH contributions, never spanning two pairs
    std::vector<int32_t> chunk_start, pair_chunk(npairs + 1, 0);
    for (int k = 0; k < npairs; k++) {
        pair_chunk[k] = (int)chunk_start.size();
        for (int q = pair_start[k]; q < pair_start[k + 1]; q += SCH) chunk_start.push_back(q);
    }
    pair_chunk[npairs] = (int)chunk_start.size();
    const int nchunks = (int)chunk_start.size();
    chunk_start.push_back(pair_start[npairs]);
    // ---------------------------------------------------------------- device layout
    osg_packer pk;
    const size_t o_fixed = pk.add(G->pose_fixed, np);
    const size_t o_epose = pk.add(G->e_pose, 4 * (size_t)ne);
    const size_t o_epoint = pk.add(G->e_point, 4 * (size_t)ne);
    const size_t o_ecam = pk.add(G->e_cam, 4 * (size_t)ne);
    const size_t o_ekind = pk.add(G->e_kind, ne);
    const size_t o_eobs = pk.add(G->e_obs, 24 * (size_t)ne);
    const size_t o_eisig = pk.add(G->e_inv_sigma2, 4 * (size_t)ne);
    const size_t o_cams = pk.add(G->cams, sizeof(osg_camera) * G->n_cams);
    const size_t o_poseh = pk.add(pose_h.data(), 4 * (size_t)np);
    const size_t o_hppose = pk.add(hp_pose.data(), 4 * (size_t)nhp);
    const size_t o_pointh = pk.add(point_h.data(), 4 * (size_t)npt);
    const size_t o_hlpoint = pk.add(hl_point.data(), 4 * (size_t)nhl);
    const size_t o_lmes = pk.add(lm_e_start.data(), 4 * (size_t)(nhl + 1));
    const size_t o_lme = pk.add(lm_e.data(), 4 * (size_t)ne);
    const size_t o_lmbs = pk.add(lm_b_start.data(), 4 * (size_t)(nhl + 1));
    const size_t o_blkpose = pk.add(blk_pose.data(), 4 * (size_t)nblk);
    const size_t o_eblk = pk.add(edge_blk.data(), 4 * (size_t)ne);
    const size_t o_hpes = pk.add(hp_e_start.data(), 4 * (size_t)(nhp + 1));
    const size_t o_hpe = pk.add(hp_e.data(), 4 * hp_e.size());
    const size_t o_hpbs = pk.add(hp_b_start.data(), 4 * (size_t)(nhp + 1));
    const size_t o_hpb = pk.add(hp_b.data(), 4 * (size_t)nblk);
    const size_t o_pairs = pk.add(pair_start.data(), 4 * (size_t)(npairs + 1));
    const size_t o_pairab = pk.add(pair_ab.data(), 4 * pair_ab.size());
    const size_t o_chs = pk.add(chunk_start.data(), 4 * chunk_start.size());
    const size_t o_blklm = pk.add(blk_lm.data(), 4 * (size_t)nblk);
    const size_t o_blkes = pk.add(blk_e_start.data(), 4 * (size_t)(nblk + 1));
    const size_t o_blke = pk.add(blk_e.data(), 4 * blk_e.size());
    const size_t o_pch = pk.add(pair_chunk.data(), 4 * pair_chunk.size());
    const size_t o_pose0 = pk.add(G->pose, 56 * (size_t)np);
    const size_t o_point0 = pk.add(G->point, 24 * (size_t)npt);
    char *pin = (char *)osg_pinned(ctx, pk.total + 4096 + sizeof(double) * (3 * NPART + 64));
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    pk.fill(pin);
    char *din = nullptr;
    OSG_ALLOC(ctx, din, SLOT_BA2, pk.total + 256);
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(din, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    // state buffers
    const int sp = 6 * nhp;
    size_t off = 0;
    size_t st_bytes = 0;
    {  // size pass
        char *z = nullptr;
        carve<double>(z, st_bytes, 7 * (size_t)np);      // pose A
        carve<double>(z, st_bytes, 7 * (size_t)np);      // pose B
        carve<double>(z, st_bytes, 3 * (size_t)npt);     // point A
        carve<double>(z, st_bytes, 3 * (size_t)npt);     // point B
        carve<double>(z, st_bytes, 3 * (size_t)ne);      // err
        carve<double>(z, st_bytes, EC * (size_t)ne);     // per-edge contributions
        carve<double>(z, st_bytes, 9 * (size_t)nhl);     // Hll
        carve<double>(z, st_bytes, 3 * (size_t)nhl);     // bl
        carve<double>(z, st_bytes, 18 * (size_t)nblk);   // Hpl
        carve<double>(z, st_bytes, 36 * (size_t)nhp);    // Hpp
        carve<double>(z, st_bytes, 6 * (size_t)nhp);     // bp
        carve<double>(z, st_bytes, 9 * (size_t)nhl);     // Dinv
        carve<double>(z, st_bytes, 18 * (size_t)nblk);   // BDinv
        carve<double>(z, st_bytes, 6 * (size_t)nblk);    // coef
        carve<double>(z, st_bytes, (size_t)sp * sp);     // Hs
        carve<double>(z, st_bytes, (size_t)sp);          // bs
        carve<double>(z, st_bytes, (size_t)sp + 3 * (size_t)nhl);  // x
        carve<double>(z, st_bytes, 3 * (size_t)NPART + 64);        // partials
        carve<double>(z, st_bytes, 36 * (size_t)std::max(nchunks, 1));  // chunk partials
        carve<double>(z, st_bytes, 3 * (size_t)nhl);                     // db
        carve<double>(z, st_bytes, (size_t)sp * CB);                     // Lkk
        carve<int>(z, st_bytes, 16);                                // flags
        carve<uint8_t>(z, st_bytes, ne);                            // edge_bad
        st_bytes += 256;
    }
    char *dst = nullptr;
    OSG_ALLOC(ctx, dst, SLOT_BA3, st_bytes);
    double *poseA = carve<double>(dst, off, 7 * (size_t)np);
    double *poseB = carve<double>(dst, off, 7 * (size_t)np);
    double *pointA = carve<double>(dst, off, 3 * (size_t)npt);
    double *pointB = carve<double>(dst, off, 3 * (size_t)npt);
    LbaDev D = {};
    D.np = np;
    D.npt = npt;
    D.ne = ne;
    D.nhp = nhp;
    D.nhl = nhl;
    D.nblk = nblk;
    D.npairs = npairs;
    D.n_cams = G->n_cams;
    D.pose_fixed = osg_dptr<uint8_t>(din, o_fixed);
    D.e_pose = osg_dptr<int32_t>(din, o_epose);
    D.e_point = osg_dptr<int32_t>(din, o_epoint);
    D.e_cam = osg_dptr<int32_t>(din, o_ecam);
    D.e_kind = osg_dptr<int8_t>(din, o_ekind);
    D.e_obs = osg_dptr<double>(din, o_eobs);
    D.e_isig2 = osg_dptr<float>(din, o_eisig);
    D.cams = osg_dptr<osg_camera>(din, o_cams);
    D.pose_h = osg_dptr<int32_t>(din, o_poseh);
    D.hp_pose = osg_dptr<int32_t>(din, o_hppose);
    D.point_h = osg_dptr<int32_t>(din, o_pointh);
    D.hl_point = osg_dptr<int32_t>(din, o_hlpoint);
    D.lm_e_start = osg_dptr<int32_t>(din, o_lmes);
    D.lm_e = osg_dptr<int32_t>(din, o_lme);
    D.lm_b_start = osg_dptr<int32_t>(din, o_lmbs);
    D.blk_pose = osg_dptr<int32_t>(din, o_blkpose);
    D.edge_blk = osg_dptr<int32_t>(din, o_eblk);
    D.hp_e_start = osg_dptr<int32_t>(din, o_hpes);
    D.hp_e = osg_dptr<int32_t>(din, o_hpe);
    D.hp_b_start = osg_dptr<int32_t>(din, o_hpbs);
    D.hp_b = osg_dptr<int32_t>(din, o_hpb);
    D.pair_start = osg_dptr<int32_t>(din, o_pairs);
    D.pair_ab = osg_dptr<int32_t>(din, o_pairab);
    D.err = carve<double>(dst, off, 3 * (size_t)ne);
    D.J = carve<double>(dst, off, EC * (size_t)ne);
    D.Hll = carve<double>(dst, off, 9 * (size_t)nhl);
    D.bl = carve<double>(dst, off, 3 * (size_t)nhl);
    D.Hpl = carve<double>(dst, off, 18 * (size_t)nblk);
    D.Hpp = carve<double>(dst, off, 36 * (size_t)nhp);
    D.bp = carve<double>(dst, off, 6 * (size_t)nhp);
    D.Dinv = carve<double>(dst, off, 9 * (size_t)nhl);
    D.BDinv = carve<double>(dst, off, 18 * (size_t)nblk);
    D.coef = carve<double>(dst, off, 6 * (size_t)nblk);
    D.Hs = carve<double>(dst, off, (size_t)sp * sp);
    D.bs = carve<double>(dst, off, (size_t)sp);
    D.x = carve<double>(dst, off, (size_t)sp + 3 * (size_t)nhl);
    D.part = carve<double>(dst, off, 3 * (size_t)NPART + 64);
    D.chunk_part = carve<double>(dst, off, 36 * (size_t)std::max(nchunks, 1));
    D.nchunks = nchunks;
    D.chunk_start = osg_dptr<int32_t>(din, o_chs);
    D.blk_lm = osg_dptr<int32_t>(din, o_blklm);
    D.blk_e_start = osg_dptr<int32_t>(din, o_blkes);
    D.blk_e = osg_dptr<int32_t>(din, o_blke);
    D.db = carve<double>(dst, off, 3 * (size_t)nhl);
    D.pair_chunk = osg_dptr<int32_t>(din, o_pch);
    D.Lkk = carve<double>(dst, off, (size_t)sp * CB);
    D.flag = carve<int>(dst, off, 16);
    uint8_t *d_bad = carve<uint8_t>(dst, off, ne);
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(poseA, din + o_pose0, 56 * (size_t)np, hipMemcpyDeviceToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(pointA, din + o_point0, 24 * (size_t)npt, hipMemcpyDeviceToDevice, ctx->stream));

    const int ge = (ne + EB - 1) / EB;
    const int gl = (nhl + EB - 1) / EB;
    const int gu = (std::max(std::max(nhl, np), npt) + EB - 1) / EB;
    OSG_REQUIRE(ctx, ge <= NPART && gu <= NPART && gl + nhp <= NPART, "graph too large for the partial buffers");
    double *h_part = (double *)(pin + ((pk.total + 255) & ~size_t(255)));
    double *cur_pose = poseA, *cur_point = pointA, *new_pose = poseB, *new_point = pointB;

    auto errors = [&](const double *poses, const double *points) -> int {
        hipLaunchKernelGGL(k_errors, dim3(ge), dim3(EB), 0, ctx->stream, D, poses, points, 0);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    };
    auto fetch = [&](size_t first, size_t count) -> int {
        if (hipMemcpyAsync(h_part + first, D.part + first, sizeof(double) * count, hipMemcpyDeviceToHost,
                           ctx->stream) != hipSuccess)
            return -1;
        return hipStreamSynchronize(ctx->stream) == hipSuccess ? 0 : -1;
    };
    auto sum_part = [&](size_t first, int count) {
        double s = 0;
        for (int i = 0; i < count; i++) s += h_part[first + i];
        return s;
    };

    const double t_upload = ms_since(tp0) - t_struct;
    const auto tp1 = std::chrono::steady_clock::now();
    // initial chi2 (activeRobustChi2 before optimising)
    D.pose_cur = cur_pose;
    D.point_cur = cur_point;
    if (errors(cur_pose, cur_point) || fetch(0, ge)) return osg_set_error(ctx, OSG_E_HIP, "k_errors");
    double currentChi = sum_part(0, ge);
    R->chi2_initial = currentChi;
    bool errors_current = true;  // err[] holds the current estimate's errors
    double lambda = 0, ni = 2;
    int nBad = 0, iters = 0, trials = 0;
    const int max_it = G->iterations;
    bool ok = true;
    for (int it = 0; it < max_it && !(stop && *stop) && ok; it++) {
        D.pose_cur = cur_pose;
        D.point_cur = cur_point;
        if (!errors_current) {
            if (errors(cur_pose, cur_point) || fetch(0, ge)) return osg_set_error(ctx, OSG_E_HIP, "k_errors");
            currentChi = sum_part(0, ge);
        }
        const double iniChi = currentChi;
        hipLaunchKernelGGL(k_linearize, dim3(ge), dim3(EB), 0, ctx->stream, D);
        hipLaunchKernelGGL(k_point_red, dim3(std::max(gl, 1)), dim3(EB), 0, ctx->stream, D);
        if (nblk > 0) hipLaunchKernelGGL(k_block_red, dim3((nblk + EB - 1) / EB), dim3(EB), 0, ctx->stream, D);
        if (nhp > 0) hipLaunchKernelGGL(k_pose_red, dim3(nhp), dim3(EB), 0, ctx->stream, D, 2 * NPART + gl);
        OSG_HIP_CHECK(ctx, hipGetLastError());
        if (it == 0) {
            if (fetch(2 * NPART, (size_t)gl + nhp)) return osg_set_error(ctx, OSG_E_HIP, "diag fetch");
            if (G->user_lambda_init > 0) lambda = G->user_lambda_init;
            else {
                double md = 0;
                for (int i = 0; i < gl + nhp; i++) md = std::max(md, h_part[2 * NPART + i]);
                lambda = 1e-5 * md;
            }
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            trials++;
            hipLaunchKernelGGL(k_schur_point, dim3(std::max(gl, 1)), dim3(EB), 0, ctx->stream, D, lambda);
            if (nblk > 0) hipLaunchKernelGGL(k_schur_block, dim3((nblk + EB - 1) / EB), dim3(EB), 0, ctx->stream, D);
            if (nhp > 0) {
                if (nchunks > 0)
                    hipLaunchKernelGGL(k_schur_chunks, dim3((nchunks * 64 + 255) / 256), dim3(256), 0, ctx->stream, D);
                hipLaunchKernelGGL(k_schur_pairs, dim3((npairs * 64 + 255) / 256), dim3(256), 0, ctx->stream, D, lambda);
                hipLaunchKernelGGL(k_bschur, dim3(nhp), dim3(256), 0, ctx->stream, D);
                const int nred = 6 * nhp;
                for (int k0 = 0; k0 < nred; k0 += CB) {
                    const int rb = (nred - k0 + CB - 1) / CB;  // row blocks at and below the diagonal
                    hipLaunchKernelGGL(k_chol_panel, dim3(rb), dim3(64), 0, ctx->stream, D, k0);
                    const int t = (nred - k0 - CB + CB - 1) / CB;
                    if (t > 0) hipLaunchKernelGGL(k_chol_syrk, dim3(t * (t + 1) / 2), dim3(256), 0, ctx->stream, D, k0);
                }
                hipLaunchKernelGGL(k_chol_back, dim3(1), dim3(1024), 0, ctx->stream, D);
            }
            D.pose_new = new_pose;
            D.point_new = new_point;
            hipLaunchKernelGGL(k_update, dim3(gu), dim3(EB), 0, ctx->stream, D, lambda);
            OSG_HIP_CHECK(ctx, hipGetLastError());
            if (errors(new_pose, new_point)) return osg_set_error(ctx, OSG_E_HIP, "k_errors");
            // one download: chi partials, scale partials, cholesky flag
            OSG_HIP_CHECK(ctx, hipMemcpyAsync(h_part, D.part, sizeof(double) * 2 * NPART, hipMemcpyDeviceToHost, ctx->stream));
            int hflag = 1;
            if (nhp > 0) OSG_HIP_CHECK(ctx, hipMemcpyAsync(&hflag, D.flag, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
            OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
            double tempChi = sum_part(0, ge);
            if (!hflag) tempChi = DBL_MAX;
            rho = currentChi - tempChi;
            double scale = sum_part(NPART, gu) + 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
                std::swap(cur_pose, new_pose);
                std::swap(cur_point, new_point);
                errors_current = true;
            } else {
                lambda *= ni;
                ni *= 2;
                errors_current = false;  // err[] holds the rejected estimate's errors
            }
            qmax++;
        } while (rho < 0 && qmax < 10 && !(stop && *stop));
        iters++;
        if (qmax == 10 || rho == 0) ok = false;
        else {
            if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
            else nBad = 0;
            if (nBad >= 3) ok = false;
        }
    }
    if (prof)
        fprintf(stderr, "[osg lba] structure %.3f ms, pack+upload %.3f ms, LM %.3f ms (%d it, %d trials), pairs %d contrib %d\n",
                t_struct, t_upload, ms_since(tp1), iters, trials, npairs, pair_start[npairs]);
    R->iterations = iters;
    R->trials = trials;
    R->aborted = (stop && *stop) ? 1 : 0;
    R->chi2_final = currentChi;
    // classification with the last computed errors; estimates out
    D.pose_cur = cur_pose;
    D.point_cur = cur_point;
    hipLaunchKernelGGL(k_classify, dim3(ge), dim3(EB), 0, ctx->stream, D, cur_pose, cur_point, d_bad);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(R->pose, cur_pose, 56 * (size_t)np, hipMemcpyDeviceToHost, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(R->point, cur_point, 24 * (size_t)npt, hipMemcpyDeviceToHost, ctx->stream));
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(R->edge_bad, d_bad, ne, hipMemcpyDeviceToHost, ctx->stream));
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    return iters;
}
