// pose.hip — Optimizer::PoseOptimization (ref:src/Optimizer.cc:71-420) for a batch of frames.
//
// NW waves (1, 2, 4 or 8 x 64 lanes) per frame, persistent over the whole call: 4 rounds x
// optimize(10) with the g2o Levenberg-Marquardt control flow (ref:Thirdparty/g2o/g2o/core/
// optimization_algorithm_levenberg.cpp:61-169) executed in-kernel.  The host picks NW: several
// waves when few frames share the chip (the drop-in's one-frame call: latency), one when a batch
// fills the chip's wave slots (throughput).
//
//   * Edge e lives on lane e % 64 of chunk e / 64; chunk c is computed by wave c % NW.  A pass
//     evaluates NW chunks per step: every lane computes its edge's terms into its wave's padded
//     LDS tile, and wave 0 sums the tiles SEQUENTIALLY IN EDGE ORDER — the order of g2o's loops
//     over _activeEdges (activeRobustChi2, ref:Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:
//     104-120; buildSystem, ref:Thirdparty/g2o/g2o/core/block_solver.hpp:529-557).  The iteration
//     pass carries 28 streams (the 21 upper entries of H, the 6 of b, and chi2), summed by lanes
//     0..27 at once; the trial pass carries chi2 only.  Together with -ffp-contract=off and the
//     correctly rounded sin / cos / cube of exact_math.h, every double the kernel forms is the one
//     the oracle forms, so iteration counts, trial counts, outlier flags and the pose are
//     identical to it (pinhole; KannalaBrandt8 differs only through the device atan2f / atan2).
//   * The first chi2 pass of an LM iteration and buildSystem run at the same pose, so they are
//     one pass (errors recomputed from the pose, never stored).  The classification after a
//     round reads each active edge's error at the pose of the LAST chi2 evaluation (a rejected
//     trial's, when the last trial was rejected), exactly as the reference reads e->chi2() from
//     the stale _error; inactive edges are re-evaluated at the final pose (computeError()).
//   * The 6x6 damped solve, exp-map update and lambda control are evaluated by every lane of
//     every wave on identical values (each wave keeps a private copy of the pose state, so none
//     can overwrite what a slower wave still reads).  Outlier flags are a per-lane register
//     bitmask, stored once at the end; the edge arrays are re-read every pass (L2 resident).
#include <algorithm>
#include <cfloat>
#include <cstdlib>
#include <vector>

#include "ba_common.h"
#include "exact_math.h"
#include "match_common.h"

using namespace osgba;

namespace {

constexpr int PW = 64;        // lanes per frame
constexpr int NT = 28;        // H upper (21) | -b terms (6) | robust chi2 (1)
constexpr int ROW = 66;       // padded tile row, 16-byte aligned (ds_read_b128 in seq_sum)

struct PoseProbDev {
    double pose[7];
    int n_edges;
    int edge_off;  // into the batched edge arrays
    osg_camera cam, cam2;
};

#ifdef OSG_POSE_PROF
// phase cycle counters of the first frames (profiling builds only: make POSE_PROF=1)
__device__ unsigned long long g_pose_prof[64][8];
#define PROF_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define PROF_ADD(slot, t0) if (threadIdx.x == 0 && blockIdx.x < 64) g_pose_prof[blockIdx.x][slot] += __builtin_amdgcn_s_memtime() - (t0)
#else
#define PROF_T(v)
#define PROF_ADD(slot, t0)
#endif

struct PoseOut {
    double pose[7];
    int n_inliers, lm_iterations, lm_trials, pad;
};

// compiler-only clobber: values read from the LDS frame state are re-read after it instead of
// being hoisted into registers for the whole kernel (they are wave-uniform broadcasts)
__device__ inline void reload_lds() { asm volatile("" ::: "memory"); }

__device__ inline double readlane_d(double v, int l)
{
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// unpivoted LDL^T of the damped 6x6 system, the oracle's ldlt_solve (require_positive)
__device__ inline bool ldlt6(double A[6][6], const double *b, double *x)
{
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double d = A[j][j];
#pragma unroll
        for (int k = 0; k < j; k++) d -= A[j][k] * A[j][k] * A[k][k];
        if (!(d > 0.0)) return false;
        A[j][j] = d;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            double s = A[i][j];
#pragma unroll
            for (int k = 0; k < j; k++) s -= A[i][k] * A[j][k] * A[k][k];
            A[i][j] = s / d;
        }
    }
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double s = b[i];
#pragma unroll
        for (int k = 0; k < i; k++) s -= A[i][k] * y[k];
        y[i] = s;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] /= A[i][i];
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double s = y[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) s -= A[k][i] * y[k];
        y[i] = s;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = y[i];
    return true;
}

// one edge of the frame, as read from the packed arrays
struct PEdge {
    double X[3], o[3];
    double w;
    int k;
};

__device__ inline PEdge load_edge(int e, const int8_t *kind, const double *xw, const double *obs,
                                  const float *isig2)
{
    PEdge E;
    E.k = kind[e];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        E.X[i] = xw[3 * e + i];
        E.o[i] = obs[3 * e + i];
    }
    E.w = (double)isig2[e];
    return E;
}

// EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose / EdgeSE3ProjectXYZOnlyPoseToBody
// computeError (ref:include/OptimizableTypes.h:74-79,139-145; types_six_dof_expmap.cpp:339-346),
// with the right camera's Trl normalised once per frame (se3_from7 is deterministic).  The
// camera structs and poses live in LDS (PoseWS) and are read where used.
__device__ inline void pose_edge_error(const PEdge &E, const osg_camera &cam, const osg_camera &cam2,
                                       const SE3 &Trl, const SE3 &T, double *ev)
{
    double Xc[3];
    if (E.k == OSG_EDGE_STEREO) {
        se3_map(T, E.X, Xc);
        const double fx = cam.fx, fy = cam.fy, cx = cam.cx, cy = cam.cy;
        const float invz = (float)(1.0f / Xc[2]);
        const double r0 = Xc[0] * invz * fx + cx;
        const double r1 = Xc[1] * invz * fy + cy;
        const double bfd = cam.bf;
        const double r2 = r0 - bfd * invz;
        ev[0] = E.o[0] - r0;
        ev[1] = E.o[1] - r1;
        ev[2] = E.o[2] - r2;
        return;
    }
    const bool body = E.k == OSG_EDGE_BODY;
    if (body) {
        const SE3 Trw = se3_mul(Trl, T);
        se3_map(Trw, E.X, Xc);
    } else {
        se3_map(T, E.X, Xc);
    }
    double uv[2];
    cam_project(body ? cam2 : cam, Xc, uv);
    ev[0] = E.o[0] - uv[0];
    ev[1] = E.o[1] - uv[1];
    ev[2] = 0.0;
}

// linearizeOplus of the three unary edges (ref:src/OptimizableTypes.cpp:110-134,238-265;
// types_six_dof_expmap.cpp:375-404); rows of Jp past the edge's dimension stay 0
__device__ inline void pose_edge_jac(const PEdge &E, const osg_camera &cam, const osg_camera &cam2, const SE3 &Trl,
                                     const SE3 &T, double Jp[3][6])
{
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) Jp[i][j] = 0.0;
    if (E.k == OSG_EDGE_STEREO) {  // OnlyPose formulas
        double Xc[3];
        se3_map(T, E.X, Xc);
        const double fx = cam.fx, fy = cam.fy, bf = cam.bf;
        const double x = Xc[0], y = Xc[1], z = Xc[2];
        const double invz = 1.0 / z;
        const double invz_2 = invz * invz;
        Jp[0][0] = x * y * invz_2 * fx;
        Jp[0][1] = -(1 + (x * x * invz_2)) * fx;
        Jp[0][2] = y * invz * fx;
        Jp[0][3] = -invz * fx;
        Jp[0][5] = x * invz_2 * fx;
        Jp[1][0] = (1 + y * y * invz_2) * fy;
        Jp[1][1] = -x * y * invz_2 * fy;
        Jp[1][2] = -x * invz * fy;
        Jp[1][4] = -invz * fy;
        Jp[1][5] = y * invz_2 * fy;
        Jp[2][0] = Jp[0][0] - bf * y * invz_2;
        Jp[2][1] = Jp[0][1] + bf * x * invz_2;
        Jp[2][2] = Jp[0][2];
        Jp[2][3] = Jp[0][3];
        Jp[2][5] = Jp[0][5] - bf * invz_2;
        return;
    }
    // mono: Xc = T X, A = -dpi(Xc); body: Xl = T X, Xr = Trl Xl, A = -dpi(Xr) Rrl; Jp = A [Xl]x-rows
    const bool body = E.k == OSG_EDGE_BODY;
    double Xl[3], Xr[3], PJ[2][3], S[3][6], A[2][3];
    se3_map(T, E.X, Xl);
    if (body) se3_map(Trl, Xl, Xr);
    else {
        Xr[0] = Xl[0];
        Xr[1] = Xl[1];
        Xr[2] = Xl[2];
    }
    cam_project_jac(body ? cam2 : cam, Xr, PJ);
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) PJ[i][j] = -PJ[i][j];
    if (body) {
        double Rrl[3][3];
        quat_to_R(Trl.q, Rrl);
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) A[i][j] = PJ[i][0] * Rrl[0][j] + PJ[i][1] * Rrl[1][j] + PJ[i][2] * Rrl[2][j];
    } else {
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) A[i][j] = PJ[i][j];
    }
    se3deriv(Xl, S);
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) Jp[i][j] = A[i][0] * S[0][j] + A[i][1] * S[1][j] + A[i][2] * S[2][j];
}

struct Huber {
    double delta_mono, delta_stereo;
    float dsqr_mono, dsqr_stereo;
};

// BaseEdge::chi2 of the error (e' (w I) e, the oracle's edge_chi2 summation order)
__device__ inline double edge_chi2_of(const double *ev, bool stereo, double w)
{
    double s = 0;
    s += ev[0] * (w * ev[0]);
    s += ev[1] * (w * ev[1]);
    if (stereo) s += ev[2] * (w * ev[2]);
    return s;
}

// sum of the first `cnt` (<= 64) entries of a 16-byte aligned LDS row, in order, onto acc.  Full
// rows go 16 entries at a time with the next 16 already loading (ds_read_b128): the add chain, one
// dependent add per edge, is the floor of every pass.
__device__ inline double seq_sum(double acc, const double *row, int cnt)
{
    if (cnt == PW) {
        const double2 *r2 = (const double2 *)row;
        double2 cur[8], nxt[8];
#pragma unroll
        for (int u = 0; u < 8; u++) cur[u] = r2[u];
#pragma unroll
        for (int blk = 0; blk < 4; blk++) {
            if (blk < 3)
#pragma unroll
                for (int u = 0; u < 8; u++) nxt[u] = r2[8 * (blk + 1) + u];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                acc += cur[u].x;
                acc += cur[u].y;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) cur[u] = nxt[u];
        }
        return acc;
    }
    int j = 0;
    for (; j + 8 <= cnt; j += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = row[j + u];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += v[u];
    }
    for (; j < cnt; j++) acc += row[j];
    return acc;
}

// sum of m >= 1 whole 64-entry LDS rows (row w at row0 + w * stride), in order, onto acc.  A row past
// its chunk's last edge holds +0.0 (every lane writes its slot, zero when it has no active edge), and
// adding +0.0 leaves acc unchanged (acc starts at +0.0, so it is never -0.0): summing rows whole is the
// same chain as summing cnt entries.  The next 16 entries are always in flight: a block's loads are
// issued before the previous block's adds (the scheduling barriers keep the compiler from sinking them
// below the adds, which it did to seq_sum: every 16 adds then waited out a whole LDS round trip), and a
// row's last block loads the next row's first.  The last row's look-ahead re-reads that row, unused.
__device__ inline double seq_sum_rows(double acc, const double *row0, int stride, int m)
{
    const double2 *r = (const double2 *)row0;
    double2 cur[8], nxt[8];
#pragma unroll
    for (int u = 0; u < 8; u++) cur[u] = r[u];
    for (int w = 0; w < m; w++) {
        const double2 *nr = (const double2 *)(row0 + (size_t)min(w + 1, m - 1) * stride);
#pragma unroll
        for (int blk = 0; blk < 4; blk++) {
            const double2 *src = blk < 3 ? r + 8 * (blk + 1) : nr;
#pragma unroll
            for (int u = 0; u < 8; u++) nxt[u] = src[u];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 8; u++) {
                acc += cur[u].x;
                acc += cur[u].y;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 8; u++) cur[u] = nxt[u];
        }
        r = nr;
    }
    return acc;
}

// frame constants and the cross-wave results (written by one wave, read by all after a barrier)
struct PoseShared {
    osg_camera cam, cam2;
    SE3 trl;
    double sys[NT];  // the last buildSystem sums: H upper (21) | b (6) | robust chi2
    double chi;      // the last trial's chi2
    int ok;          // the last trial's factorisation succeeded (wave 0's solve, broadcast)
    int n_act[8], n_bad[8];
};
// one wave's copy of the wave-uniform LM state: every wave runs the same LM control on the same
// sums, and a private copy keeps a wave that runs ahead from overwriting what another still reads
struct PoseWave {
    SE3 pose, backup, teval;
    double xs[6];  // the solver's x (kept when a factorisation fails)
};

// NW waves per frame.  Superchunk s holds chunks s*NW .. s*NW+NW-1 (64 edges each, chunk s*NW+w on
// wave w); the waves fill their LDS tiles in parallel, then wave 0 adds the tiles in edge order.
// Outlier flags live in a register bitmask per lane (bit s <-> edge (s*NW+wave)*64+lane) and are
// stored once at the end.
// ROWSUM: the edge-order sums over whole rows with the loads kept ahead (seq_sum_rows); false is the
// previous per-chunk seq_sum (OSG_POSE_ROWSUM=0, A/B runs; the same add chain, bit-identical)
template <int NW, bool ROWSUM>
__global__ __launch_bounds__(NW *PW) void k_pose_opt(const PoseProbDev *__restrict__ probs,
                                                     const int8_t *__restrict__ e_kind,
                                                     const double *__restrict__ e_xw,
                                                     const double *__restrict__ e_obs,
                                                     const float *__restrict__ e_isig2,
                                                     uint8_t *__restrict__ e_out,
                                                     PoseOut *__restrict__ out)
{
    __shared__ __attribute__((aligned(16))) double s_t[NW * NT * ROW];
    __shared__ PoseShared S;
    __shared__ PoseWave WV[NW];
    const PoseProbDev &P = probs[blockIdx.x];
    const int n = P.n_edges;
    const int8_t *kind = e_kind + P.edge_off;
    const double *xw = e_xw + 3 * (size_t)P.edge_off;
    const double *obs = e_obs + 3 * (size_t)P.edge_off;
    const float *isig2 = e_isig2 + P.edge_off;
    uint8_t *outl = e_out + P.edge_off;
    const int wave = threadIdx.x / PW, lane = threadIdx.x % PW;
    const int nsc = (n + NW * PW - 1) / (NW * PW);

    PROF_T(t_start);
    if (n < 3) {  // ref:src/Optimizer.cc:289-290
        for (int e = threadIdx.x; e < n; e += NW * PW) outl[e] = 0;
        if (threadIdx.x == 0) {
            for (int i = 0; i < 7; i++) out[blockIdx.x].pose[i] = P.pose[i];
            out[blockIdx.x].n_inliers = 0;
            out[blockIdx.x].lm_iterations = 0;
            out[blockIdx.x].lm_trials = 0;
        }
        return;
    }
    if (threadIdx.x == 0) {
        S.cam = P.cam;
        S.cam2 = P.cam2;
        S.trl = se3_from7(P.cam2.trl);
    }
    PoseWave &W = WV[wave];
#pragma unroll
    for (int i = 0; i < 6; i++) W.xs[i] = 0.0;
    __syncthreads();
    const osg_camera &cam = S.cam, &cam2 = S.cam2;
    const SE3 &Trl = S.trl;
    SE3 &pose = W.pose, &T_eval = W.teval;
    double *xs = W.xs;
    double *tile = s_t + wave * NT * ROW;
    Huber hb;
    {
        const float deltaMono = (float)sqrt(5.991);  // const float deltaMono = sqrt(5.991)
        const float deltaStereo = (float)sqrt(7.815);
        hb.delta_mono = deltaMono;
        hb.delta_stereo = deltaStereo;
        hb.dsqr_mono = (float)((double)deltaMono * (double)deltaMono);
        hb.dsqr_stereo = (float)((double)deltaStereo * (double)deltaStereo);
    }
    int robust = 1;
    int nBad = 0;
    int total_iters = 0, total_trials = 0;
    uint64_t om = 0;
    auto edge_of = [&](int s) { return (s * NW + wave) * PW + lane; };
    auto active = [&](int s) { return edge_of(s) < n && !((om >> s) & 1); };
    // the edges of chunk w of superchunk s that exist
    auto chunk_cnt = [&](int s, int w) { return min(PW, n - (s * NW + w) * PW); };
    // the chunks of superchunk s that exist (>= 1 for s < nsc)
    auto n_rows = [&](int s) { return min(NW, (n - s * NW * PW + PW - 1) / PW); };

    // activeRobustChi2 at T, summed in edge order by wave 0 lane 0, broadcast through S.chi
    auto chi_pass = [&](const SE3 &T) -> double {
        double acc = 0.0;
        for (int s = 0; s < nsc; s++) {
            reload_lds();
            PROF_T(t_pc);
            double v = 0.0;
            if (active(s)) {
                const PEdge E = load_edge(edge_of(s), kind, xw, obs, isig2);
                double ev[3];
                pose_edge_error(E, cam, cam2, Trl, T, ev);
                const bool st = E.k == OSG_EDGE_STEREO;
                const double c = edge_chi2_of(ev, st, E.w);
                v = c;
                if (robust) {
                    double r1;
                    if (st) huber(c, hb.delta_stereo, hb.dsqr_stereo, v, r1);
                    else huber(c, hb.delta_mono, hb.dsqr_mono, v, r1);
                }
            }
            tile[lane] = v;
            PROF_ADD(6, t_pc);
            __syncthreads();
            PROF_T(t_ps);
            if (threadIdx.x == 0) {
                if (ROWSUM) acc = seq_sum_rows(acc, s_t, NT * ROW, n_rows(s));
                else
                    for (int w = 0; w < NW && chunk_cnt(s, w) > 0; w++) acc = seq_sum(acc, s_t + w * NT * ROW, chunk_cnt(s, w));
            }
            PROF_ADD(7, t_ps);
            if (s + 1 < nsc) __syncthreads();  // the last superchunk's tiles are next written after the barrier below
        }
        if (threadIdx.x == 0) S.chi = acc;
        __syncthreads();
        return S.chi;
    };
    // per-wave counts -> frame total
    auto frame_count = [&](int v, int *slot) -> int {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) slot[wave] = v;
        __syncthreads();
        int t = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) t += slot[w];
        return t;
    };

    // activeRobustChi2 + buildSystem at T: the 28 sums (H upper | b | robust chi2) in edge order,
    // lane q of wave 0 adding stream q, into dst
    auto sys_pass = [&](const SE3 &T, double *dst) {
        double acc = 0.0;
        for (int s = 0; s < nsc; s++) {
            reload_lds();
            double *col = tile + lane;  // term q of this lane's edge -> tile[q * ROW + lane]
            if (active(s)) {
                const PEdge E = load_edge(edge_of(s), kind, xw, obs, isig2);
                double ev[3];
                pose_edge_error(E, cam, cam2, Trl, T, ev);
                const bool st = E.k == OSG_EDGE_STEREO;
                const double chi = edge_chi2_of(ev, st, E.w);
                double r0 = chi, rho1 = 1.0;
                if (robust) {
                    if (st) huber(chi, hb.delta_stereo, hb.dsqr_stereo, r0, rho1);
                    else huber(chi, hb.delta_mono, hb.dsqr_mono, r0, rho1);
                }
                col[27 * ROW] = r0;
                double Jp[3][6];
                pose_edge_jac(E, cam, cam2, Trl, T, Jp);
                const double ww = rho1 * E.w;
                int q = 0;
#pragma unroll
                for (int i = 0; i < 6; i++)
#pragma unroll
                    for (int j = i; j < 6; j++) {
                        double h = 0;
                        h += Jp[0][i] * ww * Jp[0][j];
                        h += Jp[1][i] * ww * Jp[1][j];
                        if (st) h += Jp[2][i] * ww * Jp[2][j];
                        col[(q++) * ROW] = h;
                    }
#pragma unroll
                for (int i = 0; i < 6; i++) {
                    double sb = 0;
                    sb += rho1 * Jp[0][i] * (E.w * ev[0]);
                    sb += rho1 * Jp[1][i] * (E.w * ev[1]);
                    if (st) sb += rho1 * Jp[2][i] * (E.w * ev[2]);
                    col[(21 + i) * ROW] = -sb;  // b -= s  ==  b + (-s), exactly
                }
            } else {
#pragma unroll
                for (int q = 0; q < NT; q++) col[q * ROW] = 0.0;
            }
            __syncthreads();
            if (wave == 0) {  // lane q < 28 adds stream q; the others repeat stream 27, unused
                const int q = lane < NT ? lane : NT - 1;
                if (ROWSUM) acc = seq_sum_rows(acc, s_t + q * ROW, NT * ROW, n_rows(s));
                else
                    for (int w = 0; w < NW && chunk_cnt(s, w) > 0; w++)
                        acc = seq_sum(acc, s_t + (w * NT + q) * ROW, chunk_cnt(s, w));
            }
            if (s + 1 < nsc) __syncthreads();  // as in chi_pass
        }
        if (wave == 0 && lane < NT) dst[lane] = acc;
        __syncthreads();
    };
    for (int it = 0; it < 4; it++) {
        // every round restarts from the input pose (ref:src/Optimizer.cc:306-307)
        pose = se3_from7(P.pose);
        T_eval = pose;
        __builtin_amdgcn_wave_barrier();
        int na = 0;
        for (int s = 0; s < nsc; s++) na += active(s) ? 1 : 0;
        const int nact = frame_count(na, S.n_act);
        if (nact > 0) {
            double lambda = 0, ni = 2;
            int nBadLM = 0;
            for (int iter = 0; iter < 10; iter++) {
                total_iters++;
                // computeActiveErrors + activeRobustChi2 + buildSystem at `pose`, one pass.  (Summing
                // buildSystem along with every trial chi2, to skip this pass after an accepted step,
                // measured slower at every frame size: the Jacobian terms cost more than the pass.)
                PROF_T(t_h);
                sys_pass(pose, S.sys);
                PROF_ADD(0, t_h);
                T_eval = pose;
                const double *sys = S.sys;  // H upper (21) | b (6) | chi2
                const double iniChi = sys[27];
                double currentChi = iniChi;
                if (iter == 0) {  // computeLambdaInit: tau * max |diag H|
                    const int dpos[6] = {0, 6, 11, 15, 18, 20};
                    double md = 0;
#pragma unroll
                    for (int i = 0; i < 6; i++) md = fmax(fabs(sys[dpos[i]]), md);
                    lambda = 1e-5 * md;
                    ni = 2;
                    nBadLM = 0;
                }
                double rho = 0;
                int qmax = 0;
                do {
                    reload_lds();
                    total_trials++;
                    W.backup = pose;  // push
                    PROF_T(t_s);
                    // the 6x6 solve and the exp-map update run on wave 0 alone and are broadcast
                    // through LDS: with 8 waves two share each SIMD, and the redundant copies of these
                    // issue-bound chains would halve its rate.  Waves 1.. take wave 0's x and pose
                    // (their copies are read-only to wave 0 until the next chi_pass barrier).
                    bool okw = true;
                    if (wave == 0) {
                        double A[6][6], bvec[6];
                        {
                            int q = 0;
#pragma unroll
                            for (int i = 0; i < 6; i++)
#pragma unroll
                                for (int j = i; j < 6; j++) {
                                    A[i][j] = sys[q] + (i == j ? lambda : 0.0);
                                    A[j][i] = A[i][j];
                                    q++;
                                }
#pragma unroll
                            for (int i = 0; i < 6; i++) bvec[i] = sys[21 + i];
                        }
                        double x[6];
                        okw = ldlt6(A, bvec, x);
                        if (okw)
#pragma unroll
                            for (int i = 0; i < 6; i++) xs[i] = x[i];
                        PROF_ADD(1, t_s);
                        PROF_T(t_x);
                        se3_oplus<true>(pose, xs);  // exp(update) * estimate (every lane holds the same update)
                        PROF_ADD(2, t_x);
                        if (lane == 0) S.ok = okw ? 1 : 0;
                    }
                    if (NW > 1) {
                        __syncthreads();
                        if (wave != 0) {
#pragma unroll
                            for (int i = 0; i < 6; i++) xs[i] = WV[0].xs[i];
                            pose = WV[0].pose;
                        }
                    }
                    const bool ok2 = wave == 0 ? okw : S.ok != 0;
                    PROF_T(t_c);
                    double tempChi = chi_pass(pose);
                    PROF_ADD(3, t_c);
                    T_eval = pose;
                    if (!ok2) tempChi = DBL_MAX;
                    rho = (currentChi - tempChi);
                    double scale = 0.;
#pragma unroll
                    for (int j = 0; j < 6; j++) scale += xs[j] * (lambda * xs[j] + sys[21 + j]);
                    scale += 1e-3;
                    rho /= scale;
                    if (rho > 0 && isfinite(tempChi)) {
                        double alpha = 1. - osgx::cube_rn(2 * rho - 1);
                        alpha = fmin(alpha, 2. / 3.);
                        const double scaleFactor = fmax(1. / 3., alpha);
                        lambda *= scaleFactor;
                        ni = 2;
                        currentChi = tempChi;
                    } else {
                        lambda *= ni;
                        ni *= 2;
                        pose = W.backup;  // pop
                    }
                    qmax++;
                } while (rho < 0 && qmax < 10);
                bool terminate = false;
                if (qmax == 10 || rho == 0) terminate = true;
                else {
                    if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
                    else nBadLM = 0;
                    if (nBadLM >= 3) terminate = true;
                }
                if (terminate) break;
            }
        }
        // classification (ref:src/Optimizer.cc:314-403): active edges read their last computed
        // error (at T_eval), inactive ones computeError() at the final pose
        PROF_T(t_cl);
        int bad = 0;
        for (int s = 0; s < nsc; s++) {
            reload_lds();
            const int e = edge_of(s);
            if (e >= n) continue;
            const PEdge E = load_edge(e, kind, xw, obs, isig2);
            const bool was_out = (om >> s) & 1;
            double ev[3];
            pose_edge_error(E, cam, cam2, Trl, was_out ? pose : T_eval, ev);
            const bool st = E.k == OSG_EDGE_STEREO;
            const float chi2 = (float)edge_chi2_of(ev, st, E.w);
            const float th = st ? 7.815f : 5.991f;
            const bool b = chi2 > th;
            om = (om & ~(uint64_t(1) << s)) | (uint64_t(b ? 1 : 0) << s);
            bad += b ? 1 : 0;
        }
        nBad = frame_count(bad, S.n_bad);
        PROF_ADD(4, t_cl);
        if (it == 2) robust = 0;
        if (n < 10) break;
        __syncthreads();  // S.n_act / S.n_bad are rewritten next round
    }
    for (int s = 0; s < nsc; s++)
        if (edge_of(s) < n) outl[edge_of(s)] = (om >> s) & 1;
    PROF_ADD(5, t_start);
    if (threadIdx.x == 0) {
        se3_to7(pose, out[blockIdx.x].pose);
        out[blockIdx.x].n_inliers = n - nBad;
        out[blockIdx.x].lm_iterations = total_iters;
        out[blockIdx.x].lm_trials = total_trials;
    }
}


}  // namespace

extern "C" {

int osg_pose_optimization_batch(osg_ctx *ctx, const osg_pose_problem *p, int32_t nb, osg_pose_result *r)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, nb >= 0 && (nb == 0 || (p && r)), "null argument");
    if (nb == 0) return 0;
    std::vector<PoseProbDev> hp(nb);
    size_t total = 0;
    for (int b = 0; b < nb; b++) {
        OSG_REQUIRE(ctx, p[b].n_edges >= 0, "n_edges");
        OSG_REQUIRE(ctx, p[b].n_edges == 0 || (p[b].kind && p[b].xw && p[b].obs && p[b].inv_sigma2 && r[b].outlier),
                    "edge arrays");
        for (int i = 0; i < 7; i++) hp[b].pose[i] = p[b].pose[i];
        hp[b].n_edges = p[b].n_edges;
        hp[b].edge_off = (int)total;
        hp[b].cam = p[b].cam;
        hp[b].cam2 = p[b].cam2;
        total += (size_t)p[b].n_edges;
    }
    OSG_REQUIRE(ctx, total < (size_t(1) << 31), "too many edges in one batch");
    // waves per frame: enough to spread a lone frame's chunks (latency), one when the batch fills
    // the chip's ~2048 wave slots (throughput); at least enough for the 64-bit outlier masks
    int nmax = 0;
    for (int b = 0; b < nb; b++) nmax = std::max(nmax, p[b].n_edges);
    const int chunks = (nmax + PW - 1) / PW;
    int nw = 1;
    if (const char *f = getenv("OSG_POSE_NW")) nw = atoi(f);  // tests pin the variant
    else {
        // waves per frame: up to one per 1.5 chunks of a lone frame's edges (latency; 8 waves share
        // 4 SIMDs and measured no faster than 4), one when the batch fills the chip's wave slots
        while (nw < 4 && 3 * nw <= 2 * chunks && (size_t)nb * 2 * nw <= 2048) nw *= 2;
        // a lone frame of >= 5 chunks (257+ edges): 8 waves, since the solve and the exp-map update run on
        // wave 0 alone (before, 8 waves ran them twice per SIMD and were slower below 9 chunks).  Measured
        // (tools/latency_probe.py): the 318-edge frame 439 -> 418 us, the 600-edge KB8 frame 816 -> 721 us
        if (nw == 4 && chunks >= 5 && (size_t)nb * 2 * 8 <= 2048) nw = 8;
        while (nw < 8 && chunks > 64 * nw) nw *= 2;
    }
    OSG_REQUIRE(ctx, nw == 1 || nw == 2 || nw == 4 || nw == 8, "OSG_POSE_NW must be 1, 2, 4 or 8");
    OSG_REQUIRE(ctx, chunks <= 64 * nw, "more than 32768 edges in one frame");
    // pack: probs | kind | xw | obs | isig2
    osg_packer pk;
    const size_t o_probs = pk.add(hp.data(), sizeof(PoseProbDev) * nb);
    const size_t o_kind = pk.total, o_xw = (o_kind + total + 255) & ~size_t(255);
    const size_t o_obs = o_xw + ((24 * total + 255) & ~size_t(255));
    const size_t o_isig = o_obs + ((24 * total + 255) & ~size_t(255));
    const size_t in_bytes = o_isig + ((4 * total + 255) & ~size_t(255)) + 256;
    const size_t o_outl = 0;
    const size_t o_res = (total + 255) & ~size_t(255);
    const size_t io_bytes = o_res + sizeof(PoseOut) * nb + 256;
    char *pin = (char *)osg_pinned(ctx, in_bytes + io_bytes);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    pk.fill(pin);
    (void)o_probs;
    for (int b = 0; b < nb; b++) {
        const size_t off = hp[b].edge_off, ne = p[b].n_edges;
        if (!ne) continue;
        std::memcpy(pin + o_kind + off, p[b].kind, ne);
        std::memcpy(pin + o_xw + 24 * off, p[b].xw, 24 * ne);
        std::memcpy(pin + o_obs + 24 * off, p[b].obs, 24 * ne);
        std::memcpy(pin + o_isig + 4 * off, p[b].inv_sigma2, 4 * ne);
    }
    char *din = nullptr, *dio = nullptr;
    OSG_ALLOC(ctx, din, SLOT_BA0, in_bytes);
    OSG_ALLOC(ctx, dio, SLOT_BA1, io_bytes);
    OSG_RC(osg_upload(ctx, din, pin, in_bytes));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    const PoseProbDev *a0 = (const PoseProbDev *)din;
    const int8_t *a1 = (const int8_t *)(din + o_kind);
    const double *a2 = (const double *)(din + o_xw), *a3 = (const double *)(din + o_obs);
    const float *a4 = (const float *)(din + o_isig);
    uint8_t *a5 = (uint8_t *)(dio + o_outl);
    PoseOut *a6 = (PoseOut *)(dio + o_res);
    const char *rs = getenv("OSG_POSE_ROWSUM");  // tests pin the variant
    const bool rowsum = !(rs && atoi(rs) == 0);
#define OSG_POSE_LAUNCH(W_)                                                                                    \
    if (rowsum)                                                                                                \
        hipLaunchKernelGGL((k_pose_opt<W_, true>), dim3(nb), dim3(W_ * PW), 0, ctx->stream, a0, a1, a2, a3, a4, a5, \
                           a6);                                                                                \
    else                                                                                                       \
        hipLaunchKernelGGL((k_pose_opt<W_, false>), dim3(nb), dim3(W_ * PW), 0, ctx->stream, a0, a1, a2, a3, a4, \
                           a5, a6)
    switch (nw) {
    case 1: OSG_POSE_LAUNCH(1); break;
    case 2: OSG_POSE_LAUNCH(2); break;
    case 4: OSG_POSE_LAUNCH(4); break;
    default: OSG_POSE_LAUNCH(8); break;
    }
#undef OSG_POSE_LAUNCH
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    char *pout = pin + in_bytes;
    OSG_RC(osg_download(ctx, pout, dio, io_bytes));
    OSG_RC(osg_wait(ctx));
    float kms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&kms, ev[0], ev[1]));
    ctx->last_kernel_ms = kms;
    const PoseOut *res = (const PoseOut *)(pout + o_res);
    int sum = 0;
    for (int b = 0; b < nb; b++) {
        for (int i = 0; i < 7; i++) r[b].pose[i] = res[b].pose[i];
        r[b].n_inliers = res[b].n_inliers;
        r[b].lm_iterations = res[b].lm_iterations;
        r[b].lm_trials = res[b].lm_trials;
        if (p[b].n_edges) std::memcpy(r[b].outlier, pout + o_outl + hp[b].edge_off, p[b].n_edges);
        sum += res[b].n_inliers;
    }
    return sum;
}

#ifdef OSG_POSE_PROF
int osg_debug_pose_prof(unsigned long long *dst, int reset)
{
    if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_pose_prof), sizeof(g_pose_prof)) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long z[64][8];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pose_prof), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif

int osg_pose_optimization(osg_ctx *ctx, const osg_pose_problem *p, osg_pose_result *r)
{
    const int rc = osg_pose_optimization_batch(ctx, p, 1, r);
    return rc < 0 ? rc : r->n_inliers;
}

}  // extern "C"
