// pose.hip — Optimizer::PoseOptimization (ref:src/Optimizer.cc:71-420) for a batch of frames.
//
// One wave (64 lanes) per frame, persistent over the whole call: 4 rounds x optimize(10) with
// the g2o Levenberg-Marquardt control flow (ref:Thirdparty/g2o/g2o/core/
// optimization_algorithm_levenberg.cpp:61-169) executed in-kernel, no workgroup barrier anywhere.
//
//   * Edge e lives on lane e % 64 of chunk e / 64.  A pass evaluates one chunk per step: every
//     lane computes its edge's terms, writes them to a padded LDS tile, and the terms are summed
//     SEQUENTIALLY IN EDGE ORDER — the order of g2o's loops over _activeEdges
//     (activeRobustChi2, ref:Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:104-120; buildSystem,
//     ref:Thirdparty/g2o/g2o/core/block_solver.hpp:529-557).  The iteration pass carries 28
//     streams (the 21 upper entries of H, the 6 of b, and chi2), summed by lanes 0..27 at once;
//     the trial pass carries chi2 only.  Together with -ffp-contract=off and the correctly
//     rounded sin / cos / cube of exact_math.h, every double the kernel forms is the one the
//     oracle forms, so iteration counts, trial counts, outlier flags and the pose are identical
//     to it (pinhole; KannalaBrandt8 differs only through the device atan2f / atan2).
//   * The first chi2 pass of an LM iteration and buildSystem run at the same pose, so they are
//     one fused pass (errors recomputed from the pose, never stored).  The classification after a
//     round reads each active edge's error at the pose of the LAST chi2 evaluation (a rejected
//     trial's, when the last trial was rejected), exactly as the reference reads e->chi2() from
//     the stale _error; inactive edges are re-evaluated at the final pose (computeError()).
//   * The 6x6 damped solve, exp-map update and lambda control are evaluated by every lane on
//     wave-uniform values (no broadcast needed).  The edge arrays are read from global memory on
//     every pass (L1/L2 resident); the only global stores are the outlier flags, once per round.
#include <cfloat>
#include <vector>

#include "ba_common.h"
#include "exact_math.h"
#include "match_common.h"

using namespace osgba;

namespace {

constexpr int PW = 64;        // lanes per frame
constexpr int NT = 28;        // H upper (21) | -b terms (6) | robust chi2 (1)
constexpr int LDS_ROW = 65;   // padded row: lane q reads row q column j -> banks 2q + 2j

struct PoseProbDev {
    double pose[7];
    int n_edges;
    int edge_off;  // into the batched edge arrays
    osg_camera cam, cam2;
};

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

// sum of the first `cnt` entries of LDS row `row` in order, onto acc
__device__ inline double seq_sum(double acc, const double *row, int cnt)
{
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

// per-frame state in LDS: read where used, so the long-lived values do not pin registers
struct PoseWS {
    SE3 pose, backup, teval, trl;
    osg_camera cam, cam2;
    double xs[6];  // the solver's x (kept when a factorisation fails)
    double sys[NT];
};

__global__ __launch_bounds__(PW) void k_pose_opt(const PoseProbDev *__restrict__ probs,
                                                 const int8_t *__restrict__ e_kind,
                                                 const double *__restrict__ e_xw,
                                                 const double *__restrict__ e_obs,
                                                 const float *__restrict__ e_isig2,
                                                 uint8_t *__restrict__ e_out,
                                                 PoseOut *__restrict__ out)
{
    __shared__ double s_t[NT * LDS_ROW];
    __shared__ PoseWS W;
    const PoseProbDev &P = probs[blockIdx.x];
    const int n = P.n_edges;
    const int8_t *kind = e_kind + P.edge_off;
    const double *xw = e_xw + 3 * (size_t)P.edge_off;
    const double *obs = e_obs + 3 * (size_t)P.edge_off;
    const float *isig2 = e_isig2 + P.edge_off;
    uint8_t *outl = e_out + P.edge_off;
    const int lane = threadIdx.x;
    const int nch = (n + PW - 1) / PW;

    for (int e = lane; e < n; e += PW) outl[e] = 0;
    if (n < 3) {  // ref:src/Optimizer.cc:289-290
        if (lane == 0) {
            for (int i = 0; i < 7; i++) out[blockIdx.x].pose[i] = P.pose[i];
            out[blockIdx.x].n_inliers = 0;
            out[blockIdx.x].lm_iterations = 0;
            out[blockIdx.x].lm_trials = 0;
        }
        return;
    }
    if (lane == 0) {
        W.cam = P.cam;
        W.cam2 = P.cam2;
        W.trl = se3_from7(P.cam2.trl);
#pragma unroll
        for (int i = 0; i < 6; i++) W.xs[i] = 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    const osg_camera &cam = W.cam, &cam2 = W.cam2;
    const SE3 &Trl = W.trl;
    SE3 &pose = W.pose;
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
    double *xs = W.xs;

    // robust chi2 of the edge on this lane for chunk c at pose T (0 when inactive / past n)
    auto chi_term = [&](int e, const SE3 &T) -> double {
        if (e >= n || outl[e]) return 0.0;
        const PEdge E = load_edge(e, kind, xw, obs, isig2);
        double ev[3];
        pose_edge_error(E, cam, cam2, Trl, T, ev);
        const bool st = E.k == OSG_EDGE_STEREO;
        const double c = edge_chi2_of(ev, st, E.w);
        if (!robust) return c;
        double r0, r1;
        if (st) huber(c, hb.delta_stereo, hb.dsqr_stereo, r0, r1);
        else huber(c, hb.delta_mono, hb.dsqr_mono, r0, r1);
        return r0;
    };

    // activeRobustChi2 at T, summed in edge order (lane 0's chain), broadcast
    auto chi_pass = [&](const SE3 &T) -> double {
        double acc = 0.0;
        for (int c = 0; c < nch; c++) {
            reload_lds();
            const double v = chi_term(c * PW + lane, T);
            s_t[lane] = v;
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) acc = seq_sum(acc, s_t, min(PW, n - c * PW));
            __builtin_amdgcn_wave_barrier();
        }
        return readlane_d(acc, 0);
    };

    for (int it = 0; it < 4; it++) {
        // every round restarts from the input pose (ref:src/Optimizer.cc:306-307)
        if (lane == 0) {
            W.pose = se3_from7(P.pose);
            W.teval = W.pose;
        }
        __builtin_amdgcn_wave_barrier();
        SE3 &T_eval = W.teval;
        int nact = 0;
        for (int e = lane; e < n; e += PW) nact += outl[e] ? 0 : 1;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) nact += __shfl_xor(nact, off);
        if (nact > 0) {
            double lambda = 0, ni = 2;
            int nBadLM = 0;
            for (int iter = 0; iter < 10; iter++) {
                total_iters++;
                // computeActiveErrors + activeRobustChi2 + buildSystem at `pose`, one pass
                double acc = 0.0;
                for (int c = 0; c < nch; c++) {
                    reload_lds();
                    const int e = c * PW + lane;
                    double *col = s_t + lane;  // term q of this lane's edge -> s_t[q * LDS_ROW + lane]
                    if (e < n && !outl[e]) {
                        const PEdge E = load_edge(e, kind, xw, obs, isig2);
                        double ev[3];
                        pose_edge_error(E, cam, cam2, Trl, pose, ev);
                        const bool st = E.k == OSG_EDGE_STEREO;
                        const double chi = edge_chi2_of(ev, st, E.w);
                        double r0 = chi, rho1 = 1.0;
                        if (robust) {
                            if (st) huber(chi, hb.delta_stereo, hb.dsqr_stereo, r0, rho1);
                            else huber(chi, hb.delta_mono, hb.dsqr_mono, r0, rho1);
                        }
                        col[27 * LDS_ROW] = r0;
                        double Jp[3][6];
                        pose_edge_jac(E, cam, cam2, Trl, pose, Jp);
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
                                col[(q++) * LDS_ROW] = h;
                            }
#pragma unroll
                        for (int i = 0; i < 6; i++) {
                            double s = 0;
                            s += rho1 * Jp[0][i] * (E.w * ev[0]);
                            s += rho1 * Jp[1][i] * (E.w * ev[1]);
                            if (st) s += rho1 * Jp[2][i] * (E.w * ev[2]);
                            col[(21 + i) * LDS_ROW] = -s;  // b -= s  ==  b + (-s), exactly
                        }
                    } else {
#pragma unroll
                        for (int q = 0; q < NT; q++) col[q * LDS_ROW] = 0.0;
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (lane < NT) acc = seq_sum(acc, s_t + lane * LDS_ROW, min(PW, n - c * PW));
                    __builtin_amdgcn_wave_barrier();
                }
                T_eval = pose;
                double *sys = W.sys;  // H upper (21) | b (6) | chi2
                if (lane < NT) sys[lane] = acc;
                __builtin_amdgcn_wave_barrier();
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
                    const bool ok2 = ldlt6(A, bvec, x);
                    if (ok2)
#pragma unroll
                        for (int i = 0; i < 6; i++) xs[i] = x[i];
                    se3_oplus(pose, xs);  // exp(update) * estimate
                    double tempChi = chi_pass(pose);
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
        int bad = 0;
        for (int e = lane; e < n; e += PW) {
            reload_lds();
            const PEdge E = load_edge(e, kind, xw, obs, isig2);
            const bool was_out = outl[e] != 0;
            double ev[3];
            pose_edge_error(E, cam, cam2, Trl, was_out ? pose : T_eval, ev);
            const bool st = E.k == OSG_EDGE_STEREO;
            const float chi2 = (float)edge_chi2_of(ev, st, E.w);
            const float th = st ? 7.815f : 5.991f;
            const bool b = chi2 > th;
            outl[e] = b ? 1 : 0;
            bad += b ? 1 : 0;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) bad += __shfl_xor(bad, off);
        nBad = bad;
        if (it == 2) robust = 0;
        if (n < 10) break;
    }
    if (lane == 0) {
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
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
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
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(din, pin, in_bytes, hipMemcpyHostToDevice, ctx->stream));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_pose_opt, dim3(nb), dim3(PW), 0, ctx->stream, (const PoseProbDev *)din,
                       (const int8_t *)(din + o_kind), (const double *)(din + o_xw), (const double *)(din + o_obs),
                       (const float *)(din + o_isig), (uint8_t *)(dio + o_outl), (PoseOut *)(dio + o_res));
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    char *pout = pin + in_bytes;
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(pout, dio, io_bytes, hipMemcpyDeviceToHost, ctx->stream));
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
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

int osg_pose_optimization(osg_ctx *ctx, const osg_pose_problem *p, osg_pose_result *r)
{
    const int rc = osg_pose_optimization_batch(ctx, p, 1, r);
    return rc < 0 ? rc : r->n_inliers;
}

}  // extern "C"
