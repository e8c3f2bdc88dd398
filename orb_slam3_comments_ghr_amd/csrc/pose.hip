// pose.hip — Optimizer::PoseOptimization (ref:src/Optimizer.cc:71-420) for a batch of frames.
//
// One 256-thread workgroup per frame, persistent over the whole call: 4 rounds x optimize(10)
// with the g2o Levenberg-Marquardt control flow (ref:Thirdparty/g2o/g2o/core/
// optimization_algorithm_levenberg.cpp:61-169) executed in-kernel:
//   * per-edge error / robust chi2 / Jacobian spread over the 256 lanes (edges strided),
//   * the 6x6 system (21 + 6 FP64 values) reduced wave-wide with DPP shuffles, then across the
//     4 waves in LDS,
//   * the damped 6x6 LDL^T solve, exp-map update, push/pop and lambda control on lane 0,
//   * inlier/outlier classification after each round with the reference's float chi2
//     compare, the robust kernel dropped after round index 2, every round restarting from the
//     input pose (ref:src/Optimizer.cc:304-307).
// Launch latency would dominate a per-iteration kernel design (<= 40 iterations x up to 10
// trials per frame); here a batch of B frames is a single launch of B workgroups.
#include <cfloat>
#include <vector>

#include "ba_common.h"
#include "match_common.h"

using namespace osgba;

namespace {

constexpr int PT = 256;

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

__device__ inline double block_sum(double v, double *s_red)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) s_red[w] = v;
    __syncthreads();
    double t = 0;
#pragma unroll
    for (int i = 0; i < PT / 64; i++) t += s_red[i];
    return t;
}

__device__ inline int block_sum_int(int v, int *s_ired)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if (lane == 0) s_ired[w] = v;
    __syncthreads();
    int t = 0;
#pragma unroll
    for (int i = 0; i < PT / 64; i++) t += s_ired[i];
    return t;
}

// unpivoted LDL^T of a 6x6 SPD matrix (upper triangle given as full), requires positive pivots
__device__ inline bool ldlt6(double A[6][6], const double *b, double *x)
{
    for (int j = 0; j < 6; j++) {
        double d = A[j][j];
        for (int k = 0; k < j; k++) d -= A[j][k] * A[j][k] * A[k][k];
        if (!(d > 0.0)) return false;
        A[j][j] = d;
        for (int i = j + 1; i < 6; i++) {
            double s = A[i][j];
            for (int k = 0; k < j; k++) s -= A[i][k] * A[j][k] * A[k][k];
            A[i][j] = s / d;
        }
    }
    double y[6];
    for (int i = 0; i < 6; i++) {
        double s = b[i];
        for (int k = 0; k < i; k++) s -= A[i][k] * y[k];
        y[i] = s;
    }
    for (int i = 0; i < 6; i++) y[i] /= A[i][i];
    for (int i = 5; i >= 0; i--) {
        double s = y[i];
        for (int k = i + 1; k < 6; k++) s -= A[k][i] * y[k];
        y[i] = s;
    }
    for (int i = 0; i < 6; i++) x[i] = y[i];
    return true;
}

__global__ __launch_bounds__(PT) void k_pose_opt(const PoseProbDev *__restrict__ probs,
                                                 const int8_t *__restrict__ e_kind,
                                                 const double *__restrict__ e_xw,
                                                 const double *__restrict__ e_obs,
                                                 const float *__restrict__ e_isig2,
                                                 double *__restrict__ e_err,
                                                 uint8_t *__restrict__ e_out,
                                                 PoseOut *__restrict__ out)
{
    __shared__ double s_red[PT / 64];
    __shared__ int s_ired[PT / 64];
    __shared__ double s_sys[27];
    __shared__ double s_part27[PT / 64][27];
    __shared__ SE3 s_pose, s_backup;
    __shared__ double s_x[6];
    __shared__ int s_flag[4];       // continue-trial, result, ok
    const PoseProbDev &P = probs[blockIdx.x];
    const int n = P.n_edges;
    const int8_t *kind = e_kind + P.edge_off;
    const double *xw = e_xw + 3 * (size_t)P.edge_off;
    const double *obs = e_obs + 3 * (size_t)P.edge_off;
    const float *isig2 = e_isig2 + P.edge_off;
    double *err = e_err + 3 * (size_t)P.edge_off;
    uint8_t *outl = e_out + P.edge_off;
    const int tid = threadIdx.x;
    const float deltaMono = (float)sqrt(5.991);    // const float deltaMono = sqrt(5.991)
    const float deltaStereo = (float)sqrt(7.815);
    const float dsqrMono = (float)((double)deltaMono * (double)deltaMono);
    const float dsqrStereo = (float)((double)deltaStereo * (double)deltaStereo);

    for (int e = tid; e < n; e += PT) {
        outl[e] = 0;
        err[3 * e] = err[3 * e + 1] = err[3 * e + 2] = 0.0;
    }
    if (n < 3) {  // ref:src/Optimizer.cc:289-290
        if (tid == 0) {
            for (int i = 0; i < 7; i++) out[blockIdx.x].pose[i] = P.pose[i];
            out[blockIdx.x].n_inliers = 0;
            out[blockIdx.x].lm_iterations = 0;
            out[blockIdx.x].lm_trials = 0;
        }
        return;
    }
    if (tid < 6) s_x[tid] = 0.0;
    int robust = 1;
    int nBad = 0;
    int total_iters = 0, total_trials = 0;
    __syncthreads();

    // per-edge helpers over the current pose in LDS -------------------------------------------
    auto edge_chi_robust = [&](int e, const SE3 &T) -> double {
        double X[3] = {xw[3 * e], xw[3 * e + 1], xw[3 * e + 2]};
        double o[3] = {obs[3 * e], obs[3 * e + 1], obs[3 * e + 2]};
        const int k = kind[e];
        const osg_camera &cam = (k == OSG_EDGE_BODY) ? P.cam2 : P.cam;
        double ev[3];
        edge_error(k, false, cam, T, X, o, ev);
        err[3 * e] = ev[0];
        err[3 * e + 1] = ev[1];
        err[3 * e + 2] = ev[2];
        const int dim = (k == OSG_EDGE_STEREO) ? 3 : 2;
        const double c = chi2_of(ev, dim, (double)isig2[e]);
        if (!robust) return c;
        double r0, r1;
        if (k == OSG_EDGE_STEREO) huber(c, (double)deltaStereo, dsqrStereo, r0, r1);
        else huber(c, (double)deltaMono, dsqrMono, r0, r1);
        return r0;
    };

    for (int it = 0; it < 4; it++) {
        if (tid == 0) s_pose = se3_from7(P.pose);
        // active edges = level 0 (non-outlier)
        int nact = 0;
        for (int e = tid; e < n; e += PT) nact += outl[e] ? 0 : 1;
        nact = block_sum_int(nact, s_ired);
        __syncthreads();
        if (nact > 0) {
            double lambda = 0, ni = 2;
            int nBadLM = 0;
            for (int iter = 0; iter < 10; iter++) {
                total_iters++;
                // computeActiveErrors + activeRobustChi2
                SE3 T = s_pose;
                double c = 0;
                for (int e = tid; e < n; e += PT)
                    if (!outl[e]) c += edge_chi_robust(e, T);
                const double iniChi = block_sum(c, s_red);
                double currentChi = iniChi;
                // buildSystem: H (upper 21) and b (6)
                double acc[27];
#pragma unroll
                for (int i = 0; i < 27; i++) acc[i] = 0.0;
                for (int e = tid; e < n; e += PT) {
                    if (outl[e]) continue;
                    double X[3] = {xw[3 * e], xw[3 * e + 1], xw[3 * e + 2]};
                    const int k = kind[e];
                    const osg_camera &cam = (k == OSG_EDGE_BODY) ? P.cam2 : P.cam;
                    double Jp[3][6], Jx[3][3];
                    edge_jacobians(k, false, cam, T, X, Jp, Jx);
                    const int dim = (k == OSG_EDGE_STEREO) ? 3 : 2;
                    const double w = (double)isig2[e];
                    const double ev[3] = {err[3 * e], err[3 * e + 1], err[3 * e + 2]};
                    double rho1 = 1.0;
                    if (robust) {
                        double r0;
                        const double chi = chi2_of(ev, dim, w);
                        if (k == OSG_EDGE_STEREO) huber(chi, (double)deltaStereo, dsqrStereo, r0, rho1);
                        else huber(chi, (double)deltaMono, dsqrMono, r0, rho1);
                    }
                    const double ww = rho1 * w;
                    int q = 0;
#pragma unroll
                    for (int i = 0; i < 6; i++)
#pragma unroll
                        for (int j = i; j < 6; j++) {
                            double h = 0;
                            for (int d = 0; d < dim; d++) h += Jp[d][i] * ww * Jp[d][j];
                            acc[q++] += h;
                        }
#pragma unroll
                    for (int i = 0; i < 6; i++) {
                        double s = 0;
                        for (int d = 0; d < dim; d++) s += rho1 * Jp[d][i] * (w * ev[d]);
                        acc[21 + i] -= s;
                    }
                }
                {  // 27 wave reductions, then one pass across the 4 waves
                    const int lane = tid & 63, w = tid >> 6;
#pragma unroll
                    for (int i = 0; i < 27; i++) acc[i] = wave_sum(acc[i]);
                    if (lane == 0)
                        for (int i = 0; i < 27; i++) s_part27[w][i] = acc[i];
                    __syncthreads();
                    if (tid < 27) {
                        double t = 0;
                        for (int ww = 0; ww < PT / 64; ww++) t += s_part27[ww][tid];
                        s_sys[tid] = t;
                    }
                    __syncthreads();
                }
                if (iter == 0) {  // computeLambdaInit: tau * max |diag H|
                    double md = 0;
                    const int dpos[6] = {0, 6, 11, 15, 18, 20};
                    for (int i = 0; i < 6; i++) md = fmax(fabs(s_sys[dpos[i]]), md);
                    lambda = 1e-5 * md;
                    ni = 2;
                    nBadLM = 0;
                }
                double rho = 0;
                int qmax = 0;
                bool cont;
                do {
                    total_trials++;
                    if (tid == 0) {
                        s_backup = s_pose;
                        double A[6][6], b[6];
                        int q = 0;
                        for (int i = 0; i < 6; i++)
                            for (int j = i; j < 6; j++) {
                                A[i][j] = s_sys[q];
                                A[j][i] = s_sys[q];
                                q++;
                            }
                        for (int i = 0; i < 6; i++) {
                            A[i][i] += lambda;
                            b[i] = s_sys[21 + i];
                        }
                        double x[6];
                        const bool ok2 = ldlt6(A, b, x);
                        if (ok2)
                            for (int i = 0; i < 6; i++) s_x[i] = x[i];
                        s_flag[2] = ok2;
                        double xx[6];
                        for (int i = 0; i < 6; i++) xx[i] = s_x[i];
                        se3_oplus(s_pose, xx);
                    }
                    __syncthreads();
                    T = s_pose;
                    double c2 = 0;
                    for (int e = tid; e < n; e += PT)
                        if (!outl[e]) c2 += edge_chi_robust(e, T);
                    double tempChi = block_sum(c2, s_red);
                    if (!s_flag[2]) tempChi = DBL_MAX;
                    rho = (currentChi - tempChi);
                    double scale = 0.;
                    for (int j = 0; j < 6; j++) scale += s_x[j] * (lambda * s_x[j] + s_sys[21 + j]);
                    scale += 1e-3;
                    rho /= scale;
                    if (rho > 0 && isfinite(tempChi)) {
                        double alpha = 1. - pow((2 * rho - 1), 3);
                        alpha = fmin(alpha, 2. / 3.);
                        const double scaleFactor = fmax(1. / 3., alpha);
                        lambda *= scaleFactor;
                        ni = 2;
                        currentChi = tempChi;
                    } else {
                        lambda *= ni;
                        ni *= 2;
                        __syncthreads();
                        if (tid == 0) s_pose = s_backup;
                    }
                    qmax++;
                    cont = (rho < 0 && qmax < 10);
                    __syncthreads();
                } while (cont);
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
        // classification (ref:src/Optimizer.cc:314-403) with the edges' last computed errors
        __syncthreads();
        const SE3 T = s_pose;
        int bad = 0;
        for (int e = tid; e < n; e += PT) {
            const int k = kind[e];
            const int dim = (k == OSG_EDGE_STEREO) ? 3 : 2;
            if (outl[e]) {
                double X[3] = {xw[3 * e], xw[3 * e + 1], xw[3 * e + 2]};
                double o[3] = {obs[3 * e], obs[3 * e + 1], obs[3 * e + 2]};
                const osg_camera &cam = (k == OSG_EDGE_BODY) ? P.cam2 : P.cam;
                double ev[3];
                edge_error(k, false, cam, T, X, o, ev);
                err[3 * e] = ev[0];
                err[3 * e + 1] = ev[1];
                err[3 * e + 2] = ev[2];
            }
            const double ev[3] = {err[3 * e], err[3 * e + 1], err[3 * e + 2]};
            const float chi2 = (float)chi2_of(ev, dim, (double)isig2[e]);
            const float th = (k == OSG_EDGE_STEREO) ? 7.815f : 5.991f;
            if (chi2 > th) {
                outl[e] = 1;
                bad++;
            } else {
                outl[e] = 0;
            }
        }
        nBad = block_sum_int(bad, s_ired);
        if (it == 2) robust = 0;
        __syncthreads();
        if (n < 10) break;
    }
    if (tid == 0) {
        se3_to7(s_pose, out[blockIdx.x].pose);
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
    // pack: probs | kind | xw | obs | isig2
    const size_t o_probs = 0;
    const size_t o_kind = (sizeof(PoseProbDev) * nb + 255) & ~size_t(255);
    const size_t o_xw = (o_kind + total + 255) & ~size_t(255);
    const size_t o_obs = o_xw + ((24 * total + 255) & ~size_t(255));
    const size_t o_isig = o_obs + ((24 * total + 255) & ~size_t(255));
    const size_t in_bytes = o_isig + ((4 * total + 255) & ~size_t(255)) + 256;
    const size_t o_err = 0;
    const size_t o_outl = (24 * total + 255) & ~size_t(255);
    const size_t o_res = o_outl + ((total + 255) & ~size_t(255));
    const size_t io_bytes = o_res + sizeof(PoseOut) * nb + 256;
    char *pin = (char *)osg_pinned(ctx, in_bytes + io_bytes);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    std::memcpy(pin + o_probs, hp.data(), sizeof(PoseProbDev) * nb);
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
    hipLaunchKernelGGL(k_pose_opt, dim3(nb), dim3(PT), 0, ctx->stream, (const PoseProbDev *)(din + o_probs),
                       (const int8_t *)(din + o_kind), (const double *)(din + o_xw), (const double *)(din + o_obs),
                       (const float *)(din + o_isig), (double *)(dio + o_err), (uint8_t *)(dio + o_outl),
                       (PoseOut *)(dio + o_res));
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    char *pout = pin + in_bytes;
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(pout + o_outl, dio + o_outl, io_bytes - o_outl, hipMemcpyDeviceToHost,
                                      ctx->stream));
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
