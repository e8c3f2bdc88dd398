/*
 * osg_ba.h — C ABI of the bundle-adjustment half of the hot path.
 *
 *   osg_pose_optimization[_batch]  ← Optimizer::PoseOptimization(Frame*)        ref:src/Optimizer.cc:71-420
 *   osg_local_bundle_adjustment    ← the g2o part of Optimizer::LocalBundleAdjustment
 *                                    (ref:src/Optimizer.cc:1877-2203: graph → optimize(10) →
 *                                    outlier classification → estimates out)
 *   osg_bundle_adjustment          ← the g2o part of Optimizer::BundleAdjustment (global BA,
 *                                    ref:src/Optimizer.cc:2850-3237)
 *
 * The caller (the ORB-SLAM3 side adapter) gathers the graph exactly as the
 * reference builds it — the same vertices, the same edges in the same insertion order, the same
 * float→double casts — and applies the returned estimates / outlier flags under the reference's
 * locks.  Inside, the g2o LM + BlockSolver_6_3 semantics are reproduced:
 * ref:Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-194,
 * ref:Thirdparty/g2o/g2o/core/block_solver.hpp:143-604, ref:Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:61-552.
 *
 * Poses are SE3 as 7 doubles {qx, qy, qz, qw, tx, ty, tz} (g2o::SE3Quat; Tcw = world→camera).
 */
#ifndef OSG_BA_H
#define OSG_BA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct osg_ctx;

/* camera model, ref:include/CameraModels/GeometricCamera.h:115 (vector<float> mvParameters) */
#define OSG_CAM_PINHOLE 0 /* ref:src/CameraModels/Pinhole.cpp:50-133 */
#define OSG_CAM_KB8 1     /* ref:src/CameraModels/KannalaBrandt8.cpp:62-260 */

/* edge kinds (ref:include/OptimizableTypes.h:32-158, ref:Thirdparty/g2o/g2o/types/types_six_dof_expmap.h:146-235) */
#define OSG_EDGE_MONO 0   /* EdgeSE3ProjectXYZ[OnlyPose]: 2-D, pCamera->project */
#define OSG_EDGE_STEREO 1 /* EdgeStereoSE3ProjectXYZ[OnlyPose]: 3-D (u, v, ur), fx fy cx cy bf */
#define OSG_EDGE_BODY 2   /* EdgeSE3ProjectXYZ[OnlyPose]ToBody: 2-D, right camera through mTrl */

typedef struct osg_camera {
    int32_t type;        /* OSG_CAM_* */
    float p[8];          /* mvParameters: fx fy cx cy [k1 k2 k3 k4] */
    float fx, fy, cx, cy, bf; /* Frame/KeyFrame fx..mbf (stereo edges copy these into doubles) */
    double trl[7];       /* right-from-left SE3 (GetRelativePoseTrl) for BODY edges */
} osg_camera;

/* ---- PoseOptimization ---------------------------------------------------------------------- */
typedef struct osg_pose_problem {
    double pose[7];           /* pFrame->GetPose() cast to double */
    int32_t n_edges;          /* one per Frame slot with a MapPoint, in slot order */
    const int8_t *kind;       /* OSG_EDGE_* per edge */
    const double *xw;         /* 3 per edge: GetWorldPos().cast<double>() */
    const double *obs;        /* 3 per edge: (u, v, ur) — ur only read for STEREO */
    const float *inv_sigma2;  /* mvInvLevelSigma2[octave] per edge */
    osg_camera cam;           /* mpCamera + stereo parameters */
    osg_camera cam2;          /* mpCamera2 + mTrl (BODY edges) */
} osg_pose_problem;

typedef struct osg_pose_result {
    double pose[7];           /* optimised Tcw (input pose when fewer than 3 edges) */
    uint8_t *outlier;         /* n_edges flags (mvbOutlier of each edge's slot) */
    int32_t n_inliers;        /* the reference's return value: nInitial - nBad */
    int32_t lm_iterations;    /* solve() calls over the 4 rounds */
    int32_t lm_trials;        /* linear solves (incl. rejected steps) */
} osg_pose_result;

int osg_pose_optimization(struct osg_ctx *ctx, const osg_pose_problem *p, osg_pose_result *r);
/* n independent frames in one launch (frame-batched tracking, sequences sharded over GPUs). */
int osg_pose_optimization_batch(struct osg_ctx *ctx, const osg_pose_problem *p, int32_t n,
                                osg_pose_result *r);

/* ---- LocalBundleAdjustment ------------------------------------------------------------------
 * Vertices are given sorted by g2o vertex id (KeyFrames: mnId; MapPoints: mnId + maxKFid + 1),
 * which fixes the Hessian index order (ref:Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:181-211,
 * 547-552).  Edges are given in insertion order (internalId order). */
typedef struct osg_ba_graph {
    int32_t n_poses;
    const double *pose;        /* 7 per pose */
    const uint8_t *pose_fixed; /* setFixed(...) */
    int32_t n_points;
    const double *point;       /* 3 per point (marginalised) */
    int32_t n_edges;
    const int32_t *e_point;    /* point index per edge (vertex 0) */
    const int32_t *e_pose;     /* pose index per edge (vertex 1) */
    const int8_t *e_kind;      /* OSG_EDGE_* */
    const int32_t *e_cam;      /* index into cams */
    const double *e_obs;       /* 3 per edge */
    const float *e_inv_sigma2;
    int32_t n_cams;
    const osg_camera *cams;
    int32_t iterations;        /* optimize(iterations): 10 in LocalBundleAdjustment */
    double user_lambda_init;   /* 0 → tau·max(diag H); 100 when the map is inertial */
    /* Huber kernels.  Zero-initialised these are LocalBundleAdjustment's: every edge robust, deltas
     * thHuberMono = sqrt(5.991) (mono and body) / thHuberStereo = sqrt(7.815) as floats
     * (ref:src/Optimizer.cc:1951-1952).  BundleAdjustment (ref:src/Optimizer.cc:2933-2934, 3000-3007,
     * 3041-3047, 3083-3085) uses sqrt(5.99) / sqrt(7.815) and attaches them to mono / stereo edges
     * only when bRobust (body edges always). */
    const uint8_t *e_robust;   /* per edge: a Huber kernel attached (NULL: every edge) */
    float huber_mono, huber_stereo; /* the deltas as stored by the reference (0: the LBA values) */
} osg_ba_graph;

typedef struct osg_ba_result {
    double *pose;              /* 7 per pose (fixed poses returned unchanged) */
    double *point;             /* 3 per point */
    uint8_t *edge_bad;         /* chi2 > 5.991 (mono/body) / 7.815 (stereo) || !isDepthPositive() */
    int32_t iterations;        /* LM solve() calls executed */
    int32_t trials;            /* linear solves incl. rejected steps */
    double chi2_initial;       /* activeRobustChi2 before the first iteration */
    double chi2_final;         /* activeRobustChi2 of the accepted state */
    int32_t aborted;           /* stop flag observed */
    double *edge_chi2;         /* optional (NULL: not written): per edge e'Ωe of its last computed error, the
                                  e->chi2() the classification reads (the merge BA's second pass needs it) */
} osg_ba_result;

/* stop_flag: the reference's bool *pbStopFlag read as one byte (nonzero = stop), polled between LM
 * iterations and trials (may be NULL). */
int osg_local_bundle_adjustment(struct osg_ctx *ctx, const osg_ba_graph *g, osg_ba_result *r,
                                const volatile uint8_t *stop_flag);

/* Optimizer::BundleAdjustment / GlobalBundleAdjustemnt (ref:src/Optimizer.cc:2831-3237): the same
 * engine on the whole map — every KeyFrame (only the map's init KeyFrame fixed), every MapPoint with
 * an edge, optimize(nIterations) with the caller's e_robust / Huber deltas, no outlier pass (edge_bad
 * is filled but the reference does not read it).  The reduced camera system is dense up to 64 free
 * KeyFrames; past that it is stored and factored on its envelope (banded maps and their loop rows).
 * Tested up to about 9 000 free KeyFrames (tests/test_ba_gpu.py::test_gba_9000_kf_loop_map_accepted,
 * no parity check at that size; parity is checked on the 1 500-KF maps).  The host structure build
 * still fills two dense pose-pair tables of nhp (nhp + 1) / 2 int32 entries each (about 160 MB each at
 * 9 000 KF, 8.6 GB each at 65 535) and walks every pair, so host memory and build time grow with nhp^2
 * (DESIGN.md §3.11). */
int osg_bundle_adjustment(struct osg_ctx *ctx, const osg_ba_graph *g, osg_ba_result *r,
                          const volatile uint8_t *stop_flag);

/* Batched form: n_graphs independent windows (e.g. the LocalMapping windows of several maps or
 * sequences) optimised in lockstep, every kernel launched once per LM trial for all of them; each
 * graph follows exactly the single-graph LM (its own lambda, accept / reject, stop rules).
 * Whole-map graphs (osg_bundle_adjustment's) are accepted too: bench.py's global_ba line runs 16
 * independent maps per batch.  Returns the summed LM iterations or a negative OSG_E_* code.  No
 * reference counterpart. */
int osg_local_bundle_adjustment_batch(struct osg_ctx *ctx, const osg_ba_graph *graphs, int32_t n_graphs,
                                      osg_ba_result *results, const volatile uint8_t *stop_flag);

/* Diagnostics: per-kernel device time of the LBA / BA engine.  enable = 1 starts timing every
 * kernel of every lockstep step with HIP events on the context's stream (and clears the sums);
 * 0 stops.  ms[OSG_LBA_NK] and steps[OSG_LBA_NK] (either may be NULL) receive the summed time and
 * the number of timed launch groups since the last enable, indexed errors, linearize, pose_red,
 * lambda_init, schur_point, schur_rows, schur_pairs, chol (every k_chol_col + k_chol_trail of a
 * step), chol_back, update, step_reduce, classify. */
#define OSG_LBA_NK 12
int osg_lba_kernel_times(struct osg_ctx *ctx, int32_t enable, double *ms, int64_t *steps);

#ifdef __cplusplus
}
#endif
#endif
