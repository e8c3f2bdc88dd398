/*
 * osg.h — C ABI of the MI355X-native ORB-SLAM3 matching + bundle-adjustment hot path.
 *
 * This is the drop-in boundary.  Every entry point replaces one reference operator
 * (Herong1212/ORB_SLAM3_comments_ghr, cited as ref:<file>:<line>) and takes plain
 * pointers and sizes only — no torch, OpenCV, Eigen or Sophus types cross it.
 *
 *   osg_descriptor_distance*   ← ORBmatcher::DescriptorDistance       ref:src/ORBmatcher.cc:2388-2408
 *   osg_hamming_top2*          ← the top-2 candidate loop shared by every matcher
 *                                (brute force over a train set, semantics of
 *                                ref:src/ORBmatcher.cc:327-355: strict '<', first index wins ties,
 *                                sentinel distance 256, best index -1)
 *   osg_search_by_bow_kf_f     ← ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
 *                                ref:src/ORBmatcher.cc:262-496
 *   osg_search_by_bow_kf_kf    ← ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)
 *                                ref:src/ORBmatcher.cc:890-1043
 *   osg_search_by_projection_mps   ← ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFar)
 *                                ref:src/ORBmatcher.cc:44-242
 *   osg_search_by_projection_last  ← ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
 *                                ref:src/ORBmatcher.cc:1957-2191
 *   osg_search_by_projection_kf    ← ORBmatcher::SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)
 *                                ref:src/ORBmatcher.cc:2203-2330
 *   osg_fuse_search*           ← the search half of ORBmatcher::Fuse (both overloads)
 *                                ref:src/ORBmatcher.cc:1330-1541, 1553-1694
 *   osg_pose_optimization*     ← Optimizer::PoseOptimization(Frame*)   ref:src/Optimizer.cc:71-420
 *   osg_local_bundle_adjustment← Optimizer::LocalBundleAdjustment(...) ref:src/Optimizer.cc:1758-2206
 *                                (graph already gathered; g2o LM + BlockSolver_6_3 inner loop on device)
 *
 * Conventions
 *  - Functions return >= 0 on success (a match / inlier count where the reference returns one)
 *    or a negative OSG_E_* code.  Nothing throws across the ABI.
 *  - Host-pointer entry points copy inputs to device memory owned by the context, run, and copy
 *    the outputs back (the reference hands host memory in).  *_dev entry points take device
 *    pointers (inputs already resident in HBM) and run asynchronously on the context's stream.
 *  - One osg_ctx per host thread (the reference calls matchers concurrently from Tracking,
 *    LocalMapping and LoopClosing).  A context owns a HIP stream and pooled device scratch.
 *  - Descriptors are ORB rows: 32 bytes, row-major, as cv::Mat CV_8UC1 rows
 *    (ref:src/ORBextractor.cc:1538), read as 8 x int32 (ref:src/ORBmatcher.cc:2390-2391).
 */
#ifndef OSG_H
#define OSG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants (ref:src/ORBmatcher.cc:34-36, ref:include/Frame.h:44-45) ------------------- */
#define OSG_TH_HIGH 100
#define OSG_TH_LOW 50
#define OSG_HISTO_LENGTH 30
#define OSG_GRID_COLS 64
#define OSG_GRID_ROWS 48
#define OSG_GRID_CELLS (OSG_GRID_COLS * OSG_GRID_ROWS)
#define OSG_DESC_BYTES 32

/* ---- error codes --------------------------------------------------------------------------- */
#define OSG_OK 0
#define OSG_E_INVALID (-1)     /* bad argument / shape */
#define OSG_E_HIP (-2)         /* HIP runtime error */
#define OSG_E_NOMEM (-3)       /* device allocation failed */
#define OSG_E_UNSUPPORTED (-4) /* configuration not implemented */
#define OSG_E_NODEVICE (-5)    /* no gfx950 device visible */

typedef struct osg_ctx osg_ctx;

/* ---- context ------------------------------------------------------------------------------- */
int osg_ctx_create(int device, osg_ctx **out);
int osg_ctx_destroy(osg_ctx *ctx);
/* Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL restores the
 * context's own stream. */
int osg_ctx_set_stream(osg_ctx *ctx, void *hip_stream);
void *osg_ctx_stream(osg_ctx *ctx);
int osg_ctx_synchronize(osg_ctx *ctx);
const char *osg_strerror(int code);
const char *osg_ctx_last_error(osg_ctx *ctx);
/* Library build identifier, e.g. "osg 0.1 gfx950". */
const char *osg_version(void);

/* ---- a1: DescriptorDistance ---------------------------------------------------------------- */
/* Host scalar form (SWAR popcount of 8 x int32 XOR, ref:src/ORBmatcher.cc:2397-2405). */
int osg_descriptor_distance(const uint8_t *a, const uint8_t *b);
/* Row-pairwise distances on device: out[i] = DescriptorDistance(a[i], b[i]), i < n. */
int osg_descriptor_distance_pairs(osg_ctx *ctx, const uint8_t *a, const uint8_t *b, int32_t n,
                                  int32_t *out);

/* ---- a1+a2: brute-force top-2 --------------------------------------------------------------
 * For every query row q: best_idx[q] = the first train index (train order) with the minimum
 * distance, best_dist[q] = that distance, second_dist[q] = the second smallest distance counted
 * with multiplicity.  Sentinels: best_idx -1, distances 256 (train empty).  Exactly the
 * (bestDist1, bestIdx, bestDist2) of ref:src/ORBmatcher.cc:316-355 with every train row a
 * candidate.  nt <= 2^24. */
int osg_hamming_top2(osg_ctx *ctx, const uint8_t *query, int32_t nq, const uint8_t *train,
                     int32_t nt, int32_t *best_idx, int32_t *best_dist, int32_t *second_dist);
/* Device form: d_query/d_train/d_out are device pointers; d_out holds nq x int32[3]
 * {best_idx, best_dist, second_dist}.  Asynchronous on the context stream. */
int osg_hamming_top2_dev(osg_ctx *ctx, const void *d_query, int32_t nq, const void *d_train,
                         int32_t nt, void *d_out);

/* Frame-batched device form: nb independent problems of equal shape in one launch, problem b's
 * queries at rows [b*nq, (b+1)*nq) of d_query, its train set at rows [b*nt, (b+1)*nt) of d_train,
 * its results at rows [b*nq, (b+1)*nq) of d_out (nq x int32[3] each, as osg_hamming_top2_dev).
 * Every problem's result is exactly the serial loop's (same semantics as osg_hamming_top2); train
 * indices are problem-local.  nt <= 2^23, nb <= 65535.  Asynchronous on the context stream.
 * No reference counterpart: the frame-batched throughput form of the loop above (SURVEY.md §8(d)
 * C2, one 2000 x 2000 problem per frame). */
int osg_hamming_top2_batch_dev(osg_ctx *ctx, const void *d_query, int32_t nq, const void *d_train,
                               int32_t nt, int32_t nb, void *d_out);

/* Diagnostics: name and grid of the kernel osg_hamming_top2[_dev] would launch for (nq, nt) in
 * this process (the launch knobs are read once).  No reference counterpart. */
int osg_hamming_top2_plan(osg_ctx *ctx, int32_t nq, int32_t nt, char *name, int32_t len);

/* Diagnostics: name of the kernel osg_hamming_top2_batch_dev launches for (nq, nt, nb) in this process,
 * with its template shape and grid (e.g. "k_top2_fp4<16,1,256,1> grid=1024 x 1024").  No reference
 * counterpart. */
int osg_hamming_top2_batch_plan(osg_ctx *ctx, int32_t nq, int32_t nt, int32_t nb, char *name, int32_t len);

/* ---- frame view (SoA gather of ORB_SLAM3::Frame / KeyFrame fields) ----------------------------
 * Grid: ref:src/Frame.cc:469-507 (AssignFeaturesToGrid), cells in CSR with cell = ix*48 + iy and
 * items in insertion (ascending feature index) order, which is GetFeaturesInArea's candidate
 * enumeration order (ix outer, iy inner; ref:src/Frame.cc:922-957). */
typedef struct osg_frame {
    int32_t n;                  /* Frame::N (left + right keypoints for a two-camera rig) */
    int32_t nleft;              /* Frame::Nleft, -1 for mono / rectified stereo */
    const uint8_t *desc;        /* n x 32 */
    const float *kp_x;          /* mvKeysUn[i].pt.x (nleft == -1) / mvKeys, mvKeysRight */
    const float *kp_y;
    const float *kp_angle;      /* cv::KeyPoint::angle, same indexing */
    const int32_t *kp_octave;   /* cv::KeyPoint::octave, same indexing */
    const float *u_right;       /* mvuRight[n] (may be NULL: treated as all < 0) */
    const int32_t *grid_start;  /* OSG_GRID_CELLS + 1 offsets into grid_idx (left camera) */
    const int32_t *grid_idx;
    const int32_t *grid_start_r;/* right camera grid (nleft != -1), indices relative to nleft */
    const int32_t *grid_idx_r;
    const int32_t *left_to_right; /* mvLeftToRightMatch[nleft] or NULL */
    const int32_t *right_to_left; /* mvRightToLeftMatch[n - nleft] or NULL */
    float min_x, max_x, min_y, max_y; /* mnMinX, mnMaxX, mnMinY, mnMaxY */
    float grid_inv_w, grid_inv_h;     /* mfGridElementWidthInv, mfGridElementHeightInv */
    const float *scale_factors;       /* mvScaleFactors[n_levels] */
    int32_t n_levels;
    float mb, mbf;                    /* baseline (m), baseline * fx */
} osg_frame;

/* Slot state of the frame being matched into (Frame::mvpMapPoints):
 *   slot_mp[i]     in/out  caller's MapPoint id in slot i, -1 = NULL
 *   slot_taken[i]  in      1 if the slot's current MapPoint blocks matching
 *                          (SearchByProjection: mvpMapPoints[i] && Observations() > 0). */

/* ---- a5: SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints) -----
 * Query fields are those Frame::isInFrustum stored on each MapPoint (ref:src/Frame.cc:676-782). */
typedef struct osg_mp_queries {
    int32_t n;
    const int32_t *mp_id;          /* caller MapPoint id written into slot_mp on a match */
    const uint8_t *desc;           /* n x 32 : MapPoint::GetDescriptor() */
    const uint8_t *usable;         /* !isBad() */
    const uint8_t *has_obs;        /* Observations() > 0 (claimed slots then block later queries) */
    const uint8_t *in_view;        /* mbTrackInView */
    const float *proj_x, *proj_y;  /* mTrackProjX, mTrackProjY */
    const float *proj_xr;          /* mTrackProjXR (stereo ur check / right-camera x) */
    const float *view_cos;         /* mTrackViewCos */
    const int32_t *pred_level;     /* mnTrackScaleLevel */
    const float *track_depth;      /* mTrackDepth (bFarPoints filter) */
    /* right camera (nleft != -1) */
    const uint8_t *in_view_r;      /* mbTrackInViewR */
    const float *proj_yr;          /* mTrackProjYR */
    const float *view_cos_r;       /* mTrackViewCosR */
    const int32_t *pred_level_r;   /* mnTrackScaleLevelR */
} osg_mp_queries;

int osg_search_by_projection_mps(osg_ctx *ctx, const osg_frame *F, const osg_mp_queries *mps,
                                 float nnratio, float th, int far_points, float th_far_points,
                                 int32_t *slot_mp, const uint8_t *slot_taken);

/* ---- a6: SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono) ------------
 * Per LastFrame slot i with a non-outlier MapPoint the caller supplies the projection the
 * reference computes with Sophus/Eigen float math (ref:src/ORBmatcher.cc:1993-2009):
 * u, v = mpCamera->project(Tcw * x3Dw), invz = 1/x3Dc(2); valid = MapPoint present, not outlier.
 * For a two-camera rig also the right-camera projection (ref:src/ORBmatcher.cc:2096-2100). */
typedef struct osg_last_queries {
    int32_t n;                     /* LastFrame.N */
    const int32_t *mp_id;          /* LastFrame.mvpMapPoints[i] id, -1 = NULL */
    const uint8_t *desc;           /* n x 32 : MapPoint::GetDescriptor() */
    const uint8_t *valid;          /* pMP && !mvbOutlier[i] */
    const uint8_t *has_obs;        /* pMP->Observations() > 0 */
    const float *u, *v, *invz;     /* projection into CurrentFrame (left camera) */
    const float *u_r, *v_r;        /* projection into right camera (nleft != -1) */
    const int32_t *octave;         /* LastFrame keypoint octave (nLastOctave) */
    const float *angle;            /* LastFrame keypoint angle (kpLF) */
    float tlc_z;                   /* (Tlw * twc)(2): forward/backward test */
} osg_last_queries;

int osg_search_by_projection_last(osg_ctx *ctx, const osg_frame *CF, const osg_last_queries *last,
                                  float th, int mono, int check_orientation, int32_t *slot_mp,
                                  const uint8_t *slot_taken);

/* ---- a7: SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>& sAlreadyFound, th, ORBdist)
 * Per KF slot: valid = pMP && !isBad() && !sAlreadyFound.count(pMP) && uv inside image &&
 * dist3D inside [minDist, maxDist]; u, v and pred_level = PredictScale(dist3D, &F) are computed
 * by the caller (ref:src/ORBmatcher.cc:2238-2262).  A match requires an empty slot
 * (ref:src/ORBmatcher.cc:2272-2273). */
typedef struct osg_kf_queries {
    int32_t n;
    const int32_t *mp_id;
    const uint8_t *desc;
    const uint8_t *valid;
    const float *u, *v;
    const int32_t *pred_level;
    const float *angle;            /* pKF->mvKeysUn[i].angle */
} osg_kf_queries;

int osg_search_by_projection_kf(osg_ctx *ctx, const osg_frame *CF, const osg_kf_queries *kfq,
                                float th, int orb_dist, int check_orientation, int32_t *slot_mp);

/* ---- a3/a4: SearchByBoW -----------------------------------------------------------------------
 * DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>, ref:Thirdparty/DBoW2/DBoW2/FeatureVector.h:24)
 * as CSR: node_id[k] ascending, feature indices feat[node_start[k] .. node_start[k+1]). */
typedef struct osg_featvec {
    int32_t n_nodes;
    const uint32_t *node_id;
    const int32_t *node_start;     /* n_nodes + 1 */
    const int32_t *feat;
} osg_featvec;

typedef struct osg_bow_side {
    int32_t n;                     /* keypoints */
    int32_t nleft;                 /* -1, or NLeft for a two-camera rig */
    const uint8_t *desc;           /* n x 32 */
    const float *angle;            /* keypoint angle as indexed by the reference at that call */
    const int32_t *mp_id;          /* GetMapPointMatches(): id, -1 = NULL (Frame side: unused) */
    const uint8_t *mp_good;        /* pMP && !pMP->isBad() */
    osg_featvec fv;
} osg_bow_side;

/* out_mp[F.n]: MapPoint id matched to each Frame keypoint, -1 = NULL. Returns nmatches. */
int osg_search_by_bow_kf_f(osg_ctx *ctx, const osg_bow_side *kf, const osg_bow_side *f,
                           float nnratio, int check_orientation, int32_t *out_mp);
/* out_mp12[kf1.n]: KF2 MapPoint id matched to each KF1 keypoint, -1 = NULL. */
int osg_search_by_bow_kf_kf(osg_ctx *ctx, const osg_bow_side *kf1, const osg_bow_side *kf2,
                            float nnratio, int check_orientation, int32_t *out_mp12);

/* ---- batched forms ----------------------------------------------------------------------------
 * B independent problems (frames / keyframe pairs) in one launch, one workgroup each; the
 * throughput path for frame batches.  F / queries / sides are arrays of B
 * structs.  The per-problem slot / output arrays are concatenated in problem order: problem b's
 * starts at the sum of the sizes (frame n / kf1 n) of problems 0..b-1.  nmatches[b] receives what
 * the single form returns for problem b.  Returns OSG_OK or an error naming the problem. */
int osg_search_by_projection_mps_batch(osg_ctx *ctx, const osg_frame *F, const osg_mp_queries *mps, int32_t B,
                                       float nnratio, float th, int far_points, float th_far_points,
                                       int32_t *slot_mp, const uint8_t *slot_taken, int32_t *nmatches);
int osg_search_by_projection_last_batch(osg_ctx *ctx, const osg_frame *CF, const osg_last_queries *last, int32_t B,
                                        float th, int mono, int check_orientation, int32_t *slot_mp,
                                        const uint8_t *slot_taken, int32_t *nmatches);
int osg_search_by_projection_kf_batch(osg_ctx *ctx, const osg_frame *CF, const osg_kf_queries *kfq, int32_t B,
                                      float th, int orb_dist, int check_orientation, int32_t *slot_mp,
                                      int32_t *nmatches);
int osg_search_by_bow_kf_f_batch(osg_ctx *ctx, const osg_bow_side *kf, const osg_bow_side *f, int32_t B,
                                 float nnratio, int check_orientation, int32_t *out_mp, int32_t *nmatches);
int osg_search_by_bow_kf_kf_batch(osg_ctx *ctx, const osg_bow_side *kf1, const osg_bow_side *kf2, int32_t B,
                                  float nnratio, int check_orientation, int32_t *out_mp12, int32_t *nmatches);

/* ---- b1/b2: Fuse — the search half ------------------------------------------------------------
 *   gated = 1  Fuse(KeyFrame*, const vector<MapPoint*>&, th, bRight)         ref:src/ORBmatcher.cc:1330-1541
 *              (LocalMapping::SearchInNeighbors, ref:src/LocalMapping.cc:1021-1063)
 *   gated = 0  Fuse(KeyFrame*, Sophus::Sim3f&, const vector<MapPoint*>&, th,
 *              vector<MapPoint*>&)                                            ref:src/ORBmatcher.cc:1553-1694
 *              (LoopClosing; right = 0)
 * The caller applies the reference's pre-search filters per MapPoint (isBad, already in the KF,
 * negative depth, outside the image, dist3D outside [min, max] invariance, viewing angle > 60 deg)
 * and projects it with the KF camera (ref:src/ORBmatcher.cc:1366-1429).  The device does the rest
 * of the loop body up to the best candidate: KeyFrame::GetFeaturesInArea(u, v, th *
 * mvScaleFactors[pred_level], right) (ref:src/KeyFrame.cc:859-907), the level window
 * [pred_level - 1, pred_level], for gated = 1 the reprojection gate (chi2 7.8 with u_right[idx]
 * >= 0, else 5.99, times mvInvLevelSigma2[octave]; ref:src/ORBmatcher.cc:1452-1486), and the
 * minimum DescriptorDistance (strict '<': the first candidate in area order wins).
 * Outputs per MapPoint: best_idx = the KF keypoint index (right camera: nleft + i) when the best
 * distance is <= TH_LOW, else -1; best_dist = the best distance (256 when no candidate).  Returns
 * the number of best_idx >= 0.  The replace / add step that follows mutates the map and stays
 * with the caller, in MapPoint order (the results stay exact under it). */
typedef struct osg_fuse_queries {
    int32_t n;
    const uint8_t *desc;           /* n x 32: MapPoint::GetDescriptor() */
    const uint8_t *valid;          /* passed the pre-search filters */
    const float *u, *v;            /* pCamera->project(Tcw * p3Dw) */
    const float *ur;               /* u - mbf * invz (gated = 1; may be NULL when no keypoint has u_right >= 0) */
    const int32_t *pred_level;     /* MapPoint::PredictScale(dist3D, pKF) */
    const float *inv_level_sigma2; /* pKF->mvInvLevelSigma2[n_levels] (gated = 1) */
} osg_fuse_queries;

int osg_fuse_search(osg_ctx *ctx, const osg_frame *KF, const osg_fuse_queries *Q, float th, int right, int gated,
                    int32_t *best_idx, int32_t *best_dist);
/* B (KeyFrame, MapPoint list) problems in one launch (SearchInNeighbors fuses one list into ~20
 * neighbours).  Outputs concatenated in problem order by Q[b].n; nfused[b] as the single form. */
int osg_fuse_search_batch(osg_ctx *ctx, const osg_frame *KF, const osg_fuse_queries *Q, int32_t B, float th,
                          int right, int gated, int32_t *best_idx, int32_t *best_dist, int32_t *nfused);

/* ---- b7: Frame::ComputeStereoMatches -------------------------------------------------------------
 * ref:src/Frame.cc:1117-1373 (rectified stereo: the Frame constructor, ref:src/Frame.cc:165).  For
 * every left keypoint: the right keypoints listed on its row (vRowIndices: each right keypoint on
 * rows floor(y - 2 s) .. ceil(y + 2 s), s = mvScaleFactors[octave]), octave within +-1, uR inside
 * [uL - mbf / mb, uL]; the first minimum DescriptorDistance below TH_HIGH, accepted below
 * (TH_HIGH + TH_LOW) / 2; then the 11 x 11 SAD (cv::NORM_L1) over incR = -5..5 at the keypoint's
 * pyramid level, the parabola fit, the disparity range test, and finally the removal of every
 * match whose SAD is >= 1.5 * 1.4 * the median SAD.  Outputs mvuRight / mvDepth (-1 = none).
 * Images: the ORBextractor pyramids (mvImagePyramid[level], 8-bit, `step` bytes per row).  The
 * SAD patches must lie inside the level image: the reference's colRange/rowRange throw otherwise
 * (ORBextractor keeps keypoints EDGE_THRESHOLD = 19 px from the border, so they do); a keypoint
 * whose patch would leave the image gets no match here. */
typedef struct osg_image_pyramid {
    int32_t n_levels;
    int32_t on_device;            /* 1: data[l] are device addresses, read in place (rows / cols / step
                                     stay host arrays); 0: host images, packed and uploaded per call */
    const uint8_t *const *data;   /* per level: the top-left pixel */
    const int32_t *rows, *cols, *step;  /* step: bytes per row (>= cols) */
} osg_image_pyramid;

typedef struct osg_stereo_frame {
    int32_t n;                    /* left keypoints (mvKeys) */
    const float *x, *y;
    const int32_t *octave;
    const uint8_t *desc;          /* n x 32 (mDescriptors) */
    int32_t n_right;              /* mvKeysRight */
    const float *xr, *yr;
    const int32_t *octave_r;
    const uint8_t *desc_r;        /* n_right x 32 (mDescriptorsRight) */
    const float *scale_factors;   /* mvScaleFactors */
    const float *inv_scale_factors; /* mvInvScaleFactors */
    int32_t n_levels;
    float mb, mbf;
    osg_image_pyramid left, right;
} osg_stereo_frame;

/* u_right[n], depth[n] out.  Returns the matches kept (accepted, then not removed by the median cut). */
int osg_compute_stereo_matches(osg_ctx *ctx, const osg_stereo_frame *F, float *u_right, float *depth);
/* B frames in one launch; outputs concatenated by F[b].n; nmatches[b] per frame. */
int osg_compute_stereo_matches_batch(osg_ctx *ctx, const osg_stereo_frame *F, int32_t B, float *u_right,
                                     float *depth, int32_t *nmatches);

/* Frame::ComputeStereoFishEyeMatches (ref:src/Frame.cc:1546-1603; the KannalaBrandt8 two-camera Frame
 * constructor, :1523): BFMatcher(NORM_HAMMING).knnMatch(k = 2) of the left stereo rows [mono_left, n_left)
 * against the right stereo rows [mono_right, n_right), Lowe's ratio 0.7, KannalaBrandt8::TriangulateMatches
 * (ref:src/CameraModels/KannalaBrandt8.cpp:438-520) with mvLevelSigma2 of both octaves, depth > 0.0001f.
 * desc_*: n x 32 bytes; kp_*: n x (x, y) float; oct_*: n octaves; cam_*: fx fy cx cy k0 k1 k2 k3;
 * Rlr (row-major 3x3), tlr: mRlr, mtlr.  Outputs mvLeftToRightMatch[n_left], mvRightToLeftMatch[n_right],
 * mvDepth[n_left] (-1 unmatched), mvStereo3Dpoints[n_left x 3] (0 unmatched; the reference leaves them
 * uninitialised).  Returns nMatches (the matches kept) or a negative error. */
int osg_compute_stereo_fisheye_matches(osg_ctx *ctx, int32_t n_left, int32_t mono_left, const uint8_t *desc_left,
                                       const float *kp_left, const int32_t *oct_left, int32_t n_right,
                                       int32_t mono_right, const uint8_t *desc_right, const float *kp_right,
                                       const int32_t *oct_right, const float *level_sigma2, int32_t n_levels,
                                       const float *cam_left, const float *cam_right, const float *Rlr,
                                       const float *tlr, int32_t *left_to_right, int32_t *right_to_left,
                                       float *depth, float *points3d);

/* ---- b6: SearchForInitialization ------------------------------------------------------------------
 * ORBmatcher::SearchForInitialization(Frame &F1, Frame &F2, vector<cv::Point2f> &vbPrevMatched,
 * vector<int> &vnMatches12, windowSize)  ref:src/ORBmatcher.cc:735-878 (monocular initialisation,
 * ref:src/Tracking.cc:2956).  F1 / F2: monocular frames (mvKeysUn; F1's grid is not read).
 * prev_xy[2 * F1.n] in/out = vbPrevMatched; matches12[F1.n] out = vnMatches12.  The reference's
 * order-dependent state (vMatchedDistance skip, vnMatches21 steal, every accepted match counted in
 * the rotation histogram even if stolen later) is reproduced exactly.  Returns nmatches.
 * F2.n <= 8192. */
int osg_search_for_initialization(osg_ctx *ctx, const osg_frame *F1, const osg_frame *F2, float *prev_xy,
                                  int window_size, float nnratio, int check_orientation, int32_t *matches12);
/* B frame pairs in one launch; prev_xy / matches12 concatenated by F1[b].n. */
int osg_search_for_initialization_batch(osg_ctx *ctx, const osg_frame *F1, const osg_frame *F2, int32_t B,
                                        float *prev_xy, int window_size, float nnratio, int check_orientation,
                                        int32_t *matches12, int32_t *nmatches);

/* ---- b5: the Sim3 projections of LoopClosing -------------------------------------------------------
 *   SearchByProjection(KeyFrame*, Sophus::Sim3f& Scw, const vector<MapPoint*>&, vector<MapPoint*>& vpMatched,
 *                      th, ratioHamming)                                  ref:src/ORBmatcher.cc:498-621
 *   SearchByProjection(KeyFrame*, Sim3f&, vpPoints, vpPointsKFs, vpMatched, vpMatchedKF, th, ratioHamming)
 *                                                                         ref:src/ORBmatcher.cc:623-733
 * (ref:src/LoopClosing.cc:1062, 1091, 1368).  Queries are osg_fuse_queries (ur and inv_level_sigma2
 * unused): valid = !isBad() && not already in vpMatched && depth >= 0 && in image && dist3D inside
 * [min, max] invariance && PO.dot(Pn) >= 0.5 dist; u, v = the Sim3 projection; pred_level =
 * PredictScale (the caller's part, :528-572).  The device walks KeyFrame::GetFeaturesInArea(u, v,
 * th * mvScaleFactors[pred_level]) skipping taken slots and keypoints outside [pred_level - 1,
 * pred_level], keeps the first minimum distance and accepts it iff bestDist <= TH_LOW * ratioHamming
 * (float); the accepted slot is taken for every later MapPoint (sequential greedy, solved exactly).
 * slot_query[KF.n] in: -2 = vpMatched[i] != NULL, -1 = free; out: the query index that took the
 * slot (the caller writes vpMatched[i] = vpPoints[q], and vpMatchedKF[i] = vpPointsKFs[q]).
 * Returns nmatches.  KF.n <= 8192. */
int osg_search_by_projection_sim3(osg_ctx *ctx, const osg_frame *KF, const osg_fuse_queries *Q, float th,
                                  float ratio_hamming, int32_t *slot_query);
int osg_search_by_projection_sim3_batch(osg_ctx *ctx, const osg_frame *KF, const osg_fuse_queries *Q, int32_t B,
                                        float th, float ratio_hamming, int32_t *slot_query, int32_t *nmatches);

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, S12, th)   ref:src/ORBmatcher.cc:1696-1939
 * (LoopClosing::DetectCommonRegionsFromBoW / DetectAndReffineSim3FromLastKF, ref:include/ORBmatcher.h:78).
 * q12: one query per KF1 keypoint: KF1's MapPoint in that slot projected into KF2 by S21 * T1w
 * (u, v, PredictScale(dist3D, pKF2)); valid = a MapPoint that is not already in vpMatches12, not
 * bad, in front of KF2, inside its image and within its distance-invariance range (:1737-1772).
 * q21: one query per KF2 keypoint, KF2's MapPoints into KF1 by S12 * T2w (:1813-1850).  Each query
 * takes the first minimum-distance keypoint of its window (KeyFrame::GetFeaturesInArea, levels
 * [pred - 1, pred]) when that distance <= TH_HIGH; match12[i1] = idx2 for the mutual pairs
 * (vnMatch2[vnMatch1[i1]] == i1), else -1: the caller sets vpMatches12[i1] = vpMapPoints2[idx2].
 * Returns nFound (>= 0) or an OSG_E_* code.  Descriptor, u/v and pred_level are read for valid
 * queries only; ur / inv_level_sigma2 are not used. */
int osg_search_by_sim3(osg_ctx *ctx, const osg_frame *kf1, const osg_frame *kf2, const osg_fuse_queries *q12,
                       const osg_fuse_queries *q21, float th, int32_t *match12);

/* ---- b3: SearchForTriangulation ---------------------------------------------------------------
 * ORBmatcher::SearchForTriangulation(KeyFrame *pKF1, KeyFrame *pKF2, vector<pair<size_t,size_t>>&,
 * bOnlyStereo, bCoarse)  ref:src/ORBmatcher.cc:1045-1328 (LocalMapping::CreateNewMapPoints,
 * ref:src/LocalMapping.cc:630).  For every KF1 keypoint without a MapPoint in a vocabulary node
 * shared with KF2: the KF2 keypoint of the same node without a MapPoint that minimises the distance
 * (<= TH_LOW; '<=' so the LAST of equal distances in node order wins, ref:src/ORBmatcher.cc:1180),
 * passing the epipole-distance test (both keypoints monocular, no second camera,
 * ref:src/ORBmatcher.cc:1189-1203) and, unless bCoarse, Pinhole::epipolarConstrain
 * (ref:src/CameraModels/Pinhole.cpp:189-219).  Then the rotation histogram + ComputeThreeMaxima.
 * In this fork vbMatched2[bestIdx2] = true is commented out (ref:src/ORBmatcher.cc:1262), so KF1
 * keypoints never compete for a KF2 keypoint: every query is independent. */
typedef struct osg_kf_side {
    int32_t n;                  /* KeyFrame::N */
    int32_t nleft;              /* NLeft, -1 without a two-camera rig */
    int32_t two_cam;            /* mpCamera2 != NULL */
    const uint8_t *desc;        /* n x 32 */
    const float *kp_x, *kp_y;   /* (NLeft == -1) ? mvKeysUn : idx < NLeft ? mvKeys : mvKeysRight[idx - NLeft] */
    const float *kp_angle;
    const int32_t *kp_octave;
    const float *u_right;       /* mvuRight[n] (NULL: all < 0) */
    const uint8_t *has_mp;      /* GetMapPoint(i) != NULL */
    const float *level_sigma2;  /* mvLevelSigma2[n_levels] */
    const float *scale_factors; /* mvScaleFactors[n_levels] */
    int32_t n_levels;
    osg_featvec fv;             /* mFeatVec */
} osg_kf_side;

/* The two-view geometry the reference computes with Sophus / Eigen before its loop
 * (ref:src/ORBmatcher.cc:1052-1083), supplied by the caller so the float values are the reference's
 * own.  F12[k] = K1^-T * [t12]x * R12 * K2^-1 (Pinhole.cpp:194-197), row-major, for the camera pair
 * k = 2 * bRight1 + bRight2 (ll, lr, rl, rr: T12 = Tll, Tlr, Trl, Trr, ref:src/ORBmatcher.cc:1205-1244);
 * only F12[0] is read without a rig.  pinhole = 0: KannalaBrandt8::epipolarConstrain (ref:src/
 * CameraModels/KannalaBrandt8.cpp:321-326 -> TriangulateMatches :438-489), which reads, for the camera
 * pair k, R12[k] / t12[k] (the Rll/tll, Rlr/tlr, Rrl/trl, Rrr/trr of :1205-1244; R12 row-major) and
 * the cameras' parameters kb[c] = {fx, fy, cx, cy, k0, k1, k2, k3}: kb[0] = pKF1->mpCamera,
 * kb[1] = pKF1->mpCamera2, kb[2] = pKF2->mpCamera, kb[3] = pKF2->mpCamera2 (only [0] and [2] are read
 * without a rig).  The triangulation's 4x4 JacobiSVD null vector is taken as the smallest-eigenvalue
 * eigenvector of A^T A (cyclic Jacobi, double) and atan2f / tanf / cosf / sinf by fixed
 * double-precision kernels rounded to float: parity with Eigen / libm is unpinned at the last ulp. */
typedef struct osg_triang_geom {
    float ep_x, ep_y;           /* pKF2->mpCamera->project(T2w * pKF1->GetCameraCenter()) */
    float F12[4][9];
    int32_t pinhole;
    float R12[4][9];            /* KannalaBrandt8 only */
    float t12[4][3];
    float kb[4][8];
} osg_triang_geom;

/* match12[kf1.n]: KF2 keypoint index per KF1 keypoint (vMatches12 after the histogram), -1 = none.
 * vMatchedPairs = the (i, match12[i] >= 0) in ascending i.  Returns nmatches. */
int osg_search_for_triangulation(osg_ctx *ctx, const osg_kf_side *kf1, const osg_kf_side *kf2,
                                 const osg_triang_geom *geom, int only_stereo, int coarse,
                                 int check_orientation, int32_t *match12);
/* B keyframe pairs in one launch (CreateNewMapPoints: the new keyframe against its ~10-20
 * neighbours).  match12 concatenated in problem order by kf1[b].n; nmatches[b] as the single form. */
int osg_search_for_triangulation_batch(osg_ctx *ctx, const osg_kf_side *kf1, const osg_kf_side *kf2,
                                       const osg_triang_geom *geom, int32_t B, int only_stereo, int coarse,
                                       int check_orientation, int32_t *match12, int32_t *nmatches);

/* ---- b4: MapPoint::ComputeDistinctiveDescriptors ------------------------------------------------
 * ref:src/MapPoint.cc:444-535, for a list of MapPoints at once (LocalMapping runs it for every MapPoint
 * of a keyframe, ref:src/LocalMapping.cc:421-436, 1066-1082).  MapPoint p's observation descriptors
 * are rows desc[start[p] .. start[p+1]) in the order the reference gathers them (mObservations
 * std::map order; per keyframe the left row, then the right row).  best_idx[p] = the row whose
 * sorted distance row (self-distance 0 included) has the smallest element [(N - 1) / 2], first row
 * on ties; -1 when N = 0 (the reference returns without touching mDescriptor).  N <= 65535. */
int osg_compute_distinctive_descriptors(osg_ctx *ctx, const uint8_t *desc, const int32_t *start, int32_t n_points,
                                        int32_t *best_idx);
/* Device form: d_desc (rows), d_start (n_points + 1), d_best_idx (n_points) in HBM; asynchronous. */
int osg_compute_distinctive_descriptors_dev(osg_ctx *ctx, const void *d_desc, const void *d_start, int32_t n_points,
                                            void *d_best_idx);

/* ---- b8: ORBextractor's per-keypoint stages --------------------------------------------------------
 * computeOrientation / IC_Angle (ref:src/ORBextractor.cc:89-136, 585-597) on mvImagePyramid[level] and
 * computeDescriptors / computeOrbDescriptor (ref:src/ORBextractor.cc:148-208, 1534-1545) on the
 * GaussianBlur'd level (ref:src/ORBextractor.cc:1628-1652), for keypoints in level coordinates (before
 * :1663-1667 scales them to level 0), e.g. from osg_orb_detect (b9).  The 7x7 Gaussian blur is
 * the caller's (OpenCV) or osg_orb_pyramid's (b10).  umax: the extractor's umax (HALF_PATCH_SIZE + 1 = 16 entries, each
 * <= 15); pattern: its 512 points (ORBextractor::pattern) as (x, y) int pairs.  The orientation box
 * (+-15 around the rounded centre) must lie inside the raw level, else OSG_E_INVALID.  The blurred
 * level is read as the reference's continuous clone (workingMat = mvImagePyramid[level].clone(),
 * :1628): offsets are linear with step = cols, so a point left of column 0 reads the previous row's
 * end; device-resident blurred levels must therefore have step == cols.  A point outside the whole
 * level buffer (the reference reads foreign heap there) reads 0.  fastAtan2 is OpenCV's (not
 * in the reference tree: its published polynomial is restated; parity with OpenCV itself
 * unpinned).  cos / sin of the angle are the host libm's cosf / sinf (the reference's std::cos(float)),
 * evaluated between the two kernels so that they agree with it bit for bit. */
typedef struct osg_orb_keypoints {
    int32_t n;
    const float *x, *y;           /* level coordinates (KeyPoint::pt before the level scale) */
    const int32_t *level;         /* KeyPoint::octave */
} osg_orb_keypoints;

/* angle[n]: written (IC_Angle) when compute_angle, else read (the keypoints' angles in degrees);
 * desc[n x 32] written.  Returns the number of keypoints that read outside their level's buffer. */
int osg_orb_describe(osg_ctx *ctx, const osg_image_pyramid *raw, const osg_image_pyramid *blurred,
                     const osg_orb_keypoints *K, const int32_t *pattern, const int32_t *umax, int32_t compute_angle,
                     float *angle, uint8_t *desc);

/* ---- b9: ORBextractor::ComputeKeyPointsOctTree --------------------------------------------------
 * ref:src/ORBextractor.cc:1065-1198 with DistributeOctTree (:716-1050), ExtractorNode::DivideNode
 * (:607-654) and compareNodes (:656-676): per level, W = 35 cells over [EDGE_THRESHOLD - 3,
 * size - EDGE_THRESHOLD + 3), each cell FAST'd as its own image (rowRange / colRange) with
 * ini_th_fast and, when that finds nothing, min_th_fast (cv::FAST with non-maximum suppression:
 * OpenCV's FAST_t<16> / cornerScore<16>, restated; not in the reference tree, so parity with OpenCV
 * itself is unpinned), then the quadtree distribution down to n_features_per_level[level]
 * (mnFeaturesPerLevel) keypoints.  Out, level by level in the reference's allKeypoints order:
 * x, y in level coordinates (after the :1190-1196 shift by the border), response (the FAST score),
 * size = (int)(PATCH_SIZE * scale_factors[level]) (mvScaleFactor); level_start[n_levels + 1].
 * Orientation and descriptors follow through osg_orb_describe.  Returns the keypoint count, or
 * OSG_E_INVALID when it exceeds `capacity` or a level is smaller than one cell. */
int osg_orb_detect(osg_ctx *ctx, const osg_image_pyramid *raw, int32_t ini_th_fast, int32_t min_th_fast,
                   const int32_t *n_features_per_level, const float *scale_factors, int32_t capacity,
                   float *x, float *y, float *response, float *size, int32_t *level_start);
/* Diagnostics: the host DistributeOctTree of osg_orb_detect alone, on nk keypoints given as (x, y,
 * response, unused) float quadruples relative to (minX, minY); kept keypoints out the same way.
 * Returns the count (no context, no GPU). */
int osg_debug_distribute_oct_tree(const float *keys4, int32_t nk, int32_t minX, int32_t maxX, int32_t minY,
                                  int32_t maxY, int32_t N, float *out4, int32_t cap);

/* ---- b10: ORBextractor::ComputePyramid + the GaussianBlur of operator() -----------------------------
 * ComputePyramid (ref:src/ORBextractor.cc:1692-1743): level l is cvRound((float)cols *
 * mvInvScaleFactor[l]) x cvRound((float)rows * ...), level 0 the image, level l >= 1 cv::resize
 * (INTER_LINEAR) of level l - 1; each level with a copyMakeBorder(EDGE_THRESHOLD = 19,
 * BORDER_REFLECT_101) border around it.  With blur, also each level's GaussianBlur(Size(7, 7), 2, 2,
 * BORDER_REFLECT_101) as operator() computes it on the level's clone (:1628-1636).  Both are OpenCV
 * calls (not in the reference tree): their 8-bit fixed-point algorithms are restated (OpenCV 4.5+,
 * no IPP; see oracle/oracle_pyramid.c), so parity with OpenCV itself is unpinned.
 * osg_orb_pyramid_layout (host only, no context): the level sizes and the byte offsets of each
 * bordered level ((rows + 38) x (cols + 38), row step cols + 38; mvImagePyramid[l] is the ROI at
 * (19, 19)) and each blurred level (rows x cols, step cols) in one buffer; returns its size in
 * bytes, or OSG_E_INVALID.  osg_orb_pyramid fills such a device buffer (dev_out, dev_bytes) from a
 * host image (image_on_device = 0; any row step) or a device one, on the context's stream, and
 * returns when it is complete.  The levels then feed osg_orb_detect (raw), osg_orb_describe (raw +
 * blurred) and osg_compute_stereo_matches as on_device pyramids.  n_levels <= 32. */
int64_t osg_orb_pyramid_layout(int32_t rows, int32_t cols, int32_t n_levels, const float *inv_scale_factors,
                               int32_t *level_rows, int32_t *level_cols, int64_t *bordered_offset,
                               int64_t *blurred_offset);
int osg_orb_pyramid(osg_ctx *ctx, const uint8_t *image, int32_t rows, int32_t cols, int32_t step,
                    int32_t image_on_device, int32_t n_levels, const float *inv_scale_factors, uint8_t *dev_out,
                    int64_t dev_bytes, int32_t blur);
/* ---- b11: ORBextractor::operator() for a batch of images -------------------------------------------
 * ref:src/ORBextractor.cc:1553-1690 (operator(): ComputePyramid, ComputeKeyPointsOctTree, the per-level
 * GaussianBlur, computeOrientation and computeDescriptors) for n_images device images of one size
 * (d_images, image_stride bytes apart, row step `step`), each image exactly as osg_orb_pyramid ->
 * osg_orb_detect -> osg_orb_describe(compute_angle = 1) produce it, with a handful of launches for the
 * whole batch (the pyramid levels, one FAST pass, one cell pass, one angle and one descriptor pass)
 * and the octrees of all (image, level) pairs on host threads.  Outputs per image b at offset
 * b * capacity: x, y in level coordinates (KeyPoint::pt before the :1663-1667 level-0 scaling),
 * angle (degrees), response, size, octave, desc (32 bytes each); counts[b] = image b's keypoints.
 * Returns the keypoints of all images, or a negative OSG_E_* code. */
typedef struct osg_orb_extract_params {
    int32_t n_levels;                      /* nlevels (<= 32) */
    const float *scale_factors;            /* mvScaleFactor */
    const float *inv_scale_factors;        /* mvInvScaleFactor */
    const int32_t *n_features_per_level;   /* mnFeaturesPerLevel */
    int32_t ini_th_fast, min_th_fast;      /* iniThFAST, minThFAST */
    const int32_t *pattern;                /* the 512 (x, y) BRIEF points */
    const int32_t *umax;                   /* 16 entries */
} osg_orb_extract_params;
int osg_orb_extract_batch(osg_ctx *ctx, const uint8_t *d_images, int64_t image_stride, int32_t rows, int32_t cols,
                          int32_t step, int32_t n_images, const osg_orb_extract_params *params, int32_t capacity,
                          float *x, float *y, float *angle, float *response, float *size, int32_t *octave,
                          uint8_t *desc, int32_t *counts);

/* Diagnostics: the 7-tap fixed-point kernel (8 fraction bits) osg_orb_pyramid blurs with. */
void osg_debug_gaussian_kernel7(int32_t *k7);

/* Diagnostics of the last search call on this context (summed / maxed over a batch): out[0]
 * candidates enumerated, out[1] Jacobi rounds, out[2] problems whose greedy was redone serially (a5 on a two-camera rig when a
 * stereo-partner write by a MapPoint without observations unblocked a slot), out[3] nmatches.
 * No reference counterpart. */
int osg_match_last_stats(osg_ctx *ctx, int32_t *out4);
/* Device time (HIP events around the launch, ms) of the last matching or pose-optimization kernel
 * this context ran: the search calls and osg_pose_optimization[_batch]. */
int osg_ctx_last_kernel_ms(osg_ctx *ctx, double *ms);
/* Device memory this context holds (its scratch arena: every slot grows to the largest call so far and
 * stays), bytes.  No reference counterpart. */
int osg_ctx_device_bytes(osg_ctx *ctx, int64_t *bytes);

#ifdef __cplusplus
}
#endif
#endif /* OSG_H */
