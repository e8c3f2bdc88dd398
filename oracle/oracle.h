/* oracle.h — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY (see
 * oracle_match.c / oracle_ba.c headers).  Never linked into the product library. */
#ifndef OSG_ORACLE_H
#define OSG_ORACLE_H
#include <stdint.h>
#include "../include/osg.h"
#include "../include/osg_ba.h"
#include "../include/osg_dbow.h"

#ifdef __cplusplus
extern "C" {
#endif

int oracle_descriptor_distance(const uint8_t *a, const uint8_t *b);
void oracle_hamming_top2(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *best_idx,
                         int32_t *best_dist, int32_t *second_dist);
void oracle_hamming_top2_mt(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *best_idx,
                            int32_t *best_dist, int32_t *second_dist, int nthreads);
int oracle_frame_features_in_area(const osg_frame *F, float x, float y, float r, int minLevel,
                                  int maxLevel, int bRight, int32_t *out);
void oracle_compute_three_maxima(const int *histo_size, int L, int *ind1, int *ind2, int *ind3);
int oracle_rot_bin(float angle_a, float angle_b);
int oracle_search_by_projection_mps(const osg_frame *F, const osg_mp_queries *Q, float nnratio,
                                    float th, int bFarPoints, float thFarPoints, int32_t *slot_mp,
                                    const uint8_t *slot_taken_in);
int oracle_search_by_projection_last(const osg_frame *CF, const osg_last_queries *L, float th,
                                     int bMono, int checkOri, int32_t *slot_mp,
                                     const uint8_t *slot_taken_in);
int oracle_search_by_projection_kf(const osg_frame *CF, const osg_kf_queries *K, float th,
                                   int ORBdist, int checkOri, int32_t *slot_mp);
int oracle_search_by_bow_kf_f(const osg_bow_side *KF, const osg_bow_side *F, float nnratio,
                              int checkOri, int32_t *out_mp);
int oracle_search_by_bow_kf_kf(const osg_bow_side *K1, const osg_bow_side *K2, float nnratio,
                               int checkOri, int32_t *out_mp12);

/* DBoW2 vocabulary transform (oracle_dbow.c) */
void oracle_dbow_transform(const osg_vocabulary_desc *V, const uint8_t *desc, int n, int levelsup, osg_bow_out *out);
/* Fuse search half (oracle_fuse.c) */
int oracle_fuse_search(const osg_frame *KF, const osg_fuse_queries *Q, float th, int right, int gated,
                       int32_t *best_idx, int32_t *best_dist);
/* SearchForInitialization (oracle_init.c); prev_xy in/out */
int oracle_search_for_initialization(const osg_frame *F1, const osg_frame *F2, float *prev_xy, int windowSize,
                                     float mfNNratio, int checkOri, int32_t *vnMatches12);
/* Sim3 projections of LoopClosing (oracle_sim3.c); slot_query as osg_search_by_projection_sim3 */
int oracle_search_by_projection_sim3(const osg_frame *KF, const osg_fuse_queries *Q, float th, float ratioHamming,
                                     int32_t *slot_query);
/* KannalaBrandt8::epipolarConstrain / unproject / project as SearchForTriangulation uses them (oracle_triang.c) */
int oracle_kb8_epipolar_constrain(const float *cam1, const float *cam2, float x1, float y1, float x2, float y2,
                                  const float *R12, const float *t12, float sigmaLevel, float unc);
void oracle_kb8_unproject(const float *cam, float u, float v, float *r);
void oracle_kb8_project(const float *cam, const float *X, float *uv);
/* ORBmatcher::SearchBySim3 (oracle_sim3.c) */
int oracle_search_by_sim3(const osg_frame *KF1, const osg_frame *KF2, const osg_fuse_queries *Q12,
                          const osg_fuse_queries *Q21, float th, int32_t *match12);
/* MapPoint::ComputeDistinctiveDescriptors over a list (oracle_desc.c) */
void oracle_compute_distinctive_descriptors(const uint8_t *desc, const int32_t *start, int n_points, int32_t *best_idx);
/* SearchForTriangulation (oracle_triang.c) */
int oracle_search_for_triangulation(const osg_kf_side *K1, const osg_kf_side *K2, const osg_triang_geom *G,
                                    int bOnlyStereo, int bCoarse, int checkOri, int32_t *vMatches12);
/* Frame::ComputeStereoMatches (oracle_stereo.c): mvuRight / mvDepth out, returns the kept matches */
int oracle_compute_stereo_matches(const osg_stereo_frame *F, float *mvuRight, float *mvDepth);

/* ORBextractor IC_Angle + computeOrbDescriptor (oracle_orb.c): the keypoints whose descriptor reads
 * leave their level's buffer, or -(k + 1) for the first keypoint k whose orientation box leaves it */
float oracle_fast_atan2(float y, float x);
int oracle_orb_describe(const osg_image_pyramid *raw, const osg_image_pyramid *blurred, const osg_orb_keypoints *K,
                        const int32_t *pattern, const int32_t *umax, int compute_angle, float *angle, uint8_t *desc);
void oracle_dbow_transform_batch(const osg_vocabulary_desc *V, const uint8_t *desc, const int32_t *n, int B,
                                 int levelsup, osg_bow_out *out);

/* ORBextractor::ComputeKeyPointsOctTree (oracle_orbdetect.cc): cv::FAST(threshold, nonmax) on one
 * image (keypoints row-major, response = score); the cell loop + DistributeOctTree over a pyramid,
 * keypoints level by level in the reference's order (level coordinates, size = (int)(31 * scale)).
 * Both return the keypoint count, or -1 when it exceeds cap. */
int oracle_fast(const uint8_t *img, int rows, int cols, int step, int threshold, int cap, float *x, float *y,
                float *response);
int oracle_orb_detect(const osg_image_pyramid *P, int ini_th, int min_th, const int32_t *n_features,
                      const float *scale_factors, int cap, float *x, float *y, float *response, float *size,
                      int32_t *level_start);

/* ORBextractor::ComputePyramid + the GaussianBlur of operator() (oracle_pyramid.c): the level sizes
 * and the byte offsets of each bordered level ((rows + 38) x (cols + 38), the ROI at (19, 19)) and
 * each blurred level (rows x cols) in one buffer; returns its size.  oracle_orb_pyramid fills such a
 * buffer from a host image (blur = 0: the bordered levels only) and returns the size, or -1. */
int64_t oracle_pyramid_layout(int32_t rows, int32_t cols, int32_t n_levels, const float *inv_scale, int32_t *lrows,
                              int32_t *lcols, int64_t *bordered_off, int64_t *blurred_off);
void oracle_gaussian_kernel7(int32_t k[7]);
int64_t oracle_orb_pyramid(const uint8_t *image, int32_t rows, int32_t cols, int32_t step, int32_t n_levels,
                           const float *inv_scale, uint8_t *out, int32_t blur);

/* bundle adjustment (oracle_ba.c) */
double oracle_ref_pow3(double t);  /* the reference's libm calls, correctly rounded */
double oracle_ref_sin(double x);
double oracle_ref_cos(double x);
void oracle_set_libm(int on);  /* 1: the host libm's sin / cos / pow / atan2 (cpu_baseline timing only) */
int oracle_pose_optimization(const osg_pose_problem *P, osg_pose_result *R);
int oracle_local_bundle_adjustment(const osg_ba_graph *G, osg_ba_result *R,
                                   const volatile uint8_t *stop_flag);

#ifdef __cplusplus
}
#endif
#endif
