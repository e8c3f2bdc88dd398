"""ctypes mirror of the C ABI in include/osg.h and include/osg_ba.h.

Only plain pointers and sizes cross the boundary; every pointer field is a ``c_void_p`` filled
from a numpy array's address by the helpers in this package.  The structures are shared by the
product bindings (liborbslam3_amd.so); the oracle's (test infrastructure) are in tests/oracle_calls.py.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# OSG_LIB_PATH points the package at another build of the same library (a profiling build)
LIB_PATH = os.environ.get("OSG_LIB_PATH") or os.path.join(_HERE, "liborbslam3_amd.so")

OSG_OK = 0
OSG_E_INVALID = -1
OSG_E_HIP = -2
OSG_E_NOMEM = -3
OSG_E_UNSUPPORTED = -4
OSG_E_NODEVICE = -5

TH_HIGH = 100
TH_LOW = 50
HISTO_LENGTH = 30
GRID_COLS = 64
GRID_ROWS = 48
GRID_CELLS = GRID_COLS * GRID_ROWS

CAM_PINHOLE = 0
CAM_KB8 = 1
EDGE_MONO = 0
EDGE_STEREO = 1
EDGE_BODY = 2

P = C.c_void_p
i32 = C.c_int32
f32 = C.c_float
f64 = C.c_double


class OsgFrame(C.Structure):
    _fields_ = [
        ("n", i32), ("nleft", i32), ("desc", P), ("kp_x", P), ("kp_y", P), ("kp_angle", P),
        ("kp_octave", P), ("u_right", P), ("grid_start", P), ("grid_idx", P),
        ("grid_start_r", P), ("grid_idx_r", P), ("left_to_right", P), ("right_to_left", P),
        ("min_x", f32), ("max_x", f32), ("min_y", f32), ("max_y", f32),
        ("grid_inv_w", f32), ("grid_inv_h", f32), ("scale_factors", P), ("n_levels", i32),
        ("mb", f32), ("mbf", f32),
    ]


class OsgMpQueries(C.Structure):
    _fields_ = [
        ("n", i32), ("mp_id", P), ("desc", P), ("usable", P), ("has_obs", P), ("in_view", P),
        ("proj_x", P), ("proj_y", P), ("proj_xr", P), ("view_cos", P), ("pred_level", P),
        ("track_depth", P), ("in_view_r", P), ("proj_yr", P), ("view_cos_r", P),
        ("pred_level_r", P),
    ]


class OsgLastQueries(C.Structure):
    _fields_ = [
        ("n", i32), ("mp_id", P), ("desc", P), ("valid", P), ("has_obs", P), ("u", P),
        ("v", P), ("invz", P), ("u_r", P), ("v_r", P), ("octave", P), ("angle", P),
        ("tlc_z", f32),
    ]


class OsgKfQueries(C.Structure):
    _fields_ = [
        ("n", i32), ("mp_id", P), ("desc", P), ("valid", P), ("u", P), ("v", P),
        ("pred_level", P), ("angle", P),
    ]


class OsgFuseQueries(C.Structure):
    _fields_ = [
        ("n", i32), ("desc", P), ("valid", P), ("u", P), ("v", P), ("ur", P), ("pred_level", P),
        ("inv_level_sigma2", P),
    ]


class OsgFeatVec(C.Structure):
    _fields_ = [("n_nodes", i32), ("node_id", P), ("node_start", P), ("feat", P)]


class OsgBowSide(C.Structure):
    _fields_ = [
        ("n", i32), ("nleft", i32), ("desc", P), ("angle", P), ("mp_id", P), ("mp_good", P),
        ("fv", OsgFeatVec),
    ]


class OsgKfSide(C.Structure):
    _fields_ = [
        ("n", i32), ("nleft", i32), ("two_cam", i32), ("desc", P), ("kp_x", P), ("kp_y", P), ("kp_angle", P),
        ("kp_octave", P), ("u_right", P), ("has_mp", P), ("level_sigma2", P), ("scale_factors", P),
        ("n_levels", i32), ("fv", OsgFeatVec),
    ]


class OsgTriangGeom(C.Structure):
    _fields_ = [("ep_x", f32), ("ep_y", f32), ("F12", f32 * 36), ("pinhole", i32), ("R12", f32 * 36),
                ("t12", f32 * 12), ("kb", f32 * 32)]


class OsgImagePyramid(C.Structure):
    _fields_ = [("n_levels", i32), ("on_device", i32), ("data", P), ("rows", P), ("cols", P), ("step", P)]


class OsgStereoFrame(C.Structure):
    _fields_ = [
        ("n", i32), ("x", P), ("y", P), ("octave", P), ("desc", P), ("n_right", i32), ("xr", P), ("yr", P),
        ("octave_r", P), ("desc_r", P), ("scale_factors", P), ("inv_scale_factors", P), ("n_levels", i32),
        ("mb", f32), ("mbf", f32), ("left", OsgImagePyramid), ("right", OsgImagePyramid),
    ]


class OsgOrbExtractParams(C.Structure):
    _fields_ = [
        ("n_levels", i32), ("scale_factors", P), ("inv_scale_factors", P), ("n_features_per_level", P),
        ("ini_th_fast", i32), ("min_th_fast", i32), ("pattern", P), ("umax", P),
    ]


class OsgOrbKeypoints(C.Structure):
    _fields_ = [("n", i32), ("x", P), ("y", P), ("level", P)]


class OsgCamera(C.Structure):
    _fields_ = [
        ("type", i32), ("p", f32 * 8), ("fx", f32), ("fy", f32), ("cx", f32), ("cy", f32),
        ("bf", f32), ("trl", f64 * 7),
    ]


class OsgPoseProblem(C.Structure):
    _fields_ = [
        ("pose", f64 * 7), ("n_edges", i32), ("kind", P), ("xw", P), ("obs", P),
        ("inv_sigma2", P), ("cam", OsgCamera), ("cam2", OsgCamera),
    ]


class OsgPoseResult(C.Structure):
    _fields_ = [
        ("pose", f64 * 7), ("outlier", P), ("n_inliers", i32), ("lm_iterations", i32),
        ("lm_trials", i32),
    ]


class OsgBaGraph(C.Structure):
    _fields_ = [
        ("n_poses", i32), ("pose", P), ("pose_fixed", P), ("n_points", i32), ("point", P),
        ("n_edges", i32), ("e_point", P), ("e_pose", P), ("e_kind", P), ("e_cam", P),
        ("e_obs", P), ("e_inv_sigma2", P), ("n_cams", i32), ("cams", P), ("iterations", i32),
        ("user_lambda_init", f64), ("e_robust", P), ("huber_mono", f32), ("huber_stereo", f32),
    ]


class OsgBaResult(C.Structure):
    _fields_ = [
        ("pose", P), ("point", P), ("edge_bad", P), ("iterations", i32), ("trials", i32),
        ("chi2_initial", f64), ("chi2_final", f64), ("aborted", i32), ("edge_chi2", P),
    ]


class OsgVocabularyDesc(C.Structure):
    _fields_ = [
        ("k", i32), ("L", i32), ("scoring", i32), ("weighting", i32), ("n_nodes", i32),
        ("parent", P), ("is_leaf", P), ("desc", P), ("weight", P),
    ]


class OsgBowOut(C.Structure):
    _fields_ = [
        ("n_words", i32), ("word", P), ("value", P), ("n_nodes", i32), ("node_id", P),
        ("node_start", P), ("feat", P),
    ]


# Every symbol include/osg.h, include/osg_ba.h and include/osg_dbow.h declare (checked by tests/test_abi.py).
EXPORTS = [
    "osg_ctx_create", "osg_ctx_destroy", "osg_ctx_set_stream", "osg_ctx_stream",
    "osg_ctx_synchronize", "osg_strerror", "osg_ctx_last_error", "osg_version",
    "osg_descriptor_distance", "osg_descriptor_distance_pairs", "osg_hamming_top2",
    "osg_hamming_top2_dev", "osg_hamming_top2_batch_dev", "osg_hamming_top2_plan", "osg_hamming_top2_batch_plan", "osg_search_by_projection_mps", "osg_search_by_projection_last",
    "osg_search_by_projection_kf", "osg_search_by_bow_kf_f", "osg_search_by_bow_kf_kf",
    "osg_search_by_projection_mps_batch", "osg_search_by_projection_last_batch",
    "osg_search_by_projection_kf_batch", "osg_search_by_bow_kf_f_batch", "osg_search_by_bow_kf_kf_batch",
    "osg_match_last_stats", "osg_ctx_last_kernel_ms", "osg_ctx_device_bytes", "osg_pose_optimization", "osg_pose_optimization_batch",
    "osg_local_bundle_adjustment", "osg_local_bundle_adjustment_batch", "osg_bundle_adjustment",
    "osg_lba_kernel_times",
    "osg_vocabulary_create", "osg_vocabulary_load_text", "osg_vocabulary_destroy", "osg_vocabulary_info",
    "osg_vocabulary_transform", "osg_vocabulary_transform_batch",
    "osg_fuse_search", "osg_fuse_search_batch", "osg_search_for_triangulation", "osg_search_for_triangulation_batch",
    "osg_compute_distinctive_descriptors", "osg_compute_distinctive_descriptors_dev",
    "osg_search_by_projection_sim3", "osg_search_by_projection_sim3_batch", "osg_search_by_sim3",
    "osg_search_for_initialization", "osg_search_for_initialization_batch",
    "osg_compute_stereo_matches", "osg_compute_stereo_matches_batch", "osg_compute_stereo_fisheye_matches",
    "osg_orb_describe", "osg_orb_detect", "osg_orb_extract_batch",
    "osg_debug_distribute_oct_tree", "osg_orb_pyramid_layout", "osg_orb_pyramid", "osg_debug_gaussian_kernel7",
]


def declare(lib: C.CDLL) -> C.CDLL:
    """Attach argtypes/restypes for the product library."""
    vp = C.c_void_p
    lib.osg_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
    lib.osg_ctx_destroy.argtypes = [vp]
    lib.osg_ctx_set_stream.argtypes = [vp, vp]
    lib.osg_ctx_stream.argtypes = [vp]
    lib.osg_ctx_stream.restype = vp
    lib.osg_ctx_synchronize.argtypes = [vp]
    lib.osg_strerror.argtypes = [C.c_int]
    lib.osg_strerror.restype = C.c_char_p
    lib.osg_ctx_last_error.argtypes = [vp]
    lib.osg_ctx_last_error.restype = C.c_char_p
    lib.osg_version.argtypes = []
    lib.osg_version.restype = C.c_char_p
    lib.osg_descriptor_distance.argtypes = [vp, vp]
    lib.osg_descriptor_distance_pairs.argtypes = [vp, vp, vp, i32, vp]
    lib.osg_hamming_top2.argtypes = [vp, vp, i32, vp, i32, vp, vp, vp]
    lib.osg_hamming_top2_dev.argtypes = [vp, vp, i32, vp, i32, vp]
    lib.osg_hamming_top2_batch_dev.argtypes = [vp, vp, i32, vp, i32, i32, vp]
    lib.osg_hamming_top2_plan.argtypes = [vp, i32, i32, C.c_char_p, i32]
    lib.osg_hamming_top2_batch_plan.argtypes = [vp, i32, i32, i32, C.c_char_p, i32]
    lib.osg_search_by_projection_mps.argtypes = [vp, C.POINTER(OsgFrame), C.POINTER(OsgMpQueries),
                                                 f32, f32, C.c_int, f32, vp, vp]
    lib.osg_search_by_projection_last.argtypes = [vp, C.POINTER(OsgFrame),
                                                  C.POINTER(OsgLastQueries), f32, C.c_int, C.c_int,
                                                  vp, vp]
    lib.osg_search_by_projection_kf.argtypes = [vp, C.POINTER(OsgFrame), C.POINTER(OsgKfQueries),
                                                f32, C.c_int, C.c_int, vp]
    lib.osg_search_by_bow_kf_f.argtypes = [vp, C.POINTER(OsgBowSide), C.POINTER(OsgBowSide), f32,
                                           C.c_int, vp]
    lib.osg_search_by_bow_kf_kf.argtypes = [vp, C.POINTER(OsgBowSide), C.POINTER(OsgBowSide), f32,
                                            C.c_int, vp]
    lib.osg_search_by_projection_mps_batch.argtypes = [vp, vp, vp, i32, f32, f32, C.c_int, f32, vp, vp, vp]
    lib.osg_search_by_projection_last_batch.argtypes = [vp, vp, vp, i32, f32, C.c_int, C.c_int, vp, vp, vp]
    lib.osg_search_by_projection_kf_batch.argtypes = [vp, vp, vp, i32, f32, C.c_int, C.c_int, vp, vp]
    lib.osg_search_by_bow_kf_f_batch.argtypes = [vp, vp, vp, i32, f32, C.c_int, vp, vp]
    lib.osg_search_by_bow_kf_kf_batch.argtypes = [vp, vp, vp, i32, f32, C.c_int, vp, vp]
    lib.osg_match_last_stats.argtypes = [vp, vp]
    lib.osg_ctx_last_kernel_ms.argtypes = [vp, vp]
    lib.osg_ctx_device_bytes.argtypes = [vp, vp]
    lib.osg_pose_optimization.argtypes = [vp, C.POINTER(OsgPoseProblem), C.POINTER(OsgPoseResult)]
    lib.osg_pose_optimization_batch.argtypes = [vp, C.POINTER(OsgPoseProblem), i32,
                                                C.POINTER(OsgPoseResult)]
    lib.osg_local_bundle_adjustment.argtypes = [vp, C.POINTER(OsgBaGraph), C.POINTER(OsgBaResult),
                                                vp]
    lib.osg_bundle_adjustment.argtypes = [vp, C.POINTER(OsgBaGraph), C.POINTER(OsgBaResult),
                                                vp]
    lib.osg_local_bundle_adjustment_batch.argtypes = [vp, vp, i32, vp, vp]
    lib.osg_lba_kernel_times.argtypes = [vp, i32, vp, vp]
    lib.osg_vocabulary_create.argtypes = [vp, C.POINTER(OsgVocabularyDesc), C.POINTER(vp)]
    lib.osg_vocabulary_load_text.argtypes = [vp, C.c_char_p, C.POINTER(vp)]
    lib.osg_vocabulary_destroy.argtypes = [vp]
    lib.osg_vocabulary_info.argtypes = [vp, vp]
    lib.osg_vocabulary_transform.argtypes = [vp, vp, vp, i32, i32, C.POINTER(OsgBowOut)]
    lib.osg_vocabulary_transform_batch.argtypes = [vp, vp, vp, vp, i32, i32, vp]
    lib.osg_fuse_search.argtypes = [vp, C.POINTER(OsgFrame), C.POINTER(OsgFuseQueries), f32, C.c_int, C.c_int,
                                    vp, vp]
    lib.osg_fuse_search_batch.argtypes = [vp, vp, vp, i32, f32, C.c_int, C.c_int, vp, vp, vp]
    lib.osg_search_for_triangulation.argtypes = [vp, C.POINTER(OsgKfSide), C.POINTER(OsgKfSide),
                                                 C.POINTER(OsgTriangGeom), C.c_int, C.c_int, C.c_int, vp]
    lib.osg_search_by_sim3.argtypes = [vp, C.POINTER(OsgFrame), C.POINTER(OsgFrame), C.POINTER(OsgFuseQueries),
                                       C.POINTER(OsgFuseQueries), f32, vp]
    lib.osg_search_by_projection_sim3.argtypes = [vp, C.POINTER(OsgFrame), C.POINTER(OsgFuseQueries), f32, f32, vp]
    lib.osg_search_by_projection_sim3_batch.argtypes = [vp, vp, vp, i32, f32, f32, vp, vp]
    lib.osg_search_for_initialization.argtypes = [vp, C.POINTER(OsgFrame), C.POINTER(OsgFrame), vp, C.c_int, f32,
                                                  C.c_int, vp]
    lib.osg_search_for_initialization_batch.argtypes = [vp, vp, vp, i32, vp, C.c_int, f32, C.c_int, vp, vp]
    lib.osg_compute_stereo_matches.argtypes = [vp, C.POINTER(OsgStereoFrame), vp, vp]
    lib.osg_compute_stereo_matches_batch.argtypes = [vp, vp, i32, vp, vp, vp]
    lib.osg_compute_stereo_fisheye_matches.argtypes = [vp, i32, i32, vp, vp, vp, i32, i32, vp, vp, vp, vp, i32,
                                                       vp, vp, vp, vp, vp, vp, vp, vp]
    lib.osg_debug_distribute_oct_tree.argtypes = [vp, i32, i32, i32, i32, i32, i32, vp, i32]
    lib.osg_orb_detect.argtypes = [vp, C.POINTER(OsgImagePyramid), i32, i32, vp, vp, i32, vp, vp, vp, vp, vp]
    lib.osg_orb_pyramid_layout.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp]
    lib.osg_orb_pyramid_layout.restype = C.c_int64
    lib.osg_orb_pyramid.argtypes = [vp, vp, i32, i32, i32, i32, i32, vp, vp, C.c_int64, i32]
    lib.osg_debug_gaussian_kernel7.argtypes = [vp]
    lib.osg_debug_gaussian_kernel7.restype = None
    lib.osg_orb_describe.argtypes = [vp, C.POINTER(OsgImagePyramid), C.POINTER(OsgImagePyramid),
                                     C.POINTER(OsgOrbKeypoints), vp, vp, i32, vp, vp]
    lib.osg_orb_extract_batch.argtypes = [vp, vp, C.c_int64, i32, i32, i32, i32, C.POINTER(OsgOrbExtractParams), i32,
                                          vp, vp, vp, vp, vp, vp, vp, vp]
    lib.osg_compute_distinctive_descriptors.argtypes = [vp, vp, vp, i32, vp]
    lib.osg_compute_distinctive_descriptors_dev.argtypes = [vp, vp, vp, i32, vp]
    lib.osg_search_for_triangulation_batch.argtypes = [vp, vp, vp, vp, i32, C.c_int, C.c_int, C.c_int, vp, vp]
    return lib
