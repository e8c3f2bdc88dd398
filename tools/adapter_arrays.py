"""Array files for the mock ORB-SLAM3 drivers (tests/adapter/adapter_driver.cpp and
tools/adapter_wall_bench.cpp read them through tests/adapter/driver_common.h).

File format: repeated {u32 name_len, name, u8 dtype ('b' u8, 'i' i32, 'f' f32, 'd' f64), u64 count,
data}.  The builders below name each problem's arrays the way driver_common.h's build_* functions
read them; `prefixed` puts a problem under "b0.", "b1.", ... (batch files) or "p0.", ... (pools).
"""
import numpy as np

_CODES = {np.dtype(np.uint8): b"b", np.dtype(np.int8): b"b", np.dtype(np.int32): b"i", np.dtype(np.uint32): b"i",
          np.dtype(np.float32): b"f", np.dtype(np.float64): b"d"}
_DTYPES = {b"b": np.uint8, b"i": np.int32, b"f": np.float32, b"d": np.float64}


def write_arrays(path, arrays):
    with open(path, "wb") as f:
        for name, a in arrays.items():
            a = np.ascontiguousarray(a)
            code = _CODES[a.dtype]
            nb = name.encode()
            f.write(np.uint32(len(nb)).tobytes() + nb + code + np.uint64(a.size).tobytes() + a.tobytes())


def read_arrays(path):
    out = {}
    with open(path, "rb") as f:
        data = f.read()
    o = 0
    while o < len(data):
        n = int(np.frombuffer(data, np.uint32, 1, o)[0]); o += 4
        name = data[o:o + n].decode(); o += n
        code = data[o:o + 1]; o += 1
        cnt = int(np.frombuffer(data, np.uint64, 1, o)[0]); o += 8
        dt = np.dtype(_DTYPES[code])
        out[name] = np.frombuffer(data, dt, cnt, o).copy(); o += cnt * dt.itemsize
    return out


def prefixed(pre, arrays):
    return {pre + k: v for k, v in arrays.items()}


def frame_arrays(F):
    """FrameSoA -> "F.*" (build_frame)."""
    d = {"F.kp_x": F.kp_x, "F.kp_y": F.kp_y, "F.kp_angle": F.kp_angle, "F.kp_octave": F.kp_octave,
         "F.desc": F.desc.reshape(-1), "F.u_right": (F.u_right if F.u_right is not None
                                                    else np.full(F.n, -1, np.float32)),
         "F.grid_start": F.grid_start, "F.grid_idx": F.grid_idx, "F.scale": F.scale,
         "F.scalars": np.array([F.min_x, F.max_x, F.min_y, F.max_y, F.inv_w, F.inv_h, F.mb, F.mbf],
                               np.float32)}
    if F.nleft != -1:
        d.update({"F.nleft": np.array([F.nleft], np.int32), "F.r_grid_start": F.grid_start_r,
                  "F.r_grid_idx": F.grid_idx_r, "F.left_to_right": F.left_to_right,
                  "F.right_to_left": F.right_to_left})
    return d


def bow_arrays(pre, S):
    """A BoW side (frames.BowSide) -> "B1.*" / "B2.*" (build_bow_kf)."""
    return {pre + "desc": S.desc.reshape(-1), pre + "angle": S.angle, pre + "mp_id": S.mp_id,
            pre + "mp_good": S.mp_good, pre + "node_id": S.node_id, pre + "node_start": S.node_start,
            pre + "feat": S.feat, pre + "nleft": np.array([S.nleft], np.int32)}


def cam_array(c):
    return np.array([c.type, *[c.p[i] for i in range(8)], c.fx, c.fy, c.cx, c.cy, c.bf], np.float32)


def slot_arrays(slot_mp, taken):
    return {"S.slot_mp": np.asarray(slot_mp, np.int32), "S.slot_taken": np.asarray(taken, np.uint8)}


LAST_KEYS = ["mp_id", "desc", "valid", "has_obs", "u", "v", "invz", "octave", "angle", "u_r", "v_r"]
MPS_KEYS = ["mp_id", "desc", "usable", "has_obs", "in_view", "proj_x", "proj_y", "proj_xr", "view_cos", "pred_level",
            "track_depth", "in_view_r", "proj_yr", "view_cos_r", "pred_level_r"]


def last_arrays(L):
    """LastFrame queries -> "L.*" (build_last_problem)."""
    return {"L." + k: np.ascontiguousarray(getattr(L, k)).reshape(-1) for k in LAST_KEYS if getattr(L, k, None) is not None}


def mps_arrays(Q):
    """Local-map queries -> "Q.*" (build_mps_problem)."""
    return {"Q." + k: np.ascontiguousarray(getattr(Q, k)).reshape(-1) for k in MPS_KEYS if getattr(Q, k, None) is not None}


def pose_arrays(P):
    """A PoseOptimization problem -> "P.*" (build_pose_problem); pass it through pose_for_mock first."""
    a = {"P.kind": P.kind.astype(np.uint8), "P.xw": P.xw.reshape(-1), "P.obs": P.obs.reshape(-1),
         "P.inv_sigma2": P.inv_sigma2, "P.pose": P.pose, "P.cam": cam_array(P.cam)}
    if (P.kind == 2).any():
        a["P.cam2"] = cam_array(P.cam2)
        a["P.cam2_trl"] = np.array([P.cam2.trl[i] for i in range(7)], np.float64)
    return a


def pose_for_mock(P):
    """Make a PoseOptimization problem representable by a Frame, in place: keypoint coordinates
    rounded to float (cv::KeyPoint); a stereo edge whose u_R is negative becomes monocular, as
    PoseOptimization reads a Frame (mvuRight < 0: no stereo observation, ref:src/Optimizer.cc:146);
    and on a two-camera problem the left-camera edges first, then the right-camera (BODY) edges, as
    Frame's slot order puts them (Nleft)."""
    P.obs = P.obs.astype(np.float32).astype(np.float64)
    P.kind = np.where((P.kind == 1) & (P.obs[:, 2] < 0), 0, P.kind).astype(P.kind.dtype)
    if (P.kind == 2).any():
        order = np.concatenate([np.nonzero(P.kind != 2)[0], np.nonzero(P.kind == 2)[0]])
        for k in ("kind", "xw", "obs", "inv_sigma2"):
            setattr(P, k, np.ascontiguousarray(getattr(P, k)[order]))
    return P


def stereo_arrays(F):
    """StereoFrame (host levels) -> "S.*", "PL.*", "PR.*" (build_stereo_problem)."""
    def dims(P):
        return np.array([[lv.shape[0], lv.shape[1]] for lv in P.levels], np.int32).reshape(-1)

    def img(P):
        return np.concatenate([np.ascontiguousarray(lv).reshape(-1) for lv in P.levels])

    return {"S.x": F.x, "S.y": F.y, "S.oct": F.octave, "S.desc": F.desc.reshape(-1), "S.xr": F.xr, "S.yr": F.yr,
            "S.oct_r": F.octave_r, "S.desc_r": F.desc_r.reshape(-1), "S.scale": F.scale, "S.inv_scale": F.inv_scale,
            "S.mb_mbf": np.array([F.mb, F.mbf], np.float32), "PL.img": img(F.left), "PL.dims": dims(F.left),
            "PR.img": img(F.right), "PR.dims": dims(F.right)}


def vocabulary_arrays(voc):
    """vocabulary.Vocabulary -> "V.*" (osg_vocabulary_create's desc)."""
    return {"V.kl": np.array([voc.k, voc.L, voc.scoring, voc.weighting], np.int32), "V.parent": voc.parent,
            "V.is_leaf": voc.is_leaf, "V.desc": np.ascontiguousarray(voc.desc, np.uint8).reshape(-1),
            "V.weight": np.ascontiguousarray(voc.weight, np.float64)}
