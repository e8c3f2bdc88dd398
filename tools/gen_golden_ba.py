"""Golden BA fixtures (tests/golden/ba_pose.npz, ba_lba.npz): seeded PoseOptimization problems and
LocalBundleAdjustment windows with the CPU oracle's results, so that tests replay a fixed reference
independent of rebuilding the oracle (tests/test_golden_ba.py: the oracle must still reproduce them
exactly on the CPU; the GPU path is compared with them under -m gpu).  Called by tools/gen_golden.py;
the cameras are stored as the bytes of their osg_camera structs."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def cam_bytes(c):
    return np.frombuffer(C.string_at(C.addressof(c), C.sizeof(c)), np.uint8).copy()


def pose_fixture(lib):
    from orb_slam3_comments_ghr_amd import optimizer as op
    from tests import oracle_calls as oc
    rng = np.random.default_rng(0x60D2)
    probs = [op.synth_pose_problem(rng, n_edges=int(rng.integers(20, 300)), stereo_frac=float(rng.uniform(0, 1)))
             for _ in range(14)]
    probs += [op.synth_pose_problem(rng, n_edges=120, cam=op.kb8_camera(), body_frac=0.3),
              op.synth_pose_problem(rng, n_edges=12, outlier_frac=1.0)]
    ref = oc.pose(lib, probs)
    d = {"n": np.array([p.n for p in probs], np.int32)}
    for k in ("kind", "xw", "obs", "inv_sigma2"):
        d[k] = np.concatenate([getattr(p, k).reshape(len(p.kind), -1) for p in probs])
    d["pose0"] = np.stack([p.pose for p in probs])
    d["cam"] = np.stack([cam_bytes(p.cam) for p in probs])
    d["cam2"] = np.stack([cam_bytes(p.cam2) for p in probs])
    d["ref_pose"] = np.stack([r.pose for r in ref])
    d["ref_outlier"] = np.concatenate([r.outlier for r in ref])
    d["ref_counts"] = np.array([[r.n_inliers, r.lm_iterations, r.lm_trials] for r in ref], np.int32)
    np.savez_compressed(os.path.join(GOLDEN, "ba_pose.npz"), **d)


def lba_fixture(lib):
    from orb_slam3_comments_ghr_amd import optimizer as op
    from tests import oracle_calls as oc
    rng = np.random.default_rng(0x60D3)
    graphs = [op.synth_lba_graph(rng, n_kf=8, n_points=500), op.synth_lba_graph(rng, n_kf=6, n_points=350,
                                                                                stereo_frac=0.4)]
    d = {"count": np.array([len(graphs)], np.int32)}
    for i, G in enumerate(graphs):
        r = oc.lba(lib, G)
        for k in ("pose", "pose_fixed", "point", "e_point", "e_pose", "e_kind", "e_cam", "e_obs", "e_inv_sigma2"):
            d[f"g{i}_{k}"] = getattr(G, k)
        d[f"g{i}_cams"] = np.stack([cam_bytes(c) for c in G.cams])
        d[f"g{i}_ref_pose"], d[f"g{i}_ref_point"], d[f"g{i}_ref_bad"] = r.pose, r.point, r.edge_bad
        d[f"g{i}_ref_counts"] = np.array([r.iterations, r.trials], np.int32)
        d[f"g{i}_ref_chi2"] = np.array([r.chi2_initial, r.chi2_final], np.float64)
    np.savez_compressed(os.path.join(GOLDEN, "ba_lba.npz"), **d)


def main(lib):
    os.makedirs(GOLDEN, exist_ok=True)
    pose_fixture(lib)
    lba_fixture(lib)


if __name__ == "__main__":
    import sys
    sys.path.insert(0, ROOT)
    from tests import oracle_calls
    main(oracle_calls.load())
