"""Frame::ComputeStereoFishEyeMatches (ref:src/Frame.cc:1546-1603) — the KannalaBrandt8 rig's stereo step.

CPU: the oracle against a numpy restatement of BFMatcher(NORM_HAMMING).knnMatch(k = 2) + Lowe's ratio, with
the triangulation verdict taken from the separately pinned KannalaBrandt8 epipolar test
(tests/test_oracle_triang.py pins it against a float64 restatement), and the true depths of the synthetic
rig.  GPU: osg_compute_stereo_fisheye_matches bit-exact against the oracle (indices, counts and the float
bit patterns of mvDepth / mvStereo3Dpoints).  Parity with OpenCV's BFMatcher itself is unpinned (its tie
order is restated: a distance equal to the first neighbour's becomes the second)."""
import numpy as np
import pytest

from orb_slam3_comments_ghr_amd import stereo as st
from tests import oracle_calls as oc  # noqa: F401  (sets the oracle's argtypes)


def run_oracle(oracle, F):
    kl, ol, dl, kr, orr, dr, s2, cl, cr, R, t = F.args()
    nl, nr = kl.shape[0], kr.shape[0]
    l2r, r2l = np.empty(nl, np.int32), np.empty(nr, np.int32)
    depth, p3d = np.empty(nl, np.float32), np.empty((nl, 3), np.float32)
    n = oracle.oracle_stereo_fisheye_matches(nl, F.mono_left, dl.ctypes.data, kl.ctypes.data, ol.ctypes.data, nr,
                                             F.mono_right, dr.ctypes.data, kr.ctypes.data, orr.ctypes.data,
                                             s2.ctypes.data, cl.ctypes.data, cr.ctypes.data, R.ctypes.data,
                                             t.ctypes.data, l2r.ctypes.data, r2l.ctypes.data, depth.ctypes.data,
                                             p3d.ctypes.data)
    return l2r, r2l, depth, p3d, n


def numpy_knn2(dl, dr):
    bits = np.unpackbits(dl[:, None, :] ^ dr[None, :, :], axis=2).sum(2)
    j1 = bits.argmin(1)  # first minimum: a tie never displaces the first neighbour
    srt = np.sort(bits, 1)
    return j1, srt[:, 0], srt[:, 1]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_fisheye_vs_numpy(oracle, seed):
    F = st.synth_fisheye_stereo(np.random.default_rng(seed))
    l2r, r2l, depth, p3d, n = run_oracle(oracle, F)
    ml, mr = F.mono_left, F.mono_right
    j1, d1, d2 = numpy_knn2(F.desc_left[ml:], F.desc_right[mr:])
    ratio = d1.astype(np.float32).astype(np.float64) < d2.astype(np.float32).astype(np.float64) * 0.7
    kl, ol, dl, kr, orr, dr, s2, cl, cr, R, t = F.args()
    want = np.full(len(kl), -1, np.int32)
    for q in np.nonzero(ratio)[0]:
        i, j = ml + q, mr + j1[q]
        ok = oracle.oracle_kb8_epipolar_constrain(cl.ctypes.data, cr.ctypes.data, float(kl[i, 0]), float(kl[i, 1]),
                                                  float(kr[j, 0]), float(kr[j, 1]), R.ctypes.data, t.ctypes.data,
                                                  float(s2[ol[i]]), float(s2[orr[j]]))
        if ok:
            want[i] = j
    assert np.array_equal(l2r, want)
    assert n == int((want >= 0).sum()) and n > 100 and ratio.sum() > n  # the ratio test and triangulation both cut
    r2l_want = np.full(len(kr), -1, np.int32)
    for i in np.nonzero(want >= 0)[0]:
        r2l_want[want[i]] = i  # later queries overwrite
    assert np.array_equal(r2l, r2l_want)
    assert np.all(depth[want < 0] == -1.0) and np.all(p3d[want < 0] == 0)
    assert np.all(depth[want >= 0] > 1e-4) and np.array_equal(depth[want >= 0], p3d[want >= 0, 2])
    # geometry: the left camera point of a true pair is recovered (depth 1-8 m, 0.3 px noise)
    good = want >= 0
    assert np.median(np.abs(np.linalg.norm(p3d[good], axis=1))) > 1.0


def test_oracle_fisheye_edges(oracle):
    F = st.synth_fisheye_stereo(np.random.default_rng(9), n_points=50)
    # fewer than two right stereo rows: knnMatch returns < 2 neighbours, nothing is matched
    F1 = st.FishEyeStereoFrame(**{**F.__dict__, "mono_right": len(F.kp_right) - 1})
    l2r, r2l, depth, _, n = run_oracle(oracle, F1)
    assert n == 0 and np.all(l2r == -1) and np.all(r2l == -1) and np.all(depth == -1)
    # no left stereo rows
    F2 = st.FishEyeStereoFrame(**{**F.__dict__, "mono_left": len(F.kp_left)})
    assert run_oracle(oracle, F2)[4] == 0


def _same(ctx, oracle, F):
    got = st.ComputeStereoFishEyeMatches(ctx, F)
    want = run_oracle(oracle, F)
    assert got[4] == want[4]
    for g, w in zip(got[:4], want[:4]):
        assert np.array_equal(g.view(np.int32), w.view(np.int32))
    return got[4]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_gpu_fisheye_vs_oracle(ctx, oracle, seed):
    assert _same(ctx, oracle, st.synth_fisheye_stereo(np.random.default_rng(seed))) > 100


@pytest.mark.gpu
def test_gpu_fisheye_large_and_edges(ctx, oracle):
    rng = np.random.default_rng(11)
    _same(ctx, oracle, st.synth_fisheye_stereo(rng, n_points=1500, n_distract=400, flip=0.08))
    F = st.synth_fisheye_stereo(rng, n_points=40)
    _same(ctx, oracle, st.FishEyeStereoFrame(**{**F.__dict__, "mono_right": len(F.kp_right) - 1}))
    _same(ctx, oracle, st.FishEyeStereoFrame(**{**F.__dict__, "mono_left": len(F.kp_left)}))
    _same(ctx, oracle, st.FishEyeStereoFrame(**{**F.__dict__, "mono_left": 0, "mono_right": 0}))
