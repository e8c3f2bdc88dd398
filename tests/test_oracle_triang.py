"""Pinning the SearchForTriangulation oracle (oracle/oracle_triang.c, test infrastructure) against the
independent pure-Python restatement (tests/pyref_match.py) and a hand-derived case.  CPU only."""
import numpy as np
import pytest

from orb_slam3_comments_ghr_amd import frames as fr
from tests import oracle_calls as oc
from tests import pyref_match as pr


def same(a, b):
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("forward", [False, True])
@pytest.mark.parametrize("coarse,only_stereo,ori", [(False, False, True), (True, False, True),
                                                    (False, True, True), (False, False, False)])
def test_oracle_triang_vs_python(oracle, seed, forward, coarse, only_stereo, ori):
    rng = np.random.default_rng(7000 + seed)
    K1, K2, g = fr.synth_triang_pair(rng, n1=300, n2=280, n_nodes=30, forward=forward)
    ref = oc.triangulation(oracle, K1, K2, g, only_stereo, coarse, ori)
    same(ref, pr.search_for_triangulation(K1, K2, g, only_stereo, coarse, ori))
    assert ref[0] > (0 if only_stereo else 10)


@pytest.mark.parametrize("coarse", [False, True])
def test_oracle_triang_two_cam_vs_python(oracle, coarse):
    rng = np.random.default_rng(7100)
    K1, K2, g = fr.synth_triang_pair(rng, n1=300, n2=300, n_nodes=30, two_cam=True)
    ref = oc.triangulation(oracle, K1, K2, g, coarse=coarse)
    same(ref, pr.search_for_triangulation(K1, K2, g, coarse=coarse))
    assert ref[0] > 5


def hand_pair(stereo1=False):
    """KF1: one keypoint without a MapPoint at (100, 100).  KF2 (same vocabulary node), descriptor
    distances 10, 10, 5, 3: keypoint 0 (150, 101) and 1 (180, 101.5) lie on the epipolar line
    (F12 = [t]x for K = I, R = I, t = (1, 0, 0): the line is y2 = y1, pass iff dy^2 < 3.84);
    2 (200, 103) is 3 px off it; 3 (300, 100) is on it but 5 px from the epipole (305, 100)
    (25 < 100 * mvScaleFactors[0])."""
    d1 = np.zeros((1, 32), np.uint8)
    d2 = np.zeros((4, 32), np.uint8)
    for i, k in enumerate([10, 10, 5, 3]):
        bits = np.zeros(256, np.uint8)
        bits[i * 20: i * 20 + k] = 1
        d2[i] = np.packbits(bits)
    node = dict(node_id=np.array([7], np.uint32), node_start=np.array([0, 1], np.int32))
    K1 = fr.KFSide(desc=d1, kp_x=[100.0], kp_y=[100.0], kp_angle=[10.0], kp_octave=[0],
                   u_right=[50.0 if stereo1 else -1.0], has_mp=[0], feat=np.array([0], np.int32), **node)
    node2 = dict(node_id=np.array([7], np.uint32), node_start=np.array([0, 4], np.int32))
    K2 = fr.KFSide(desc=d2, kp_x=[150.0, 180.0, 200.0, 300.0], kp_y=[101.0, 101.5, 103.0, 100.0],
                   kp_angle=[5.0] * 4, kp_octave=[0] * 4, u_right=None, has_mp=[0] * 4,
                   feat=np.arange(4, dtype=np.int32), **node2)
    F = np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32)[None]
    return K1, K2, fr.TriangGeom(ep=(305.0, 100.0), F12=F)


def test_oracle_triang_hand_case(oracle):
    K1, K2, g = hand_pair()
    # equal distances: the later keypoint in node order wins ('<=', ref:src/ORBmatcher.cc:1180)
    assert oc.triangulation(oracle, K1, K2, g)[1].tolist() == [[0, 1]]
    # bCoarse: no epipolar test, keypoint 2 (d 5) wins; keypoint 3 still fails the epipole test
    assert oc.triangulation(oracle, K1, K2, g, coarse=True)[1].tolist() == [[0, 2]]
    # a stereo KF1 keypoint skips the epipole test: keypoint 3 (d 3) wins
    K1s, K2s, gs = hand_pair(stereo1=True)
    assert oc.triangulation(oracle, K1s, K2s, gs)[1].tolist() == [[0, 3]]
    # bOnlyStereo: KF2 has no stereo keypoint, nothing matches
    assert oc.triangulation(oracle, K1s, K2s, gs, only_stereo=True)[0] == 0
    # a MapPoint on the KF1 keypoint removes it from the search
    K1.has_mp[:] = 1
    assert oc.triangulation(oracle, K1, K2, g)[0] == 0
    for args in [(False, False), (True, False)]:
        K1, K2, g = hand_pair()
        same(oc.triangulation(oracle, K1, K2, g, *args), pr.search_for_triangulation(K1, K2, g, *args))
