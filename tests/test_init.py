"""ORBmatcher::SearchForInitialization (ref:src/ORBmatcher.cc:735-878): the oracle pinned by the pure-Python
restatement and a hand case (CPU); the GPU one-wave sequential walk bit-exact against the oracle."""
import numpy as np
import pytest

from orb_slam3_comments_ghr_amd import frames as fr
from orb_slam3_comments_ghr_amd.matcher import ORBmatcher
from tests import oracle_calls as oc
from tests import pyref_match as pr


def same(a, b):
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("window,ori", [(100, True), (50, True), (100, False)])
def test_oracle_vs_python(oracle, seed, window, ori):
    F1, F2, prev = fr.synth_init_pair(np.random.default_rng(9500 + seed), n1=400, n2=400)
    ref = oc.initialization(oracle, F1, F2, prev, window, 0.9, ori)
    same(ref, pr.search_for_initialization(F1, F2, prev, window, 0.9, ori))
    assert ref[0] > 20


def bits(k):
    b = np.zeros(256, np.uint8)
    b[:k] = 1
    return np.packbits(b)


def hand_case():
    """F2 keypoints 0 (100, 100, d0 = bits 0) and 1 (130, 100, bits 30), octave 0.  F1 keypoint 0 (bits 4)
    takes F2 0 (d 4 vs 26: 4 < 0.9 * 26).  F1 keypoint 1 (octave 1) is skipped.  F1 keypoint 2 (bits 1) steals
    F2 0 (d 1 < vMatchedDistance 4).  F1 keypoint 3 (bits 2): F2 0 is skipped (vMatchedDistance 1 <= 2), so its
    best is F2 1 (d 28) alone: 28 <= 50 and the second is INT_MAX -> accepted."""
    F1 = fr.FrameSoA(desc=np.stack([bits(4), bits(0), bits(1), bits(2)]), kp_x=np.full(4, 100, np.float32),
                     kp_y=np.full(4, 100, np.float32), kp_angle=np.zeros(4, np.float32),
                     kp_octave=np.array([0, 1, 0, 0], np.int32))
    F2 = fr.FrameSoA(desc=np.stack([bits(0), bits(30)]), kp_x=np.array([100, 130], np.float32),
                     kp_y=np.array([100, 100], np.float32), kp_angle=np.zeros(2, np.float32),
                     kp_octave=np.zeros(2, np.int32))
    prev = np.stack([F1.kp_x, F1.kp_y], axis=1).astype(np.float32)
    return F1, F2, prev


def test_oracle_hand_case(oracle):
    F1, F2, prev = hand_case()
    n, m12, p = oc.initialization(oracle, F1, F2, prev, 100, 0.9, True)
    assert m12.tolist() == [-1, -1, 0, 1] and n == 2
    assert p[3].tolist() == [130.0, 100.0] and p[0].tolist() == [100.0, 100.0]
    same((n, m12, p), pr.search_for_initialization(F1, F2, prev, 100, 0.9, True))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("window,ori", [(100, True), (50, True), (100, False)])
def test_gpu_vs_oracle(ctx, oracle, seed, window, ori):
    """Monocular initialisation shape: 2 x 5000 keypoints (the 5 x nFeatures initialisation extractor,
    ref:src/Tracking.cc:667), ~22 % at level 0, windowSize 100, nnratio 0.9 (ref:src/Tracking.cc:2951)."""
    F1, F2, prev = fr.synth_init_pair(np.random.default_rng(9600 + seed), n1=5000, n2=5000, level0=0.22)
    ref = oc.initialization(oracle, F1, F2, prev, window, 0.9, ori)
    p = prev.copy()
    n, m12 = ORBmatcher(ctx, nnratio=0.9, checkOri=ori).SearchForInitialization(F1, F2, p, window)
    same((n, m12, p), ref)
    assert n > 200
    st = ctx.match_last_stats()
    assert st["rounds"] >= 2 and not st["serial"]  # the fixed point ran (and resolved steals)


@pytest.mark.gpu
def test_gpu_serial_paths(ctx, oracle):
    """The one-wave sequential walk: (a) more level-0 F2 keypoints than the claim tables hold; (b) a
    pile-up of 12 F1 keypoints stealing one F2 keypoint in turn (claim-list overflow)."""
    m = ORBmatcher(ctx, nnratio=0.9)
    F1, F2, prev = fr.synth_init_pair(np.random.default_rng(9800), n1=3000, n2=6000, level0=1.0)
    ref = oc.initialization(oracle, F1, F2, prev, 100, 0.9, True)
    p = prev.copy()
    same((*m.SearchForInitialization(F1, F2, p, 100), p), ref)
    assert ctx.match_last_stats()["serial"]
    # (b): F1 keypoint k has a copy of F2 0's descriptor with 12 - k flipped bits
    d2 = np.stack([bits(0), bits(200)])
    d1 = np.stack([bits(12 - k) for k in range(12)])
    F1 = fr.FrameSoA(desc=d1, kp_x=np.full(12, 100, np.float32), kp_y=np.full(12, 100, np.float32),
                     kp_angle=np.zeros(12, np.float32), kp_octave=np.zeros(12, np.int32))
    F2 = fr.FrameSoA(desc=d2, kp_x=np.array([100, 110], np.float32), kp_y=np.array([100, 100], np.float32),
                     kp_angle=np.zeros(2, np.float32), kp_octave=np.zeros(2, np.int32))
    prev = np.stack([F1.kp_x, F1.kp_y], axis=1).astype(np.float32)
    ref = oc.initialization(oracle, F1, F2, prev, 100, 0.9, True)
    p = prev.copy()
    same((*m.SearchForInitialization(F1, F2, p, 100), p), ref)
    assert ref[1].tolist() == [-1] * 11 + [0]
    assert ctx.match_last_stats()["serial"]


@pytest.mark.gpu
def test_gpu_hand_case_and_edges(ctx, oracle):
    m = ORBmatcher(ctx, nnratio=0.9)
    F1, F2, prev = hand_case()
    n, m12 = m.SearchForInitialization(F1, F2, prev, 100)
    assert m12.tolist() == [-1, -1, 0, 1] and n == 2
    rng = np.random.default_rng(9700)
    F1, F2, prev = fr.synth_init_pair(rng, n1=500, n2=500)
    E = fr.FrameSoA(desc=np.zeros((0, 32), np.uint8), kp_x=[], kp_y=[], kp_angle=[], kp_octave=[])
    assert m.SearchForInitialization(E, F2, np.zeros((0, 2), np.float32), 100)[0] == 0
    n, m12 = m.SearchForInitialization(F1, E, prev.copy(), 100)
    assert n == 0 and (m12 == -1).all()
    far = np.full_like(prev, -5000.0)
    ref = oc.initialization(oracle, F1, F2, far, 100, 0.9, True)
    got = m.SearchForInitialization(F1, F2, far.copy(), 100)
    assert got[0] == ref[0] == 0
