"""Frame::ComputeStereoMatches (ref:src/Frame.cc:1117-1373): the C oracle pinned by the pure-Python
restatement and two hand cases (CPU); the GPU path bit-exact against the oracle (mvuRight / mvDepth bit
patterns and match counts) on EuRoC-shaped stereo pairs, batches, device-resident pyramids and edges."""
import numpy as np
import pytest

from orb_slam3_comments_ghr_amd import stereo as st
from tests import oracle_calls as oc
from tests import pyref_stereo as ps

MBF = 47.9


def same(a, b):
    np.testing.assert_array_equal(np.asarray(a[0]).view(np.int32), np.asarray(b[0]).view(np.int32))
    np.testing.assert_array_equal(np.asarray(a[1]).view(np.int32), np.asarray(b[1]).view(np.int32))
    assert int(a[2]) == int(b[2])


def hand_frame(noisy):
    """40 x 80 single-level pair.  Columns < 44 of the right image are the left image shifted 4 px
    (plus +-6 noise when `noisy`); columns >= 44 are identical and mirror-symmetric about column 60.
    Keypoints (16, 10), (22, 20), (28, 30) match right keypoints 4 px to the left; keypoint (60, 20)
    matches (60, 20) at zero disparity (noisy case only)."""
    rng = np.random.default_rng(4242)
    L = rng.integers(0, 256, (40, 80)).astype(np.int64)
    for k in range(1, 16):
        L[:, 60 + k] = L[:, 60 - k]
    R = L.copy()
    R[:, :44] = L[:, 4:48] + (rng.integers(-6, 7, (40, 44)) if noisy else 0)
    L, R = (np.clip(a, 0, 255).astype(np.uint8) for a in (L, R))
    u = [16.0, 22.0, 28.0] + ([60.0] if noisy else [])
    v = [10.0, 20.0, 30.0] + ([20.0] if noisy else [])
    ur = [x - 4 for x in u[:3]] + ([60.0] if noisy else [])
    desc = rng.integers(0, 256, (len(u), 32), dtype=np.uint8)
    one = st.ImagePyramid
    return st.StereoFrame(desc=desc, x=u, y=v, octave=np.zeros(len(u)), desc_r=desc.copy(), xr=ur, yr=v,
                          octave_r=np.zeros(len(u)), left=one([L]), right=one([R]), scale=[1.0], mbf=MBF)


def check_hand(res):
    """noise-free: every SAD minimum is 0, so the median is 0 and `dist < 0` never holds — the
    reference's cut removes every match.  Noisy: the three shifted matches land within half a pixel
    of 4 px, the zero-disparity one takes the 0.01 clamp (bestuR = uL - 0.01 in double)."""
    (ur0, d0, n0), (ur1, d1, n1) = res
    assert n0 == 0 and (ur0 == -1).all() and (d0 == -1).all()
    assert n1 == 4
    np.testing.assert_allclose(ur1[:3], [12, 18, 24], atol=0.5)
    np.testing.assert_array_equal(d1[:3], (np.float32(MBF) / (np.float32([16, 22, 28]) - ur1[:3])).astype(np.float32))
    assert ur1[3] == np.float32(60.0 - 0.01) and d1[3] == np.float32(np.float32(MBF) / np.float32(0.01))


@pytest.mark.parametrize("seed", range(3))
def test_oracle_vs_python(oracle, seed):
    F = st.synth_stereo_frame(np.random.default_rng(9900 + seed), n=300, bordered=seed == 2)
    ref = oc.stereo(oracle, F)
    ur, d, n, accepted = ps.compute_stereo_matches(F, stats=True)
    same(ref, (ur, d, n))
    assert n > 150 and accepted > n  # the median cut removed some
    assert (np.abs(ur[ur >= 0] - np.round(ur[ur >= 0])) > 1e-3).mean() > 0.5  # sub-pixel positions


def test_oracle_hand_cases(oracle):
    res = [oc.stereo(oracle, hand_frame(False)), oc.stereo(oracle, hand_frame(True))]
    check_hand(res)
    for noisy, r in zip((False, True), res):
        same(r, ps.compute_stereo_matches(hand_frame(noisy)))


def test_oracle_empty_and_edges(oracle):
    F = st.synth_stereo_frame(np.random.default_rng(9910), n=200, edge=0.0)
    same(oc.stereo(oracle, F), ps.compute_stereo_matches(F))  # patches leaving the image: no match
    E = st.StereoFrame(desc=F.desc[:0], x=[], y=[], octave=[], desc_r=F.desc_r, xr=F.xr, yr=F.yr,
                       octave_r=F.octave_r, left=F.left, right=F.right)
    assert oc.stereo(oracle, E)[2] == 0
    R0 = st.StereoFrame(desc=F.desc, x=F.x, y=F.y, octave=F.octave, desc_r=F.desc_r[:0], xr=[], yr=[], octave_r=[],
                        left=F.left, right=F.right)
    ur, d, n = oc.stereo(oracle, R0)
    assert n == 0 and (ur == -1).all() and (d == -1).all()


# ----------------------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_vs_oracle(ctx, oracle, seed):
    """EuRoC stereo shape: 752 x 480, 8 levels x 1.2, 1200 keypoints per side (nFeatures 1200)."""
    F = st.synth_stereo_frame(np.random.default_rng(9950 + seed), n=1200, bordered=bool(seed % 2))
    ref = oc.stereo(oracle, F)
    same(st.ComputeStereoMatches(ctx, F), ref)
    assert ref[2] > 500


@pytest.mark.gpu
def test_gpu_batch_and_device_pyramids(ctx, oracle):
    rng = np.random.default_rng(9970)
    frames = [st.synth_stereo_frame(rng, n=int(rng.integers(200, 1500)), bordered=bool(i % 3 == 0)) for i in range(10)]
    F = frames[0]
    frames.append(st.StereoFrame(desc=F.desc[:0], x=[], y=[], octave=[], desc_r=F.desc_r, xr=F.xr, yr=F.yr,
                                 octave_r=F.octave_r, left=F.left, right=F.right))
    frames.append(st.StereoFrame(desc=F.desc, x=F.x, y=F.y, octave=F.octave, desc_r=F.desc_r[:0], xr=[], yr=[],
                                 octave_r=[], left=F.left, right=F.right))
    refs = [oc.stereo(oracle, f) for f in frames]
    outs, nm = st.ComputeStereoMatchesBatch(ctx, frames)
    for (ur, d), k, r in zip(outs, nm, refs):
        same((ur, d, k), r)
    # the same frames with both pyramids resident in HBM (read in place, torch row strides)
    dev = [f.to_device() for f in frames[:6]]
    outs, nm = st.ComputeStereoMatchesBatch(ctx, dev)
    for (ur, d), k, r in zip(outs, nm, refs[:6]):
        same((ur, d, k), r)
    assert st.ComputeStereoMatchesBatch(ctx, [])[1].size == 0


@pytest.mark.gpu
def test_gpu_hand_cases_and_edges(ctx, oracle):
    check_hand([st.ComputeStereoMatches(ctx, hand_frame(False)), st.ComputeStereoMatches(ctx, hand_frame(True))])
    rng = np.random.default_rng(9980)
    F = st.synth_stereo_frame(rng, n=600, edge=0.0)  # patches leaving the level images
    same(st.ComputeStereoMatches(ctx, F), oc.stereo(oracle, F))
    # one dense row band: every left keypoint on row 200 sees all 700 right keypoints (> 64 per lane pass)
    F = st.synth_stereo_frame(rng, n=500, n_right=700)
    D = st.StereoFrame(desc=F.desc, x=F.x, y=np.full(F.n, 200.3, np.float32), octave=F.octave, desc_r=F.desc_r,
                       xr=F.xr, yr=np.full(F.n_right, 200.6, np.float32), octave_r=F.octave_r, left=F.left,
                       right=F.right)
    ref = oc.stereo(oracle, D)
    same(st.ComputeStereoMatches(ctx, D), ref)
    assert ref[2] > 50


@pytest.mark.gpu
def test_gpu_device_row_index(ctx, oracle):
    """vRowIndices built on the device (k_stereo_rows: LDS counts, block scan, atomic fill in any order):
    * a 1100-row image (more rows than the workgroup's 1024 threads: two rows per scan segment);
    * keypoints 2 px from the top and bottom, whose row bands the reference would index past (clipped);
    * 30 % exact duplicates on the same row: Hamming ties resolve to the lowest right index, as the
      reference's ascending candidate vector does."""
    rng = np.random.default_rng(9995)
    F = st.synth_stereo_frame(rng, n=900, width=800, height=1100, edge=2.0, dup=0.3)
    yr = np.array(F.yr, np.float32)
    yr[:20] = rng.uniform(0.0, 1.5, 20)
    yr[20:40] = 1099.0 - rng.uniform(0.0, 1.5, 20)
    F = st.StereoFrame(desc=F.desc, x=F.x, y=F.y, octave=F.octave, desc_r=F.desc_r, xr=F.xr, yr=yr,
                       octave_r=F.octave_r, left=F.left, right=F.right)
    ref = oc.stereo(oracle, F)
    same(st.ComputeStereoMatches(ctx, F), ref)
    assert ref[2] > 200
    outs, nm = st.ComputeStereoMatchesBatch(ctx, [F, F])
    for (ur, d), k in zip(outs, nm):
        same((ur, d, k), ref)
