"""GPU parity: the ORBmatcher search operators through the C ABI against the CPU oracle —
bit-exact match assignments and counts, on seeded synthetic frames (SURVEY.md §8d C3 shapes)."""
import numpy as np
import pytest

from tests import oracle_calls as oc
from orb_slam3_comments_ghr_amd import frames as fr
from orb_slam3_comments_ghr_amd.matcher import ORBmatcher

pytestmark = pytest.mark.gpu


def assert_same(name, got_n, got_s, ref_n, ref_s):
    bad = np.nonzero(got_s != ref_s)[0]
    assert bad.size == 0, f"{name}: {bad.size} slots differ, first {bad[:8]}: got {got_s[bad[:8]]} ref {ref_s[bad[:8]]}"
    assert got_n == ref_n, f"{name}: nmatches {got_n} != {ref_n}"


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("th,nn,far", [(1.0, 0.8, False), (3.0, 0.8, False), (5.0, 0.6, True)])
def test_search_by_projection_mps(ctx, oracle, seed, th, nn, far):
    rng = np.random.default_rng(1000 + seed)
    F = fr.synth_frame(rng, n=1200, stereo=(seed % 2 == 0))
    Q = fr.synth_mp_queries(rng, F, m=3000)
    slot_mp, taken = fr.synth_slots(rng, F.n)
    ref = oc.mps(oracle, F, Q, nn, th, far, 20.0, slot_mp, taken)
    s = slot_mp.copy()
    n = ORBmatcher(ctx, nn).SearchByProjection(F, Q, th, far, 20.0, slot_mp=s, slot_taken=taken)
    assert_same("mps", n, s, *ref)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("th,mono,tlc", [(7.0, False, 0.0), (15.0, True, 0.0), (7.0, False, 1.0), (14.0, False, -1.0)])
def test_search_by_projection_last(ctx, oracle, seed, th, mono, tlc):
    rng = np.random.default_rng(2000 + seed)
    F = fr.synth_frame(rng, n=1200, stereo=not mono)
    L = fr.synth_last_queries(rng, F, n_last=1100, tlc_z=tlc)
    slot_mp, taken = fr.synth_slots(rng, F.n)
    for ori in (True, False):
        ref = oc.last(oracle, F, L, th, mono, ori, slot_mp, taken)
        s = slot_mp.copy()
        n = ORBmatcher(ctx, 0.9, ori).SearchByProjection(F, L, th, mono, slot_mp=s, slot_taken=taken)
        assert_same(f"last ori={ori}", n, s, *ref)


@pytest.mark.parametrize("prepass", ["0", "1"])
def test_candidate_overflow_retry(ctx, oracle, monkeypatch, prepass):
    """More than 32 candidates per query (the first candidate-buffer guess): the launch reports the
    overflow and the host retries with the exact size, with and without the prepass."""
    monkeypatch.setenv("OSG_MATCH_PREPASS", prepass)
    rng = np.random.default_rng(79)
    F = fr.synth_frame(rng, n=3000, stereo=False)
    Q = fr.synth_mp_queries(rng, F, m=300)
    Q.in_view[:] = 1
    Q.usable[:] = 1
    slot_mp, taken = fr.synth_slots(rng, F.n)
    ref = oc.mps(oracle, F, Q, 0.9, 40.0, False, 50.0, slot_mp, taken)
    s = slot_mp.copy()
    n = ORBmatcher(ctx, 0.9).SearchByProjection(F, Q, 40.0, slot_mp=s, slot_taken=taken)
    assert ctx.match_last_stats()["candidates"] > 32 * 300
    assert_same("overflow", n, s, *ref)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("th,orb", [(10.0, 100), (3.0, 64)])
def test_search_by_projection_kf(ctx, oracle, seed, th, orb):
    rng = np.random.default_rng(3000 + seed)
    F = fr.synth_frame(rng, n=1200)
    K = fr.synth_kf_queries(rng, F, n_kf=1000)
    slot_mp, _ = fr.synth_slots(rng, F.n, frac_assigned=0.2)
    for ori in (True, False):
        ref = oc.kf(oracle, F, K, th, orb, ori, slot_mp)
        s = slot_mp.copy()
        n = ORBmatcher(ctx, 0.75, ori).SearchByProjection(F, K, th, orb, slot_mp=s)
        assert_same(f"kf ori={ori}", n, s, *ref)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("nn", [0.7, 0.75, 0.9])
def test_search_by_bow_kf_f(ctx, oracle, seed, nn):
    rng = np.random.default_rng(4000 + seed)
    KF, F = fr.synth_bow_pair(rng, n_kf=1200, n_f=1200, n_nodes=100)
    for ori in (True, False):
        ref = oc.bow_kf_f(oracle, KF, F, nn, ori)
        n, out = ORBmatcher(ctx, nn, ori).SearchByBoW(KF, F)
        assert_same(f"bow kf-f ori={ori}", n, out, *ref)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("nn", [0.75, 0.9])
def test_search_by_bow_kf_kf(ctx, oracle, seed, nn):
    rng = np.random.default_rng(5000 + seed)
    K1, K2 = fr.synth_bow_pair(rng, n_kf=1100, n_f=1300, n_nodes=80, f_is_kf=True)
    for ori in (True, False):
        ref = oc.bow_kf_kf(oracle, K1, K2, nn, ori)
        n, out = ORBmatcher(ctx, nn, ori).SearchByBoW(K1, K2, kf2=True)
        assert_same(f"bow kf-kf ori={ori}", n, out, *ref)


@pytest.mark.parametrize("prepass", ["0", "1"])
def test_dense_conflicts_many_rounds(ctx, oracle, monkeypatch, prepass):
    """Adversarial greedy: many map points project onto the same few keypoints with nearly equal
    descriptors, forcing long claim chains in the fixed-point resolve.  With and without the
    multi-workgroup prepass (k_grid_*)."""
    monkeypatch.setenv("OSG_MATCH_PREPASS", prepass)
    rng = np.random.default_rng(77)
    F = fr.synth_frame(rng, n=400, stereo=False)
    Q = fr.synth_mp_queries(rng, F, m=4000, noise_px=0.5, match_frac=1.0)
    Q.in_view[:] = 1
    Q.usable[:] = 1
    Q.has_obs[:] = 1
    slot_mp = np.full(F.n, -1, np.int32)
    taken = np.zeros(F.n, np.uint8)
    ref = oc.mps(oracle, F, Q, 0.9, 4.0, False, 50.0, slot_mp, taken)
    s = slot_mp.copy()
    n = ORBmatcher(ctx, 0.9).SearchByProjection(F, Q, 4.0, slot_mp=s, slot_taken=taken)
    assert_same("dense", n, s, *ref)


def test_empty_inputs(ctx):
    rng = np.random.default_rng(5)
    F = fr.synth_frame(rng, n=50)
    Q = fr.synth_mp_queries(rng, F, m=0)
    s = np.full(F.n, -1, np.int32)
    assert ORBmatcher(ctx).SearchByProjection(F, Q, 3.0, slot_mp=s, slot_taken=np.zeros(F.n, np.uint8)) == 0
    assert (s == -1).all()


# ---- two-camera rigs (Frame::Nleft != -1)

def two_cam(rng, nl=700, nr=650):
    return fr.synth_frame_two_cam(rng, n_left=nl, n_right=nr, stereo_frac=0.6)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("th,nn,far", [(1.0, 0.8, False), (3.0, 0.8, False), (5.0, 0.6, True)])
def test_search_by_projection_mps_two_cam(ctx, oracle, seed, th, nn, far):
    """a5 right-camera pass: stereo-partner writes, the ratio-failure skip, own-left blocking.
    Seeds with every MapPoint observed run the Jacobi resolve alone; the others include
    observation-less MapPoints whose partner writes unblock slots (serial redo)."""
    rng = np.random.default_rng(6000 + seed)
    F = two_cam(rng)
    Q = fr.synth_mp_queries_two_cam(rng, F, m=2000)
    if seed < 2:
        Q.has_obs[:] = 1
    slot_mp, taken = fr.synth_slots(rng, F.n, frac_assigned=0.15)
    ref = oc.mps(oracle, F, Q, nn, th, far, 20.0, slot_mp, taken)
    s = slot_mp.copy()
    n = ORBmatcher(ctx, nn).SearchByProjection(F, Q, th, far, 20.0, slot_mp=s, slot_taken=taken)
    assert_same("mps two-cam", n, s, *ref)
    if seed < 2:
        assert not ctx.match_last_stats()["serial"]


@pytest.mark.parametrize("prepass", ["0", "1"])
def test_search_by_projection_mps_two_cam_paths(ctx, oracle, monkeypatch, prepass):
    """Both resolve paths are exercised: all-observed (Jacobi only) and a run that must be redone
    serially because an observation-less MapPoint's partner write unblocks a slot; with the candidate
    lists from k_match itself and from the k_grid_* prepass."""
    monkeypatch.setenv("OSG_MATCH_PREPASS", prepass)
    seen = set()
    for seed in range(12):
        rng = np.random.default_rng(6100 + seed)
        F = two_cam(rng, 400, 380)
        Q = fr.synth_mp_queries_two_cam(rng, F, m=1500, noise_px=1.0, match_frac=0.9)
        Q.has_obs[:] = rng.random(len(Q.mp_id)) < 0.6
        slot_mp, taken = fr.synth_slots(rng, F.n, frac_assigned=0.4, frac_taken=0.9)
        ref = oc.mps(oracle, F, Q, 0.9, 3.0, False, 20.0, slot_mp, taken)
        s = slot_mp.copy()
        n = ORBmatcher(ctx, 0.9).SearchByProjection(F, Q, 3.0, False, 20.0, slot_mp=s, slot_taken=taken)
        assert_same(f"mps two-cam seed {seed}", n, s, *ref)
        seen.add(ctx.match_last_stats()["serial"])
    assert True in seen


@pytest.mark.parametrize("seed", range(4))
def test_search_by_projection_mps_two_cam_dense_conflicts(ctx, oracle, seed):
    """The serial redo's 64-query speculative batches under heavy conflicts: few keypoints, many
    queries on the same slots, so most batches stop early and commit a prefix."""
    rng = np.random.default_rng(6200 + seed)
    F = two_cam(rng, 70, 60)
    Q = fr.synth_mp_queries_two_cam(rng, F, m=900, noise_px=1.0, match_frac=0.95)
    Q.has_obs[:] = rng.random(len(Q.mp_id)) < 0.5
    slot_mp, taken = fr.synth_slots(rng, F.n, frac_assigned=0.3, frac_taken=0.5)
    ref = oc.mps(oracle, F, Q, 0.95, 5.0, False, 20.0, slot_mp, taken)
    s = slot_mp.copy()
    n = ORBmatcher(ctx, 0.95).SearchByProjection(F, Q, 5.0, False, 20.0, slot_mp=s, slot_taken=taken)
    assert_same(f"mps two-cam dense seed {seed}", n, s, *ref)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("th,mono,tlc", [(7.0, False, 0.0), (15.0, True, 0.0), (7.0, False, 1.0), (14.0, False, -1.0)])
def test_search_by_projection_last_two_cam(ctx, oracle, seed, th, mono, tlc):
    rng = np.random.default_rng(7000 + seed)
    F = two_cam(rng)
    L = fr.synth_last_queries_two_cam(rng, F, n_last=1000, tlc_z=tlc)
    slot_mp, taken = fr.synth_slots(rng, F.n)
    for ori in (True, False):
        ref = oc.last(oracle, F, L, th, mono, ori, slot_mp, taken)
        s = slot_mp.copy()
        n = ORBmatcher(ctx, 0.9, ori).SearchByProjection(F, L, th, mono, slot_mp=s, slot_taken=taken)
        assert_same(f"last two-cam ori={ori}", n, s, *ref)


def test_search_by_projection_kf_two_cam(ctx, oracle):
    rng = np.random.default_rng(7500)
    F = two_cam(rng)
    K = fr.synth_kf_queries(rng, F, n_kf=900)
    slot_mp, _ = fr.synth_slots(rng, F.n, frac_assigned=0.2)
    for ori in (True, False):
        ref = oc.kf(oracle, F, K, 10.0, 100, ori, slot_mp)
        s = slot_mp.copy()
        n = ORBmatcher(ctx, 0.75, ori).SearchByProjection(F, K, 10.0, 100, slot_mp=s)
        assert_same(f"kf two-cam ori={ori}", n, s, *ref)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("nn", [0.7, 0.9])
def test_search_by_bow_two_cam(ctx, oracle, seed, nn):
    rng = np.random.default_rng(8000 + seed)
    KF, F = fr.synth_bow_pair(rng, n_kf=1200, n_f=1200, n_nodes=100, nleft_kf=640, nleft_f=600)
    K1, K2 = fr.synth_bow_pair(rng, n_kf=1100, n_f=1300, n_nodes=80, f_is_kf=True, nleft_kf=560, nleft_f=700)
    for ori in (True, False):
        ref = oc.bow_kf_f(oracle, KF, F, nn, ori)
        n, out = ORBmatcher(ctx, nn, ori).SearchByBoW(KF, F)
        assert_same(f"bow kf-f two-cam ori={ori}", n, out, *ref)
        ref = oc.bow_kf_kf(oracle, K1, K2, nn, ori)
        n, out = ORBmatcher(ctx, nn, ori).SearchByBoW(K1, K2, kf2=True)
        assert_same(f"bow kf-kf two-cam ori={ori}", n, out, *ref)


# ---- batched forms: B problems in one launch equal B single calls (and the oracle)

@pytest.mark.parametrize("prepass", [None, "0", "1"])
def test_batch_projection_all_overloads(ctx, oracle, monkeypatch, prepass):
    """Batches of a5 / a6 / a7 problems (one- and two-camera, an empty query set): every problem
    equals the oracle, with the k_grid_* prepass pinned on or off, and by default (on for <= 64)."""
    if prepass is not None:
        monkeypatch.setenv("OSG_MATCH_PREPASS", prepass)
    rng = np.random.default_rng(9000)
    B = 24
    m = ORBmatcher(ctx, 0.8, True)
    # a5, mixing one-camera and two-camera frames, and an empty query set
    Fs = [fr.synth_frame(rng, n=900, stereo=(b % 2 == 0)) if b % 3 else two_cam(rng, 500, 450) for b in range(B)]
    Qs = [fr.synth_mp_queries_two_cam(rng, F, m=1200) if F.nleft != -1 else fr.synth_mp_queries(rng, F, m=1500)
          for F in Fs]
    Qs[5] = fr.synth_mp_queries(rng, Fs[5], m=0)
    slots = [fr.synth_slots(rng, F.n) for F in Fs]
    s_in = [s.copy() for s, _ in slots]
    nm = m.SearchByProjectionBatch(Fs, Qs, 3.0, False, 20.0, slot_mps=s_in, slot_takens=[t for _, t in slots])
    for b in range(B):
        ref = oc.mps(oracle, Fs[b], Qs[b], 0.8, 3.0, False, 20.0, slots[b][0], slots[b][1])
        assert_same(f"mps batch [{b}]", int(nm[b]), s_in[b], *ref)
    # a6
    Ls = [fr.synth_last_queries_two_cam(rng, F, n_last=600) if F.nleft != -1 else fr.synth_last_queries(rng, F, 700)
          for F in Fs]
    s_in = [s.copy() for s, _ in slots]
    nm = m.SearchByProjectionBatch(Fs, Ls, 7.0, False, slot_mps=s_in, slot_takens=[t for _, t in slots])
    for b in range(B):
        ref = oc.last(oracle, Fs[b], Ls[b], 7.0, False, True, slots[b][0], slots[b][1])
        assert_same(f"last batch [{b}]", int(nm[b]), s_in[b], *ref)
    # a7
    Ks = [fr.synth_kf_queries(rng, F, n_kf=500) for F in Fs]
    s_in = [s.copy() for s, _ in slots]
    nm = m.SearchByProjectionBatch(Fs, Ks, 10.0, 100, slot_mps=s_in)
    for b in range(B):
        ref = oc.kf(oracle, Fs[b], Ks[b], 10.0, 100, True, slots[b][0])
        assert_same(f"kf batch [{b}]", int(nm[b]), s_in[b], *ref)


@pytest.mark.parametrize("kf2", [False, True])
def test_batch_bow(ctx, oracle, kf2):
    rng = np.random.default_rng(9100 + kf2)
    B = 40
    pairs = [fr.synth_bow_pair(rng, n_kf=800 + 10 * b, n_f=900, n_nodes=60, f_is_kf=kf2,
                               nleft_kf=(400 if b % 4 == 0 else -1), nleft_f=(450 if b % 4 == 0 else -1))
             for b in range(B)]
    m = ORBmatcher(ctx, 0.75, True)
    nm, outs = m.SearchByBoWBatch([p[0] for p in pairs], [p[1] for p in pairs], kf2=kf2)
    for b, (A, Bs) in enumerate(pairs):
        ref = (oc.bow_kf_kf if kf2 else oc.bow_kf_f)(oracle, A, Bs, 0.75, True)
        assert_same(f"bow batch [{b}]", int(nm[b]), outs[b], *ref)


def test_pinned_staging_reused_back_to_back(ctx, oracle):
    """The pinned staging block is rewritten at the same offsets by consecutive calls (uploads and
    downloads by copy kernels over PCIe): alternating different frames through one context, every
    call must see its own inputs and return its own results (no stale line from the previous call)."""
    rng = np.random.default_rng(4242)
    cases = []
    for k in range(4):
        F = fr.synth_frame(rng, n=600, stereo=(k % 2 == 0))
        Q = fr.synth_mp_queries(rng, F, m=900)
        slot_mp, taken = fr.synth_slots(rng, F.n)
        cases.append((F, Q, slot_mp, taken, oc.mps(oracle, F, Q, 0.8, 3.0, False, 20.0, slot_mp, taken)))
    m = ORBmatcher(ctx, 0.8)
    for rep in range(3):
        for i, (F, Q, slot_mp, taken, ref) in enumerate(cases):
            s = slot_mp.copy()
            n = m.SearchByProjection(F, Q, 3.0, False, 20.0, slot_mp=s, slot_taken=taken)
            assert_same(f"rep {rep} case {i}", n, s, *ref)
