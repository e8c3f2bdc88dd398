"""bench.py's cpu_baseline workers (tests/cpu_mt.py): every workload's oracle worker runs on 1 and on
2 threads with its arguments packed per thread, and a worker's outputs equal the oracle helpers'
(tests/oracle_calls.py) on the same frame, so the N-thread rate times the same computation."""
import numpy as np
import pytest

import bench
from orb_slam3_comments_ghr_amd import frames as fr
from orb_slam3_comments_ghr_amd import optimizer as op
from orb_slam3_comments_ghr_amd import orb, stereo as st, vocabulary as vb
from tests import cpu_mt


@pytest.fixture(autouse=True)
def _libm_off_after():
    """bench._oracle() switches the shared oracle library to the host libm (the cpu_baseline legs time
    the reference's own arithmetic); later tests in the session hold it to the correctly rounded path."""
    yield
    for lib, _ in bench._ORACLE:
        lib.oracle_set_libm(0)
    bench._ORACLE.clear()


def _runs(worker):
    for n in (1, 2):
        calls, el = cpu_mt.run(worker, n, 0.05)
        assert calls >= n and el > 0


def test_host_threads():
    n = cpu_mt.host_threads()
    assert 1 <= n <= (__import__("os").cpu_count() or 1)
    assert isinstance(cpu_mt.cpu_model(), str)


def test_baseline_object():
    q = np.random.default_rng(1).integers(0, 256, (64, 32), dtype=np.uint8)
    t = np.random.default_rng(2).integers(0, 256, (128, 32), dtype=np.uint8)
    cb = bench.cpu_baseline(q, t, 0.3)
    assert cb["cores"] == cpu_mt.host_threads() and cb["value"] > 0 and cb["value_1thread"] > 0
    assert cb["node_estimate"]["threads"] == __import__("os").cpu_count()


def test_c3_worker():
    rng = np.random.default_rng(3)
    pairs = [fr.synth_bow_pair(rng, n_kf=300, n_f=300, n_nodes=20) for _ in range(2)]
    probs = [op.synth_pose_problem(rng, n_edges=50) for _ in range(2)]
    _runs(bench._c3_worker(pairs, probs))


def test_c5_worker():
    rng = np.random.default_rng(4)
    F = [fr.synth_frame_two_cam(rng, n_left=200, n_right=200, stereo_frac=0.5, width=512, height=512)
         for _ in range(2)]
    L = [fr.synth_last_queries_two_cam(rng, f, n_last=300) for f in F]
    Q = [fr.synth_mp_queries_two_cam(rng, f, m=300) for f in F]
    S = [fr.synth_slots(rng, f.n, frac_assigned=0.05) for f in F]
    probs = [op.synth_pose_problem(rng, n_edges=60, cam=op.kb8_camera(), body_frac=0.4) for _ in range(2)]
    _runs(bench._c5_worker(F, L, Q, S, probs))


def test_dbow_worker():
    rng = np.random.default_rng(5)
    voc = vb.synth_vocabulary(rng, k=4, L=3, min_children=2, min_leaf_depth=3)
    pool = [vb.synth_features(rng, voc, n=100) for _ in range(3)]
    _runs(bench._dbow_worker(voc, pool))


def test_stereo_worker():
    rng = np.random.default_rng(6)
    pool = [st.synth_stereo_frame(rng, n=200) for _ in range(2)]
    _runs(bench._stereo_worker(pool))


def test_orb_worker():
    rng = np.random.default_rng(7)
    pool = [orb.synth_orb_frame(rng, n=200, edge=16) for _ in range(2)]
    _runs(bench._orb_worker(pool, orb.synth_pattern(rng)))


def test_lba_worker_matches_oracle_helper():
    from tests import oracle_calls as oc
    rng = np.random.default_rng(8)
    G = op.synth_lba_graph(rng, n_kf=6, n_points=200)
    _runs(bench._lba_worker([G]))
    # the worker's call is the helper's call: same graph -> same iterations as oc.lba
    lib = oc.load()
    assert oc.lba(lib, G).iterations == oc.lba(lib, G).iterations


@pytest.mark.parametrize("n", [1, 3])
def test_run_counts_every_thread(n):
    seen = set()

    def worker(tid):
        return lambda i: seen.add(tid)
    calls, _ = cpu_mt.run(worker, n, 0.02)
    assert seen == set(range(n)) and calls >= n
