"""MapPoint::ComputeDistinctiveDescriptors (ref:src/MapPoint.cc:444-535): the oracle pinned by a numpy
restatement and hand cases (CPU), and the GPU list form bit-exact against the oracle."""
import numpy as np
import pytest

from orb_slam3_comments_ghr_amd import mappoint as mp
from tests import oracle_calls as oc
from tests import pyref_match as pr


def rows(*bit_counts):
    out = np.zeros((len(bit_counts), 32), np.uint8)
    for i, k in enumerate(bit_counts):
        b = np.zeros(256, np.uint8)
        b[:k] = 1
        out[i] = np.packbits(b)
    return out


@pytest.mark.parametrize("seed", range(3))
def test_oracle_vs_numpy(oracle, seed):
    lists = mp.synth_observations(np.random.default_rng(8000 + seed), n_points=300, n_max=40)
    desc, start = mp.to_csr(lists)
    np.testing.assert_array_equal(oc.distinctive(oracle, desc, start), pr.distinctive(lists))


def test_hand_cases(oracle):
    """N = 0 -> -1; N = 1, 2 -> row 0 (the median of a 2-row includes the self-distance 0); rows with
    0, 10, 20, 30 set bits (distances |i - j| * 10): medians at index 1 are 10, 10, 10, 10 -> row 0;
    with a far row 200 added (N = 5, index 2): medians 20, 10, 10, 20, 180 -> row 1."""
    lists = [np.zeros((0, 32), np.uint8), rows(5), rows(5, 40), rows(0, 10, 20, 30), rows(0, 10, 20, 30, 200)]
    desc, start = mp.to_csr(lists)
    want = [-1, 0, 0, 0, 1]
    assert oc.distinctive(oracle, desc, start).tolist() == want
    assert pr.distinctive(lists).tolist() == want


@pytest.mark.gpu
@pytest.mark.parametrize("n_max", [4, 30, 64, 200])
def test_gpu_vs_oracle(ctx, oracle, n_max):
    lists = mp.synth_observations(np.random.default_rng(8100 + n_max), n_points=3000, n_max=n_max)
    desc, start = mp.to_csr(lists)
    np.testing.assert_array_equal(mp.ComputeDistinctiveDescriptors(ctx, lists), oc.distinctive(oracle, desc, start))


@pytest.mark.gpu
def test_gpu_edges(ctx, oracle):
    lists = [np.zeros((0, 32), np.uint8), rows(5), rows(5, 40), rows(0, 10, 20, 30), rows(0, 10, 20, 30, 200)]
    assert mp.ComputeDistinctiveDescriptors(ctx, lists).tolist() == [-1, 0, 0, 0, 1]
    assert mp.ComputeDistinctiveDescriptors(ctx, []).tolist() == []
    same = [np.repeat(rows(77), 65, 0)]  # 65 identical rows: every median 0, row 0 wins
    assert mp.ComputeDistinctiveDescriptors(ctx, same).tolist() == [0]
