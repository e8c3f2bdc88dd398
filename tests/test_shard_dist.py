"""Multi-GPU partitioning (orb_slam3_comments_ghr_amd/shard.py) checked against one
process: the train-sharded top-2 merge is bit-exact with the serial loop over the whole train set,
and C5-style sequences sharded over ranks and gathered give every sequence's single-process result.

CPU: world_size 2 over gloo (127.0.0.1) with the oracle as the per-rank compute.  GPU: the same
partitioning with the C-ABI kernel as the compute — in one process over K simulated shards, and
over 2 gloo ranks sharing cuda:0."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from orb_slam3_comments_ghr_amd import shard, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_top2(lib):
    def top2(q, t):
        nq = q.shape[0]
        out = [np.empty(nq, np.int32) for _ in range(3)]
        lib.oracle_hamming_top2(q.ctypes.data, nq, t.ctypes.data, t.shape[0], *[o.ctypes.data for o in out])
        return tuple(out)
    return top2


def _split(n, cuts):
    b = [0] + sorted(cuts) + [n]
    return list(zip(b[:-1], b[1:]))


def test_shard_rows_cover_in_order():
    for n in (0, 1, 7, 2000):
        for world in (1, 2, 3, 8):
            rs = [shard.shard_rows(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs[:-1], rs[1:]))
            assert max(e - b for b, e in rs) - min(e - b for b, e in rs) <= 1


def test_shard_units_round_robin():
    assert shard.shard_units(5, 0, 2) == [0, 2, 4] and shard.shard_units(5, 1, 2) == [1, 3]
    assert sorted(sum((shard.shard_units(11, r, 4) for r in range(4)), [])) == list(range(11))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_merge_top2_equals_serial_loop(oracle, seed):
    """Shards of the C2 generator's train set (planted near-duplicates, 5 % exact duplicate rows:
    ties across shard borders), including empty shards, merged == one serial pass."""
    rng = np.random.default_rng(seed)
    q, t = synth.descriptors_c2(300, 900, seed=synth.SEED_C2 + seed)
    # duplicates straddling shard borders: copy rows across the cut points
    cuts = sorted(rng.choice(np.arange(1, 900), size=4, replace=False).tolist()) + [450, 450]
    for c in cuts[:4]:
        t[c] = t[c - 1]
    top2 = _oracle_top2(oracle)
    want = top2(q, t)
    parts = []
    for b, e in _split(900, cuts):
        bi, bd, sd = top2(q, np.ascontiguousarray(t[b:e]))
        parts.append((np.where(bi >= 0, bi + b, -1), bd, sd))
    got = shard.merge_top2(parts)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


def test_merge_top2_no_row_below_sentinel(oracle):
    """A query whose every train row is its bitwise complement (distance 256): idx stays -1."""
    q = np.random.default_rng(5).integers(0, 256, (3, 32), dtype=np.uint8)
    t = np.ascontiguousarray(np.repeat(~q[:1], 6, axis=0))
    top2 = _oracle_top2(oracle)
    want = top2(q, t)
    parts = [(np.where(p[0] >= 0, p[0] + b, -1), p[1], p[2])
             for b, e in _split(6, [2, 4]) for p in [top2(q, np.ascontiguousarray(t[b:e]))]]
    got = shard.merge_top2(parts)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    assert got[0][0] == -1 and got[1][0] == 256


# ---------------------------------------------------------------- world_size 2 over gloo (CPU)
def _c5_units(n_seq, frames_per_seq=2, full=False):
    """C5-style sequences: per frame, a two-camera KB8 frame with LastF and local-map queries and a pose
    problem (seeded by sequence, SURVEY.md §8(d) C5: seeds 0x0B5EED10 + seq).  Small frames for the CPU
    gloo test; full=True the bench's C5 frame (2 x 1000 keypoints, 2000 LastF and 1500 local-map
    queries, a 600-edge pose problem)."""
    nk, nl, nm, ne = (1000, 2000, 1500, 600) if full else (150, 200, 200, 60)
    from orb_slam3_comments_ghr_amd import frames as fr, optimizer as op
    seqs = []
    for s in range(n_seq):
        rng = np.random.default_rng(0x0B5EED10 + s)
        frames = []
        for _ in range(frames_per_seq):
            F = fr.synth_frame_two_cam(rng, n_left=nk, n_right=nk, stereo_frac=0.5, width=512, height=512)
            frames.append((F, fr.synth_last_queries_two_cam(rng, F, n_last=nl),
                           fr.synth_mp_queries_two_cam(rng, F, m=nm), fr.synth_slots(rng, F.n, frac_assigned=0.05),
                           op.synth_pose_problem(rng, n_edges=ne, cam=op.kb8_camera(), body_frac=0.4)))
        seqs.append(frames)
    return seqs


def _c5_oracle_sequence(lib, frames):
    from tests import oracle_calls as oc
    out = []
    for F, L, Q, S, P in frames:
        n1, s1 = oc.last(lib, F, L, 7.0, False, True, S[0], S[1])
        n2, s2 = oc.mps(lib, F, Q, 0.9, 3.0, False, 20.0, S[0], S[1])
        r = oc.pose(lib, [P])[0]
        out.append((int(n1), s1.tolist(), int(n2), s2.tolist(), r.pose.tolist(), r.outlier.tolist(), int(r.n_inliers)))
    return out


def _gloo_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from tests import oracle_calls as oc
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = oc.load()
    # train-sharded C2': this rank holds rows [b, e) of the train set, queries replicated
    qd, td = synth.descriptors_c2(200, 1001, seed=synth.SEED_C2_STREAM)
    b, e = shard.shard_rows(td.shape[0], rank, world)
    merged = shard.train_sharded_top2(_oracle_top2(lib), qd, np.ascontiguousarray(td[b:e]), b, dist)
    # C5: one sequence per rank (round-robin), results gathered once at the end
    seqs = _c5_units(3)
    local = shard.run_sharded(lambda fr_: _c5_oracle_sequence(lib, fr_), seqs, dist)
    everything = shard.gather_results(local, dist)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, [m.tolist() for m in merged], sorted(local), everything))


def test_sharded_paths_gloo_world2(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    qd, td = synth.descriptors_c2(200, 1001, seed=synth.SEED_C2_STREAM)
    want = [w.tolist() for w in _oracle_top2(oracle)(qd, td)]
    seqs = _c5_units(3)
    want_seq = {i: _c5_oracle_sequence(oracle, s) for i, s in enumerate(seqs)}
    owned = set()
    for rank, merged, mine, everything in res:
        assert merged == want, f"rank {rank}: train-sharded top-2 != one serial pass"
        assert mine == shard.shard_units(3, rank, world)
        owned |= set(mine)
        assert everything == want_seq, f"rank {rank}: gathered sequences != single-process run"
    assert owned == {0, 1, 2}


# ---------------------------------------------------------------- the GPU kernel as the compute
def _gpu_top2(ctx):
    return lambda q, t: ctx.hamming_top2(q, t)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 3, 8])
def test_train_sharded_top2_gpu(ctx, oracle, k):
    """K train shards through the C-ABI kernel, merged: bit-exact with the oracle's serial pass."""
    qd, td = synth.descriptors_c2(1000, 20000, seed=synth.SEED_C2_STREAM + k)
    parts = []
    for r in range(k):
        b, e = shard.shard_rows(td.shape[0], r, k)
        parts.append(shard.train_sharded_top2(_gpu_top2(ctx), qd, np.ascontiguousarray(td[b:e]), b))
    got = shard.merge_top2(parts)
    want = _oracle_top2(oracle)(qd, td)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


def _gpu_gloo_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from orb_slam3_comments_ghr_amd import Context
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = Context(0)
    qd, td = synth.descriptors_c2(500, 30001, seed=synth.SEED_C2_STREAM + 9)
    b, e = shard.shard_rows(td.shape[0], rank, world)
    merged = shard.train_sharded_top2(_gpu_top2(ctx), qd, np.ascontiguousarray(td[b:e]), b, dist)
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, [m.tolist() for m in merged]))


@pytest.mark.gpu
def test_train_sharded_top2_gpu_two_ranks(oracle):
    """Two processes on cuda:0, each with half the train rows, exchanging over gloo: every rank's
    merged result is the oracle's serial pass."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    qd, td = synth.descriptors_c2(500, 30001, seed=synth.SEED_C2_STREAM + 9)
    want = [w.tolist() for w in _oracle_top2(oracle)(qd, td)]
    for rank, merged in res:
        assert merged == want


# ------------------------------------------- config 5 on the HIP path: sequences sharded over ranks
def _c5_gpu_sequence(ctx, frames):
    """_c5_oracle_sequence through the C-ABI kernels: per frame, two-camera KB8
    SearchByProjection(F, LastF) and SearchByProjection(F, local map) (k_match) and
    PoseOptimization (k_pose_opt), with the same arguments as the oracle run."""
    from orb_slam3_comments_ghr_amd import optimizer as op
    from orb_slam3_comments_ghr_amd.matcher import ORBmatcher
    out = []
    for F, L, Q, S, P in frames:
        s1 = S[0].copy()
        n1 = ORBmatcher(ctx, 0.6, True).SearchByProjection(F, L, 7.0, False, slot_mp=s1, slot_taken=S[1])
        s2 = S[0].copy()
        n2 = ORBmatcher(ctx, 0.9, True).SearchByProjection(F, Q, 3.0, False, 20.0, slot_mp=s2, slot_taken=S[1])
        r = op.Optimizer(ctx).PoseOptimization(P)
        out.append((int(n1), s1.tolist(), int(n2), s2.tolist(), r.pose.tolist(), r.outlier.tolist(), int(r.n_inliers)))
    return out


N_SEQ_GPU = 6
FRAMES_GPU = 4  # full-size C5 frames


def _gpu_c5_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from orb_slam3_comments_ghr_amd import Context
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = Context(0)
    seqs = _c5_units(N_SEQ_GPU, frames_per_seq=FRAMES_GPU, full=True)
    local = shard.run_sharded(lambda fr_: _c5_gpu_sequence(ctx, fr_), seqs, dist)
    everything = shard.gather_results(local, dist)
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, sorted(local), everything))


@pytest.mark.gpu
def test_c5_sequences_sharded_gpu_two_ranks(oracle):
    """BASELINE config 5 in its sharded form on the HIP path: C5 sequences of full-size frames (two-camera
    KB8 2 x 1000 keypoints, SearchByProjection x2 + a 600-edge PoseOptimization per frame, 6 sequences
    x 4 frames) round-robin over two processes sharing
    cuda:0, each through the C-ABI kernels, gathered once at the end; every rank's gathered results
    equal the single-process oracle run, sequence by sequence, bit for bit."""
    world = 2
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_gpu_c5_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=110) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seqs = _c5_units(N_SEQ_GPU, frames_per_seq=FRAMES_GPU, full=True)
    want = {i: _c5_oracle_sequence(oracle, s) for i, s in enumerate(seqs)}
    owned = set()
    for rank, mine, everything in res:
        assert mine == shard.shard_units(N_SEQ_GPU, rank, world)
        owned |= set(mine)
        assert sorted(everything) == list(range(N_SEQ_GPU))
        for i in range(N_SEQ_GPU):
            assert everything[i] == want[i], f"rank {rank}: sequence {i} != the single-process oracle run"
    assert owned == set(range(N_SEQ_GPU))
