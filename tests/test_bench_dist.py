"""The multi-GPU bench path on CPU: world_size 2 over gloo (127.0.0.1).  bench.py shards
independent frames / windows over ranks (weak scaling, no data-path collective); the whole-job
figures are the slowest rank's time and the sum of all ranks' units (bench.job_totals)."""
import hashlib
import os
import socket
import sys

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from orb_slam3_comments_ghr_amd import synth
    # per-rank synthetic frame, as bench.py seeds it
    qd, td = synth.descriptors_c2(128, 128, seed=synth.SEED_C2 + rank)
    digest = hashlib.sha1(qd.tobytes() + td.tobytes()).hexdigest()
    digests = [None] * world
    dist.all_gather_object(digests, digest)
    elapsed, units = bench.job_totals(1.0 + 0.5 * rank, 1000 * (rank + 1), world, dist, "cpu")
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, elapsed, units, digests))


def test_bench_job_totals_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, elapsed, units, digests in res:
        assert elapsed == 1.5           # max over ranks
        assert units == 3000            # sum over ranks
        assert len(set(digests)) == world, "every rank matches its own independent frame"


def test_bench_job_totals_single_rank():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.job_totals(2.0, 7, 1) == (2.0, 7.0)
