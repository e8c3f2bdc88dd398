"""Multi-GPU partitioning of the hot path, one process per GPU over
torch.distributed (RCCL over xGMI on the box, gloo in the CPU tests).

* Independent units (C3 / C5 frames, TUM-VI sequences, LBA windows): round-robin over ranks, no
  collective in the data path; results are gathered once at the end (``gather_results``).  A CPU
  deployment of the reference runs one Tracking thread per sequence (ref:src/System.cc:240-268,
  ref:src/Tracking.cc:2009); here one rank owns each sequence.
* Brute-force Hamming top-2 over a train set too large for one GPU (C2' streaming): the train set is
  sharded by row ranges, queries replicated; each rank's kernel gives (best_idx, best_dist,
  second_dist) over its rows, one all-gather exchanges the 12 B/query triples and every rank merges
  them (``merge_top2``) into exactly what one serial pass over the whole train set gives
  (ref:src/ORBmatcher.cc:327-355: strict ``<`` updates in train order).

The compute step is a parameter: the GPU path passes the C-ABI kernels, the CPU tests pass the
oracle, so the same partitioning and merge code runs in both.
"""
from __future__ import annotations

import numpy as np

SENTINEL = 256  # TH no-match distance the top-2 loop starts from (ref:src/ORBmatcher.cc:327-329)


def shard_units(n_units: int, rank: int, world: int) -> list[int]:
    """The unit indices rank owns: round-robin, so every rank gets floor or ceil of n / world."""
    return list(range(rank, n_units, world))


def shard_rows(n_rows: int, rank: int, world: int) -> tuple[int, int]:
    """[begin, end) of rank's contiguous row range of an n_rows train set (first ranks take the
    remainder), so concatenating the ranks' ranges in rank order is the train order."""
    base, rem = divmod(n_rows, world)
    b = rank * base + min(rank, rem)
    return b, b + base + (1 if rank < rem else 0)


def merge_top2(parts) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Merge per-shard top-2 triples (best_idx [global], best_dist, second_dist), listed in train
    order, into the serial loop's result.  The serial loop keeps the first index of the minimum
    (strict <) and the second-smallest distance of the whole multiset, and each shard's two
    smallest are its (best, second), so: best = the first shard reaching the minimum; second = the
    smallest of every other shard's best and every shard's second."""
    idx = np.stack([np.asarray(p[0], np.int64) for p in parts])      # (K, Q)
    bd = np.stack([np.asarray(p[1], np.int64) for p in parts])
    sd = np.stack([np.asarray(p[2], np.int64) for p in parts])
    k = np.argmin(bd, axis=0)  # argmin returns the first minimum: train order tie-break
    q = np.arange(bd.shape[1])
    best = bd[k, q]
    others = bd.copy()
    others[k, q] = SENTINEL
    second = np.minimum(others.min(axis=0), sd.min(axis=0))
    bi = idx[k, q]
    bi = np.where(best < SENTINEL, bi, -1)  # no row with distance < 256: the loop's initial -1
    return bi.astype(np.int32), best.astype(np.int32), second.astype(np.int32)


def merge_top2_torch(parts):
    """merge_top2 on device tensors: parts (K, Q, 3) int32 [global idx, best, second] in train order
    -> (Q, 3).  Same rule as merge_top2 (first shard at the minimum; second = the smallest of the
    other shards' bests and every shard's second)."""
    import torch
    bd, sd = parts[:, :, 1], parts[:, :, 2]
    k = torch.argmin(bd, dim=0)  # first minimum along the shard axis (train order)
    best = bd.gather(0, k[None]).squeeze(0)
    others = bd.scatter(0, k[None], SENTINEL)
    second = torch.minimum(others.min(dim=0).values, sd.min(dim=0).values)
    bi = parts[:, :, 0].gather(0, k[None]).squeeze(0)
    bi = torch.where(best < SENTINEL, bi, torch.full_like(bi, -1))
    return torch.stack([bi, best, second], dim=1)


def train_sharded_top2(top2, query, train_shard, row0: int, dist=None):
    """Top-2 of `query` against the whole train set when this rank holds rows [row0, row0 + len).
    `top2(q, t) -> (idx, best, second)` is the local kernel (GPU C-ABI or oracle); the one exchange
    is an all-gather of the (Q, 3) int32 triples (8 B of key + 4 B of second per query, as
    SURVEY §8(e) sizes it), then every rank merges locally."""
    bi, bd, sd = top2(query, train_shard)
    bi = np.where(bi >= 0, bi + row0, -1).astype(np.int32)
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return bi, bd.astype(np.int32), sd.astype(np.int32)
    import torch
    mine = torch.from_numpy(np.stack([bi, bd, sd], axis=1).astype(np.int32))
    backend = dist.get_backend()
    if backend == "nccl":
        mine = mine.cuda()
    parts = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, mine)
    parts = [p.cpu().numpy() for p in parts]
    return merge_top2([(p[:, 0], p[:, 1], p[:, 2]) for p in parts])


def run_sharded(process, units, dist=None):
    """Run process(unit) for the units this rank owns (round-robin); returns {unit index: result}
    for this rank's units.  No collective."""
    rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    return {i: process(units[i]) for i in shard_units(len(units), rank, world)}


def gather_results(local: dict, dist=None) -> dict:
    """All ranks' {unit index: result} merged (all_gather_object: one small exchange at the end)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return dict(local)
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, local)
    out = {}
    for p in parts:
        out.update(p)
    return out
