"""Host mirror of ``MapPoint::ComputeDistinctiveDescriptors`` (ref:src/MapPoint.cc:444-535) over a list of
MapPoints, on top of the C ABI (``osg_compute_distinctive_descriptors``).  LocalMapping calls it for
every MapPoint of a keyframe (ref:src/LocalMapping.cc:421-436, 1066-1082); here that loop is one launch.

    best = ComputeDistinctiveDescriptors(ctx, desc_lists)     # desc_lists[p]: N_p x 32 observation rows
    mDescriptor[p] = desc_lists[p][best[p]]                   # (best -1: N_p == 0, left unchanged)
"""
from __future__ import annotations

import numpy as np

from . import Context


def to_csr(desc_lists):
    """Observation descriptor lists -> (rows (total x 32), start (n_points + 1))."""
    start = np.zeros(len(desc_lists) + 1, np.int32)
    start[1:] = np.cumsum([len(d) for d in desc_lists])
    rows = [np.ascontiguousarray(d, np.uint8).reshape(-1, 32) for d in desc_lists]
    desc = np.concatenate(rows) if rows else np.zeros((0, 32), np.uint8)
    return np.ascontiguousarray(desc, np.uint8), start


def ComputeDistinctiveDescriptors(ctx: Context, desc_lists=None, *, desc=None, start=None) -> np.ndarray:
    """best_idx[p] per MapPoint: the observation row with the least median distance to the others
    (first on ties), -1 for a point without observations.  Pass the per-point lists, or the CSR
    (``desc`` rows, ``start`` offsets)."""
    if desc_lists is not None:
        desc, start = to_csr(desc_lists)
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    start = np.ascontiguousarray(start, np.int32)
    n = len(start) - 1
    out = np.full(n, -1, np.int32)
    rc = ctx.lib.osg_compute_distinctive_descriptors(ctx.handle, desc.ctypes.data, start.ctypes.data, n,
                                                     out.ctypes.data)
    ctx.check(rc, "ComputeDistinctiveDescriptors")
    return out


def synth_observations(rng, n_points=1000, n_min=1, n_max=30, flip=0.08, outlier=0.15):
    """Per MapPoint: N ~ U{n_min..n_max} observation descriptors, noisy copies (flip p) of one
    descriptor, ``outlier`` of them unrelated; a few exact duplicates exercise ties."""
    lists = []
    for _ in range(n_points):
        n = int(rng.integers(n_min, n_max + 1))
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        bits = np.unpackbits(np.repeat(base[None], n, 0), axis=1)
        d = np.packbits(bits ^ (rng.random(bits.shape) < flip).astype(np.uint8), axis=1)
        out = rng.random(n) < outlier
        d[out] = rng.integers(0, 256, (int(out.sum()), 32), dtype=np.uint8)
        if n >= 3 and rng.random() < 0.3:
            d[-1] = d[0]
        lists.append(d)
    return lists
