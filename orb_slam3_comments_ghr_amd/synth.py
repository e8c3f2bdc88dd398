"""Seeded synthetic workloads for the benchmark configs.

EuRoC / TUM-VI images, yaml files and ORBvoc.txt are not available, so every config runs on
synthetic data of the documented shape.  All generators are deterministic in their seed.
"""
from __future__ import annotations

import numpy as np

SEED_C2 = 0x0B5EED01
SEED_C2_STREAM = 0x0B5EED02
SEED_C3 = 0x0B5EED03
SEED_C4 = 0x0B5EED04

# EuRoC cam0 intrinsics (upstream ORB-SLAM3 Examples/Stereo/EuRoC.yaml; not in the fork)
EUROC_W, EUROC_H = 752, 480
EUROC_FX, EUROC_FY, EUROC_CX, EUROC_CY = 458.654, 457.296, 367.215, 248.375
EUROC_BF = 47.9


def _flip_bits(rng: np.random.Generator, rows: np.ndarray, p: float) -> np.ndarray:
    bits = np.unpackbits(rows, axis=1)
    flips = (rng.random(bits.shape) < p).astype(np.uint8)
    return np.packbits(bits ^ flips, axis=1)


def descriptors_c2(nq: int = 2000, nt: int = 2000, seed: int = SEED_C2):
    """C2: queries uniform; 60 % of train rows are noisy copies (flip p = 0.08, d ~ 20) of a
    random query, the rest uniform (d ~ 128); 5 % of train rows exactly duplicate another train
    row (tie-breaking on the first index)."""
    rng = np.random.default_rng(seed)
    q = rng.integers(0, 256, size=(nq, 32), dtype=np.uint8)
    t = rng.integers(0, 256, size=(nt, 32), dtype=np.uint8)
    n_plant = int(0.6 * nt)
    plant_rows = rng.choice(nt, size=n_plant, replace=False)
    src = rng.integers(0, nq, size=n_plant)
    t[plant_rows] = _flip_bits(rng, q[src], 0.08)
    n_dup = int(0.05 * nt)
    if nt > 1 and n_dup > 0:
        dst = rng.choice(nt, size=n_dup, replace=False)
        srcr = rng.integers(0, nt, size=n_dup)
        t[dst] = t[srcr]
    return q, t


def descriptors_stream(nq: int = 4, nt: int = 1 << 24, seed: int = SEED_C2_STREAM):
    """C2': a few queries against a train set far larger than the 256 MiB Infinity Cache."""
    rng = np.random.default_rng(seed)
    q = rng.integers(0, 256, size=(nq, 32), dtype=np.uint8)
    t = rng.integers(0, 256, size=(nt, 32), dtype=np.uint8)
    # plant a few near-duplicates so the answer is not arbitrary
    for j in range(nq):
        rows = rng.integers(0, nt, size=3)
        t[rows] = _flip_bits(rng, np.repeat(q[j:j + 1], 3, axis=0), 0.05)
    return q, t
