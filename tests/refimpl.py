"""Independent numpy implementations used to cross-check the C oracle (not the product).

These restate the reference semantics a second way (vectorised, np.bitwise_count) so that the
oracle's line-by-line C restatement is pinned by something other than itself.
"""
import numpy as np


def hamming_matrix(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a64 = np.ascontiguousarray(a, dtype=np.uint8).reshape(-1, 32).view(np.uint64)
    b64 = np.ascontiguousarray(b, dtype=np.uint8).reshape(-1, 32).view(np.uint64)
    out = np.zeros((a64.shape[0], b64.shape[0]), np.int32)
    for k in range(4):
        out += np.bitwise_count(a64[:, k:k + 1] ^ b64[None, :, k]).astype(np.int32)
    return out


def top2_from_matrix(D: np.ndarray):
    """(best_idx, best_dist, second_dist) with the reference's semantics: strict '<' from the
    sentinel 256 (so distance 256 never enters), first index wins ties, second counts
    multiplicity."""
    nq, nt = D.shape
    bi = np.full(nq, -1, np.int32)
    bd = np.full(nq, 256, np.int32)
    sd = np.full(nq, 256, np.int32)
    if nt == 0:
        return bi, bd, sd
    order = np.argsort(D, axis=1, kind="stable")
    d_sorted = np.take_along_axis(D, order, axis=1)
    has1 = d_sorted[:, 0] < 256
    bi[has1] = order[has1, 0]
    bd[has1] = d_sorted[has1, 0]
    if nt > 1:
        has2 = d_sorted[:, 1] < 256
        sd[has2] = d_sorted[has2, 1]
    return bi, bd, sd
