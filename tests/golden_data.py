"""The committed fixtures under tests/golden/ that hold the reference's own data (not oracle outputs)."""
import hashlib
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BIT_PATTERN_SHA256 = "7e645581387b82784797e8adddb9b6f0c12611859fda09ca8a9bec96d767a05f"


def bit_pattern_31() -> np.ndarray:
    """ORBextractor's BRIEF sampling pattern, ref:src/ORBextractor.cc:212 (`bit_pattern_31_`, copied
    into `pattern` at ref:src/ORBextractor.cc:536-541) as int32 (512, 2): extracted as data by
    tools/gen_bit_pattern.py, checked here against the SHA-256 recorded at extraction."""
    with np.load(os.path.join(GOLDEN, "orb_bit_pattern_31.npz")) as d:
        pat = np.ascontiguousarray(d["pattern"], np.int32)
        sha = str(d["sha256"])
    got = hashlib.sha256(pat.tobytes()).hexdigest()
    if got != sha or sha != BIT_PATTERN_SHA256:
        raise AssertionError(f"orb_bit_pattern_31.npz: sha256 {got} != {BIT_PATTERN_SHA256}")
    return pat
