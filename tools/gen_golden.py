"""Regenerate tests/golden/*.npz from the CPU oracle (the reference itself cannot be built or
run here: SURVEY.md §8c).  Each fixture stores inputs and the oracle's outputs; the numpy
cross-checks in tests/ pin the oracle independently."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orb_slam3_comments_ghr_amd import synth  # noqa: E402
from tests import oracle_calls  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    lib = oracle_calls.load()
    q, t = synth.descriptors_c2(400, 600, seed=0x60D1)
    n = q.shape[0]
    bi, bd, sd = (np.empty(n, np.int32) for _ in range(3))
    lib.oracle_hamming_top2(q.ctypes.data, n, t.ctypes.data, t.shape[0], bi.ctypes.data,
                            bd.ctypes.data, sd.ctypes.data)
    np.savez_compressed(os.path.join(GOLDEN, "top2_c2_400x600.npz"), query=q, train=t,
                        best_idx=bi, best_dist=bd, second_dist=sd)
    import importlib
    for mod in ("tools.gen_golden_match", "tools.gen_golden_ba"):
        try:
            m = importlib.import_module(mod)
        except ModuleNotFoundError:
            continue
        m.main(lib)
    print("golden fixtures written to", GOLDEN)


if __name__ == "__main__":
    main()
