#!/usr/bin/env python3
"""Probe the host CPU resources a GPU-box command actually gets (affinity, cgroup quota, model)
and how the oracle's brute-force top-2 scales with host threads.  Used to size bench.py's
multi-threaded cpu_baseline.  Prints one JSON object."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def read(path):
    try:
        return open(path).read().strip()
    except OSError:
        return None


def main():
    out = {"os_cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
           "cgroup_cpu_max": read("/sys/fs/cgroup/cpu.max"), "cgroup_pids_max": read("/sys/fs/cgroup/pids.max"),
           "omp": os.environ.get("OMP_NUM_THREADS")}
    model = None
    for line in (read("/proc/cpuinfo") or "").splitlines():
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    out["cpu_model"] = model
    from tests import oracle_calls
    from orb_slam3_comments_ghr_amd import synth
    lib = oracle_calls.load()
    q, t = synth.descriptors_c2(2000, 2000, seed=1)
    bi, bd, sd = (np.empty(2000, np.int32) for _ in range(3))
    scale = {}
    for nth in [1, 8, 16, 32, 64, 128, 256]:
        if nth > (os.cpu_count() or 1):
            break
        reps = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 1.5:
            # query slices of one 2000 x 2000 problem, one slice per thread
            lib.oracle_hamming_top2_mt(q.ctypes.data, 2000, t.ctypes.data, 2000, bi.ctypes.data,
                                       bd.ctypes.data, sd.ctypes.data, nth)
            reps += 1
        el = time.perf_counter() - t0
        scale[nth] = round(reps * 4e6 / el / 1e6, 1)
        print(nth, scale[nth], flush=True)
    out["top2_mmatches_by_threads"] = scale
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
