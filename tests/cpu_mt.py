"""The multi-threaded CPU baseline (test infrastructure, used only by bench.py's cpu_baseline legs
and tests): the oracle run with one independent problem per host thread, as a CPU deployment of the
reference serves independent frames / windows (one Tracking or LocalMapping thread per sequence,
ref:src/System.cc:240-268), so the GPU's frame-batched throughput is priced against every core the
box gives this process, not against one.

Each worker thread calls the oracle through ctypes (CDLL: the GIL is released for the whole C call)
with its arguments packed before the timed region, so the only Python on the timed path is the
loop and the ctypes dispatch (a few microseconds against 0.1-10 ms of C work per call).
"""
from __future__ import annotations

import os
import platform
import threading
import time


# the compiler flags of the oracle build the workers call (bench.py sets it when it loads the timing
# build; every baseline object carries it as `flags`)
ORACLE_FLAGS = "-O3 -ffp-contract=off -fno-fast-math (the checker build)"


def cgroup_cpus():
    """The CPU quota of this process's cgroup (cpu.max quota / period), or None when unlimited."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return None


def host_threads():
    """Threads the CPU baseline may keep busy: the cgroup quota when one is set (the GPU box gives
    each one-GPU job 16 CPUs of a 256-thread host), else the affinity set."""
    aff = len(os.sched_getaffinity(0))
    q = cgroup_cpus()
    return min(aff, q) if q else aff


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def run(make_worker, n_threads, seconds):
    """Run make_worker(tid) -> call(i) on n_threads threads for ~seconds; returns (calls, elapsed).
    Every worker is built (its outputs allocated) before the clock starts."""
    barrier = threading.Barrier(n_threads + 1)
    stop = threading.Event()
    counts = [0] * n_threads
    errors = []

    def body(tid):
        try:
            call = make_worker(tid)
        except BaseException as e:  # noqa: BLE001 - surfaced below
            errors.append(e)
            barrier.abort()
            return
        try:
            barrier.wait()
        except threading.BrokenBarrierError:
            return
        i = 0
        try:
            while not stop.is_set() or i == 0:
                call(i)
                i += 1
        except BaseException as e:  # noqa: BLE001
            errors.append(e)
        counts[tid] = i

    th = [threading.Thread(target=body, args=(t,), daemon=True) for t in range(n_threads)]
    for t in th:
        t.start()
    try:
        barrier.wait()
    except threading.BrokenBarrierError:
        pass
    t0 = time.perf_counter()
    time.sleep(seconds)
    stop.set()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    if errors:
        raise errors[0]
    return sum(counts), el


def baseline(make_worker, units_per_call, unit, seconds, label, threads=None):
    """The cpu_baseline object: the oracle on 1 thread and on `threads` threads (default: every CPU
    this process may use), one independent problem per thread.  `value` is the N-thread rate."""
    n = threads or host_threads()
    c1, e1 = run(make_worker, 1, seconds / 3)
    cn, en = run(make_worker, n, seconds * 2 / 3)
    v1 = c1 * units_per_call / e1
    vn = cn * units_per_call / en
    host = os.cpu_count()
    return {"value": round(vn, 2), "unit": unit, "cores": n, "kind": "port", "flags": ORACLE_FLAGS,
            "value_1thread": round(v1, 2), "thread_scaling": round(vn / v1, 2) if v1 else None,
            "host_cpus": host, "cgroup_cpu_quota": cgroup_cpus(), "cpu_model": cpu_model(),
            "node_estimate": {"threads": host, "value": round(vn * host / n, 1),
                              "note": "linear extrapolation of the N-thread rate to every hardware thread of "
                                      "the host (the box's cgroup caps this job at `cores`)"},
            "sample": f"{label}: {cn} calls on {n} threads in {en:.1f} s (+ {c1} calls on 1 thread in {e1:.1f} s), "
                      f"oracle gcc {ORACLE_FLAGS}, one independent problem per thread"}
