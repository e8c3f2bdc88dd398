"""Host runtime of the product library, on the CPU (no GPU calls): the process-wide worker pool behind
osg_parallel_for under concurrent callers, and the LBA / GBA structure build's two paths (the windows'
sequential passes and the maps' worker-pool passes) giving the same arrays.  Drives
tools/micro/lba_host_time.hip, which compiles ba.hip's host code against the built library."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

from orb_slam3_comments_ghr_amd import optimizer as op

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "orb_slam3_comments_ghr_amd")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = str(tmp_path_factory.mktemp("lht") / "liblba_host_time.so")
    cmd = [hipcc, "--offload-arch=gfx950", "-O2", "-shared", "-fPIC", os.path.join(ROOT, "tools/micro/lba_host_time.hip"),
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(LIBDIR, "csrc"), "-L" + LIBDIR, "-lorbslam3_amd",
           "-Wl,-rpath," + LIBDIR, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lib = C.CDLL(out)
    lib.lba_host_struct_hash.restype = C.c_ulonglong
    lib.lba_host_struct_hash.argtypes = [C.c_void_p]
    lib.pool_stress.restype = C.c_int
    lib.pool_stress.argtypes = [C.c_int, C.c_int, C.c_int]
    return lib


@pytest.fixture(scope="module")
def packer(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = str(tmp_path_factory.mktemp("pk") / "libpacker_check.so")
    cmd = [hipcc, "--offload-arch=gfx950", "-O2", "-shared", "-fPIC", os.path.join(ROOT, "tools/micro/packer_check.hip"),
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(LIBDIR, "csrc"), "-L" + LIBDIR, "-lorbslam3_amd",
           "-Wl,-rpath," + LIBDIR, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lib = C.CDLL(out)
    lib.packer_check.restype = C.c_int
    lib.packer_check.argtypes = [C.c_uint, C.c_int, C.c_int]
    return lib


@pytest.mark.parametrize("seed,n_items,threads", [(1, 3, 1), (2, 12, 4), (3, 40, 8), (4, 25, 16)])
def test_packer_row_gathers(packer, seed, n_items, threads):
    """The matcher's pinned-block packer: row-gather items (SearchByBoW's query rows) and plain items, by
    fill() and by fill_parallel()'s 4 MiB pieces (rows split across pieces), equal a reference pack."""
    assert packer.packer_check(seed, n_items, threads) == 0


@pytest.mark.parametrize("threads,loops,n", [(1, 500, 1), (1, 500, 37), (8, 300, 5), (8, 100, 1000), (24, 100, 33)])
def test_worker_pool_concurrent_callers(harness, threads, loops, n):
    assert harness.pool_stress(threads, loops, n) == 0


def test_structure_map_path_equals_window_path(harness, monkeypatch):
    graphs = [op.synth_lba_graph(np.random.default_rng(0x0B5EED04), n_kf=50, n_points=10000),
              op.synth_lba_graph(np.random.default_rng(5), n_kf=20, n_points=2500, stereo_frac=0.3),
              op.synth_map_graph(np.random.default_rng(7), n_kf=150, n_points=20000, loop=True)]
    for G in graphs:
        monkeypatch.delenv("OSG_LBA_MAP_MODE", raising=False)
        h_window = harness.lba_host_struct_hash(C.byref(G.struct()))
        monkeypatch.setenv("OSG_LBA_MAP_MODE", "1")
        h_map = harness.lba_host_struct_hash(C.byref(G.struct()))
        assert h_window != 0 and h_window == h_map


def test_structure_build_concurrent_callers(harness, monkeypatch):
    """8 host threads building structures at once (as bench.py's global_ba stage
    drives lba_batch from 8 threads), each on its own graph, through the worker pool's map path with its
    thread_local scratch vectors: every hash equals the same graph's single-threaded build."""
    import threading
    monkeypatch.setenv("OSG_LBA_MAP_MODE", "1")
    graphs = [op.synth_map_graph(np.random.default_rng(70 + i), n_kf=150 + 40 * i, n_points=15000, loop=(i % 2 == 1))
              for i in range(4)] + [op.synth_lba_graph(np.random.default_rng(80 + i), n_kf=50, n_points=10000)
                                    for i in range(4)]
    structs = [G.struct() for G in graphs]
    want = [harness.lba_host_struct_hash(C.byref(s)) for s in structs]
    assert all(want)
    got = [[] for _ in graphs]

    def run(i):
        for _ in range(6):
            got[i].append(harness.lba_host_struct_hash(C.byref(structs[i])))
    th = [threading.Thread(target=run, args=(i,)) for i in range(len(graphs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for i in range(len(graphs)):
        assert got[i] == [want[i]] * 6, i
