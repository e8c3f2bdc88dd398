"""GPU parity: brute-force top-2 (DescriptorDistance + the top-2 candidate loop) through the C ABI
against the CPU oracle — bit-exact indices and distances."""
import numpy as np
import pytest

from tests.conftest import ptr
from orb_slam3_comments_ghr_amd import synth

pytestmark = pytest.mark.gpu


def otop2(oracle, q, t, threads=8):
    q = np.ascontiguousarray(q, np.uint8).reshape(-1, 32)
    t = np.ascontiguousarray(t, np.uint8).reshape(-1, 32)
    n = q.shape[0]
    bi, bd, sd = (np.empty(n, np.int32) for _ in range(3))
    oracle.oracle_hamming_top2_mt(ptr(q), n, ptr(t), t.shape[0], ptr(bi), ptr(bd), ptr(sd), threads)
    return bi, bd, sd


def check(ctx, oracle, q, t):
    got = ctx.hamming_top2(q, t)
    ref = otop2(oracle, q, t)
    for name, g, r in zip(("best_idx", "best_dist", "second_dist"), got, ref):
        bad = np.nonzero(g != r)[0]
        assert bad.size == 0, f"{name}: {bad.size} mismatches, first {bad[:5]} got {g[bad[:5]]} ref {r[bad[:5]]}"


def test_c2_2000x2000(ctx, oracle):
    q, t = synth.descriptors_c2(2000, 2000)
    check(ctx, oracle, q, t)


@pytest.mark.parametrize("nq,nt", [(1, 1), (1, 7), (63, 65), (64, 64), (65, 1000), (129, 3),
                                   (3000, 257), (257, 5000), (8, 2000), (9, 70000)])
def test_shapes(ctx, oracle, nq, nt):
    q, t = synth.descriptors_c2(nq, nt, seed=nq * 7919 + nt)
    check(ctx, oracle, q, t)


def test_empty_train(ctx):
    q, _ = synth.descriptors_c2(10, 1)
    bi, bd, sd = ctx.hamming_top2(q, np.zeros((0, 32), np.uint8))
    assert (bi == -1).all() and (bd == 256).all() and (sd == 256).all()


def test_all_at_256(ctx, oracle):
    # train rows are exact complements of the query: every distance 256 -> never enters
    q = np.random.default_rng(3).integers(0, 256, (5, 32), dtype=np.uint8)
    t = np.repeat(~q[:1], 300, axis=0)
    check(ctx, oracle, q[:1], t)
    bi, bd, sd = ctx.hamming_top2(q[:1], t)
    assert bi[0] == -1 and bd[0] == 256 and sd[0] == 256


def test_ties_first_index(ctx, oracle):
    rng = np.random.default_rng(11)
    q = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    t = np.repeat(q, 40, axis=0)  # 40 exact duplicates per query, interleaved in chunks
    rng.shuffle(t, axis=0)
    check(ctx, oracle, q, t)


@pytest.mark.parametrize("nq", [1, 2, 4, 8])
def test_stream_shape(ctx, oracle, nq):
    q, t = synth.descriptors_stream(nq, 1 << 20, seed=100 + nq)
    check(ctx, oracle, q, t)


def test_stream_full_size_c2prime(ctx, oracle):
    q, t = synth.descriptors_stream(4, 1 << 24)
    check(ctx, oracle, q, t)


def test_repeated_calls_reset_counters(ctx, oracle):
    q, t = synth.descriptors_c2(2000, 2000, seed=5)
    ref = otop2(oracle, q, t)
    for _ in range(20):
        got = ctx.hamming_top2(q, t)
        for g, r in zip(got, ref):
            np.testing.assert_array_equal(g, r)


def test_pairwise_distance(ctx, oracle):
    rng = np.random.default_rng(2)
    a = rng.integers(0, 256, (10001, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (10001, 32), dtype=np.uint8)
    got = ctx.descriptor_distance_pairs(a, b)
    ref = np.array([oracle.oracle_descriptor_distance(ptr(a[i]), ptr(b[i])) for i in range(len(a))])
    np.testing.assert_array_equal(got, ref)


def test_alternating_problems_no_stale_partials(ctx, oracle):
    """Partials and counters are reused between calls: alternate two different problems so a
    stale partial from the previous call would show up as a mismatch."""
    p1 = synth.descriptors_c2(2000, 2000, seed=21)
    p2 = synth.descriptors_c2(2000, 2000, seed=22)
    r1 = otop2(oracle, *p1)
    r2 = otop2(oracle, *p2)
    for i in range(30):
        q, t = (p1, p2)[i % 2]
        ref = (r1, r2)[i % 2]
        got = ctx.hamming_top2(q, t)
        for g, r in zip(got, ref):
            np.testing.assert_array_equal(g, r)


@pytest.mark.parametrize("variant,waves,wg", [("0", "4", ""), ("1", "8", ""), ("4", "16", ""), ("4", "4", ""),
                                               ("3", "16", ""), ("3", "16", "64"), ("3", "16", "4096"),
                                               ("2", "8", "")])
def test_tile_variants(oracle, variant, waves, wg):
    """Every top-2 variant in a fresh process (the knobs are read once per process): tile kernel
    with scalar/LDS staging x fence/write-through merge x 4/8/16 waves, and the query-split kernel
    at several queries-per-workgroup (OSG_TOP2_QS_WG target 64 -> 32 queries per workgroup at
    nq = 2000, 4096 -> 1 query per workgroup)."""
    import subprocess, sys, os, json
    code = (
        "import numpy as np, json\n"
        "from orb_slam3_comments_ghr_amd import Context, synth\n"
        "c = Context(0)\n"
        "out = []\n"
        "for seed, (nq, nt) in enumerate([(2000, 2000), (300, 20000), (5000, 600), (70, 4097)]):\n"
        "    q, t = synth.descriptors_c2(nq, nt, seed=900 + seed)\n"
        "    out.append([a.tolist() for a in c.hamming_top2(q, t)])\n"
        "print(json.dumps(out))\n")
    env = dict(os.environ, OSG_TOP2_VARIANT=variant, OSG_TOP2_WAVES=waves)
    if wg:
        env["OSG_TOP2_WG"] = env["OSG_TOP2_QS_WG"] = wg
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    for seed, (nq, nt) in enumerate([(2000, 2000), (300, 20000), (5000, 600), (70, 4097)]):
        q, t = synth.descriptors_c2(nq, nt, seed=900 + seed)
        ref = otop2(oracle, q, t)
        for g, rr in zip(got[seed], ref):
            np.testing.assert_array_equal(np.array(g, np.int32), rr)


# ---- frame-batched form (osg_hamming_top2_batch_dev): nb independent problems in one launch
def _batch(ctx, qs, ts, ql=None, monkeypatch=None):
    import torch
    nb, nq, nt = len(qs), qs[0].shape[0], ts[0].shape[0]
    dq = torch.from_numpy(np.ascontiguousarray(np.concatenate(qs))).cuda()
    dt = torch.from_numpy(np.ascontiguousarray(np.concatenate(ts) if nt else np.zeros((0, 32), np.uint8))).cuda()
    do = torch.full((nb * nq, 3), -7, dtype=torch.int32, device="cuda")
    ctx.hamming_top2_batch_dev(dq, nq, dt, nt, nb, do)
    torch.cuda.synchronize()
    return do.cpu().numpy().reshape(nb, nq, 3)


@pytest.mark.parametrize("nb,nq,nt", [(1, 2000, 2000), (7, 2000, 2000), (3, 1, 1), (5, 129, 3), (4, 300, 2049),
                                      (2, 257, 5000), (64, 64, 200)])
def test_batch_equals_serial_loop(ctx, oracle, nb, nq, nt):
    qs, ts = zip(*[synth.descriptors_c2(nq, nt, seed=synth.SEED_C2 + 1000 * b + nq + nt) for b in range(nb)])
    got = _batch(ctx, qs, ts)
    for b in range(nb):
        for k, r in enumerate(otop2(oracle, qs[b], ts[b])):
            np.testing.assert_array_equal(got[b, :, k], r, err_msg=f"problem {b} column {k}")


def test_batch_ties_and_sentinels(ctx, oracle):
    """Exact duplicates straddling the 2048-row LDS chunk and the 16 waves' row slices, and a
    problem whose every distance is 256 (idx -1), next to ordinary problems."""
    rng = np.random.default_rng(12)
    q0 = rng.integers(0, 256, (100, 32), dtype=np.uint8)
    t0 = np.repeat(q0, 30, axis=0)
    rng.shuffle(t0, axis=0)
    q1 = rng.integers(0, 256, (100, 32), dtype=np.uint8)
    t1 = np.repeat(~q1[:1], 3000, axis=0)
    q2, t2 = synth.descriptors_c2(100, 3000, seed=99)
    got = _batch(ctx, [q0, q1[:1].repeat(100, 0), q2], [t0, t1, t2])
    for b, (q, t) in enumerate([(q0, t0), (q1[:1].repeat(100, 0), t1), (q2, t2)]):
        for k, r in enumerate(otop2(oracle, q, t)):
            np.testing.assert_array_equal(got[b, :, k], r)
    assert (got[1, :, 0] == -1).all() and (got[1, :, 1] == 256).all()


def test_batch_empty_train(ctx):
    q, _ = synth.descriptors_c2(50, 1)
    got = _batch(ctx, [q, q], [np.zeros((0, 32), np.uint8)] * 2)
    assert (got[..., 0] == -1).all() and (got[..., 1:] == 256).all()


_VARIANTS = [{"OSG_TOP2_BATCH_MFMA": "0", "OSG_TOP2_BATCH_QL": ql, "OSG_TOP2_BATCH_SCALAR": sc}
             for ql, sc in [("1", "0"), ("2", "0"), ("4", "0"), ("1", "1"), ("4", "1")]]
_VARIANTS += [{"OSG_TOP2_FP4": "0", "OSG_TOP2_MFMA_SHAPE": sh} for sh in ("0", "1", "2", "3", "4")]
_VARIANTS += [{"OSG_TOP2_FP4": "1", "OSG_TOP2_MFMA_SHAPE": sh} for sh in ("0", "1", "2", "4", "5", "6", "7", "8", "9", "10", "11", "12", "13")]


@pytest.mark.parametrize("env", _VARIANTS, ids=lambda e: "-".join(f"{k[9:]}={v}" for k, v in e.items()))
def test_batch_query_per_lane_variants(oracle, env):
    """The popcount kernel's queries-per-lane (OSG_TOP2_BATCH_QL) and scalar-load (OSG_TOP2_BATCH_SCALAR)
    instantiations, the I8-MFMA kernel's workgroup shapes (OSG_TOP2_FP4=0, OSG_TOP2_MFMA_SHAPE) and the
    FP4 block-scaled kernel's (the default), read once per process.
    nt = 2100: a partial LDS chunk and a partial 32-row tile."""
    import subprocess
    import sys
    out = f"/tmp/_osg_batch_ql_{__import__('os').getpid()}.npy"  # per process: concurrent suites do not share it
    code = ("import numpy as np, torch\n"
            "from orb_slam3_comments_ghr_amd import Context, synth\n"
            "from tests.test_top2_gpu import _batch\n"
            "ctx = Context(0)\n"
            "qs, ts = zip(*[synth.descriptors_c2(333, 2100, seed=5 + b) for b in range(3)])\n"
            f"np.save({out!r}, _batch(ctx, qs, ts))\n")
    env = dict(__import__("os").environ, **env)
    root = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.load(out)
    __import__("os").remove(out)
    qs, ts = zip(*[synth.descriptors_c2(333, 2100, seed=5 + b) for b in range(3)])
    for b in range(3):
        for k, ref in enumerate(otop2(oracle, qs[b], ts[b])):
            np.testing.assert_array_equal(got[b, :, k], ref)


def test_batch_mfma_edges(ctx, oracle):
    """The matrix-core form's edge cases (the default, k_top2_fp4), each problem against the serial loop:
    * exact duplicates of the best row straddling the 32-row tiles and the 256-row LDS chunks (first index wins);
    * the query itself in the train set (H = 0), its complement (H = 256, never enters), all-zero and all-one
      descriptors (|q| = 0 and 256 shift the key by the most);
    * nt = 8192, the largest train set the 13-bit row field holds, and nt = 1."""
    rng = np.random.default_rng(2024)
    probs = []
    q = rng.integers(0, 256, (96, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (600, 32), dtype=np.uint8)
    for j, rows in enumerate([(31, 32), (255, 256, 257), (0, 511), (63, 64, 512)]):
        for rr in rows:
            t[rr] = q[j]
    t[100] = ~q[10]
    probs.append((q, t))
    z = np.zeros((1, 32), np.uint8)
    o = np.full((1, 32), 255, np.uint8)
    q2 = np.concatenate([z, o, q[:94]])
    t2 = np.concatenate([o, z, t[:598]])
    probs.append((q2, t2))
    for qq, tt in probs:
        got = _batch(ctx, [qq], [tt])
        for k, r in enumerate(otop2(oracle, qq, tt)):
            np.testing.assert_array_equal(got[0, :, k], r)
    assert got[0, 0, 1] == 0 and got[0, 1, 1] == 0   # the zero / one rows found at H = 0
    q3, t3 = synth.descriptors_c2(200, 8192, seed=77)
    q4, t4 = synth.descriptors_c2(200, 1, seed=78)
    for qq, tt in [(q3, t3), (q4, t4)]:
        got = _batch(ctx, [qq, qq], [tt, tt])
        for b in range(2):
            for k, r in enumerate(otop2(oracle, qq, tt)):
                np.testing.assert_array_equal(got[b, :, k], r)


def _edge_problems():
    """test_batch_mfma_edges' problems: duplicates across tiles / chunks, H = 0 and 256, |q| = 0 and 256,
    nt = 8192 and nt = 1."""
    rng = np.random.default_rng(2024)
    q = rng.integers(0, 256, (96, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (600, 32), dtype=np.uint8)
    for j, rows in enumerate([(31, 32), (255, 256, 257), (0, 511), (63, 64, 512)]):
        for rr in rows:
            t[rr] = q[j]
    t[100] = ~q[10]
    z = np.zeros((1, 32), np.uint8)
    o = np.full((1, 32), 255, np.uint8)
    probs = [(q, t), (np.concatenate([z, o, q[:94]]), np.concatenate([o, z, t[:598]]))]
    probs += [synth.descriptors_c2(200, 8192, seed=77), synth.descriptors_c2(200, 1, seed=78)]
    return probs


@pytest.mark.parametrize("env", [{"OSG_TOP2_FP4": "0"}, {"OSG_TOP2_FP4": "0", "OSG_TOP2_MFMA_SHAPE": "1"},
                                 {"OSG_TOP2_FP4": "1", "OSG_TOP2_MFMA_SHAPE": "1"}, {"OSG_TOP2_FP4": "1", "OSG_TOP2_MFMA_SHAPE": "8"},
                                 {"OSG_TOP2_FP4": "1", "OSG_TOP2_MFMA_SHAPE": "9"}, {"OSG_TOP2_FP4": "1", "OSG_TOP2_MFMA_SHAPE": "10"},
                                 {"OSG_TOP2_FP4": "1", "OSG_TOP2_MFMA_SHAPE": "11"}, {"OSG_TOP2_FP4": "1", "OSG_TOP2_MFMA_SHAPE": "12"},
                                 {"OSG_TOP2_FP4": "1", "OSG_TOP2_MFMA_SHAPE": "13"}],
                         ids=lambda e: "-".join(f"{k[9:]}={v}" for k, v in e.items()))
def test_batch_fp4_edges(oracle, env, tmp_path):
    """The same edge cases on the other matrix-core forms, each against the serial loop: the I8 form
    (k_top2_mfma, OSG_TOP2_FP4=0, integer keys) and a second FP4 shape (keys carried in f32 in [2^23, 2^24),
    exact)."""
    import os
    import subprocess
    import sys
    code = ("import numpy as np\n"
            "from orb_slam3_comments_ghr_amd import Context\n"
            "from tests.test_top2_gpu import _batch, _edge_problems\n"
            "ctx = Context(0)\n"
            "out = {}\n"
            "for i, (q, t) in enumerate(_edge_problems()):\n"
            "    out[f'p{i}'] = _batch(ctx, [q, q], [t, t])\n"
            "import sys\n"
            "np.savez(sys.argv[1], **out)\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = str(tmp_path / f"fp4_edges_{os.getpid()}.npz")
    r = subprocess.run([sys.executable, "-c", code, path], cwd=root, env=dict(os.environ, **env), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.load(path)
    for i, (q, t) in enumerate(_edge_problems()):
        for b in range(2):
            for k, ref in enumerate(otop2(oracle, q, t)):
                np.testing.assert_array_equal(got[f"p{i}"][b, :, k], ref, err_msg=f"problem {i} column {k}")
