#!/usr/bin/env python3
"""Probe of the C++ adapter's wall rate (bench infrastructure): builds bench.py's C3 / C5 problem pools,
then runs tools/adapter_wall_bench at several host-thread counts, with OSG_WALL_SPLIT=1 (the adapter's
gathers timed alone) and OSG_MATCH_PROFILE=2 (the library's host phases per call).  One JSON line per
run on stdout; the library's phase lines go to the .err files under --out.

    python tools/wall_probe.py --out gpurun_out/wallp [--threads 1,8,16] [--workloads c3,c5]
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tools.adapter_arrays import (bow_arrays, frame_arrays, last_arrays, mps_arrays, pose_arrays,  # noqa: E402
                                  pose_for_mock, prefixed, slot_arrays, stereo_arrays, write_arrays)


def c3_pool(n_pool=32):
    from orb_slam3_comments_ghr_amd import frames as fr, optimizer as op
    rng = np.random.default_rng(0x0B5EED03)
    pairs = [fr.synth_bow_pair(rng, n_kf=1200, n_f=1200, n_nodes=100) for _ in range(n_pool)]
    for pair in pairs:
        for S in pair:
            S.mp_good = (S.mp_good.astype(bool) & (S.mp_id >= 0)).astype(np.uint8)
    probs = [pose_for_mock(op.synth_pose_problem(rng, n_edges=300)) for _ in range(n_pool)]
    arrays = {"pool.n": np.array([n_pool], np.int32)}
    for i in range(n_pool):
        arrays.update(prefixed(f"p{i}.", {**bow_arrays("B1.", pairs[i][0]), **bow_arrays("B2.", pairs[i][1]),
                                          **pose_arrays(probs[i])}))
    return arrays


def c5_pool(n_pool=32):
    from orb_slam3_comments_ghr_amd import frames as fr, optimizer as op
    rng = np.random.default_rng(0x0B5EED10)
    F = [fr.synth_frame_two_cam(rng, n_left=1000, n_right=1000, stereo_frac=0.5, width=512, height=512)
         for _ in range(n_pool)]
    L = [fr.synth_last_queries_two_cam(rng, f, n_last=2000) for f in F]
    for x in L:
        x.valid = (x.valid.astype(bool) & (x.mp_id >= 0)).astype(np.uint8)
    Q = [fr.synth_mp_queries_two_cam(rng, f, m=1500) for f in F]
    for x in Q:
        x.has_obs[:] = 1
    S = [fr.synth_slots(rng, f.n, frac_assigned=0.05) for f in F]
    probs = [pose_for_mock(op.synth_pose_problem(rng, n_edges=600, cam=op.kb8_camera(), body_frac=0.4))
             for _ in range(n_pool)]
    arrays = {"pool.n": np.array([n_pool], np.int32)}
    for i in range(n_pool):
        arrays.update(prefixed(f"p{i}.", {**frame_arrays(F[i]), **slot_arrays(*S[i]), **last_arrays(L[i]),
                                          **mps_arrays(Q[i]), **pose_arrays(probs[i])}))
    return arrays


def stereo_pool(n_pool=16):
    from orb_slam3_comments_ghr_amd import stereo as st
    rng = np.random.default_rng(0x0B5EED20)
    pool = [st.synth_stereo_frame(rng, n=1200) for _ in range(n_pool)]
    arrays = {"pool.n": np.array([n_pool], np.int32)}
    for i, f in enumerate(pool):
        arrays.update(prefixed(f"p{i}.", stereo_arrays(f)))
    return arrays


POOLS = {"c3": c3_pool, "c5": c5_pool, "stereo": stereo_pool}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "wallp"))
    ap.add_argument("--threads", default="1,8,16")
    ap.add_argument("--workloads", default="c3,c5")
    ap.add_argument("--frames", default="256", help="frames per batched call, comma-separated list")
    ap.add_argument("--no-split", action="store_true", help="skip the OSG_WALL_SPLIT runs")
    ap.add_argument("--reps", type=int, default=12)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    exe = os.path.join(ROOT, "tools", "adapter_wall_bench")
    for wl in a.workloads.split(","):
        path = os.path.join(a.out, f"{wl}.arrays")
        write_arrays(path, POOLS[wl]())
        for t, fr in [(int(x), int(f)) for x in a.threads.split(",") for f in a.frames.split(",")]:
            for split in ((0,) if a.no_split else (0, 1)):
                env = dict(os.environ, OSG_WALL_SPLIT=str(split))
                if t == 1 and split:
                    env["OSG_MATCH_PROFILE"] = "2"
                    env["OSG_STEREO_PROFILE"] = "1"
                errf = os.path.join(a.out, f"{wl}_t{t}_f{fr}_s{split}.err")
                with open(errf, "w") as ef:
                    r = subprocess.run([exe, wl, path, str(fr), str(a.reps * 256 // fr), str(t)], stdout=subprocess.PIPE,
                                       stderr=ef, text=True, timeout=300, env=env)
                if r.returncode != 0:
                    print(json.dumps({"workload": wl, "threads": t, "split": split, "rc": r.returncode}), flush=True)
                    sys.exit(1)
                w = json.loads(r.stdout.strip().splitlines()[-1])
                w.pop("first_rep", None)
                w["split"] = split
                print(json.dumps(w), flush=True)


if __name__ == "__main__":
    main()
