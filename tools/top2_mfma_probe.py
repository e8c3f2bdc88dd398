#!/usr/bin/env python3
"""A/B of the frame-batched C2 top-2 forms: the I8-MFMA kernel (shapes OSG_TOP2_MFMA_SHAPE 0..3) against
the popcount kernel (OSG_TOP2_BATCH_MFMA=0).  Each configuration runs in its own child process (the
library reads its knobs once); every child checks its result against the popcount kernel's output saved
by the first child.  One JSON line per configuration.

    python tools/top2_mfma_probe.py [--frames 256] [--reps 50]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, numpy as np, torch
sys.path.insert(0, ROOT)
from orb_slam3_comments_ghr_amd import Context, synth
B, reps, ref = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
nq = nt = 2000
dev = torch.device('cuda', 0)
ctx = Context(0)
stream = torch.cuda.Stream(dev); torch.cuda.set_stream(stream); ctx.set_stream(stream.cuda_stream)
fr = [synth.descriptors_c2(nq, nt, seed=synth.SEED_C2 + 7919 * b) for b in range(B)]
dq = torch.from_numpy(np.concatenate([f[0] for f in fr])).to(dev)
dt = torch.from_numpy(np.concatenate([f[1] for f in fr])).to(dev)
do = torch.empty((B * nq, 3), dtype=torch.int32, device=dev)
for _ in range(3): ctx.hamming_top2_batch_dev(dq, nq, dt, nt, B, do)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda._sleep(int(2e6))
e0.record(stream)
for _ in range(reps): ctx.hamming_top2_batch_dev(dq, nq, dt, nt, B, do)
e1.record(stream)
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / reps
got = do.cpu().numpy()
if not os.path.exists(ref): np.save(ref, got); eq = None
else: eq = bool((np.load(ref) == got).all())
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith('OSG_TOP2')}, "frames": B, "kernel_us": round(us, 2),
                  "Mmatches_per_s": round(B * nq * nt / us, 1), "equal_to_popcount_kernel": eq}), flush=True)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--shapes", default="0,1,2,3,4")
    a = ap.parse_args()
    ref = "/tmp/_top2_mfma_probe_ref.npy"
    if os.path.exists(ref):
        os.remove(ref)
    confs = [{"OSG_TOP2_BATCH_MFMA": "0"}] + [{"OSG_TOP2_MFMA_SHAPE": s} for s in a.shapes.split(",")]
    rc = 0
    for c in confs:
        env = dict(os.environ, **c)
        r = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT)), str(a.frames), str(a.reps), ref],
                           env=env, capture_output=True, text=True, timeout=300)
        sys.stdout.write(r.stdout)
        if r.returncode != 0:
            sys.stdout.write(json.dumps({"env": c, "error": r.stderr[-1500:]}) + "\n")
            rc = 1
            break
        sys.stdout.flush()
    sys.exit(rc)


if __name__ == "__main__":
    main()
