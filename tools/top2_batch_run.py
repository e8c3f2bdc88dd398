#!/usr/bin/env python3
"""Runs the frame-batched C2 top-2 (osg_hamming_top2_batch_dev) `reps` times on 256 resident 2000 x 2000
frames: the target program of the rocprofv3 passes over the headline kernel (tools/gpu/top2_pmc.sh).
The kernel form follows the library's knobs (OSG_TOP2_BATCH_MFMA, OSG_TOP2_MFMA_SHAPE)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_comments_ghr_amd import Context, synth  # noqa: E402

B = int(os.environ.get("FRAMES", "256"))
reps = int(os.environ.get("REPS", "10"))
nq = nt = 2000
ctx = Context(0)
fr = [synth.descriptors_c2(nq, nt, seed=synth.SEED_C2 + 7919 * b) for b in range(B)]
dq = torch.from_numpy(np.concatenate([f[0] for f in fr])).cuda()
dt = torch.from_numpy(np.concatenate([f[1] for f in fr])).cuda()
do = torch.empty((B * nq, 3), dtype=torch.int32, device="cuda")
for _ in range(reps):
    ctx.hamming_top2_batch_dev(dq, nq, dt, nt, B, do)
torch.cuda.synchronize()
print("ok", int(do[:, 1].sum()))
