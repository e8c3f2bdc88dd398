"""Per-phase host times of the batched ORB extractor (OSG_ORB_PROFILE=1 prints them to stderr):
B EuRoC-shaped images per osg_orb_extract_batch call.  Run on the GPU box:
    OSG_ORB_PROFILE=1 python tools/orb_batch_probe.py [B] [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_comments_ghr_amd import Context, orb  # noqa: E402


def main():
    import torch
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rng = np.random.default_rng(0x0B5EED41)
    imgs = [orb.synth_fast_pyramid(rng, n_levels=1)[0] for _ in range(4)]
    batch = torch.stack([torch.from_numpy(imgs[i % 4]) for i in range(B)]).cuda()
    pattern = orb.synth_pattern(np.random.default_rng(5))
    ctx = Context(0)
    for _ in range(3):
        orb.ORBExtractBatch(ctx, batch, pattern=pattern)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        orb.ORBExtractBatch(ctx, batch, pattern=pattern, sync=False)
    el = time.perf_counter() - t0
    print(f"B={B}: {el / reps * 1e3:.2f} ms per call, {B * reps / el:.0f} frames/s", flush=True)


if __name__ == "__main__":
    main()
