"""osg_orb_pyramid timing probe: ComputePyramid (+ blur) on a 752x480 device image, N calls; prints the
event-timed device ms per call (first launch to last).  Run under rocprofv3 --kernel-trace --stats for
the per-kernel split."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_comments_ghr_amd import Context, orb


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    ctx = Context(0)
    img = torch.from_numpy(orb.synth_fast_pyramid(np.random.default_rng(1), n_levels=1)[0]).cuda()
    inv = orb.inv_scale_factors(8, 1.2)
    P = orb.ComputePyramid(ctx, img, inv)
    torch.cuda.synchronize()
    ms = 0.0
    t0 = time.perf_counter()
    for _ in range(n):
        orb.ComputePyramid(ctx, img, inv, out=P.buffer, sync=False)
        ms += ctx.last_kernel_ms()
    wall = time.perf_counter() - t0
    print({"calls": n, "device_us_per_call": round(ms * 1e3 / n, 2), "wall_us_per_call": round(wall * 1e6 / n, 2)})
    ctx.close()


if __name__ == "__main__":
    main()
