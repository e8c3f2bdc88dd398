"""Where a global BA's time goes: host phases (OSG_LBA_PROFILE=1 prints structure build, pack + upload,
LM and download per call) for whole-map graphs of growing size.  python tools/gba_profile.py"""
import os
import sys
import time

os.environ.setdefault("OSG_LBA_PROFILE", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from orb_slam3_comments_ghr_amd import Context, optimizer as op  # noqa: E402


def main():
    ctx = Context(0)
    opt = op.Optimizer(ctx)
    for n_kf, n_pts in ((50, 10000), (150, 20000), (300, 40000)):
        G = op.synth_gba_graph(np.random.default_rng(n_kf), n_kf=n_kf, n_points=n_pts)
        opt.BundleAdjustment(G)
        t = time.perf_counter()
        r = opt.BundleAdjustment(G)
        el = time.perf_counter() - t
        print(f"gba n_kf={n_kf} points={len(G.point)} edges={len(G.e_point)} n={6 * (n_kf - 1)}: {el * 1e3:.2f} ms, "
              f"{r.iterations} iterations, {r.trials} trials", flush=True)


if __name__ == "__main__":
    main()
