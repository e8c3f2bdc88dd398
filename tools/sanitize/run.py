"""Host runtime under ASan / TSan, CPU only: writes the graphs (C4 windows, a stereo
window, 150- and 190-KF maps open and loop-closed), builds tools/sanitize/host_san.hip twice with
runtime.hip (host code sanitized: -Xarch_host -fsanitize=address / thread) and runs both.

    python tools/sanitize/run.py [--out profiles/r06_host_sanitizers.txt]
"""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from orb_slam3_comments_ghr_amd import optimizer as op  # noqa: E402
from tools.adapter_arrays import write_arrays  # noqa: E402

CSRC = os.path.join(ROOT, "orb_slam3_comments_ghr_amd", "csrc")


def graphs():
    g = [op.synth_lba_graph(np.random.default_rng(80 + i), n_kf=50, n_points=10000) for i in range(2)]
    g.append(op.synth_lba_graph(np.random.default_rng(5), n_kf=20, n_points=2500, stereo_frac=0.3))
    g += [op.synth_map_graph(np.random.default_rng(70 + i), n_kf=150 + 40 * i, n_points=15000, loop=(i % 2 == 1))
          for i in range(2)]
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_host_sanitizers.txt"))
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="osg_san_")
    files = []
    for i, G in enumerate(graphs()):
        p = os.path.join(d, f"g{i}.arrays")
        write_arrays(p, {"pose": G.pose.reshape(-1), "point": G.point.reshape(-1), "e_obs": G.e_obs.reshape(-1),
                         "pose_fixed": G.pose_fixed, "e_point": G.e_point, "e_pose": G.e_pose, "e_cam": G.e_cam,
                         "e_kind": G.e_kind.view(np.uint8), "e_inv_sigma2": G.e_inv_sigma2,
                         "cams": np.frombuffer(bytes(G._cams), np.uint8)})
        files.append(p)
    log = []
    rc_all = 0
    for san in ("address", "thread"):
        exe = os.path.join(d, f"host_san_{san}")
        cmd = ["hipcc", "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer",
               "-Xarch_host", f"-fsanitize={san}", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
               os.path.join(ROOT, "tools", "sanitize", "host_san.hip"), os.path.join(CSRC, "runtime.hip"),
               "-o", exe, "-Xarch_host", f"-fsanitize={san}", "-pthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        log.append(f"== build -fsanitize={san}: rc {r.returncode}\n" + (r.stderr[-3000:] if r.returncode else ""))
        if r.returncode:
            rc_all = 1
            continue
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
                   TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1", OSG_HOST_THREADS="16")
        r = subprocess.run([exe] + files, capture_output=True, text=True, env=env, timeout=3000)
        log.append(f"== run -fsanitize={san}: rc {r.returncode}\n{r.stdout}{r.stderr[-6000:]}")
        rc_all |= r.returncode != 0
    text = "\n".join(log)
    print(text)
    with open(a.out, "w") as f:
        f.write("tools/sanitize/run.py: host code of liborbslam3_amd (runtime.hip worker pool, ba.hip structure build, "
                "match_common.h packer) under ASan / TSan on the CPU\n" + text)
    sys.exit(rc_all)


if __name__ == "__main__":
    main()
