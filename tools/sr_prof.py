"""k_schur_rows_c's per-workgroup timeline (a `make SR_PROF=1` library, OSG_SR_PROF_OUT=file): graph 0's row
segments of one LM step, wall-clock ticks at 100 MHz.

    python tools/sr_prof.py sr.bin
"""
import sys

import numpy as np


def main(path):
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 13).astype(np.int64)
    a = a[a[:, 0] > 0]
    t0 = a[:, 0].min()
    st = (a[:, 0] - t0) * 0.01
    stage = (a[:, 1] - a[:, 0]) * 0.01
    ends = (a[:, 2:10] - a[:, 1:2]) * 0.01
    wg = (a[:, 2:10].max(1) - a[:, 0]) * 0.01
    ch, nr = a[:, 10], a[:, 11]
    xcc = a[:, 12] & 0xF
    cu = (a[:, 12] >> 32) & 0xFF
    print(f"workgroups {len(a)}  span {((a[:, 2:10].max() - t0) * 0.01):.1f} us  starts {st.min():.1f}..{st.max():.1f} us")
    for name, v in [("staging us", stage), ("chunk loop us (wave mean)", ends.mean(1)),
                    ("chunk loop us (slowest wave)", ends.max(1)), ("workgroup us", wg),
                    ("chunks per segment", ch), ("blocks per segment", nr)]:
        print(f"{name:30s} mean {v.mean():8.2f}  p10 {np.percentile(v, 10):8.2f}  p50 {np.median(v):8.2f}  "
              f"p90 {np.percentile(v, 90):8.2f}  max {v.max():8.2f}")
    print("staging share of workgroup time: %.3f" % (stage.sum() / wg.sum()))
    print("slowest / mean wave loop: %.2f" % (ends.max(1).sum() / ends.mean(1).sum()))
    print("XCCs", np.bincount(xcc, minlength=8).tolist())
    key = xcc * 256 + cu
    _, per = np.unique(key, return_counts=True)
    print("distinct CUs %d, workgroups per CU mean %.2f max %d" % (len(per), per.mean(), per.max()))
    # chunk-loop time per chunk of the wave (8 waves take every 8th chunk)
    print("loop us per chunk (wave mean / (chunks/8)): %.3f" % np.mean(ends.mean(1) / np.maximum(ch / 8.0, 1)))


if __name__ == "__main__":
    main(sys.argv[1])
