#!/usr/bin/env python3
"""Extract the reference's BRIEF sampling table as DATA into tests/golden/orb_bit_pattern_31.npz.

ref:src/ORBextractor.cc:212 holds `static int bit_pattern_31_[256 * 4]`: 256 point pairs (x1, y1, x2, y2),
which ORBextractor's constructor copies into `pattern` (512 cv::Point, ref:src/ORBextractor.cc:536-541)
and computeOrbDescriptor reads pair by pair.  This script reads the initialiser's integers as text (the
C comments after each row dropped) and stores them as an int32 (512, 2) array -- the layout
orb.ORBDescribe takes -- with a SHA-256 of the raw int32 bytes.  It needs /root/reference (this
container only); the .npz it writes is the committed fixture the tests load.

    python tools/gen_bit_pattern.py [--reference /root/reference]
"""
import argparse
import hashlib
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def extract(src_text: str) -> np.ndarray:
    start = src_text.index("bit_pattern_31_[256 * 4]")
    body = src_text[src_text.index("{", start) + 1:]
    body = body[:body.index("};")]
    body = re.sub(r"/\*.*?\*/", " ", body, flags=re.S)   # the per-row mean / correlation comments
    body = re.sub(r"//[^\n]*", " ", body)
    vals = [int(v) for v in re.findall(r"-?\d+", body)]
    if len(vals) != 1024:
        raise ValueError(f"expected 1024 integers, found {len(vals)}")
    a = np.array(vals, np.int32).reshape(512, 2)
    if np.abs(a).max() > 13:
        raise ValueError("a sampling offset outside the 31 x 31 patch")
    return a


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "orb_bit_pattern_31.npz"))
    a = ap.parse_args()
    src = os.path.join(a.reference, "src", "ORBextractor.cc")
    with open(src, encoding="utf-8", errors="replace") as f:
        pat = extract(f.read())
    sha = hashlib.sha256(pat.tobytes()).hexdigest()
    np.savez(a.out, pattern=pat, sha256=np.array(sha), source=np.array("ref:src/ORBextractor.cc:212"))
    print(f"{a.out}: {pat.shape} int32, sha256 {sha}")


if __name__ == "__main__":
    main()
