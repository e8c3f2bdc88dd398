"""Independent pure-Python restatement of ORBextractor::ComputeKeyPointsOctTree
(ref:src/ORBextractor.cc:1065-1198) that pins the C++ oracle (oracle/oracle_orbdetect.cc).  TEST
INFRASTRUCTURE ONLY.

Written differently from the oracle on purpose:
  * FAST by its definition instead of OpenCV's code: a pixel is a corner at threshold t when 9
    contiguous pixels of its 16-pixel circle are all < v - t or all > v + t; its score is the largest
    t' >= t at which it is still a corner (found by counting up), which is what cornerScore<16>
    computes.  Suppression keeps a corner whose score is strictly above its 8 neighbours' (0 outside
    the tested range), row by row.
  * DistributeOctTree's node list as a Python list (index 0 = front), and std::sort restated as
    libstdc++'s introsort (median-of-three quicksort above 16 elements, then insertion sort), so
    that nodes of equal (size, UL.x) come out in the order the reference's std::sort gives them.
"""
import math

import numpy as np

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def _run9(flags):
    f = flags + flags
    run = 0
    for b in f:
        run = run + 1 if b else 0
        if run >= 9:
            return True
    return False


def is_corner(img, y, x, t):
    v = int(img[y, x])
    c = [int(img[y + dy, x + dx]) for dx, dy in CIRCLE]
    return _run9([p < v - t for p in c]) or _run9([p > v + t for p in c])


def fast(img, t):
    """cv::FAST(img, t, nonmax = true) on one image: [(x, y, score)] in row-major order."""
    t = min(max(int(t), 0), 255)
    rows, cols = img.shape
    score = np.zeros((rows, cols), np.int32)
    for y in range(3, rows - 3):
        for x in range(3, cols - 3):
            if is_corner(img, y, x, t):
                s = t
                while s + 1 <= 255 and is_corner(img, y, x, s + 1):
                    s += 1
                score[y, x] = s
    out = []
    for y in range(3, rows - 3):
        for x in range(3, cols - 3):
            s = score[y, x]
            if s and all(s > score[y + dy, x + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dy or dx):
                out.append((float(x), float(y), float(s)))
    return out


# ---- std::sort (libstdc++ bits/stl_algo.h) --------------------------------------------------------
def std_sort(a, less):
    def insertion_sort(lo, hi):
        for i in range(lo + 1, hi):
            if less(a[i], a[lo]):
                v = a[i]
                a[lo + 1:i + 1] = a[lo:i]
                a[lo] = v
            else:
                linear_insert(i)

    def linear_insert(i):
        v = a[i]
        j = i - 1
        while less(v, a[j]):
            a[j + 1] = a[j]
            j -= 1
        a[j + 1] = v

    def median_to_first(r, x, y, z):
        if less(a[x], a[y]):
            if less(a[y], a[z]):
                a[r], a[y] = a[y], a[r]
            elif less(a[x], a[z]):
                a[r], a[z] = a[z], a[r]
            else:
                a[r], a[x] = a[x], a[r]
        elif less(a[x], a[z]):
            a[r], a[x] = a[x], a[r]
        elif less(a[y], a[z]):
            a[r], a[z] = a[z], a[r]
        else:
            a[r], a[y] = a[y], a[r]

    def partition(lo, hi, p):
        while True:
            while less(a[lo], a[p]):
                lo += 1
            hi -= 1
            while less(a[p], a[hi]):
                hi -= 1
            if not lo < hi:
                return lo
            a[lo], a[hi] = a[hi], a[lo]
            lo += 1

    def introsort(lo, hi, depth):
        while hi - lo > 16:
            if depth == 0:
                raise NotImplementedError("heapsort fallback")
            depth -= 1
            mid = lo + (hi - lo) // 2
            median_to_first(lo, lo + 1, mid, hi - 1)
            cut = partition(lo + 1, hi, lo)
            introsort(cut, hi, depth)
            hi = cut

    n = len(a)
    if n < 2:
        return
    introsort(0, n, 2 * (n.bit_length() - 1))
    if n > 16:
        insertion_sort(0, 16)
        for i in range(16, n):
            linear_insert(i)
    else:
        insertion_sort(0, n)


# ---- DistributeOctTree ----------------------------------------------------------------------------
class Node:
    def __init__(self, ul, ur, bl, br):
        self.UL, self.UR, self.BL, self.BR = ul, ur, bl, br
        self.keys = []
        self.no_more = False

    def divide(self):
        hx = math.ceil(np.float32(self.UR[0] - self.UL[0]) / np.float32(2))
        hy = math.ceil(np.float32(self.BR[1] - self.UL[1]) / np.float32(2))
        ul, ur, bl, br = self.UL, self.UR, self.BL, self.BR
        n1 = Node(ul, (ul[0] + hx, ul[1]), (ul[0], ul[1] + hy), (ul[0] + hx, ul[1] + hy))
        n2 = Node(n1.UR, ur, n1.BR, (ur[0], ul[1] + hy))
        n3 = Node(n1.BL, n1.BR, bl, (n1.BR[0], bl[1]))
        n4 = Node(n3.UR, n2.BR, n3.BR, br)
        for k in self.keys:
            if k[0] < n1.UR[0]:
                (n1 if k[1] < n1.BR[1] else n3).keys.append(k)
            elif k[1] < n1.BR[1]:
                n2.keys.append(k)
            else:
                n4.keys.append(k)
        for n in (n1, n2, n3, n4):
            n.no_more = len(n.keys) == 1
        return n1, n2, n3, n4


def distribute_oct_tree(keys, minX, maxX, minY, maxY, N):
    n_ini = int(np.round(np.float32(maxX - minX) / np.float32(maxY - minY)))
    hX = np.float32(maxX - minX) / np.float32(n_ini)
    nodes = []
    for i in range(n_ini):
        ul = (int(hX * np.float32(i)), 0)
        ur = (int(hX * np.float32(i + 1)), 0)
        nodes.append(Node(ul, ur, (ul[0], maxY - minY), (ur[0], maxY - minY)))
    ini = list(nodes)
    for k in keys:
        ini[int(np.float32(k[0]) / hX)].keys.append(k)
    nodes = [n for n in nodes if n.keys]
    for n in nodes:
        n.no_more = len(n.keys) == 1

    def push_children(parent, expand):
        for c in parent.divide():
            if c.keys:
                nodes.insert(0, c)
                if len(c.keys) > 1:
                    expand.append((len(c.keys), c))

    finish = False
    expand = []
    while not finish:
        prev = len(nodes)
        expand = []
        i = 0
        while i < len(nodes):
            n = nodes[i]
            if n.no_more:
                i += 1
                continue
            before = len(nodes)
            push_children(n, expand)
            i += len(nodes) - before
            del nodes[i]
        n_to_expand = len(expand)
        if len(nodes) >= N or len(nodes) == prev:
            finish = True
        elif len(nodes) + 3 * n_to_expand > N:
            while not finish:
                prev2 = len(nodes)
                work = list(expand)
                expand = []
                std_sort(work, lambda a, b: a[0] < b[0] or (a[0] == b[0] and a[1].UL[0] < b[1].UL[0]))
                for _, n in reversed(work):
                    push_children(n, expand)
                    nodes.remove(n)
                    if len(nodes) >= N:
                        break
                if len(nodes) >= N or len(nodes) == prev2:
                    finish = True
    out = []
    for n in nodes:
        best = n.keys[0]
        for k in n.keys[1:]:
            if k[2] > best[2]:
                best = k
        out.append(best)
    return out


def orb_detect(levels, n_features, scales, ini_th=20, min_th=7):
    """The whole of ComputeKeyPointsOctTree's keypoint part: [(x, y, response, size, level)]."""
    out = []
    for level, img in enumerate(levels):
        rows, cols = img.shape
        minBX = minBY = 19 - 3
        maxBX, maxBY = cols - 19 + 3, rows - 19 + 3
        width, height = np.float32(maxBX - minBX), np.float32(maxBY - minBY)
        n_cols, n_rows = int(width / np.float32(35)), int(height / np.float32(35))
        w_cell, h_cell = math.ceil(width / np.float32(n_cols)), math.ceil(height / np.float32(n_rows))
        keys = []
        for i in range(n_rows):
            ini_y = minBY + i * h_cell
            max_y = min(ini_y + h_cell + 6, maxBY)
            if ini_y >= maxBY - 3:
                continue
            for j in range(n_cols):
                ini_x = minBX + j * w_cell
                max_x = min(ini_x + w_cell + 6, maxBX)
                if ini_x >= maxBX - 6:
                    continue
                cell = img[ini_y:max_y, ini_x:max_x]
                ks = fast(cell, ini_th) or fast(cell, min_th)
                keys += [(x + j * w_cell, y + i * h_cell, r) for x, y, r in ks]
        kept = distribute_oct_tree(keys, minBX, maxBX, minBY, maxBY, int(n_features[level]))
        size = float(int(np.float32(31) * np.float32(scales[level])))
        out += [(x + minBX, y + minBY, r, size, level) for x, y, r in kept]
    return out
