"""Pure-Python restatement of Frame::ComputeStereoMatches (ref:src/Frame.cc:1117-1373), written apart
from oracle/oracle_stereo.c to pin it: Python lists for vRowIndices, numpy bit counts for
DescriptorDistance, numpy slices for the SAD, Python's tuple sort for vDistIdx, float32 scalars for
the reference's float arithmetic.  Test infrastructure only (small frames)."""
import numpy as np

f32 = np.float32
TH_HIGH, TH_LOW = 100, 50


def _cround(v):
    """C round() on a float value: half away from zero."""
    v = float(v)
    return f32(np.floor(v + 0.5) if v >= 0 else np.ceil(v - 0.5))


def _hamming(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def compute_stereo_matches(F, stats=False):
    """(mvuRight, mvDepth, kept) [+ accepted before the median cut]."""
    N = F.n
    ur = np.full(N, -1, f32)
    depth = np.full(N, -1, f32)
    nRows = F.left.levels[0].shape[0]
    vRowIndices = [[] for _ in range(nRows)]
    for iR in range(F.n_right):
        r = f32(2.0) * F.scale[F.octave_r[iR]]
        maxr = int(np.ceil(f32(F.yr[iR] + r)))
        minr = int(np.floor(f32(F.yr[iR] - r)))
        for yi in range(minr, maxr + 1):
            if 0 <= yi < nRows:  # (the reference indexes past vRowIndices here: undefined)
                vRowIndices[yi].append(iR)
    minZ = f32(F.mb)
    minD = f32(0)
    maxD = f32(f32(F.mbf) / minZ)
    vDistIdx = []
    for iL in range(N):
        levelL = int(F.octave[iL])
        vL, uL = F.y[iL], F.x[iL]
        if not vL >= 0 or int(vL) >= nRows:
            continue
        cands = vRowIndices[int(vL)]
        if not cands:
            continue
        minU, maxU = f32(uL - maxD), f32(uL - minD)
        if maxU < 0:
            continue
        bestDist, bestIdxR = TH_HIGH, 0
        for iR in cands:
            if F.octave_r[iR] < levelL - 1 or F.octave_r[iR] > levelL + 1:
                continue
            if minU <= F.xr[iR] <= maxU:
                d = _hamming(F.desc[iL], F.desc_r[iR])
                if d < bestDist:
                    bestDist, bestIdxR = d, iR
        if bestDist >= (TH_HIGH + TH_LOW) // 2:
            continue
        sf = F.inv_scale[levelL]
        suL, svL, suR0 = _cround(f32(uL * sf)), _cround(f32(vL * sf)), _cround(f32(F.xr[bestIdxR] * sf))
        ImL, ImR = F.left.levels[levelL], F.right.levels[levelL]
        if suR0 < 0 or suR0 + 11 >= ImR.shape[1]:  # iniu / endu, :1280-1284
            continue
        pu, pv, pr = int(suL), int(svL), int(suR0)
        if (pv - 5 < 0 or pv + 5 >= min(ImL.shape[0], ImR.shape[0]) or pu - 5 < 0 or pu + 5 >= ImL.shape[1]
                or pr - 10 < 0 or pr + 10 >= ImR.shape[1]):
            continue  # the reference's rowRange / colRange would throw
        IL = ImL[pv - 5:pv + 6, pu - 5:pu + 6].astype(np.int64)
        dists = [f32(np.abs(IL - ImR[pv - 5:pv + 6, pr + inc - 5:pr + inc + 6].astype(np.int64)).sum())
                 for inc in range(-5, 6)]
        k = dists.index(min(dists))  # the first minimum
        inc = k - 5
        if inc in (-5, 5):
            continue
        d1, d2, d3 = dists[k - 1], dists[k], dists[k + 1]
        with np.errstate(divide="ignore", invalid="ignore"):
            deltaR = f32(f32(d1 - d3) / f32(f32(2.0) * f32(f32(d1 + d3) - f32(f32(2.0) * d2))))
        if deltaR < -1 or deltaR > 1:
            continue
        bestuR = f32(F.scale[levelL] * f32(f32(suR0 + f32(inc)) + deltaR))
        disparity = f32(uL - bestuR)
        if minD <= disparity < maxD:
            if disparity <= 0:
                disparity = f32(0.01)
                bestuR = f32(float(uL) - 0.01)
            depth[iL] = f32(f32(F.mbf) / disparity)
            ur[iL] = bestuR
            vDistIdx.append((int(dists[k]), iL))
    kept = len(vDistIdx)
    if vDistIdx:
        vDistIdx.sort()
        thDist = f32(f32(f32(1.5) * f32(1.4)) * f32(vDistIdx[len(vDistIdx) // 2][0]))
        for dist, iL in vDistIdx:
            if not f32(dist) < thDist:
                ur[iL] = depth[iL] = -1
                kept -= 1
    return (ur, depth, kept, len(vDistIdx)) if stats else (ur, depth, kept)
