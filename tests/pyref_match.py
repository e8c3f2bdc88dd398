"""Second, independent restatement of the reference matchers in pure Python (float32 scalars for
the reference's float arithmetic).  Slow — small inputs only.  Used to pin the C oracle
(tests/test_oracle_match.py); never used by the product."""
import math

import numpy as np

f32 = np.float32
TH_HIGH, TH_LOW, HISTO = 100, 50, 30


def dist(a, b):
    return int(np.bitwise_count(np.bitwise_xor(a, b)).sum())


def features_in_area(F, x, y, r, minL=-1, maxL=-1, right=False):
    """Frame::GetFeaturesInArea; ``right`` walks mGridRight (indices relative to Nleft)."""
    x, y, r = f32(x), f32(y), f32(r)
    out = []
    minCX = max(0, int(math.floor(f32(f32(x - f32(F.min_x)) - r) * F.inv_w)))
    if minCX >= 64:
        return out
    maxCX = min(63, int(math.ceil(f32(f32(x - f32(F.min_x)) + r) * F.inv_w)))
    if maxCX < 0:
        return out
    minCY = max(0, int(math.floor(f32(f32(y - f32(F.min_y)) - r) * F.inv_h)))
    if minCY >= 48:
        return out
    maxCY = min(47, int(math.ceil(f32(f32(y - f32(F.min_y)) + r) * F.inv_h)))
    if maxCY < 0:
        return out
    chk = (minL > 0) or (maxL >= 0)
    gs, gi = (F.grid_start_r, F.grid_idx_r) if right else (F.grid_start, F.grid_idx)
    off = F.nleft if right else 0
    for ix in range(minCX, maxCX + 1):
        for iy in range(minCY, maxCY + 1):
            c = ix * 48 + iy
            for j in range(gs[c], gs[c + 1]):
                idx = int(gi[j])
                k = idx + off
                o = int(F.kp_octave[k])
                if chk:
                    if o < minL:
                        continue
                    if maxL >= 0 and o > maxL:
                        continue
                if abs(f32(F.kp_x[k] - x)) < r and abs(f32(F.kp_y[k] - y)) < r:
                    out.append(idx)
    return out


def rot_bin(a, b):
    rot = f32(f32(a) - f32(b))
    if rot < 0.0:
        rot = f32(rot + f32(360.0))
    v = float(f32(rot * f32(f32(1.0) / f32(30))))
    b_ = int(math.floor(v + 0.5))  # round half away from zero, v >= 0
    return 0 if b_ == 30 else b_


def three_maxima(sizes):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(sizes):
        if s > m1:
            m3, m2, m1 = m2, m1, s
            i3, i2, i1 = i2, i1, i
        elif s > m2:
            m3, m2 = m2, s
            i3, i2 = i2, i
        elif s > m3:
            m3, i3 = s, i
    if m2 < f32(0.1) * f32(m1):
        i2 = i3 = -1
    elif m3 < f32(0.1) * f32(m1):
        i3 = -1
    return i1, i2, i3


def apply_hist(hist, slots, nm):
    keep = three_maxima([len(h) for h in hist])
    for i in range(HISTO):
        if i in keep:
            continue
        for s in hist[i]:
            slots[s] = -1
            nm -= 1
    return nm


class _Top2:
    def __init__(self):
        self.b, self.bl, self.b2, self.bl2, self.bi = 256, -1, 256, -1, -1

    def push(self, d, lvl, idx):
        if d < self.b:
            self.b2, self.bl2, self.b, self.bl, self.bi = self.b, self.bl, d, lvl, idx
        elif d < self.b2:
            self.b2, self.bl2 = d, lvl


def search_mps(F, Q, nn, th, far, thfar, slot_mp, slot_taken):
    slots = slot_mp.copy()
    taken = slot_taken.copy()
    nm = 0
    nn = f32(nn)
    two = F.nleft != -1

    def assign(s, i):
        slots[s] = Q.mp_id[i]
        taken[s] = Q.has_obs[i]

    for i in range(len(Q.mp_id)):
        in_r = Q.in_view_r is not None and bool(Q.in_view_r[i])
        if not Q.in_view[i] and not in_r:
            continue
        if far and Q.track_depth[i] > f32(thfar):
            continue
        if not Q.usable[i]:
            continue
        if Q.in_view[i]:
            lvl = int(Q.pred_level[i])
            r = f32(2.5) if float(Q.view_cos[i]) > 0.998 else f32(4.0)
            if f32(th) != f32(1.0):
                r = f32(r * f32(th))
            R = f32(r * F.scale[lvl])
            t = _Top2()
            for idx in features_in_area(F, Q.proj_x[i], Q.proj_y[i], R, lvl - 1, lvl):
                if slots[idx] >= 0 and taken[idx]:
                    continue
                if not two and F.u_right is not None and F.u_right[idx] > 0:
                    if abs(f32(Q.proj_xr[i] - F.u_right[idx])) > R:
                        continue
                t.push(dist(Q.desc[i], F.desc[idx]), int(F.kp_octave[idx]), idx)
            if t.b <= TH_HIGH:
                if t.bl == t.bl2 and f32(t.b) > nn * f32(t.b2):
                    continue  # skips the right-camera pass too
                assign(t.bi, i)
                nm += 1
                if two and F.left_to_right is not None and F.left_to_right[t.bi] != -1:
                    assign(F.left_to_right[t.bi] + F.nleft, i)
                    nm += 1
        if two and in_r:
            lvl = int(Q.pred_level_r[i])
            if lvl == -1:
                continue
            r = f32(2.5) if float(Q.view_cos_r[i]) > 0.998 else f32(4.0)
            R = f32(r * F.scale[lvl])
            t = _Top2()
            for idx in features_in_area(F, Q.proj_xr[i], Q.proj_yr[i], R, lvl - 1, lvl, right=True):
                s_ = idx + F.nleft
                if slots[s_] >= 0 and taken[s_]:
                    continue
                t.push(dist(Q.desc[i], F.desc[s_]), int(F.kp_octave[s_]), idx)
            if t.b <= TH_HIGH:
                if t.bl == t.bl2 and f32(t.b) > nn * f32(t.b2):
                    continue
                if F.right_to_left is not None and F.right_to_left[t.bi] != -1:
                    assign(F.right_to_left[t.bi], i)
                    nm += 1
                assign(t.bi + F.nleft, i)
                nm += 1
    return nm, slots


def search_last(F, L, th, mono, ori, slot_mp, slot_taken):
    slots = slot_mp.copy()
    taken = slot_taken.copy()
    hist = [[] for _ in range(HISTO)]
    nm = 0
    two = F.nleft != -1
    fwd = f32(L.tlc_z) > f32(F.mb) and not mono
    bwd = -f32(L.tlc_z) > f32(F.mb) and not mono

    def window(u, v, rad, o, right):
        if fwd:
            return features_in_area(F, u, v, rad, o, -1, right)
        if bwd:
            return features_in_area(F, u, v, rad, 0, o, right)
        return features_in_area(F, u, v, rad, o - 1, o + 1, right)

    for i in range(len(L.mp_id)):
        if not L.valid[i]:
            continue
        invz = L.invz[i]
        if invz < 0:
            continue
        u, v = L.u[i], L.v[i]
        if u < f32(F.min_x) or u > f32(F.max_x) or v < f32(F.min_y) or v > f32(F.max_y):
            continue
        o = int(L.octave[i])
        rad = f32(f32(th) * F.scale[o])
        c = window(u, v, rad, o, False)
        if not c:
            continue
        b, bi = 256, -1
        for i2 in c:
            if slots[i2] >= 0 and taken[i2]:
                continue
            if not two and F.u_right is not None and F.u_right[i2] > 0:
                ur = f32(u - f32(f32(F.mbf) * invz))
                if abs(f32(ur - F.u_right[i2])) > rad:
                    continue
            d = dist(L.desc[i], F.desc[i2])
            if d < b:
                b, bi = d, i2
        if b <= TH_HIGH:
            slots[bi] = L.mp_id[i]
            taken[bi] = L.has_obs[i]
            nm += 1
            if ori:
                hist[rot_bin(L.angle[i], F.kp_angle[bi])].append(bi)
        if two:
            b, bi = 256, -1
            for i2 in window(L.u_r[i], L.v_r[i], rad, o, True):
                s_ = i2 + F.nleft
                if slots[s_] >= 0 and taken[s_]:
                    continue
                d = dist(L.desc[i], F.desc[s_])
                if d < b:
                    b, bi = d, s_
            if b <= TH_HIGH:
                slots[bi] = L.mp_id[i]
                taken[bi] = L.has_obs[i]
                nm += 1
                if ori:
                    hist[rot_bin(L.angle[i], F.kp_angle[bi])].append(bi)
    if ori:
        nm = apply_hist(hist, slots, nm)
    return nm, slots


def search_kf(F, K, th, orb, ori, slot_mp):
    slots = slot_mp.copy()
    hist = [[] for _ in range(HISTO)]
    nm = 0
    for i in range(len(K.mp_id)):
        if not K.valid[i]:
            continue
        lvl = int(K.pred_level[i])
        rad = f32(f32(th) * F.scale[lvl])
        c = features_in_area(F, K.u[i], K.v[i], rad, lvl - 1, lvl + 1)
        if not c:
            continue
        b, bi = 256, -1
        for i2 in c:
            if slots[i2] >= 0:
                continue
            d = dist(K.desc[i], F.desc[i2])
            if d < b:
                b, bi = d, i2
        if b <= orb:
            slots[bi] = K.mp_id[i]
            nm += 1
            if ori:
                hist[rot_bin(K.angle[i], F.kp_angle[bi])].append(bi)
    if ori:
        nm = apply_hist(hist, slots, nm)
    return nm, slots


def _shared_nodes(A, B):
    ma = {int(n): (A.node_start[k], A.node_start[k + 1]) for k, n in enumerate(A.node_id)}
    mb = {int(n): (B.node_start[k], B.node_start[k + 1]) for k, n in enumerate(B.node_id)}
    for n in sorted(set(ma) & set(mb)):
        yield ma[n], mb[n]


def search_bow_kf_f(KF, F, nn, ori):
    out = np.full(F.n, -1, np.int32)
    hist = [[] for _ in range(HISTO)]
    nm = 0
    nn = f32(nn)
    for (a0, a1), (b0, b1) in _shared_nodes(KF, F):
        for a in range(a0, a1):
            ik = int(KF.feat[a])
            if not KF.mp_good[ik]:
                continue
            tl, tr = _Top2(), _Top2()
            for j in range(b0, b1):
                jf = int(F.feat[j])
                if out[jf] >= 0:
                    continue
                d = dist(KF.desc[ik], F.desc[jf])
                (tl if F.nleft == -1 or jf < F.nleft else tr).push(d, 0, jf)
            if tl.b <= TH_LOW:
                if f32(tl.b) < nn * f32(tl.b2):
                    out[tl.bi] = KF.mp_id[ik]
                    nm += 1
                    if ori:
                        hist[rot_bin(KF.angle[ik], F.angle[tl.bi])].append(tl.bi)
                if tr.b <= TH_LOW:  # right match: ratio test disabled ('|| true')
                    out[tr.bi] = KF.mp_id[ik]
                    nm += 1
                    if ori:
                        hist[rot_bin(KF.angle[ik], F.angle[tr.bi])].append(tr.bi)
    if ori:
        nm = apply_hist(hist, out, nm)
    return nm, out


def search_bow_kf_kf(K1, K2, nn, ori):
    """Two-camera keyframes: indices >= mvKeysUn.size() == NLeft are skipped on both sides."""
    out = np.full(K1.n, -1, np.int32)
    matched2 = np.zeros(K2.n, bool)
    hist = [[] for _ in range(HISTO)]
    nm = 0
    nn = f32(nn)
    for (a0, a1), (b0, b1) in _shared_nodes(K1, K2):
        for a in range(a0, a1):
            i1 = int(K1.feat[a])
            if K1.nleft != -1 and i1 >= K1.nleft:
                continue
            if not K1.mp_good[i1]:
                continue
            b, bi, b2 = 256, -1, 256
            for j in range(b0, b1):
                i2 = int(K2.feat[j])
                if K2.nleft != -1 and i2 >= K2.nleft:
                    continue
                if matched2[i2] or K2.mp_id[i2] < 0 or not K2.mp_good[i2]:
                    continue
                d = dist(K1.desc[i1], K2.desc[i2])
                if d < b:
                    b2, b, bi = b, d, i2
                elif d < b2:
                    b2 = d
            if b < TH_LOW and f32(b) < nn * f32(b2):
                out[i1] = K2.mp_id[bi]
                matched2[bi] = True
                nm += 1
                if ori:
                    hist[rot_bin(K1.angle[i1], K2.angle[bi])].append(i1)
    if ori:
        nm = apply_hist(hist, out, nm)
    return nm, out


def fuse_search(F, Q, th, right=False, gated=True):
    """Search half of ORBmatcher::Fuse (both overloads): KeyFrame::GetFeaturesInArea (no levels),
    level window [pred-1, pred], chi2 gate (gated), strict '<' best, accept <= TH_LOW."""
    n = len(Q.valid)
    bi = np.full(n, -1, np.int32)
    bd = np.full(n, 256, np.int32)
    off = F.nleft if right else 0
    nf = 0
    for i in range(n):
        if not Q.valid[i]:
            continue
        lvl = int(Q.pred_level[i])
        rad = f32(f32(th) * F.scale[lvl])
        u, v = f32(Q.u[i]), f32(Q.v[i])
        best, besti = (256 if gated else 2 ** 31 - 1), -1
        for idx in features_in_area(F, u, v, rad, -1, -1, right=right):
            k = idx + off
            o = int(F.kp_octave[k])
            if o < lvl - 1 or o > lvl:
                continue
            if gated:
                ex, ey = f32(u - F.kp_x[k]), f32(v - F.kp_y[k])
                inv = f32(Q.inv_level_sigma2[o])
                kr = F.u_right[idx] if F.u_right is not None else f32(-1)
                if kr >= 0:
                    er = f32(f32(Q.ur[i]) - f32(kr))
                    e2 = f32(f32(f32(ex * ex) + f32(ey * ey)) + f32(er * er))
                    if float(f32(e2 * inv)) > 7.8:
                        continue
                else:
                    e2 = f32(f32(ex * ex) + f32(ey * ey))
                    if float(f32(e2 * inv)) > 5.99:
                        continue
            d = dist(Q.desc[i], F.desc[k])
            if d < best:
                best, besti = d, k
        bd[i] = min(best, 256)
        if best <= TH_LOW:
            bi[i] = besti
            nf += 1
    return nf, bi, bd


def search_for_triangulation(K1, K2, geom, only_stereo=False, coarse=False, ori=True):
    """ORBmatcher::SearchForTriangulation (ref:src/ORBmatcher.cc:1045-1328) with
    Pinhole::epipolarConstrain (ref:src/CameraModels/Pinhole.cpp:189-219).  Node pairing by set
    intersection (not the reference's lower_bound walk); returns (nmatches, pairs)."""
    nodes1 = {int(K1.node_id[k]): K1.feat[K1.node_start[k]:K1.node_start[k + 1]] for k in range(len(K1.node_id))}
    nodes2 = {int(K2.node_id[k]): K2.feat[K2.node_start[k]:K2.node_start[k + 1]] for k in range(len(K2.node_id))}
    m12 = [-1] * K1.n
    hist = [[] for _ in range(HISTO)]
    nm = 0
    F = geom.F12

    def stereo(K, i):
        return (not K.two_cam) and K.u_right is not None and K.u_right[i] >= 0

    def right(K, i):
        return not (K.nleft == -1 or i < K.nleft)

    for node in sorted(set(nodes1) & set(nodes2)):
        for idx1 in nodes1[node]:
            idx1 = int(idx1)
            if K1.has_mp[idx1]:
                continue
            s1 = stereo(K1, idx1)
            if only_stereo and not s1:
                continue
            x1, y1 = f32(K1.kp_x[idx1]), f32(K1.kp_y[idx1])
            best_d, best = TH_LOW, -1
            for idx2 in nodes2[node]:
                idx2 = int(idx2)
                if K2.has_mp[idx2]:
                    continue
                s2 = stereo(K2, idx2)
                if only_stereo and not s2:
                    continue
                d = dist(K1.desc[idx1], K2.desc[idx2])
                if d > TH_LOW or d > best_d:
                    continue
                x2, y2 = f32(K2.kp_x[idx2]), f32(K2.kp_y[idx2])
                o2 = int(K2.kp_octave[idx2])
                if not s1 and not s2 and not K1.two_cam:
                    ex, ey = f32(f32(geom.ep[0]) - x2), f32(f32(geom.ep[1]) - y2)
                    if f32(f32(ex * ex) + f32(ey * ey)) < f32(f32(100) * K2.scale[o2]):
                        continue
                k = (2 * right(K1, idx1) + right(K2, idx2)) if (K1.two_cam and K2.two_cam) else 0
                ok = coarse
                if not ok:
                    Fk = F[k]
                    a = f32(f32(f32(x1 * Fk[0, 0]) + f32(y1 * Fk[1, 0])) + Fk[2, 0])
                    b = f32(f32(f32(x1 * Fk[0, 1]) + f32(y1 * Fk[1, 1])) + Fk[2, 1])
                    c = f32(f32(f32(x1 * Fk[0, 2]) + f32(y1 * Fk[1, 2])) + Fk[2, 2])
                    num = f32(f32(f32(a * x2) + f32(b * y2)) + c)
                    den = f32(f32(a * a) + f32(b * b))
                    ok = den != 0 and float(f32(f32(num * num) / den)) < 3.84 * float(K2.level_sigma2[o2])
                if ok:
                    best, best_d = idx2, d
            if best >= 0:
                m12[idx1] = best
                nm += 1
                if ori:
                    hist[rot_bin(K1.kp_angle[idx1], K2.kp_angle[best])].append(idx1)
    if ori:
        nm = apply_hist(hist, m12, nm)
    pairs = [(i, j) for i, j in enumerate(m12) if j >= 0]
    return nm, np.array(pairs, np.int64).reshape(-1, 2)


def distinctive(desc_lists):
    """MapPoint::ComputeDistinctiveDescriptors (ref:src/MapPoint.cc:444-535) with numpy: the distance
    matrix by bitwise_count, per-row sorted median at int(0.5 * (N - 1)), first minimum."""
    out = []
    for d in desc_lists:
        d = np.asarray(d, np.uint8).reshape(-1, 32)
        n = len(d)
        if n == 0:
            out.append(-1)
            continue
        M = np.bitwise_count(d[:, None, :] ^ d[None, :, :]).sum(axis=2)
        med = np.sort(M, axis=1)[:, int(0.5 * (n - 1))]
        out.append(int(np.argmin(med)))
    return np.array(out, np.int32)


def search_sim3(F, Q, th, ratio, slot_query):
    """SearchByProjection(KeyFrame*, Sim3f&, ...) (ref:src/ORBmatcher.cc:498-621) from the area walk on:
    vpMatched written as soon as a MapPoint is accepted.  slot_query: -2 taken, -1 free."""
    s = np.array(slot_query, np.int32).copy()
    n = 0
    for q in range(Q.n):
        if not Q.valid[q]:
            continue
        lvl = int(Q.pred_level[q])
        r = f32(f32(th) * F.scale[lvl])
        bd, bi = 256, -1
        for idx in features_in_area(F, Q.u[q], Q.v[q], r):
            if s[idx] != -1:
                continue
            o = int(F.kp_octave[idx])
            if o < lvl - 1 or o > lvl:
                continue
            d = dist(Q.desc[q], F.desc[idx])
            if d < bd:
                bd, bi = d, idx
        if float(bd) <= float(f32(f32(TH_LOW) * f32(ratio))):
            s[bi] = q
            n += 1
    return n, s


def search_by_sim3(F1, F2, Q12, Q21, th):
    """ORBmatcher::SearchBySim3 (ref:src/ORBmatcher.cc:1696-1939) from the area walk on: each direction's
    strict-'<' minimum from INT_MAX, accepted iff <= TH_HIGH; the mutual pairs in KF1 order."""
    def direction(F, Q):
        out = [-1] * Q.n
        for q in range(Q.n):
            if not Q.valid[q]:
                continue
            lvl = int(Q.pred_level[q])
            r = f32(f32(th) * F.scale[lvl])
            bd, bi = 2147483647, -1
            for idx in features_in_area(F, Q.u[q], Q.v[q], r):
                o = int(F.kp_octave[idx])
                if o < lvl - 1 or o > lvl:
                    continue
                d = dist(Q.desc[q], F.desc[idx])
                if d < bd:
                    bd, bi = d, idx
            if bd <= TH_HIGH:
                out[q] = bi
        return out
    m1, m2 = direction(F2, Q12), direction(F1, Q21)
    m12 = [(i2 if i2 >= 0 and m2[i2] == i1 else -1) for i1, i2 in enumerate(m1)]
    return sum(1 for x in m12 if x >= 0), np.array(m12, np.int32)


def search_for_initialization(F1, F2, prev, window=100, nn=0.9, ori=True):
    """ORBmatcher::SearchForInitialization (ref:src/ORBmatcher.cc:735-878): (nmatches, vnMatches12, prev)."""
    INT_MAX = 2147483647
    n1, n2 = F1.n, F2.n
    m12 = [-1] * n1
    md = [INT_MAX] * n2
    m21 = [-1] * n2
    hist = [[] for _ in range(HISTO)]
    nm = 0
    for i1 in range(n1):
        if F1.kp_octave[i1] > 0:
            continue
        cand = features_in_area(F2, prev[i1, 0], prev[i1, 1], float(window), 0, 0)
        if not cand:
            continue
        b1 = b2 = INT_MAX
        bi = -1
        for i2 in cand:
            d = dist(F1.desc[i1], F2.desc[i2])
            if md[i2] <= d:
                continue
            if d < b1:
                b1, b2, bi = d, b1, i2
            elif d < b2:
                b2 = d
        if b1 <= TH_LOW and float(f32(b1)) < float(f32(f32(b2) * f32(nn))):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                nm -= 1
            m12[i1] = bi
            m21[bi] = i1
            md[bi] = b1
            nm += 1
            if ori:
                hist[rot_bin(F1.kp_angle[i1], F2.kp_angle[bi])].append(i1)
    if ori:
        keep = three_maxima([len(h) for h in hist])
        for i in range(HISTO):
            if i in keep:
                continue
            for i1 in hist[i]:
                if m12[i1] >= 0:
                    m12[i1] = -1
                    nm -= 1
    p = np.array(prev, np.float32).copy()
    for i1 in range(n1):
        if m12[i1] >= 0:
            p[i1] = (F2.kp_x[m12[i1]], F2.kp_y[m12[i1]])
    return nm, np.array(m12, np.int32), p
