"""Helpers that run the C oracle (test infrastructure) on the SoA containers."""
import ctypes as C

import numpy as np


def mps(oracle, F, Q, nn, th, far, thfar, slot_mp, slot_taken):
    s = slot_mp.copy()
    fs, qs = F.struct(), Q.struct()
    t = np.ascontiguousarray(slot_taken, np.uint8)
    n = oracle.oracle_search_by_projection_mps(C.byref(fs), C.byref(qs), nn, th, int(far), thfar,
                                               s.ctypes.data, t.ctypes.data)
    return n, s


def last(oracle, F, L, th, mono, ori, slot_mp, slot_taken):
    s = slot_mp.copy()
    fs, qs = F.struct(), L.struct()
    t = np.ascontiguousarray(slot_taken, np.uint8)
    n = oracle.oracle_search_by_projection_last(C.byref(fs), C.byref(qs), th, int(mono), int(ori),
                                                s.ctypes.data, t.ctypes.data)
    return n, s


def kf(oracle, F, K, th, orb, ori, slot_mp):
    s = slot_mp.copy()
    fs, qs = F.struct(), K.struct()
    n = oracle.oracle_search_by_projection_kf(C.byref(fs), C.byref(qs), th, int(orb), int(ori), s.ctypes.data)
    return n, s


def bow_kf_f(oracle, KF, F, nn, ori):
    out = np.full(F.n, -1, np.int32)
    a, b = KF.struct(), F.struct()
    n = oracle.oracle_search_by_bow_kf_f(C.byref(a), C.byref(b), nn, int(ori), out.ctypes.data)
    return n, out


def bow_kf_kf(oracle, K1, K2, nn, ori):
    out = np.full(K1.n, -1, np.int32)
    a, b = K1.struct(), K2.struct()
    n = oracle.oracle_search_by_bow_kf_kf(C.byref(a), C.byref(b), nn, int(ori), out.ctypes.data)
    return n, out
