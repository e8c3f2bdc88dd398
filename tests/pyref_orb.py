"""Pure-Python restatement of IC_Angle (ref:src/ORBextractor.cc:89-136) and computeOrbDescriptor
(ref:src/ORBextractor.cc:148-208), written independently of oracle/oracle_orb.c to pin it on small
cases.  float32 arithmetic step by step (numpy scalars round every operation to single precision);
cos / sin are libm's cosf / sinf through ctypes, as the reference's std::cos(float).  fastAtan2 is
OpenCV's published polynomial (OpenCV is not in the reference tree: parity with it is unpinned)."""
import ctypes as C
import ctypes.util

import numpy as np

_libm = C.CDLL(ctypes.util.find_library("m"))
_libm.cosf.restype = _libm.sinf.restype = C.c_float
_libm.cosf.argtypes = _libm.sinf.argtypes = [C.c_float]

f32 = np.float32


def fast_atan2(y, x):
    r2d = f32(180 / 3.1415926535897932384626433832795)
    p1, p3 = f32(0.9997878412794807) * r2d, f32(-0.3258083974640975) * r2d
    p5, p7 = f32(0.1555786518463281) * r2d, f32(-0.04432655554792128) * r2d
    y, x = f32(y), f32(x)
    ax, ay = abs(x), abs(y)
    eps = f32(np.finfo(np.float64).eps)
    if ax >= ay:
        c = ay / (ax + eps)
        c2 = c * c
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c
    else:
        c = ax / (ay + eps)
        c2 = c * c
        a = f32(90) - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c
    if x < 0:
        a = f32(180) - a
    if y < 0:
        a = f32(360) - a
    return f32(a)


def ic_angle(img, x, y, umax):
    cx, cy = int(np.rint(f32(x))), int(np.rint(f32(y)))
    I = img.astype(np.int64)
    m10 = sum(u * I[cy, cx + u] for u in range(-15, 16))
    m01 = 0
    for v in range(1, 16):
        d = int(umax[v])
        vs = 0
        for u in range(-d, d + 1):
            p, m = I[cy + v, cx + u], I[cy - v, cx + u]
            vs += p - m
            m10 += u * (p + m)
        m01 += v * vs
    return fast_atan2(f32(m01), f32(m10))


def orb_descriptor(img, x, y, angle, pattern):
    factor = f32(3.1415926535897932384626433832795 / f32(180))
    t = f32(angle) * factor
    a, b = f32(_libm.cosf(t)), f32(_libm.sinf(t))
    cx, cy = int(np.rint(f32(x))), int(np.rint(f32(y)))
    pts = np.asarray(pattern, np.int32).reshape(-1, 2)
    out = np.zeros(32, np.uint8)
    for i in range(32):
        val = 0
        for j in range(8):
            t2 = []
            for s in range(2):
                px, py = f32(pts[16 * i + 2 * j + s, 0]), f32(pts[16 * i + 2 * j + s, 1])
                dy = int(np.rint(px * b + py * a))
                dx = int(np.rint(px * a - py * b))
                flat = np.ascontiguousarray(img).reshape(-1)   # the continuous clone: rows wrap
                off = (cy + dy) * img.shape[1] + (cx + dx)
                t2.append(int(flat[off]) if 0 <= off < flat.size else 0)   # outside the buffer: 0
            val |= int(t2[0] < t2[1]) << j
        out[i] = val
    return out
