"""numpy restatement of ComputePyramid + the per-level GaussianBlur (ref:src/ORBextractor.cc:1692-1743,
1628-1636), written independently of oracle/oracle_pyramid.c to pin it: whole-array cv::resize
INTER_LINEAR fixed-point tables and passes, np.pad(mode="reflect") for BORDER_REFLECT_101, and the
7-tap fixed-point Gaussian derived with Python floats.  OpenCV's own code is not in the reference tree,
so this pins the restatement, not OpenCV."""
import math

import numpy as np

EDGE = 19


def gaussian_kernel7(sigma=2.0):
    xs = [-3, -2, -1]
    v = [math.exp(-(x * x) / (2 * sigma * sigma)) for x in xs]
    s = 2 * sum(v) + 1
    err, out = 0.0, []
    for t in v:
        adj = t / s * 256 + err
        q = round(adj)  # Python round: ties to even, like lrint
        err = adj - q
        out.append(q)
    return out + [256 - 2 * sum(out)] + out[::-1]


def _axis(sn, dn):
    scale = 1.0 / (dn / sn)
    d = np.arange(dn, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    return s, f


def _weights(f):
    w0 = np.rint((np.float32(1) - f).astype(np.float32) * np.float32(2048)).astype(np.int64)
    w1 = np.rint(f * np.float32(2048)).astype(np.int64)
    return w0, w1


def vector_columns(w):
    x = 16 * (w // 16)
    return x + 8 if w - x > 8 else x


def resize(src, dw, dh):
    sh, sw = src.shape
    S = src.astype(np.int64)
    sx, fx = _axis(sw, dw)
    left = sx < 0
    fx[left], sx[left] = 0, 0
    right = sx + 1 >= sw
    xmax = int(np.argmax(right)) if right.any() else dw
    clamp = sx >= sw - 1
    fx[clamp], sx[clamp] = 0, sw - 1
    a0, a1 = _weights(fx)
    H = S[:, sx] * a0 + S[:, np.minimum(sx + 1, sw - 1)] * a1
    H[:, xmax:] = S[:, sx[xmax:]] * 2048
    sy, fy = _axis(sh, dh)
    b0, b1 = _weights(fy)
    D0 = H[np.clip(sy, 0, sh - 1)]
    D1 = H[np.clip(sy + 1, 0, sh - 1)]
    vec = (((D0 >> 4) * b0[:, None]) >> 16) + (((D1 >> 4) * b1[:, None]) >> 16)
    vec = (vec + 2) >> 2
    sca = (D0 * b0[:, None] + D1 * b1[:, None] + (1 << 21)) >> 22
    xv = vector_columns(dw)
    out = np.where(np.arange(dw)[None, :] < xv, vec, sca)
    return np.clip(out, 0, 255).astype(np.uint8)


def blur(img):
    k = np.array(gaussian_kernel7(), np.int64)
    h, w = img.shape
    P = np.pad(img.astype(np.int64), 3, mode="reflect")
    H = sum(k[j] * P[:, j:j + w] for j in range(7))
    V = sum(k[i] * H[i:i + h, :] for i in range(7))
    return ((V + (1 << 15)) >> 16).astype(np.uint8)


def pyramid(image, inv_scale):
    """(bordered levels, ROI levels, blurred levels)."""
    rows, cols = image.shape
    bordered, roi = [], []
    for l, s in enumerate(np.asarray(inv_scale, np.float32)):
        w = int(np.rint(np.float32(cols) * s))
        h = int(np.rint(np.float32(rows) * s))
        lv = image.copy() if l == 0 else resize(roi[-1], w, h)
        assert lv.shape == (h, w)
        roi.append(lv)
        bordered.append(np.pad(lv, EDGE, mode="reflect"))
    return bordered, roi, [blur(r) for r in roi]
