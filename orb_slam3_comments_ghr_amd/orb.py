"""Host mirror of ORBextractor's per-keypoint stages on the C ABI (``osg_orb_describe``, include/osg.h
b8): computeOrientation / IC_Angle (ref:src/ORBextractor.cc:89-136, 585-597) on mvImagePyramid and
computeDescriptors / computeOrbDescriptor (ref:src/ORBextractor.cc:148-208, 1534-1545) on the blurred
levels (ref:src/ORBextractor.cc:1628-1652).  The caller passes the extractor's ``umax`` and
``pattern``.

ComputePyramid + the per-level GaussianBlur (``osg_orb_pyramid``, include/osg.h b10; OpenCV's
fixed-point resize / blur restated, parity with OpenCV itself unpinned):

    P = ComputePyramid(ctx, image, inv_scale_factors(8, 1.2))     # P.raw, P.blurred on the GPU

ComputeKeyPointsOctTree (``osg_orb_detect``, include/osg.h b9): FAST per W = 35 cell with
iniThFAST / minThFAST and DistributeOctTree down to mnFeaturesPerLevel (ref:src/ORBextractor.cc:
716-1198):

    x, y, response, size, level_start = ORBDetect(ctx, raw, features_per_level(1000, 8, 1.2),
                                                  scale_factors(8, 1.2))

    angle, desc, n_out = ORBDescribe(ctx, raw, blurred, x, y, level, pattern, umax)     # IC_Angle + rBRIEF
    _, desc, n_out = ORBDescribe(ctx, None, blurred, x, y, level, pattern, angle=angle) # given angles

n_out counts the keypoints whose rotated pattern left their level's buffer (read as 0 there; the
reference reads foreign heap).  The blurred levels are addressed as the reference's continuous clone.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import Context, _abi, load_library
from .stereo import ImagePyramid

HALF_PATCH_SIZE = 15
EDGE_THRESHOLD = 19


def ic_umax(half_patch_size: int = HALF_PATCH_SIZE) -> np.ndarray:
    """The row half-widths of the circular orientation patch, as the ORBextractor constructor builds
    them (ref:src/ORBextractor.cc:548-575): cvRound(sqrt(hp^2 - v^2)) up to vmax, then mirrored about
    the diagonal so the patch is symmetric."""
    hp = half_patch_size
    r = float(np.float32(hp) * np.float32(math.sqrt(2.0)) / np.float32(2))  # HALF_PATCH_SIZE * sqrt(2.f) / 2
    vmax, vmin = math.floor(r + 1), math.ceil(r)
    umax = [0] * (hp + 1)
    for v in range(vmax + 1):
        umax[v] = int(np.rint(math.sqrt(hp * hp - v * v)))
    v0 = 0
    for v in range(hp, vmin - 1, -1):
        while umax[v0] == umax[v0 + 1]:
            v0 += 1
        umax[v] = v0
        v0 += 1
    return np.array(umax, np.int32)


def synth_pattern(rng, npoints: int = 512, radius: int = 13) -> np.ndarray:
    """A BRIEF test pattern of the reference's shape (ORBextractor::pattern: 512 points, 256 pairs,
    coordinates within +-13).  The real bit_pattern_31_ comes from the caller's extractor."""
    return rng.integers(-radius, radius + 1, (npoints, 2)).astype(np.int32)


def ORBDescribe(ctx: Context, raw, blurred, x, y, level, pattern, umax=None, angle=None):
    """IC_Angle (when ``angle`` is None) and the 256-bit steered BRIEF descriptor of every keypoint.
    raw / blurred: ImagePyramid (mvImagePyramid and its GaussianBlur'd levels) or lists of levels;
    x, y: level coordinates; level: KeyPoint::octave.  Returns (angle float32[n], desc uint8[n, 32],
    keypoints that read outside their level's buffer)."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    level = np.ascontiguousarray(level, np.int32)
    n = len(x)
    assert len(y) == n and len(level) == n
    pattern = np.ascontiguousarray(pattern, np.int32).reshape(-1)
    assert pattern.size == 1024, "ORBextractor::pattern: 512 (x, y) points"
    compute = angle is None
    if compute:
        umax = ic_umax() if umax is None else np.ascontiguousarray(umax, np.int32)
        assert umax.size == HALF_PATCH_SIZE + 1
        ang = np.zeros(n, np.float32)
    else:
        ang = np.array(angle, np.float32).reshape(-1)
        assert ang.size == n
    if blurred is not None and not isinstance(blurred, ImagePyramid):
        blurred = ImagePyramid(blurred)
    if raw is not None and not isinstance(raw, ImagePyramid):
        raw = ImagePyramid(raw)
    assert blurred is not None and (raw is not None or not compute)
    desc = np.zeros((n, 32), np.uint8)
    K = _abi.OsgOrbKeypoints(n, x.ctypes.data, y.ctypes.data, level.ctypes.data)
    rs = raw.struct() if raw is not None else _abi.OsgImagePyramid()
    bs = blurred.struct()
    n_out = ctx.check(ctx.lib.osg_orb_describe(ctx.handle, C.byref(rs), C.byref(bs), C.byref(K), pattern.ctypes.data,
                                       umax.ctypes.data if compute else None, int(compute), ang.ctypes.data,
                                       desc.ctypes.data), "osg_orb_describe")
    return ang, desc, n_out


def scale_factors(n_levels: int = 8, factor: float = 1.2) -> np.ndarray:
    """mvScaleFactor as the ORBextractor constructor builds it (ref:src/ORBextractor.cc:484-491):
    float products of scaleFactor."""
    s = [np.float32(1.0)]
    for _ in range(1, n_levels):
        s.append(np.float32(s[-1] * np.float32(factor)))
    return np.array(s, np.float32)


def features_per_level(nfeatures: int = 1000, n_levels: int = 8, factor: float = 1.2) -> np.ndarray:
    """mnFeaturesPerLevel (ref:src/ORBextractor.cc:505-528): a geometric share per level in float,
    cvRound'ed, the last level taking the rest."""
    f = np.float32(1.0) / np.float32(factor)
    d = np.float32(np.float32(nfeatures * (np.float32(1) - f)) /
                   (np.float32(1) - np.float32(math.pow(float(f), float(n_levels)))))
    out, total = [], 0
    for _ in range(n_levels - 1):
        n = int(np.rint(d))
        out.append(n)
        total += n
        d = np.float32(d * f)
    out.append(max(nfeatures - total, 0))
    return np.array(out, np.int32)


def ORBDetect(ctx: Context, raw, n_features, scales, ini_th: int = 20, min_th: int = 7, capacity: int | None = None):
    """ORBextractor::ComputeKeyPointsOctTree on the GPU (FAST scores and per-cell suppression) and the
    host (DistributeOctTree).  raw: ImagePyramid or a list of levels (mvImagePyramid); n_features:
    mnFeaturesPerLevel; scales: mvScaleFactor.  Returns (x, y, response, size, level_start) with the
    keypoints of level l at [level_start[l], level_start[l + 1]) in the reference's order, in level
    coordinates."""
    if not isinstance(raw, ImagePyramid):
        raw = ImagePyramid(raw)
    L = len(raw.levels)
    n_features = np.ascontiguousarray(n_features, np.int32)
    scales = np.ascontiguousarray(scales, np.float32)
    assert n_features.size >= L and scales.size >= L
    cap = int(capacity if capacity is not None else max(int(n_features[:L].sum()) * 2 + 16, 64))
    x, y, resp, size = (np.zeros(cap, np.float32) for _ in range(4))
    ls = np.zeros(L + 1, np.int32)
    rs = raw.struct()
    n = ctx.check(ctx.lib.osg_orb_detect(ctx.handle, C.byref(rs), int(ini_th), int(min_th), n_features.ctypes.data,
                                         scales.ctypes.data, cap, x.ctypes.data, y.ctypes.data, resp.ctypes.data,
                                         size.ctypes.data, ls.ctypes.data), "osg_orb_detect")
    return x[:n], y[:n], resp[:n], size[:n], ls


def inv_scale_factors(n_levels: int = 8, factor: float = 1.2) -> np.ndarray:
    """mvInvScaleFactor: 1.0f / mvScaleFactor[i] in float (ref:src/ORBextractor.cc ORBextractor())."""
    return (np.float32(1) / scale_factors(n_levels, factor)).astype(np.float32)


def pyramid_layout(rows: int, cols: int, inv_scale):
    """Level sizes and byte offsets of ``osg_orb_pyramid``'s buffer (include/osg.h b10): returns
    (level_rows, level_cols, bordered_offset, blurred_offset, total_bytes)."""
    inv_scale = np.ascontiguousarray(inv_scale, np.float32)
    L = inv_scale.size
    lr, lc = np.zeros(L, np.int32), np.zeros(L, np.int32)
    bo, bl = np.zeros(L, np.int64), np.zeros(L, np.int64)
    total = load_library().osg_orb_pyramid_layout(int(rows), int(cols), L, inv_scale.ctypes.data, lr.ctypes.data,
                                                  lc.ctypes.data, bo.ctypes.data, bl.ctypes.data)
    if total < 0:
        raise ValueError(f"osg_orb_pyramid_layout({rows}, {cols}, {L} levels) = {total}")
    return lr, lc, bo, bl, int(total)


class OrbPyramid:
    """The device buffer ``ComputePyramid`` fills: ``raw`` is mvImagePyramid (ImagePyramid of the ROI
    views, row step cols + 38), ``bordered`` the whole bordered levels, ``blurred`` the GaussianBlur'd
    levels (continuous, as the reference's clone) or None."""

    def __init__(self, buffer, lr, lc, bo, bl, blur):
        E = EDGE_THRESHOLD
        self.buffer = buffer
        self.level_rows, self.level_cols = lr, lc
        self.bordered = [buffer[int(bo[l]):int(bo[l]) + (int(lr[l]) + 2 * E) * (int(lc[l]) + 2 * E)]
                         .view(int(lr[l]) + 2 * E, int(lc[l]) + 2 * E) for l in range(lr.size)]
        self.raw = ImagePyramid([b[E:E + int(lr[l]), E:E + int(lc[l])] for l, b in enumerate(self.bordered)])
        self.blurred = ImagePyramid([buffer[int(bl[l]):int(bl[l]) + int(lr[l]) * int(lc[l])]
                                     .view(int(lr[l]), int(lc[l])) for l in range(lr.size)]) if blur else None


def ComputePyramid(ctx: Context, image, inv_scale, blur: bool = True, out=None, sync: bool = True) -> OrbPyramid:
    """ORBextractor::ComputePyramid (ref:src/ORBextractor.cc:1692-1743) and, with blur, the per-level
    GaussianBlur(7 x 7, 2, 2, BORDER_REFLECT_101) of operator() (:1628-1636), on the GPU
    (``osg_orb_pyramid``, include/osg.h b10).  image: 8-bit numpy array (any row step) or a uint8
    torch tensor on the GPU; inv_scale: mvInvScaleFactor.  out: a reusable uint8 device buffer of at
    least the layout's size.  sync=False skips the device synchronisation before the call (the caller
    knows a device image is complete)."""
    import torch

    on_device = hasattr(image, "data_ptr")
    if on_device:
        assert image.is_cuda and image.dtype == torch.uint8 and image.dim() == 2 and image.stride(1) == 1
        rows, cols, step, ptr = image.shape[0], image.shape[1], image.stride(0), image.data_ptr()
        if sync:
            torch.cuda.synchronize(image.device)  # the kernels run on the context's own stream
    else:
        assert image.dtype == np.uint8 and image.ndim == 2 and image.strides[1] == 1, "8-bit rows"
        rows, cols, step, ptr = image.shape[0], image.shape[1], image.strides[0], image.ctypes.data
    inv_scale = np.ascontiguousarray(inv_scale, np.float32)
    lr, lc, bo, bl, total = pyramid_layout(rows, cols, inv_scale)
    if out is None or out.numel() < total:
        out = torch.empty(total, dtype=torch.uint8, device=image.device if on_device else "cuda")
        torch.cuda.synchronize(out.device)
    ctx.check(ctx.lib.osg_orb_pyramid(ctx.handle, ptr, rows, cols, step, int(on_device), inv_scale.size,
                                      inv_scale.ctypes.data, out.data_ptr(), out.numel(), int(bool(blur))),
              "osg_orb_pyramid")
    return OrbPyramid(out, lr, lc, bo, bl, blur)


class OrbBatchKeypoints:
    """What ``ORBExtractBatch`` returns: per-image arrays [B, capacity] (x, y in level coordinates,
    angle in degrees, response, size, octave) and desc [B, capacity, 32]; image b's keypoints are the
    first counts[b] of its row, level by level in the reference's order."""

    def __init__(self, counts, x, y, angle, response, size, octave, desc):
        self.counts, self.x, self.y, self.angle = counts, x, y, angle
        self.response, self.size, self.octave, self.desc = response, size, octave, desc

    def image(self, b: int):
        """(x, y, angle, response, size, octave, desc) of image b."""
        n = int(self.counts[b])
        return (self.x[b, :n], self.y[b, :n], self.angle[b, :n], self.response[b, :n], self.size[b, :n],
                self.octave[b, :n], self.desc[b, :n])

    def level_coordinates_to_image(self, scales):
        """KeyPoint::pt *= mvScaleFactor[octave] for octave > 0 (ref:src/ORBextractor.cc:1663-1667)."""
        s = np.asarray(scales, np.float32)[self.octave]
        return self.x * s, self.y * s


def ORBExtractBatch(ctx: Context, images, n_features: int = 1000, n_levels: int = 8, factor: float = 1.2,
                    ini_th: int = 20, min_th: int = 7, pattern=None, umax=None, capacity: int | None = None,
                    sync: bool = True) -> OrbBatchKeypoints:
    """ORBextractor::operator() (ref:src/ORBextractor.cc:1553-1690) for a batch of same-size images
    on the GPU (``osg_orb_extract_batch``, include/osg.h b11): each image's keypoints, angles and
    descriptors equal ComputePyramid -> ORBDetect -> ORBDescribe on that image alone.
    images: uint8 torch tensor [B, rows, cols] on the GPU (row stride 1 element apart, any image
    stride); pattern: ORBextractor::pattern (512 (x, y) points)."""
    import torch

    assert hasattr(images, "data_ptr") and images.is_cuda and images.dtype == torch.uint8, "device uint8 images"
    assert images.dim() == 3 and images.stride(2) == 1
    B, rows, cols = images.shape
    if sync:
        torch.cuda.synchronize(images.device)  # the kernels run on the context's own stream
    scales = scale_factors(n_levels, factor)
    inv = inv_scale_factors(n_levels, factor)
    nfl = features_per_level(n_features, n_levels, factor)
    assert pattern is not None, "ORBextractor::pattern"
    pattern = np.ascontiguousarray(pattern, np.int32).reshape(-1)
    assert pattern.size == 1024, "ORBextractor::pattern: 512 (x, y) points"
    umax = ic_umax() if umax is None else np.ascontiguousarray(umax, np.int32)
    assert umax.size == HALF_PATCH_SIZE + 1
    cap = int(capacity if capacity is not None else max(int(nfl.sum()) * 2 + 16, 64))
    prm = _abi.OsgOrbExtractParams(n_levels, scales.ctypes.data, inv.ctypes.data, nfl.ctypes.data, int(ini_th),
                                   int(min_th), pattern.ctypes.data, umax.ctypes.data)
    x, y, ang, resp, size = (np.zeros((B, cap), np.float32) for _ in range(5))
    octave = np.zeros((B, cap), np.int32)
    desc = np.zeros((B, cap, 32), np.uint8)
    counts = np.zeros(B, np.int32)
    # a size-1 batch dimension may carry any stride (numpy's new axes have 0)
    istride = images.stride(0) if B > 1 else rows * images.stride(1)
    ctx.check(ctx.lib.osg_orb_extract_batch(ctx.handle, images.data_ptr(), istride, rows, cols,
                                            images.stride(1), B, C.byref(prm), cap, x.ctypes.data, y.ctypes.data,
                                            ang.ctypes.data, resp.ctypes.data, size.ctypes.data, octave.ctypes.data,
                                            desc.ctypes.data, counts.ctypes.data), "osg_orb_extract_batch")
    return OrbBatchKeypoints(counts, x, y, ang, resp, size, octave, desc)


def synth_fast_pyramid(rng, width=752, height=480, n_levels=8, factor=1.2, n_blobs=400):
    """A synthetic image pyramid with FAST corners: a smooth random background plus bright and dark
    rectangles and discs (corners and blobs at every scale), each level a box-filtered 2x2 resample
    of the base image at size cvRound(size / scale) (ComputePyramid's shape,
    ref:src/ORBextractor.cc:1692-1745; cv::resize itself is OpenCV's)."""
    img = rng.normal(128, 6, (height, width)).astype(np.float32)
    for _ in range(n_blobs):
        cx, cy = rng.integers(0, width), rng.integers(0, height)
        r = int(rng.integers(2, 14))
        val = float(rng.choice([30.0, 70.0, 190.0, 235.0]))
        if rng.random() < 0.5:
            img[max(0, cy - r):cy + r, max(0, cx - r):cx + r] = val
        else:
            yy, xx = np.ogrid[:height, :width]
            img[(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = val
    base = np.clip(img + rng.normal(0, 3, img.shape), 0, 255).astype(np.uint8)
    levels = [base]
    sc = scale_factors(n_levels, factor)
    for l in range(1, n_levels):
        w, h = int(np.rint(np.float32(width) / sc[l])), int(np.rint(np.float32(height) / sc[l]))
        ys = np.minimum((np.arange(h) * sc[l]).astype(np.int64), height - 1)
        xs = np.minimum((np.arange(w) * sc[l]).astype(np.int64), width - 1)
        levels.append(np.ascontiguousarray(base[np.ix_(ys, xs)]))
    return levels


def synth_orb_frame(rng, n=1200, width=752, height=480, n_levels=8, factor=1.2, fractional=False,
                    edge=EDGE_THRESHOLD):
    """A synthetic extractor output of EuRoC shape: per level a smooth random image (raw) and a second
    one standing in for its blur, and n keypoints spread over the levels in proportion to their area
    (ref:src/ORBextractor.cc:474-494), ``edge`` px inside each level (FAST's own margin is
    EDGE_THRESHOLD - 3 = 16, where rotated pattern points can fall off the row and wrap).  ``fractional``
    adds sub-pixel offsets including exact .5 ties (cvRound is round-half-even)."""
    raw, blur = [], []
    scale = 1.0
    areas = []
    for _ in range(n_levels):
        w, h = int(round(width / scale)), int(round(height / scale))
        base = rng.integers(0, 256, (h // 4 + 2, w // 4 + 2)).astype(np.float32)
        img = np.kron(base, np.ones((4, 4), np.float32))[:h, :w] + rng.normal(0, 12, (h, w))
        raw.append(np.clip(img, 0, 255).astype(np.uint8))
        b = img.copy()
        b[1:-1, 1:-1] = (img[:-2, 1:-1] + img[2:, 1:-1] + img[1:-1, :-2] + img[1:-1, 2:] + 4 * img[1:-1, 1:-1]) / 8
        blur.append(np.clip(b, 0, 255).astype(np.uint8))
        areas.append(w * h)
        scale *= factor
    share = np.array(areas, np.float64) / sum(areas)
    level = rng.choice(n_levels, size=n, p=share).astype(np.int32)
    x = np.empty(n, np.float32)
    y = np.empty(n, np.float32)
    for l in range(n_levels):
        m = level == l
        h, w = raw[l].shape
        x[m] = rng.integers(edge, w - edge, m.sum())
        y[m] = rng.integers(edge, h - edge, m.sum())
    if fractional:
        off = rng.choice(np.array([0.0, 0.25, 0.5, -0.5, 0.45, -0.3], np.float32), size=(2, n))
        x += off[0]
        y += off[1]
    return raw, blur, x, y, level
