"""Host mirror of ``Frame::ComputeStereoMatches`` (ref:src/Frame.cc:1117-1373) on the C ABI
(``osg_compute_stereo_matches[_batch]``, include/osg.h b7): the rectified-stereo step of the stereo
Frame constructor (ref:src/Frame.cc:165).  ``StereoFrame`` holds the Frame fields it reads — mvKeys /
mvKeysRight (x, y, octave), mDescriptors / mDescriptorsRight, mvScaleFactors / mvInvScaleFactors,
mb / mbf — and both ORBextractor pyramids (mvImagePyramid: host arrays with any row step, or torch
tensors already on the GPU).  The call returns mvuRight and mvDepth (-1 = no match) and the number
of matches kept.

    ur, depth, n = ComputeStereoMatches(ctx, F)
    outs, n = ComputeStereoMatchesBatch(ctx, [F0, F1, ...])     # B frames, one launch
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field, replace

import numpy as np

from . import Context, _abi
from .frames import scale_factors
from .synth import EUROC_BF, EUROC_FX, EUROC_H, EUROC_W


class ImagePyramid:
    """ORBextractor::mvImagePyramid: one 8-bit image per level.  numpy levels may be row-strided views
    (the reference's levels are ROIs of bordered buffers, ref:src/ORBextractor.cc:1692-1700); torch
    levels on the GPU are read in place."""

    def __init__(self, levels):
        self.levels = list(levels)
        self.on_device = bool(self.levels) and hasattr(self.levels[0], "data_ptr")
        ptrs, rows, cols, step = [], [], [], []
        for lv in self.levels:
            if self.on_device:
                assert lv.is_cuda and lv.element_size() == 1 and lv.dim() == 2 and lv.stride(1) == 1
                ptrs.append(lv.data_ptr())
                step.append(lv.stride(0))
            else:
                assert lv.dtype == np.uint8 and lv.ndim == 2 and lv.strides[1] == 1, "8-bit rows, unit column stride"
                ptrs.append(lv.ctypes.data)
                step.append(lv.strides[0])
            rows.append(lv.shape[0])
            cols.append(lv.shape[1])
        self._ptrs = (C.c_void_p * max(len(ptrs), 1))(*ptrs)
        self._rows, self._cols, self._step = (np.array(v, np.int32) for v in (rows, cols, step))

    def struct(self):
        s = _abi.OsgImagePyramid()
        s.n_levels = len(self.levels)
        s.on_device = int(self.on_device)
        s.data = C.addressof(self._ptrs)
        s.rows, s.cols, s.step = self._rows.ctypes.data, self._cols.ctypes.data, self._step.ctypes.data
        return s

    def to_device(self, device="cuda"):
        import torch
        levels = [torch.from_numpy(np.ascontiguousarray(lv)).to(device) for lv in self.levels]
        torch.cuda.synchronize(device)  # the kernels run on the context's own stream
        return ImagePyramid(levels)


@dataclass
class StereoFrame:
    desc: np.ndarray          # mDescriptors, n x 32
    x: np.ndarray             # mvKeys[i].pt.x
    y: np.ndarray
    octave: np.ndarray
    desc_r: np.ndarray        # mDescriptorsRight, n_right x 32
    xr: np.ndarray            # mvKeysRight[i].pt.x
    yr: np.ndarray
    octave_r: np.ndarray
    left: ImagePyramid        # mpORBextractorLeft->mvImagePyramid
    right: ImagePyramid       # mpORBextractorRight->mvImagePyramid
    scale: np.ndarray = field(default_factory=scale_factors)
    mb: float = EUROC_BF / EUROC_FX
    mbf: float = EUROC_BF

    def __post_init__(self):
        self.desc = np.ascontiguousarray(self.desc, np.uint8).reshape(-1, 32)
        self.desc_r = np.ascontiguousarray(self.desc_r, np.uint8).reshape(-1, 32)
        for k, dt in (("x", np.float32), ("y", np.float32), ("octave", np.int32), ("xr", np.float32),
                      ("yr", np.float32), ("octave_r", np.int32), ("scale", np.float32)):
            setattr(self, k, np.ascontiguousarray(getattr(self, k), dt))
        # mvInvScaleFactor[i] = 1.0f / mvScaleFactor[i] (ref:src/ORBextractor.cc:504)
        self.inv_scale = (np.float32(1.0) / self.scale).astype(np.float32)

    @property
    def n(self):
        return self.desc.shape[0]

    @property
    def n_right(self):
        return self.desc_r.shape[0]

    def struct(self):
        s = _abi.OsgStereoFrame()
        s.n, s.n_right = self.n, self.n_right
        s.x, s.y, s.octave, s.desc = (a.ctypes.data for a in (self.x, self.y, self.octave, self.desc))
        s.xr, s.yr, s.octave_r, s.desc_r = (a.ctypes.data for a in (self.xr, self.yr, self.octave_r, self.desc_r))
        s.scale_factors = self.scale.ctypes.data
        s.inv_scale_factors = self.inv_scale.ctypes.data
        s.n_levels = len(self.scale)
        s.mb, s.mbf = self.mb, self.mbf
        s.left, s.right = self.left.struct(), self.right.struct()
        return s

    def to_device(self, device="cuda"):
        """The same frame with both pyramids resident on the GPU (read in place by the kernel)."""
        return replace(self, left=self.left.to_device(device), right=self.right.to_device(device))


def ComputeStereoMatches(ctx: Context, F: StereoFrame):
    """``Frame::ComputeStereoMatches()``: (mvuRight, mvDepth, matches kept)."""
    ur = np.empty(F.n, np.float32)
    depth = np.empty(F.n, np.float32)
    s = F.struct()
    n = ctx.check(ctx.lib.osg_compute_stereo_matches(ctx.handle, C.byref(s), ur.ctypes.data, depth.ctypes.data),
                  "ComputeStereoMatches")
    return ur, depth, n


def ComputeStereoMatchesBatch(ctx: Context, frames):
    """B frames in one launch (a batch of stereo Frame constructions); ([(mvuRight, mvDepth)], kept[B])."""
    B = len(frames)
    arr = (_abi.OsgStereoFrame * max(B, 1))(*[f.struct() for f in frames])
    off = np.zeros(B + 1, np.int64)
    off[1:] = np.cumsum([f.n for f in frames])
    ur = np.empty(int(off[-1]), np.float32)
    depth = np.empty(int(off[-1]), np.float32)
    nm = np.zeros(max(B, 1), np.int32)
    ctx.check(ctx.lib.osg_compute_stereo_matches_batch(ctx.handle, C.addressof(arr), B, ur.ctypes.data,
                                                       depth.ctypes.data, nm.ctypes.data), "ComputeStereoMatchesBatch")
    return [(ur[off[i]:off[i + 1]], depth[off[i]:off[i + 1]]) for i in range(B)], nm[:B]


# ------------------------------------------------------------------------------- generators

def _field(g, ys, xs, step):
    """Bilinear sample of the coarse random field g (one node every `step` px) at (ys, xs)."""
    gy, gx = ys / step, xs / step
    y0 = np.clip(np.floor(gy).astype(np.int64), 0, g.shape[0] - 2)
    x0 = np.clip(np.floor(gx).astype(np.int64), 0, g.shape[1] - 2)
    fy, fx = np.clip(gy - y0, 0, 1), np.clip(gx - x0, 0, 1)
    return (g[y0, x0] * (1 - fy) * (1 - fx) + g[y0 + 1, x0] * fy * (1 - fx) + g[y0, x0 + 1] * (1 - fy) * fx
            + g[y0 + 1, x0 + 1] * fy * fx)


def _flip1(rng, d, p):
    bits = np.unpackbits(d)
    return np.packbits(bits ^ (rng.random(bits.shape) < p).astype(np.uint8))


def synth_stereo_frame(rng, n=1200, n_right=None, width=EUROC_W, height=EUROC_H, n_levels=8, match=0.75,
                       edge=16.0, dup=0.03, confuse=0.15, bordered=False, mb=EUROC_BF / EUROC_FX, mbf=EUROC_BF,
                       noise=2.0, step=3.0):
    """A rectified EuRoC-like stereo pair (752 x 480, bf 47.9): a textured scene of 12 fronto-parallel
    planes (Z 1.5-12 m), both pyramids sampled from it (+ pixel noise; level sizes as ORBextractor's
    cvRound(cols / scale)); n left keypoints, octave ~ geometric(1/1.2), `edge` x scale px from the
    border.  `match` of them are seen in the right image at their plane's disparity (+ sub-pixel noise,
    descriptor flips p = 0.04, octave +-1 for 15 %); `confuse` of those get a weaker copy (flips
    p = 0.2) on the same row, `dup` an exact duplicate 2 x scale px to the left (a Hamming tie: the
    lower right index wins); the remaining right keypoints are unrelated.  `bordered`: levels are ROI
    views of buffers with a 19-px border, as the reference's are (row step != cols)."""
    n_right = n if n_right is None else n_right
    scale = scale_factors(n_levels)
    inv = (np.float32(1.0) / scale).astype(np.float32)
    g = rng.uniform(0, 255, (int(height / step) + 3, int(width / step) + 3))
    zb = rng.uniform(1.5, 12.0, (3, 4))

    def disparity(ys, xs):
        by = np.clip((ys * 3 / height).astype(np.int64), 0, 2)
        bx = np.clip((xs * 4 / width).astype(np.int64), 0, 3)
        return mbf / zb[by, bx]

    def pyramid(right):
        levels = []
        for s, iv in zip(scale, inv):
            w = int(np.floor(float(np.float32(width) * iv) + 0.5))
            h = int(np.floor(float(np.float32(height) * iv) + 0.5))
            ys, xs = np.meshgrid(np.arange(h) * float(s), np.arange(w) * float(s), indexing="ij")
            if right:
                xs = xs + disparity(ys, xs)
            img = np.clip(np.rint(_field(g, ys, xs, step) + rng.normal(0, noise, (h, w))), 0, 255).astype(np.uint8)
            if bordered:
                buf = np.zeros((h + 38, w + 38), np.uint8)
                buf[19:19 + h, 19:19 + w] = img
                img = buf[19:19 + h, 19:19 + w]
            levels.append(img)
        return ImagePyramid(levels)

    p = np.array([1.2 ** -i for i in range(n_levels)])
    oct_ = rng.choice(n_levels, size=n, p=p / p.sum()).astype(np.int32)
    s = scale[oct_].astype(np.float64)
    x = rng.uniform(edge * s, width - edge * s).astype(np.float32)
    y = rng.uniform(edge * s, height - edge * s).astype(np.float32)
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    d = disparity(y.astype(np.float64), x.astype(np.float64))
    rx, ry, ro, rd = [], [], [], []
    for i in np.nonzero(rng.random(n) < match)[0]:
        o = int(np.clip(oct_[i] + (rng.choice([-1, 1]) if rng.random() < 0.15 else 0), 0, n_levels - 1))
        xr_ = float(x[i]) - d[i] + rng.normal(0, 0.3 * s[i])
        yr_ = float(np.clip(float(y[i]) + rng.normal(0, 0.4 * s[i]), 0, height - 1))
        if not 0 <= xr_ < width:
            continue
        rx.append(xr_), ry.append(yr_), ro.append(o), rd.append(_flip1(rng, desc[i], 0.04))
        if rng.random() < dup and xr_ - 2 * s[i] >= 0:
            rx.append(xr_ - 2 * s[i]), ry.append(yr_), ro.append(o), rd.append(rd[-1].copy())
        if rng.random() < confuse:
            rx.append(float(np.clip(xr_ + rng.uniform(-20, 20) * s[i], 0, width - 1))), ry.append(yr_)
            ro.append(o), rd.append(_flip1(rng, desc[i], 0.2))
    while len(rx) < n_right:
        rx.append(rng.uniform(0, width)), ry.append(rng.uniform(0, height))
        ro.append(int(rng.choice(n_levels, p=p / p.sum()))), rd.append(rng.integers(0, 256, 32, dtype=np.uint8))
    perm = rng.permutation(len(rx))[:n_right]
    desc_r = np.stack(rd)[perm] if n_right else np.zeros((0, 32), np.uint8)
    return StereoFrame(desc=desc, x=x, y=y, octave=oct_, desc_r=desc_r, xr=np.array(rx, np.float32)[perm],
                       yr=np.array(ry, np.float32)[perm], octave_r=np.array(ro, np.int32)[perm], left=pyramid(False),
                       right=pyramid(True), scale=scale, mb=mb, mbf=mbf)


# ------------------------------------------------------------------ the KannalaBrandt8 rig's stereo step

@dataclass
class FishEyeStereoFrame:
    """The inputs of ``Frame::ComputeStereoFishEyeMatches()`` (ref:src/Frame.cc:1546-1603): both cameras'
    keypoints (x, y, octave) and descriptors with the stereo rows from monoLeft / monoRight on, mvLevelSigma2,
    the two KannalaBrandt8 parameter vectors and the rig's mRlr / mtlr."""
    kp_left: np.ndarray    # (Nleft, 2) float32
    oct_left: np.ndarray   # (Nleft,) int32
    desc_left: np.ndarray  # (Nleft, 32) uint8
    mono_left: int
    kp_right: np.ndarray
    oct_right: np.ndarray
    desc_right: np.ndarray
    mono_right: int
    level_sigma2: np.ndarray  # float32
    cam_left: np.ndarray      # fx fy cx cy k0 k1 k2 k3, float32
    cam_right: np.ndarray
    Rlr: np.ndarray           # (3, 3) float32
    tlr: np.ndarray           # (3,) float32

    def args(self):
        f = lambda a, t: np.ascontiguousarray(a, t)  # noqa: E731
        return (f(self.kp_left, np.float32), f(self.oct_left, np.int32), f(self.desc_left, np.uint8),
                f(self.kp_right, np.float32), f(self.oct_right, np.int32), f(self.desc_right, np.uint8),
                f(self.level_sigma2, np.float32), f(self.cam_left, np.float32), f(self.cam_right, np.float32),
                f(self.Rlr, np.float32), f(self.tlr, np.float32))


def ComputeStereoFishEyeMatches(ctx: Context, F: FishEyeStereoFrame):
    """``Frame::ComputeStereoFishEyeMatches()`` through ``osg_compute_stereo_fisheye_matches``:
    (mvLeftToRightMatch, mvRightToLeftMatch, mvDepth, mvStereo3Dpoints, nMatches)."""
    kl, ol, dl, kr, orr, dr, s2, cl, cr, R, t = F.args()
    nl, nr = kl.shape[0], kr.shape[0]
    l2r, r2l = np.empty(nl, np.int32), np.empty(nr, np.int32)
    depth, p3d = np.empty(nl, np.float32), np.empty((nl, 3), np.float32)
    n = ctx.check(ctx.lib.osg_compute_stereo_fisheye_matches(
        ctx.handle, nl, F.mono_left, dl.ctypes.data, kl.ctypes.data, ol.ctypes.data, nr, F.mono_right,
        dr.ctypes.data, kr.ctypes.data, orr.ctypes.data, s2.ctypes.data, s2.size, cl.ctypes.data, cr.ctypes.data,
        R.ctypes.data, t.ctypes.data, l2r.ctypes.data, r2l.ctypes.data, depth.ctypes.data, p3d.ctypes.data),
        "ComputeStereoFishEyeMatches")
    return l2r, r2l, depth, p3d, n


def synth_fisheye_stereo(rng, n_points=600, n_mono_left=150, n_mono_right=140, n_distract=120, flip=0.04,
                         n_levels=8, factor=1.2):
    """A TUM-VI-like KannalaBrandt8 rig (EuRoC-sized intrinsics, 10 cm baseline, 1-2 degree relative
    rotation): n_points 3-D points seen by both cameras (right descriptor = left with `flip` of the bits
    flipped, pixel noise 0.3 px), mono rows first on each side, unrelated right distractors, right stereo rows
    shuffled.  Some pairs duplicate a descriptor so the knn ties and the ratio test both occur."""
    from .frames import KB8_TRIANG, kb8_project
    cam = KB8_TRIANG.astype(np.float32)
    a = np.deg2rad(rng.uniform(1, 2))
    Rlr = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]], np.float64)
    tlr = np.array([0.10, 0.002, -0.001])
    X = np.stack([rng.uniform(-3, 3, n_points), rng.uniform(-2, 2, n_points), rng.uniform(1.0, 8.0, n_points)], 1)
    Xr = (X - tlr) @ Rlr  # Rlr^T (X - tlr): left-camera point in the right camera
    uvl = kb8_project(cam.astype(np.float64), X) + rng.normal(0, 0.3, (n_points, 2))
    uvr = kb8_project(cam.astype(np.float64), Xr) + rng.normal(0, 0.3, (n_points, 2))
    dl = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    dup = rng.choice(n_points, n_points // 20, replace=False)
    dl[dup[1::2]] = dl[dup[0::2][:len(dup[1::2])]]  # equal descriptors: knn ties / failed ratio
    dr = np.stack([_flip1(rng, d, flip) for d in dl])
    nd = n_distract
    dr = np.concatenate([dr, rng.integers(0, 256, (nd, 32), dtype=np.uint8)])
    uvr = np.concatenate([uvr, rng.uniform([0, 0], [752, 480], (nd, 2))])
    perm = rng.permutation(len(dr))
    dr, uvr = dr[perm], uvr[perm]
    octl = rng.integers(0, n_levels, n_points).astype(np.int32)
    octr = rng.integers(0, n_levels, len(dr)).astype(np.int32)
    ml = rng.uniform([0, 0], [752, 480], (n_mono_left, 2))
    mr = rng.uniform([0, 0], [752, 480], (n_mono_right, 2))
    sf = scale_factors(n_levels, factor)
    return FishEyeStereoFrame(
        kp_left=np.concatenate([ml, uvl]).astype(np.float32),
        oct_left=np.concatenate([rng.integers(0, n_levels, n_mono_left), octl]).astype(np.int32),
        desc_left=np.concatenate([rng.integers(0, 256, (n_mono_left, 32), dtype=np.uint8), dl]),
        mono_left=n_mono_left,
        kp_right=np.concatenate([mr, uvr]).astype(np.float32),
        oct_right=np.concatenate([rng.integers(0, n_levels, n_mono_right), octr]).astype(np.int32),
        desc_right=np.concatenate([rng.integers(0, 256, (n_mono_right, 32), dtype=np.uint8), dr]),
        mono_right=n_mono_right,
        level_sigma2=(np.asarray(sf, np.float32) ** 2).astype(np.float32),
        cam_left=cam, cam_right=cam.copy(), Rlr=Rlr.astype(np.float32), tlr=tlr.astype(np.float32))
