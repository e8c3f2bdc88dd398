"""orb_slam3_comments_ghr_amd — MI355X-native ORB-SLAM3 matching + bundle-adjustment hot path.

The product is ``liborbslam3_amd.so`` (hand-written HIP kernels for gfx950 behind the C ABI in
``include/osg.h`` / ``include/osg_ba.h``).  This package loads it with ctypes and mirrors the
reference operator API (``ORBmatcher``, ``Optimizer``) on top of it.  There is no CPU fallback:
if the library or a gfx950 device is missing, every operation raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi
from ._abi import LIB_PATH

__all__ = ["load_library", "Context", "OsgError", "LIB_PATH"]

_lib = None


class OsgError(RuntimeError):
    pass


def load_library() -> C.CDLL:
    """Load liborbslam3_amd.so (built by ``make`` / ``__graft_entry__.build()``)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OsgError(
                f"{LIB_PATH} is missing: build it with `make` (hipcc --offload-arch=gfx950); "
                "there is no CPU fallback for the hot path")
        _torch_device_first()
        _lib = _abi.declare(C.CDLL(LIB_PATH))
    return _lib


def _ptr(a) -> int | None:
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if hasattr(a, "data_ptr"):  # torch tensor
        return int(a.data_ptr())
    assert isinstance(a, np.ndarray) and a.flags["C_CONTIGUOUS"], "need a C-contiguous ndarray"
    return int(a.ctypes.data)


def _torch_device_first():
    """torch ships its own libamdhip64 (same soname as /opt/rocm's).  Measured on the MI355X box: when
    the library's HIP runtime is loaded or initialised before torch's, torch reports no GPU for the
    rest of the process (and the other way round the library does); when torch is imported and
    initialised first, both share torch's runtime and device tensors pass through the ABI (bench.py's
    order).  So the library is loaded after torch has opened the device."""
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()


class Context:
    """One ``osg_ctx`` (device, HIP stream, pooled scratch).  One per host thread."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.osg_ctx_create(int(device), C.byref(h))
        if rc != 0:
            raise OsgError(f"osg_ctx_create(device={device}) failed: "
                           f"{self.lib.osg_strerror(rc).decode()}")
        self.handle = h
        self.device = device

    def close(self):
        if getattr(self, "handle", None):
            self.lib.osg_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def check(self, rc: int, what: str) -> int:
        if rc < 0:
            msg = self.lib.osg_ctx_last_error(self.handle).decode()
            raise OsgError(f"{what}: {self.lib.osg_strerror(rc).decode()} ({msg})")
        return rc

    def set_stream(self, stream_handle: int | None):
        self.check(self.lib.osg_ctx_set_stream(self.handle, stream_handle), "set_stream")

    def synchronize(self):
        self.check(self.lib.osg_ctx_synchronize(self.handle), "synchronize")

    # ---- a1/a2 ---------------------------------------------------------------------------
    def hamming_top2(self, query: np.ndarray, train: np.ndarray):
        """Brute-force top-2 (best_idx, best_dist, second_dist) per query row."""
        q = np.ascontiguousarray(query, dtype=np.uint8).reshape(-1, 32)
        t = np.ascontiguousarray(train, dtype=np.uint8).reshape(-1, 32)
        nq, nt = q.shape[0], t.shape[0]
        bi = np.empty(nq, np.int32)
        bd = np.empty(nq, np.int32)
        sd = np.empty(nq, np.int32)
        self.check(self.lib.osg_hamming_top2(self.handle, _ptr(q), nq, _ptr(t), nt, _ptr(bi),
                                             _ptr(bd), _ptr(sd)), "osg_hamming_top2")
        return bi, bd, sd

    def hamming_top2_dev(self, d_query, nq: int, d_train, nt: int, d_out):
        """Device-resident form (torch tensors or raw device addresses); async on the stream."""
        self.check(self.lib.osg_hamming_top2_dev(self.handle, _ptr(d_query), int(nq),
                                                 _ptr(d_train), int(nt), _ptr(d_out)),
                   "osg_hamming_top2_dev")

    def hamming_top2_batch_dev(self, d_query, nq: int, d_train, nt: int, nb: int, d_out):
        """nb equal-shape problems in one launch (device pointers / tensors; problem b at rows b*nq of
        d_query and d_out, b*nt of d_train); async on the stream."""
        self.check(self.lib.osg_hamming_top2_batch_dev(self.handle, _ptr(d_query), int(nq), _ptr(d_train), int(nt),
                                                       int(nb), _ptr(d_out)), "osg_hamming_top2_batch_dev")

    def hamming_top2_plan(self, nq: int, nt: int) -> str:
        """Name and grid of the kernel a (nq, nt) top-2 launch uses in this process."""
        import ctypes
        buf = ctypes.create_string_buffer(160)
        self.check(self.lib.osg_hamming_top2_plan(self.handle, int(nq), int(nt), buf, 160), "osg_hamming_top2_plan")
        return buf.value.decode()

    def hamming_top2_batch_plan(self, nq: int, nt: int, nb: int) -> str:
        """The kernel osg_hamming_top2_batch_dev launches for (nq, nt, nb), with its shape and grid."""
        buf = C.create_string_buffer(160)
        self.check(self.lib.osg_hamming_top2_batch_plan(self.handle, int(nq), int(nt), int(nb), buf, 160),
                   "osg_hamming_top2_batch_plan")
        return buf.value.decode()

    def match_last_stats(self) -> dict:
        """Diagnostics of the last search call: candidates, Jacobi rounds, serial redo, nmatches."""
        out = np.zeros(4, np.int32)
        self.check(self.lib.osg_match_last_stats(self.handle, _ptr(out)), "osg_match_last_stats")
        return dict(candidates=int(out[0]), rounds=int(out[1]), serial=bool(out[2]), nmatches=int(out[3]),
                    kernel_ms=self.last_kernel_ms())

    def last_kernel_ms(self) -> float:
        """Device time of the last matching / pose-optimization kernel (HIP events), ms."""
        ms = np.zeros(1, np.float64)
        self.check(self.lib.osg_ctx_last_kernel_ms(self.handle, _ptr(ms)), "osg_ctx_last_kernel_ms")
        return float(ms[0])

    def device_bytes(self) -> int:
        """Device memory this context's scratch arena holds (slots grow to the largest call and stay)."""
        b = np.zeros(1, np.int64)
        self.check(self.lib.osg_ctx_device_bytes(self.handle, _ptr(b)), "osg_ctx_device_bytes")
        return int(b[0])

    def descriptor_distance_pairs(self, a: np.ndarray, b: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=np.uint8).reshape(-1, 32)
        b = np.ascontiguousarray(b, dtype=np.uint8).reshape(-1, 32)
        assert a.shape == b.shape
        out = np.empty(a.shape[0], np.int32)
        self.check(self.lib.osg_descriptor_distance_pairs(self.handle, _ptr(a), _ptr(b),
                                                          a.shape[0], _ptr(out)),
                   "osg_descriptor_distance_pairs")
        return out


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    """ORBmatcher::DescriptorDistance on one pair (host scalar, ref:src/ORBmatcher.cc:2388-2408)."""
    lib = load_library()
    a = np.ascontiguousarray(a, dtype=np.uint8).reshape(32)
    b = np.ascontiguousarray(b, dtype=np.uint8).reshape(32)
    return int(lib.osg_descriptor_distance(_ptr(a), _ptr(b)))
