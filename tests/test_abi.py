"""CPU: the C-ABI library loads and exports every symbol include/*.h declares (no GPU compute)."""
import ctypes
import os
import re

import pytest

from orb_slam3_comments_ghr_amd import _abi, load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    syms = set()
    for h in ("osg.h", "osg_ba.h", "osg_dbow.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(osg_[a-z0-9_]+)\s*\(", text):
            syms.add(m.group(1))
    return syms


def test_header_symbols_match_binding_table():
    assert header_symbols() == set(_abi.EXPORTS)


def test_library_exports_every_symbol():
    lib = load_library()
    for s in _abi.EXPORTS:
        assert hasattr(lib, s), s


def test_every_symbol_has_argtypes():
    # pointers through an undeclared ctypes call would be truncated to C int
    lib = load_library()
    missing = [s for s in _abi.EXPORTS if getattr(lib, s).argtypes is None]
    assert not missing, missing


def test_host_only_entry_points():
    lib = load_library()
    assert b"gfx950" in lib.osg_version()
    assert lib.osg_strerror(-4) == b"unsupported configuration"
    import numpy as np
    a = np.zeros(32, np.uint8)
    b = np.full(32, 255, np.uint8)
    assert lib.osg_descriptor_distance(a.ctypes.data, b.ctypes.data) == 256


def test_ctx_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU visible")
    lib = load_library()
    h = ctypes.c_void_p()
    rc = lib.osg_ctx_create(0, ctypes.byref(h))
    assert rc in (_abi.OSG_E_NODEVICE, _abi.OSG_E_HIP) and not h.value
