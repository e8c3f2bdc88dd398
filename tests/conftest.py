import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import oracle_calls as oc  # noqa: E402



def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the HIP library")


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement (test infrastructure only): the checker for every parity test."""
    return oc.load()


@pytest.fixture(scope="session")
def ctx():
    """A product context on cuda:0.  Fails loudly (no fallback) if the library or GPU is absent."""
    from orb_slam3_comments_ghr_amd import Context
    c = Context(0)
    yield c
    c.close()


def ptr(a):
    return None if a is None else int(a.ctypes.data)
