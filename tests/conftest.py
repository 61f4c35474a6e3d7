import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")


@pytest.fixture(scope="session")
def oracle():
    import _oracle
    _oracle.lib()
    return _oracle


@pytest.fixture(scope="session")
def gpu_lib():
    """The HIP library; GPU tests fail loudly (never fall back) when it is missing or no device is visible."""
    from pinot_amd import _lib as L
    from pinot_amd.build import build
    build()
    lib = L.load()
    import ctypes
    n = ctypes.c_int()
    L.check(lib.pgpu_device_count(ctypes.byref(n)))
    assert n.value > 0, "no HIP device visible"
    return lib
