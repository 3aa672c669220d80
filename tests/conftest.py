import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cypher-for-apache-spark_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libcapsmi kernels on the device)")


def gpu_available() -> bool:
    try:
        import capsmi._lib as L
        import ctypes
        lib = L.load()
        s = ctypes.c_void_p()
        if lib.capsmi_session_create(0, ctypes.byref(s)) != 0:
            return False
        lib.capsmi_session_destroy(s)
        return True
    except Exception:
        return False


@pytest.fixture(scope="session")
def session():
    from capsmi import Session
    s = Session(0)
    yield s
    s.close()
