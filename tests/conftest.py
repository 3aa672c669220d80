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
    """One session for the GPU tests, bound to torch's current stream: the tests hand torch buffers
    (``torch.zeros(...).data_ptr()``) to library calls, and a zero-fill queued on torch's stream is
    only ordered before the library's copies when both run on one stream (include/capsmi.h, the
    external-buffer contract).  On the session's own non-blocking stream a late fill could overwrite
    words the library had already copied (GPUTEST_r05: test_bitmap_scan_of_exact_node_table)."""
    import torch
    from capsmi import Session
    s = Session(0)
    s.set_stream(torch.cuda.current_stream().cuda_stream)
    yield s
    s.close()


@pytest.fixture
def knobs():
    """``knobs(session, CAPSMI_COUNT="atomic")``: CAPSMI_* configuration knobs on a session for one test
    (capsmi_session_set_config -- the library reads the environment only at session create), put back to
    the environment's values when the test ends."""
    done = []

    def set_(sess, **kv):
        for k, v in kv.items():
            sess.set_config(k, v)
            done.append((sess, k))

    yield set_
    for sess, k in reversed(done):
        try:
            sess.set_config(k, None)
        except Exception:  # a session the test closed
            pass
