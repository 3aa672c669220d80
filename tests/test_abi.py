"""CPU checks of the drop-in boundary: libcapsmi.so loads, exports every entry point declared in
include/capsmi.h, and fails loudly (no CPU fallback) when there is no GPU."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    with open(os.path.join(ROOT, "include", "capsmi.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^(?:capsmi_status|size_t|const char\*)\s+(capsmi_\w+)\s*\(", text, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    assert len(names) >= 45
    assert "capsmi_join" in names and "capsmi_two_hop_count_distinct" in names


def test_library_exports_every_declared_symbol():
    from capsmi import _lib
    lib = _lib.load()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    # the ctypes signature table covers the whole header too
    assert sorted(_lib.EXPORTED) == _declared()


def test_library_exports_only_c_symbols():
    """the boundary is C: every capsmi_* dynamic symbol is unmangled"""
    import subprocess
    so = os.path.join(ROOT, "cypher-for-apache-spark_amd", "capsmi", "libcapsmi.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(_declared()) <= syms


def test_version_string():
    from capsmi import _lib
    assert b"gfx950" in _lib.load().capsmi_version()


def test_no_silent_cpu_fallback_without_gpu():
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("a GPU is present")
    from capsmi import _lib
    lib = _lib.load()
    s = ctypes.c_void_p()
    rc = lib.capsmi_session_create(0, ctypes.byref(s))
    assert rc == _lib.ERR_DEVICE
    assert "HIP" in _lib.last_error()
    with pytest.raises(_lib.DeviceError):
        from capsmi import Session
        Session(0)


def test_null_arguments_are_rejected():
    from capsmi import _lib
    lib = _lib.load()
    out = ctypes.c_int64()
    assert lib.capsmi_table_size(None, ctypes.byref(out)) == _lib.ERR_ILLEGAL_ARGUMENT
    assert "null argument" in _lib.last_error()
    b, e = ctypes.c_int64(), ctypes.c_int64()
    assert lib.capsmi_owner_words(1 << 20, 3, 8, ctypes.byref(b), ctypes.byref(e)) == 0
    assert (b.value, e.value) == (3 * 32768 // 8, 4 * 32768 // 8)


def test_config_knobs_are_checked():
    """capsmi_config_check: the session configuration's names and values, refused when
    unknown -- the removed A/B variants' knobs included -- or unparsable."""
    from capsmi import _lib
    lib = _lib.load()
    ok = [("CAPSMI_JOIN", "radix"), ("CAPSMI_JOIN", "auto"), ("CAPSMI_COUNT", "atomic"), ("CAPSMI_COUNT", "rec"),
          ("CAPSMI_REC_FULL", "0"), ("CAPSMI_GROUPED", "keys"), ("CAPSMI_PAIRS", "uint2"), ("CAPSMI_TRI_BUILD", "sorted"),
          ("CAPSMI_TRI_DEG_SAMPLE", "32"), ("CAPSMI_TRI_SPLIT", "0"), ("CAPSMI_TRI_VMODE_T", "0"),
          ("CAPSMI_UND", "stream"), ("CAPSMI_VL_BITS", "16"), ("CAPSMI_VL_SUBLOG", "3"), ("CAPSMI_VL_F2", "1"),
          ("CAPSMI_COLL_CHUNK", "64"), ("CAPSMI_INGEST_THREADS", "4"), ("CAPSMI_JOIN", None)]
    for k, v in ok:
        assert lib.capsmi_config_check(k.encode(), None if v is None else v.encode()) == _lib.OK, (k, v)
    bad = [("CAPSMI_JOIN", "sideways"), ("CAPSMI_COUNT", "pairs"), ("CAPSMI_VL_BITS", "1"), ("CAPSMI_TRI_SPLIT", "x"),
           ("CAPSMI_COLL_CHUNK", "0"), ("CAPSMI_P1", "6"), ("CAPSMI_SORT", "onesweep"), ("CAPSMI_TRI_WALK", "flat"),
           ("CAPSMI_RADIX_ORDER", "probe"), ("CAPSMI_NOPE", None)]
    for k, v in bad:
        assert lib.capsmi_config_check(k.encode(), None if v is None else v.encode()) == _lib.ERR_ILLEGAL_ARGUMENT, (k, v)
        assert "configuration" in _lib.last_error()


def test_profiling_names_need_a_session():
    """capsmi_session_set_profiling_names refuses a null session (no device needed to check)."""
    from capsmi import _lib
    lib = _lib.load()
    assert lib.capsmi_session_set_profiling_names(None, b"part_scatter1") == _lib.ERR_ILLEGAL_ARGUMENT
    assert lib.capsmi_session_set_profiling_names(None, None) == _lib.ERR_ILLEGAL_ARGUMENT
