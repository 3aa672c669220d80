"""Sanitizer runs of the host code (SURVEY.md §5 "ASan/UBSan on the C++ host code"), on the CPU:
- the oracle's C restatement (oracle/rmat.c, closed.c) under AddressSanitizer + UndefinedBehaviorSanitizer,
  every closed form against enumeration (tests/sanitize/oracle_san.c);
- the CSV reader's host half (csrc/csv_parse.h: chunking, the threaded parser, Spark row ids) under
  ASan + UBSan and under ThreadSanitizer, 1 vs 2 / 3 / 8 threads equal (tests/sanitize/csv_san.cpp).
GPU code is not instrumented (GPU sanitizers are unavailable on this pool); the harnesses are built from the
sources into a temporary directory, nothing is committed."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")
ASAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


def _build(cmd, tmp_path):
    if not shutil.which(cmd[0]):
        pytest.skip(f"{cmd[0]} not installed")
    p = subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True)
    if p.returncode != 0 and "cannot find" in (p.stderr + p.stdout) and "san" in (p.stderr + p.stdout):
        pytest.skip("sanitizer runtime not installed: " + p.stderr[-300:])
    assert p.returncode == 0, p.stderr[-3000:]


def _run(exe, *args, timeout=240):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1", OMP_NUM_THREADS="4")
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=timeout, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-6000:])
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-6000:]
    assert "WARNING: ThreadSanitizer" not in p.stderr, p.stderr[-6000:]
    return p.stdout


def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_san")
    _build(["gcc", *ASAN, "-fopenmp", "-std=c11", os.path.join(SAN, "oracle_san.c"),
            os.path.join(ROOT, "oracle", "rmat.c"), os.path.join(ROOT, "oracle", "closed.c"), "-o", exe], tmp_path)
    out = _run(exe)
    assert "0 mismatches" in out, out


def test_csv_reader_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "csv_san")
    _build(["g++", *ASAN, "-std=c++17", "-pthread", os.path.join(SAN, "csv_san.cpp"), "-o", exe], tmp_path)
    out = _run(exe, "300")
    assert "0 mismatches" in out, out


def test_csv_reader_under_tsan(tmp_path):
    exe = str(tmp_path / "csv_tsan")
    _build(["g++", "-fsanitize=thread", "-g", "-O1", "-std=c++17", "-pthread", os.path.join(SAN, "csv_san.cpp"),
            "-o", exe], tmp_path)
    out = _run(exe, "60")
    assert "0 mismatches" in out, out
