"""ctypes binding of oracle/liboracle.so (oracle/rmat.c) -- TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

I64P = ctypes.POINTER(ctypes.c_int64)
U8P = ctypes.POINTER(ctypes.c_uint8)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        lib = ctypes.CDLL(_LIB)
        lib.orc_splitmix64.restype = ctypes.c_uint64
        lib.orc_splitmix64.argtypes = [ctypes.c_uint64]
        lib.orc_rmat_edges.restype = None
        lib.orc_rmat_edges.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                       ctypes.c_int64, ctypes.c_int64, I64P, I64P]
        lib.orc_is_person.restype = ctypes.c_int
        lib.orc_is_person.argtypes = [ctypes.c_int64]
        lib.orc_age.restype = ctypes.c_int64
        lib.orc_age.argtypes = [ctypes.c_int64, ctypes.c_uint64]
        lib.orc_row_hash.restype = ctypes.c_uint64
        lib.orc_row_hash.argtypes = [I64P, ctypes.c_int]
        lib.orc_two_hop_enumerate.restype = ctypes.c_int
        lib.orc_two_hop_enumerate.argtypes = [ctypes.c_int64, ctypes.c_int64, I64P, I64P, U8P, U8P, U8P, I64P, I64P,
                                              I64P, I64P, ctypes.c_int]
        lib.orc_two_hop_closed_form.restype = ctypes.c_int
        lib.orc_two_hop_closed_form.argtypes = [ctypes.c_int64, ctypes.c_int64, I64P, I64P, U8P, U8P, U8P, I64P, I64P]
        lib.orc_expand_filter.restype = None
        lib.orc_expand_filter.argtypes = [ctypes.c_int64, I64P, I64P, U8P, U8P, I64P,
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        lib.orc_triangle_enumerate.restype = ctypes.c_int
        lib.orc_triangle_enumerate.argtypes = [ctypes.c_int64, ctypes.c_int64, I64P, I64P, I64P, ctypes.c_int]
        lib.orc_var_length_count.restype = ctypes.c_int
        lib.orc_var_length_count.argtypes = [ctypes.c_int64, ctypes.c_int64, I64P, I64P, U8P, U8P, ctypes.c_int,
                                             ctypes.c_int, I64P, I64P, ctypes.c_int]
        lib.orc_two_hop_undirected_enumerate.restype = ctypes.c_int
        lib.orc_two_hop_undirected_enumerate.argtypes = [ctypes.c_int64, ctypes.c_int64, I64P, I64P, U8P, U8P, U8P,
                                                         I64P, I64P, I64P, ctypes.c_int]
        # closed.c
        lib.orc_c2_masks.restype = None
        lib.orc_c2_masks.argtypes = [ctypes.c_int64, ctypes.c_uint64, U8P, U8P]
        lib.orc_two_hop_closed_form_mt.restype = ctypes.c_int
        lib.orc_two_hop_closed_form_mt.argtypes = [ctypes.c_int64, ctypes.c_int64, I64P, I64P, U8P, U8P, U8P, I64P,
                                                   I64P, ctypes.c_int]
        lib.orc_var_length_closed_form.restype = ctypes.c_int
        lib.orc_var_length_closed_form.argtypes = [ctypes.c_int64, ctypes.c_int64, I64P, I64P, U8P, U8P, ctypes.c_int,
                                                   ctypes.c_int, I64P, I64P, ctypes.c_int]
        lib.orc_vl4_t14.restype = ctypes.c_int
        lib.orc_vl4_t14.argtypes = [ctypes.c_int64, ctypes.c_int64, I64P, I64P, U8P, I64P, ctypes.c_int]
        lib.orc_triangle_closed_form.restype = ctypes.c_int
        lib.orc_triangle_closed_form.argtypes = [ctypes.c_int64, ctypes.c_int64, I64P, I64P, U8P, I64P, ctypes.c_int]
        _lib = lib
    return _lib


def _p64(a):
    return a.ctypes.data_as(I64P) if a is not None else None


def _p8(a):
    return a.ctypes.data_as(U8P) if a is not None else None


def splitmix64(x: int) -> int:
    return load().orc_splitmix64(x & 0xFFFFFFFFFFFFFFFF)


def rmat_edges(scale: int, e_begin: int, e_end: int, probs=(57, 19, 19), seed: int = 42):
    n = e_end - e_begin
    src = np.empty(n, dtype=np.int64)
    dst = np.empty(n, dtype=np.int64)
    load().orc_rmat_edges(scale, probs[0], probs[1], probs[2], seed, e_begin, e_end, _p64(src), _p64(dst))
    return src, dst


def person_mask(n: int) -> np.ndarray:
    lib = load()
    return np.array([lib.orc_is_person(i) for i in range(n)], dtype=np.uint8)


def ages(ids: np.ndarray, seed: int = 42) -> np.ndarray:
    lib = load()
    return np.array([lib.orc_age(int(i), seed) for i in ids], dtype=np.int64)


def row_hash(row) -> int:
    a = np.ascontiguousarray(np.asarray(row, dtype=np.int64))
    return load().orc_row_hash(_p64(a), len(a))


def fingerprint(cols) -> tuple:
    """(count, sum, xor) of row hashes over int64 columns (vectorised restatement of orc_row_hash)."""
    cols = [np.asarray(c, dtype=np.int64).astype(np.uint64) for c in cols]
    n = len(cols[0]) if cols else 0
    h = np.full(n, 0x243F6A8885A308D3, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for c in cols:
            z = (h ^ c) + np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            h = z ^ (z >> np.uint64(31))
        s = int(h.sum(dtype=np.uint64)) if n else 0
    x = int(np.bitwise_xor.reduce(h)) if n else 0
    return n, s, x


def two_hop_enumerate(n, src, dst, a_ok=None, b_ok=None, c_ok=None, grouped=False, threads=0):
    lib = load()
    rows, dist = ctypes.c_int64(), ctypes.c_int64()
    grows = np.zeros(n, dtype=np.int64) if grouped else None
    gdist = np.zeros(n, dtype=np.int64) if grouped else None
    rc = lib.orc_two_hop_enumerate(n, len(src), _p64(src), _p64(dst), _p8(a_ok), _p8(b_ok), _p8(c_ok),
                                   ctypes.byref(rows), ctypes.byref(dist), _p64(grows), _p64(gdist), threads)
    if rc:
        raise MemoryError("orc_two_hop_enumerate")
    if grouped:
        return rows.value, dist.value, grows, gdist
    return rows.value, dist.value


def two_hop_undirected_enumerate(n, src, dst, a_ok=None, b_ok=None, c_ok=None, threads=0):
    """(count(*), count(DISTINCT c), count(DISTINCT a)) of MATCH (a)-[r1]-(b)-[r2]-(c) by enumeration."""
    rows, dc, da = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    if load().orc_two_hop_undirected_enumerate(n, len(src), _p64(src), _p64(dst), _p8(a_ok), _p8(b_ok), _p8(c_ok),
                                               ctypes.byref(rows), ctypes.byref(dc), ctypes.byref(da), threads):
        raise MemoryError("orc_two_hop_undirected_enumerate")
    return rows.value, dc.value, da.value


def two_hop_closed_form(n, src, dst, a_ok=None, b_ok=None, c_ok=None):
    lib = load()
    rows, dist = ctypes.c_int64(), ctypes.c_int64()
    rc = lib.orc_two_hop_closed_form(n, len(src), _p64(src), _p64(dst), _p8(a_ok), _p8(b_ok), _p8(c_ok),
                                     ctypes.byref(rows), ctypes.byref(dist))
    if rc:
        raise MemoryError("orc_two_hop_closed_form")
    return rows.value, dist.value


def expand_filter(src, dst, a_ok=None, b_ok=None):
    lib = load()
    rows, s, x = ctypes.c_int64(), ctypes.c_uint64(), ctypes.c_uint64()
    lib.orc_expand_filter(len(src), _p64(src), _p64(dst), _p8(a_ok), _p8(b_ok), ctypes.byref(rows), ctypes.byref(s),
                          ctypes.byref(x))
    return rows.value, s.value, x.value


def triangle_enumerate(n, src, dst, threads=0):
    rows = ctypes.c_int64()
    if load().orc_triangle_enumerate(n, len(src), _p64(src), _p64(dst), ctypes.byref(rows), threads):
        raise MemoryError("orc_triangle_enumerate")
    return rows.value


def var_length_count(n, src, dst, lo, hi, a_ok=None, b_ok=None, threads=0):
    rows = ctypes.c_int64()
    g = np.zeros(n, dtype=np.int64)
    rc = load().orc_var_length_count(n, len(src), _p64(src), _p64(dst), _p8(a_ok), _p8(b_ok), lo, hi, _p64(g),
                                     ctypes.byref(rows), threads)
    if rc:
        raise ValueError(f"orc_var_length_count rc={rc}")
    return rows.value, g


def c2_masks(n: int, seed: int = 42):
    """(person, adult) uint8 masks of the C2 node tables (closed.c orc_c2_masks)."""
    person = np.empty(n, dtype=np.uint8)
    adult = np.empty(n, dtype=np.uint8)
    load().orc_c2_masks(n, seed, _p8(person), _p8(adult))
    return person, adult


def two_hop_closed_form_mt(n, src, dst, a_ok=None, b_ok=None, c_ok=None, threads=0):
    rows, dist = ctypes.c_int64(), ctypes.c_int64()
    if load().orc_two_hop_closed_form_mt(n, len(src), _p64(src), _p64(dst), _p8(a_ok), _p8(b_ok), _p8(c_ok),
                                         ctypes.byref(rows), ctypes.byref(dist), threads):
        raise MemoryError("orc_two_hop_closed_form_mt")
    return rows.value, dist.value


def var_length_closed_form(n, src, dst, lo, hi, a_ok=None, b_ok=None, threads=0):
    rows = ctypes.c_int64()
    g = np.zeros(n, dtype=np.int64)
    rc = load().orc_var_length_closed_form(n, len(src), _p64(src), _p64(dst), _p8(a_ok), _p8(b_ok), lo, hi, _p64(g),
                                           ctypes.byref(rows), threads)
    if rc:
        raise ValueError(f"orc_var_length_closed_form rc={rc}")
    return rows.value, g


def var_length4_closed_form(n, src, dst, a_ok=None, b_ok=None):
    """Per start node a: the relationship-distinct paths of exactly 4 hops a -> ... -> z with a_ok(a), b_ok(z)
    (MATCH (a)-[*4..4]->(b); paths never repeat a relationship: VarLengthExpandPlanner.scala:97,133,179-180),
    by inclusion-exclusion over the 15 set partitions of the hop positions {1,2,3,4} (Mobius weights
    prod (-1)^(|B|-1) (|B|-1)!).  A block {i, j} forces r_i = r_j, which makes the walk between them a closed
    walk: adjacent positions a self-loop, {1,3} / {2,4} a reciprocal pair, {1,4} a 2-walk back along a
    relationship (a directed triangle through it -- the one term that is not a product of per-node vectors and
    pair multiplicities).  Scipy sparse over the multiplicity matrix A (A[x, y] = m(x, y), self-loops on the
    diagonal); test infrastructure.  Returns (total, per-node counts)."""
    import scipy.sparse as sp
    src = np.ascontiguousarray(src, np.int64)
    dst = np.ascontiguousarray(dst, np.int64)
    A = sp.csr_matrix((np.ones(len(src), np.int64), (src, dst)), shape=(n, n))
    A.sum_duplicates()
    s = A.diagonal().astype(np.int64)
    b = np.ones(n, np.int64) if b_ok is None else np.asarray(b_ok).astype(np.int64)
    a = np.ones(n, np.int64) if a_ok is None else np.asarray(a_ok).astype(np.int64)
    Ab = A @ b
    A2b = A @ Ab
    M = A.multiply(A.T).tocsr()  # m(x, y) m(y, x)
    W4 = A @ (A @ A2b)
    pair1 = (s * A2b) + (A @ (s * Ab)) + (A @ (A @ (s * b)))      # {12} {23} {34}
    t14 = np.zeros(n, np.int64)  # {14}: sum_y A(a, y) b(y) (A A)(y, a), by merges (closed.c orc_vl4_t14)
    if load().orc_vl4_t14(n, len(src), _p64(src), _p64(dst), _p8(None if b_ok is None else np.ascontiguousarray(b_ok, np.uint8)),
                          _p64(t14), 0):
        raise MemoryError("orc_vl4_t14")
    pair2 = (M @ Ab) + (A @ (M @ b)) + t14  # {13} {24} {14}
    two = s * s * b * 2 + b * np.asarray(M.sum(axis=1)).ravel()     # {12}{34} {14}{23}; {13}{24}
    three = (s * Ab) + 2 * (s * s * b) + (A @ (s * b))             # {123}; {124} {134}; {234}
    per = (W4 - pair1 - pair2 + two + 2 * three - 6 * (s * b)) * a
    return int(per.sum()), per


def two_hop_undirected_closed_form(n, src, dst, a_ok=None, b_ok=None, c_ok=None, threads=0):
    """(count(*), count(DISTINCT c)) of (a)-[r1]-(b)-[r2]-(c), r1 <> r2 (closed.c)."""
    rows, d = ctypes.c_int64(), ctypes.c_int64()
    if load().orc_two_hop_undirected_closed_form(n, len(src), _p64(src), _p64(dst), _p8(a_ok), _p8(b_ok), _p8(c_ok),
                                                 ctypes.byref(rows), ctypes.byref(d), threads):
        raise MemoryError("orc_two_hop_undirected_closed_form")
    return rows.value, d.value


def triangle_closed_form(n, src, dst, n_ok=None, threads=0):
    rows = ctypes.c_int64()
    rc = load().orc_triangle_closed_form(n, len(src), _p64(src), _p64(dst), _p8(n_ok), ctypes.byref(rows), threads)
    if rc:
        raise ValueError(f"orc_triangle_closed_form rc={rc}")
    return rows.value
