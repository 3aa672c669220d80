"""The generic equi-join (Table.join, SparkTable.scala:205-229) on its radix-partitioned LDS path
and direct-address path (csrc/k_rjoin.hip), at sizes that exercise several partitions, build chunks
larger than one LDS table and probe partitions spread over many tiles.  Expected pairs: pandas' merge on the non-null
keys (null keys never match; an unmatched or null-key row of the preserved side is padded with
nulls); every strategy (CAPSMI_JOIN=radix|hash|direct and the automatic choice) must give the
same pairs.  Bit-exact."""
import os

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


def _table(session, name, keys, valid=None, types=None):
    from capsmi import ColumnData
    from capsmi.expr import I64
    cols = [ColumnData(f"{name}_row", I64, np.arange(len(keys[0]), dtype=np.int64))]
    for i, k in enumerate(keys):
        cols.append(ColumnData(f"{name}_k{i}", (types or {}).get(i, I64), k, None if valid is None else valid[i]))
    return session.table(cols)


def _expected(lk, lv, rk, rv, jt):
    def frame(keys, valid, tag):
        d = {f"k{i}": k for i, k in enumerate(keys)}
        d[tag] = np.arange(len(keys[0]))
        f = pd.DataFrame(d)
        ok = np.ones(len(keys[0]), bool)
        for v in valid or []:
            if v is not None:
                ok &= v
        return f[ok], f[~ok]
    lf, lnull = frame(lk, lv, "l")
    rf, rnull = frame(rk, rv, "r")
    on = [f"k{i}" for i in range(len(lk))]
    how = {"inner": "inner", "left_outer": "left", "right_outer": "right"}[jt]
    m = lf.merge(rf, on=on, how=how)
    pairs = [np.stack([m["l"].fillna(-1).to_numpy(np.int64), m["r"].fillna(-1).to_numpy(np.int64)], 1)]
    if jt == "left_outer":
        pairs.append(np.stack([lnull["l"].to_numpy(np.int64), np.full(len(lnull), -1)], 1))
    if jt == "right_outer":
        pairs.append(np.stack([np.full(len(rnull), -1), rnull["r"].to_numpy(np.int64)], 1))
    p = np.concatenate(pairs)
    return p[np.lexsort((p[:, 1], p[:, 0]))]


def _pairs(t):
    cl, cr = t.column("l_row"), t.column("r_row")
    a = np.where(cl.valid, cl.values, -1) if cl.valid is not None else cl.values
    b = np.where(cr.valid, cr.values, -1) if cr.valid is not None else cr.values
    p = np.stack([a, b], 1).astype(np.int64)
    return p[np.lexsort((p[:, 1], p[:, 0]))]


def _join(session, L, R, jt, nkeys, mode):
    """mode: a CAPSMI_JOIN strategy (session configuration)"""
    with session.configured(CAPSMI_JOIN=mode):
        t = L.join(R, jt, *[(f"l_k{i}", f"r_k{i}") for i in range(nkeys)])
        return _pairs(t)


def _check(session, lk, rk, jt, lv=None, rv=None, types=None):
    L = _table(session, "l", lk, lv, types)
    R = _table(session, "r", rk, rv, types)
    want = _expected(lk, lv, rk, rv, jt)
    for mode in ("radix", "hash", "direct", "auto"):
        got = _join(session, L, R, jt, len(lk), mode)
        assert got.shape == want.shape, mode
        np.testing.assert_array_equal(got, want, err_msg=mode)
    return len(want)


@pytest.mark.parametrize("jt", ["inner", "left_outer", "right_outer"])
def test_unique_build_keys(session, jt):
    """Node-scan shaped: a unique id side (many partitions) joined with a larger foreign-key side."""
    rng = np.random.default_rng(1)
    ids = rng.permutation(1 << 18).astype(np.int64) * 7 - (1 << 40)
    fk = ids[rng.integers(0, len(ids), 1 << 20)]
    fk[::97] = 5  # keys with no partner
    assert _check(session, [fk], [ids], jt) >= (1 << 20) - (1 << 20) // 97 - 1


@pytest.mark.parametrize("jt", ["inner", "left_outer", "right_outer"])
def test_dense_unique_keys_direct(session, jt):
    """Node ids (unique, dense range with holes) joined with relationship endpoints: the direct-address
    table is the strategy taken, with null and out-of-range probe keys."""
    import ctypes
    from capsmi import _lib
    rng = np.random.default_rng(5)
    base = 1 << 41
    ids = base + rng.permutation(1 << 19)[: 400_000].astype(np.int64)
    fk = base + rng.integers(-1000, (1 << 19) + 1000, 1 << 20)
    valid = rng.random(1 << 20) > 0.05
    _lib.call("capsmi_session_set_profiling", session.handle, 1)
    try:
        cnt, ms = ctypes.c_int64(), ctypes.c_double()
        _lib.call("capsmi_session_kernel_time", session.handle, b"direct_join_probe", ctypes.byref(cnt), ctypes.byref(ms))
        _check(session, [fk], [ids], jt, [valid], None)
        _lib.call("capsmi_session_kernel_time", session.handle, b"direct_join_probe", ctypes.byref(cnt), ctypes.byref(ms))
        if jt != "right_outer":  # right outer builds on the left (foreign-key) side: not unique
            assert cnt.value >= 2  # the direct and auto runs
    finally:
        _lib.call("capsmi_session_set_profiling", session.handle, 0)


@pytest.mark.parametrize("jt", ["inner", "left_outer"])
def test_skewed_duplicate_keys(session, jt):
    """Zipf keys on both sides: hub keys put more than one LDS table of build rows in a partition
    and more than one tile of probe rows."""
    rng = np.random.default_rng(2)
    rk = (rng.zipf(1.3, 60_000) % 5000).astype(np.int64)      # build: key 1 ~ 18k rows (9 LDS chunks)
    lk = rng.integers(0, 6000, 120_000).astype(np.int64)      # probe: uniform (some keys unmatched) ...
    lk[:50], lk[50:150], lk[150:3150] = 1, 2, 7               # ... plus hubs: key 7 spans two probe tiles
    rng.shuffle(lk)
    assert _check(session, [lk], [rk], jt) < 8_000_000


@pytest.mark.parametrize("jt", ["inner", "left_outer", "right_outer"])
def test_multi_key_with_nulls(session, jt):
    rng = np.random.default_rng(3)
    n1, n2 = 200_000, 150_000
    lk = [rng.integers(0, 300, n1), rng.integers(-50, 50, n1)]
    rk = [rng.integers(0, 300, n2), rng.integers(-50, 50, n2)]
    lv = [rng.random(n1) > 0.1, None]
    rv = [None, rng.random(n2) > 0.2]
    _check(session, lk, rk, jt, lv, rv)


def test_double_keys_and_empty_sides(session):
    from capsmi.expr import F64
    rng = np.random.default_rng(4)
    lk = [rng.integers(0, 1000, 50_000).astype(np.float64) / 4]
    rk = [rng.integers(0, 1000, 20_000).astype(np.float64) / 4]
    _check(session, lk, rk, "inner", types={0: F64})
    e = [np.zeros(0, np.int64)]
    for jt in ["inner", "left_outer", "right_outer"]:
        _check(session, e, [np.arange(5000, dtype=np.int64)], jt)
        _check(session, [np.arange(5000, dtype=np.int64)], e, jt)
