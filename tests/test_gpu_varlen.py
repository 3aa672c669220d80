"""Fused var-length grouped count (C5 shape) vs edge-distinct path enumeration (oracle/rmat.c)."""
import numpy as np
import pytest

from oracle import cpu

pytestmark = pytest.mark.gpu


def _table(session, src, dst):
    from capsmi import ColumnData, I64
    return session.table([ColumnData("id", I64, np.arange(len(src))), ColumnData("source", I64, src),
                          ColumnData("target", I64, dst)])


def _check(session, n, src, dst, a_mask, b_mask, lo, hi, rels=None):
    from capsmi import ColumnData, I64, graph
    rels = rels or [_table(session, src, dst)]
    a_nodes = session.table([ColumnData("id", I64, np.nonzero(a_mask)[0])])
    b_nodes = session.table([ColumnData("id", I64, np.nonzero(b_mask)[0])])
    a_ok = graph.NodeBitmap(session, 0, n).add_scan(a_nodes)
    b_ok = graph.NodeBitmap(session, 0, n).add_scan(b_nodes)
    out = graph.var_length_count(session, rels, a_ok, b_ok, lo, hi, "a", "cnt")
    _, g = cpu.var_length_count(n, src, dst, lo, hi, a_mask.astype(np.uint8), b_mask.astype(np.uint8))
    want = {int(i): int(g[i]) for i in np.nonzero(g)[0]}
    ids, cnt = out.column("a").values, out.column("cnt").values
    got = dict(zip(ids.tolist(), cnt.tolist()))
    assert got == want


@pytest.mark.parametrize("seed", range(6))
def test_random_multigraphs(session, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(5, 300))
    m = int(rng.integers(0, 3000))
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    src[: m // 5] = dst[: m // 5]  # self-loops
    a_mask = rng.random(n) < 0.7
    b_mask = rng.random(n) < 0.6
    for lo, hi in [(1, 1), (1, 2), (1, 3), (2, 3), (3, 3)]:
        _check(session, n, src, dst, a_mask, b_mask, lo, hi)


@pytest.mark.parametrize("scale", [8, 11])
def test_ldbc_shaped_rmat(session, scale):
    """C5 generator at small scale: R-MAT (0.45, 0.15, 0.15, 0.25), edge factor 32, all Person."""
    from capsmi import graph
    n, m = 1 << scale, 32 << scale
    rels = graph.rmat_rels(session, scale, 0, m, graph.RMAT_LDBC, 42)
    src, dst = cpu.rmat_edges(scale, 0, m, graph.RMAT_LDBC, 42)
    ones = np.ones(n, dtype=bool)
    _check(session, n, src, dst, ones, ones, 1, 3, rels=[rels])


def test_split_rel_tables_union(session):
    rng = np.random.default_rng(9)
    n, m = 100, 2000
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    t1, t2 = _table(session, src[:700], dst[:700]), _table(session, src[700:], dst[700:])
    ones = np.ones(n, dtype=bool)
    _check(session, n, src, dst, ones, ones, 1, 3, rels=[t1, t2])


@pytest.mark.parametrize("seed", [0, 1])
def test_many_source_slices(session, seed):
    """Domain of several 8192-id source slices (LDS accumulators flushed per slice segment),
    reciprocal pairs and multi-edges (the (source, target) pair-count table), hub sources."""
    rng = np.random.default_rng(100 + seed)
    n, m = 45_000, 150_000
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    hubs = rng.integers(0, n, 8)
    src[: m // 10] = rng.choice(hubs, m // 10)
    k = m // 5  # reciprocal copies and repeats
    src[k:2 * k], dst[k:2 * k] = dst[:k].copy(), src[:k].copy()
    src[2 * k:2 * k + 500], dst[2 * k:2 * k + 500] = src[:500], dst[:500]
    src[-300:] = dst[-300:]  # self-loops
    a_mask = rng.random(n) < 0.8
    b_mask = rng.random(n) < 0.7
    for lo, hi in [(1, 3), (2, 2), (3, 3)]:
        _check(session, n, src, dst, a_mask, b_mask, lo, hi)


def test_large_domain_atomic_path(session):
    """n > 2^24 ids takes the atomic passes; the answer is the same."""
    rng = np.random.default_rng(3)
    n, m = (1 << 24) + 77, 20_000
    nodes = rng.integers(0, n, 3000)
    src = rng.choice(nodes, m).astype(np.int64)
    dst = rng.choice(nodes, m).astype(np.int64)
    ones = np.ones(n, dtype=bool)
    _check(session, n, src, dst, ones, ones, 1, 3)
