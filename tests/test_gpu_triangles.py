"""Fused cyclic triangle count (C4 shape) vs binding enumeration (oracle/rmat.c)."""
import numpy as np
import pytest

from oracle import cpu

pytestmark = pytest.mark.gpu


def _count(session, n, src, dst, mask=None, nparts=1):
    from capsmi import ColumnData, I64, graph
    rels = session.table([ColumnData("id", I64, np.arange(len(src))), ColumnData("source", I64, src),
                          ColumnData("target", I64, dst)])
    ids = np.arange(n) if mask is None else np.nonzero(mask)[0]
    nodes = session.table([ColumnData("id", I64, ids)])
    ok = graph.NodeBitmap(session, 0, n).add_scan(nodes)
    if nparts == 1:
        return graph.triangle_count(session, [rels], ok)
    g = graph.TriGraph(session, [rels], ok)
    return sum(g.count(p, nparts) for p in range(nparts))


VMODE = ["0", "2", "default"]  # CAPSMI_TRI_VMODE_T: every edge from u / almost every edge from v / 256
# walks: lists over the direction-split lists (default), lists over the combined out-lists, the flat
# prefix-sum walk
WALKS = ["lists", "lists-nosplit", "flat"]


def _vmode(monkeypatch, t):
    if t != "default":
        monkeypatch.setenv("CAPSMI_TRI_VMODE_T", t)


def _walk(monkeypatch, walk):
    if walk == "flat":
        monkeypatch.setenv("CAPSMI_TRI_WALK", "flat")
    elif walk == "lists-nosplit":
        monkeypatch.setenv("CAPSMI_TRI_SPLIT", "0")


@pytest.mark.parametrize("vmode", VMODE)
@pytest.mark.parametrize("seed", range(8))
def test_random_multigraphs(session, monkeypatch, seed, vmode):
    _vmode(monkeypatch, vmode)
    rng = np.random.default_rng(seed)
    n = int(rng.integers(3, 60))
    m = int(rng.integers(0, 600))
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    src[: m // 6] = dst[: m // 6]
    assert _count(session, n, src, dst) == cpu.triangle_enumerate(n, src, dst)


@pytest.mark.parametrize("vmode", VMODE)
def test_node_filter_and_parts(session, monkeypatch, vmode):
    _vmode(monkeypatch, vmode)
    rng = np.random.default_rng(42)
    n, m = 200, 4000
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    mask = rng.random(n) < 0.7
    keep = mask[src] & mask[dst]
    want = cpu.triangle_enumerate(n, src[keep], dst[keep])
    assert _count(session, n, src, dst, mask) == want
    assert _count(session, n, src, dst, mask, nparts=4) == want


@pytest.mark.parametrize("vmode", VMODE)
@pytest.mark.parametrize("walk", WALKS)
@pytest.mark.parametrize("scale", [9, 12])
def test_rmat(session, monkeypatch, scale, walk, vmode):
    _vmode(monkeypatch, vmode)
    _walk(monkeypatch, walk)
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    assert _count(session, 1 << scale, src, dst) == cpu.triangle_enumerate(1 << scale, src, dst)


@pytest.mark.parametrize("vmode", VMODE)
@pytest.mark.parametrize("walk", WALKS)
def test_dense_big_vertices(session, monkeypatch, walk, vmode):
    """Out-degrees above 64 (one workgroup per vertex) on a dense random multigraph; every wedge walk
    (wave-per-list over split or combined lists, CAPSMI_TRI_WALK=flat prefix-sum walk)."""
    _vmode(monkeypatch, vmode)
    _walk(monkeypatch, walk)
    rng = np.random.default_rng(11)
    n, m = 300, 40000
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    assert _count(session, n, src, dst) == cpu.triangle_enumerate(n, src, dst)


@pytest.mark.parametrize("vmode", VMODE)
@pytest.mark.parametrize("walk", ["lists", "lists-nosplit"])
@pytest.mark.parametrize("mult", [False, True])
def test_complete_digraph_chunks(session, monkeypatch, mult, walk, vmode):
    _vmode(monkeypatch, vmode)
    _walk(monkeypatch, walk)
    """Complete digraph on 2200 nodes: out-degrees up to 2199 exceed one LDS chunk (2048).
    Loop-free, so count(*) = trace(M^3) for the multiplicity matrix M (exact in float64 here)."""
    n = 2200
    rng = np.random.default_rng(5)
    M = np.ones((n, n), dtype=np.int64)
    if mult:
        M = rng.integers(1, 4, (n, n))
    np.fill_diagonal(M, 0)
    a, b = np.nonzero(M)
    reps = M[a, b]
    src = np.repeat(a, reps).astype(np.int64)
    dst = np.repeat(b, reps).astype(np.int64)
    Mf = M.astype(np.float64)
    want = int(round(np.trace(Mf @ Mf @ Mf)))
    assert _count(session, n, src, dst) == want
    assert _count(session, n, src, dst, nparts=3) == want


def test_wide_id_range(session):
    """Ids spread over [0, 2^25 + 3): the undirected sort keys carry the direction bit below the
    target (bits > 24) instead of in the unsorted bit 31.  The count is label-invariant, so the
    oracle enumerates the compacted ids."""
    from capsmi import ColumnData, I64, graph
    rng = np.random.default_rng(21)
    n = (1 << 25) + 3
    ids = np.unique(rng.integers(0, n, 700)).astype(np.int64)
    ids[-1] = n - 1
    k = len(ids)
    a = rng.integers(0, k, 9000)
    b = rng.integers(0, k, 9000)
    b[:300] = a[:300]  # self-loops
    src, dst = ids[a], ids[b]
    rels = session.table([ColumnData("id", I64, np.arange(len(src))), ColumnData("source", I64, src),
                          ColumnData("target", I64, dst)])
    nodes = session.table([ColumnData("id", I64, ids)])
    ok = graph.NodeBitmap(session, 0, n).add_scan(nodes)
    assert graph.triangle_count(session, [rels], ok) == cpu.triangle_enumerate(k, a.astype(np.int64), b.astype(np.int64))


@pytest.mark.parametrize("vmode", VMODE)
def test_exception_multiplicities(session, monkeypatch, vmode):
    """Multiplicities from 1 to 40 in both directions: the 4-bit codes of the oriented targets saturate
    (>= 15) for many edges, whose exact payloads are placed after the key-only sort (k_exc_place) and
    read on hits from either side of a wedge."""
    _vmode(monkeypatch, vmode)
    rng = np.random.default_rng(17)
    n = 90
    a, b = np.nonzero(rng.random((n, n)) < 0.25)
    keep = a != b
    a, b = a[keep], b[keep]
    reps = rng.integers(1, 41, len(a)) * (rng.random(len(a)) < 0.3) + 1
    src = np.repeat(a, reps).astype(np.int64)
    dst = np.repeat(b, reps).astype(np.int64)
    assert _count(session, n, src, dst) == cpu.triangle_closed_form(n, src, dst)


@pytest.mark.parametrize("vmode", VMODE)
@pytest.mark.parametrize("walk", ["lists", "lists-nosplit"])
def test_split_word_cap(session, monkeypatch, walk, vmode):
    """Ids above 2^16 (24 id bits): a split-list word holds 8 multiplicity bits, so multiplicities of
    255 and more are read exactly from the combined list."""
    _vmode(monkeypatch, vmode)
    _walk(monkeypatch, walk)
    rng = np.random.default_rng(23)
    n = 70000
    k = 120
    a, b = np.nonzero(rng.random((k, k)) < 0.3)
    keep = a != b
    a, b = a[keep], b[keep]
    reps = np.where(rng.random(len(a)) < 0.1, rng.integers(250, 320, len(a)), rng.integers(1, 3, len(a)))
    src = np.repeat(a, reps).astype(np.int64)
    dst = np.repeat(b, reps).astype(np.int64)
    far = rng.integers(k, n, 2000).astype(np.int64)  # ids up to 70000, a few edges into the dense part
    src = np.concatenate([src, far, [n - 1]])
    dst = np.concatenate([dst, rng.integers(0, k, 2000).astype(np.int64), [0]])
    assert _count(session, n, src, dst) == cpu.triangle_closed_form(n, src, dst)
