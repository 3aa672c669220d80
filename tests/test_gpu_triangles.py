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
# walks: lists over the direction-split lists (default), lists over the combined out-lists (the form when the
# split codes do not fit; config CAPSMI_TRI_SPLIT=0)
WALKS = ["lists", "lists-nosplit"]


def _vmode(knobs, session, t):
    if t != "default":
        knobs(session, CAPSMI_TRI_VMODE_T=t)


def _walk(knobs, session, walk):
    if walk == "lists-nosplit":
        knobs(session, CAPSMI_TRI_SPLIT="0")


@pytest.mark.parametrize("vmode", VMODE)
@pytest.mark.parametrize("seed", range(8))
def test_random_multigraphs(session, knobs, seed, vmode):
    _vmode(knobs, session, vmode)
    rng = np.random.default_rng(seed)
    n = int(rng.integers(3, 60))
    m = int(rng.integers(0, 600))
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    src[: m // 6] = dst[: m // 6]
    assert _count(session, n, src, dst) == cpu.triangle_enumerate(n, src, dst)


@pytest.mark.parametrize("vmode", VMODE)
def test_node_filter_and_parts(session, knobs, vmode):
    _vmode(knobs, session, vmode)
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
def test_rmat(session, knobs, scale, walk, vmode):
    _vmode(knobs, session, vmode)
    _walk(knobs, session, walk)
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    assert _count(session, 1 << scale, src, dst) == cpu.triangle_enumerate(1 << scale, src, dst)


@pytest.mark.parametrize("vmode", VMODE)
@pytest.mark.parametrize("walk", WALKS)
def test_dense_big_vertices(session, knobs, walk, vmode):
    """Out-degrees above 64 (one workgroup per vertex) on a dense random multigraph; every wedge walk
    (wave-per-list over split or combined lists)."""
    _vmode(knobs, session, vmode)
    _walk(knobs, session, walk)
    rng = np.random.default_rng(11)
    n, m = 300, 40000
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    assert _count(session, n, src, dst) == cpu.triangle_enumerate(n, src, dst)


@pytest.mark.parametrize("vmode", VMODE)
@pytest.mark.parametrize("walk", ["lists", "lists-nosplit"])
@pytest.mark.parametrize("mult", [False, True])
def test_complete_digraph_chunks(session, knobs, mult, walk, vmode):
    _vmode(knobs, session, vmode)
    _walk(knobs, session, walk)
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
def test_exception_multiplicities(session, knobs, vmode):
    """Multiplicities from 1 to 40 in both directions: the 4-bit codes of the oriented targets saturate
    (>= 15) for many edges, whose exact payloads are placed after the key-only sort (k_exc_place) and
    read on hits from either side of a wedge."""
    _vmode(knobs, session, vmode)
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
def test_split_word_cap(session, knobs, walk, vmode):
    """Ids above 2^16 (24 id bits): a split-list word holds 8 multiplicity bits, so multiplicities of
    255 and more are read exactly from the combined list."""
    _vmode(knobs, session, vmode)
    _walk(knobs, session, walk)
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


@pytest.mark.parametrize("vmode", VMODE)
def test_run_passes_across_tiles(session, knobs, vmode):
    """The direct build's fused run passes (k_or_count / k_or_write / k_or_long) over ~60 sort tiles of 4096
    keys: runs of one pair's relationships from 1 to 90 keys in either or both directions (long runs past
    kShortRun, runs crossing tile ends), self-loops (the pair terms), filtered nodes (dropped keys sorted
    last), and the CSR offsets of vertices without out-edges filled from the next one."""
    _vmode(knobs, session, vmode)
    rng = np.random.default_rng(29)
    n = 5000
    a = rng.integers(0, n, 24000)
    b = rng.integers(0, n, 24000)
    keep = a != b
    a, b = a[keep], b[keep]
    kind = rng.random(len(a))
    f = np.where(kind < 0.6, 1, np.where(kind < 0.8, rng.integers(2, 60, len(a)), rng.integers(1, 45, len(a))))
    r = np.where(kind < 0.8, 0, rng.integers(1, 45, len(a)))
    src = np.concatenate([np.repeat(a, f), np.repeat(b, r)]).astype(np.int64)
    dst = np.concatenate([np.repeat(b, f), np.repeat(a, r)]).astype(np.int64)
    loops = rng.choice(n, n // 10, replace=False)
    ls = np.repeat(loops, rng.integers(1, 6, len(loops))).astype(np.int64)
    src = np.concatenate([src, ls])
    dst = np.concatenate([dst, ls])
    perm = rng.permutation(len(src))
    src, dst = src[perm], dst[perm]
    mask = rng.random(n) < 0.8
    keep = mask[src] & mask[dst]
    want = cpu.triangle_closed_form(n, src[keep], dst[keep])
    assert want > 0
    assert _count(session, n, src, dst, mask) == want
    assert _count(session, n, src, dst, mask, nparts=3) == want


def _mix32(x):
    """k_tri.hip mix32 (the degree sample's hashed offset), vectorised over uint64."""
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(33)
    x = x * np.uint64(0xFF51AFD7ED558CCD)
    x ^= x >> np.uint64(33)
    return (x & np.uint64(0xFFFFFFFF)).astype(np.uint64)


@pytest.mark.parametrize("vmode", VMODE)
@pytest.mark.parametrize("graph_kind", ["rmat12", "random"])
def test_sampled_degree_order(session, knobs, graph_kind, vmode):
    """The direct build's degree order estimated from 1 in 32 relationships (config CAPSMI_TRI_DEG_SAMPLE=32,
    the C4 default above 2^22 relationships) -- any total order gives the same count."""
    _vmode(knobs, session, vmode)
    knobs(session, CAPSMI_TRI_DEG_SAMPLE="32")
    if graph_kind == "rmat12":
        n = 1 << 12
        src, dst = cpu.rmat_edges(12, 0, 16 << 12)
    else:
        rng = np.random.default_rng(31)
        n, m = 3000, 200_000
        src = rng.integers(0, n, m).astype(np.int64)
        dst = (src + rng.integers(-40, 41, m)) % n  # local neighbourhoods: many triangles
        src[:2000] = dst[:2000]  # self-loops
    assert _count(session, n, src, dst) == cpu.triangle_closed_form(n, src, dst)


def test_sampled_order_misranks_a_hub(session, knobs):
    """A hub whose relationships all sit at positions the 1-in-32 degree sample skips: it ranks below its
    70,000 neighbours (each of which has a sampled relationship), so every one of its edges is oriented out of
    it -- an out-degree of 70,000 >= 2^16 breaks the sqrt(2m) bound of an exact degree order, the build
    checks it (k_max_od) and takes the unpacked in-keys and the combined walks.  The count must not change
    (ADVICE r05).  Padding relationships whose nodes are filtered out fill the rest of the blocks."""
    knobs(session, CAPSMI_TRI_DEG_SAMPLE="32")
    k = 70_000
    hub, w = 0, np.arange(1, k + 1, dtype=np.int64)
    pad = k + 1  # a node outside the scanned node table
    n = k + 2
    blocks = k
    m = 32 * blocks
    sampled = np.arange(blocks, dtype=np.uint64) * np.uint64(32) + (_mix32(np.arange(blocks, dtype=np.uint64)) & np.uint64(31))
    sampled = sampled.astype(np.int64)
    free = np.ones(m, bool)
    free[sampled] = False
    slots = np.nonzero(free)[0]
    src = np.full(m, pad, np.int64)
    dst = np.full(m, pad, np.int64)
    # sampled slots: w_i -> w_{i+3} (every neighbour gets a sampled relationship)
    src[sampled], dst[sampled] = w, w[(np.arange(k) + 3) % k]
    # unsampled slots: hub -> w_i, w_i -> w_{i+1}, and w_j -> hub for every 13th j (directed triangles through the hub)
    back = w[::13]
    extra_s = np.concatenate([np.full(k, hub), w, back])
    extra_d = np.concatenate([w, w[(np.arange(k) + 1) % k], np.full(len(back), hub)])
    assert len(extra_s) <= len(slots)
    src[slots[:len(extra_s)]], dst[slots[:len(extra_s)]] = extra_s, extra_d
    assert not np.isin(np.nonzero((src == hub) | (dst == hub))[0], sampled).any()
    mask = np.ones(n, bool)
    mask[pad] = False
    keep = mask[src] & mask[dst]
    want = cpu.triangle_closed_form(n, src[keep], dst[keep])
    assert want > 0
    assert _count(session, n, src, dst, mask) == want
