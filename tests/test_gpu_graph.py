"""Device parity for the fused graph kernels (the hot path) against the CPU oracle.

All comparisons are exact (integer ids and counts).  Sizes are small enough for the oracle's
binding enumeration; at full size the bench checks size-independent properties instead.
"""
import numpy as np
import pytest

from oracle import cpu

pytestmark = pytest.mark.gpu


def _rels(session, scale, ef=16, probs=(57, 19, 19), seed=42):
    from capsmi import graph
    return graph.rmat_rels(session, scale, 0, ef << scale, probs, seed)


def _bitmaps(session, scale, kind):
    from capsmi import graph
    n = 1 << scale
    if kind == "all":
        nodes = graph.rmat_nodes(session, scale, graph.NODES_ALL)
    else:
        nodes = graph.rmat_nodes(session, scale, graph.NODES_PERSON)
    bm = graph.NodeBitmap(session, 0, n).add_scan(nodes, "id")
    return bm, nodes


@pytest.mark.parametrize("scale", [6, 10, 13])
def test_rmat_matches_oracle(session, scale):
    t = _rels(session, scale)
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    assert t.size == 16 << scale
    np.testing.assert_array_equal(t.column("source").values, src)
    np.testing.assert_array_equal(t.column("target").values, dst)
    np.testing.assert_array_equal(t.column("id").values, np.arange(16 << scale))


@pytest.mark.parametrize("part_col", [0, 1])
def test_rmat_partitions_cover_graph(session, part_col):
    from capsmi import graph
    scale, nparts = 11, 4
    full = cpu.rmat_edges(scale, 0, 16 << scale)
    seen = []
    for p in range(nparts):
        t = graph.rmat_rels(session, scale, 0, 16 << scale, part_col=part_col, part=p, nparts=nparts)
        ids = t.column("id").values
        key = (t.column("source") if part_col == 0 else t.column("target")).values
        wb, we = graph.owner_words(1 << scale, p, nparts)
        assert np.all((key >> 5) >= wb) and np.all((key >> 5) < we)
        np.testing.assert_array_equal(t.column("source").values, full[0][ids])
        seen.append(ids)
    allids = np.sort(np.concatenate(seen))
    np.testing.assert_array_equal(allids, np.arange(16 << scale))


@pytest.mark.parametrize("scale,kind", [(6, "all"), (9, "person"), (12, "all"), (12, "person"), (14, "all")])
def test_two_hop_count_distinct(session, scale, kind):
    from capsmi import graph
    n = 1 << scale
    rels = _rels(session, scale)
    bm, _ = _bitmaps(session, scale, kind)
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    mask = None if kind == "all" else cpu.person_mask(n)
    rows, dist = cpu.two_hop_enumerate(n, src, dst, mask, mask, mask)
    assert graph.two_hop_count_distinct(session, [rels], bm, bm, bm) == dist
    assert graph.two_hop_count(session, [rels], bm, bm, bm) == rows
    # clustered (Cache analogue) copy gives the same answer
    cl = graph.cluster_by(rels, "target", 0, n)
    assert cl.fingerprint(["id", "source", "target"]) == rels.fingerprint(["id", "source", "target"])
    assert graph.two_hop_count_distinct(session, [cl], bm, bm, bm) == dist


def test_two_hop_self_loop_rules(session):
    """Hand-made multigraph exercising the r1 <> r2 rule through self-loops."""
    from capsmi import ColumnData, I64, graph
    # node 0: one self-loop only; node 1: two self-loops; node 2 <- 3 plus a self-loop at 2;
    # node 4 -> 5 -> 5 (self-loop at 5 reached from 4); node 6 isolated
    edges = [(0, 0), (1, 1), (1, 1), (3, 2), (2, 2), (4, 5), (5, 5), (5, 6)]
    src = np.array([e[0] for e in edges], dtype=np.int64)
    dst = np.array([e[1] for e in edges], dtype=np.int64)
    n = 8
    t = session.table([ColumnData("id", I64, np.arange(len(edges))), ColumnData("source", I64, src),
                       ColumnData("target", I64, dst)])
    nodes = session.table([ColumnData("id", I64, np.arange(n))])
    bm = graph.NodeBitmap(session, 0, n).add_scan(nodes)
    rows, dist = cpu.two_hop_enumerate(n, src, dst)
    assert cpu.two_hop_closed_form(n, src, dst) == (rows, dist)
    assert graph.two_hop_count_distinct(session, [t], bm, bm, bm) == dist
    assert graph.two_hop_count(session, [t], bm, bm, bm) == rows
    # split over two tables (a union rel scan) gives the same result
    t1 = session.table([ColumnData("id", I64, np.arange(4)), ColumnData("source", I64, src[:4]),
                        ColumnData("target", I64, dst[:4])])
    t2 = session.table([ColumnData("id", I64, np.arange(4, 8)), ColumnData("source", I64, src[4:]),
                        ColumnData("target", I64, dst[4:])])
    assert graph.two_hop_count_distinct(session, [t1, t2], bm, bm, bm) == dist


@pytest.mark.parametrize("scale,kind", [(8, "all"), (12, "person"), (15, "all"), (16, "person")])
def test_two_hop_partitioned(session, scale, kind):
    """Radix-partitioned layout (cold and cached) vs the oracle; more than one target slice at 2^20+."""
    from capsmi import graph
    n = 1 << scale
    rels = _rels(session, scale)
    bm, _ = _bitmaps(session, scale, kind)
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    mask = None if kind == "all" else cpu.person_mask(n)
    rows, dist = cpu.two_hop_closed_form(n, src, dst, mask, mask, mask)
    rp = graph.RelPartition(session, [rels], 0, n)
    assert rp.size == 16 << scale
    assert rp.count_distinct(bm, bm, bm) == dist
    assert graph.two_hop_count_distinct(session, [rels], bm, bm, bm) == dist


def test_two_hop_partitioned_multislice(session):
    """id domain of 2^21 (4 target slices, all 8 source super-slices) with a sparse edge set,
    plus ids outside the domain that the partition must drop."""
    from capsmi import ColumnData, I64, graph
    rng = np.random.default_rng(5)
    n = 1 << 21
    m = 200000
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    hubs = rng.integers(0, n, 50)
    src[: m // 4] = hubs[rng.integers(0, 50, m // 4)]
    dst[m // 4: m // 2] = hubs[rng.integers(0, 50, m // 4)]
    src[:20] = dst[:20]  # self-loops
    src[20:30] = dst[20:30] = dst[10]
    outside = np.array([n + 5, -3, 7], dtype=np.int64)
    s_all = np.concatenate([src, outside, [1, 2]])
    d_all = np.concatenate([dst, [4, 5, n + 1], outside[:2]])
    t = session.table([ColumnData("id", I64, np.arange(len(s_all))), ColumnData("source", I64, s_all),
                       ColumnData("target", I64, d_all)])
    person = (rng.random(n) < 0.8).astype(np.uint8)
    nodes = session.table([ColumnData("id", I64, np.nonzero(person)[0])])
    bm = graph.NodeBitmap(session, 0, n).add_scan(nodes)
    keep = (s_all >= 0) & (s_all < n) & (d_all >= 0) & (d_all < n)
    rows, dist = cpu.two_hop_closed_form(n, s_all[keep], d_all[keep], person, person, person)
    rp = graph.RelPartition(session, [t], 0, n)
    assert rp.size == int(keep.sum())
    assert rp.count_distinct(bm, bm, bm) == dist
    assert graph.two_hop_count_distinct(session, [t], bm, bm, bm) == dist


def test_two_hop_phased_matches_fused(session):
    """The multi-GPU phase entry points, run as one 'rank', equal the fused call."""
    import torch
    from capsmi import graph
    scale = 12
    n = 1 << scale
    rels = _rels(session, scale)
    bm, _ = _bitmaps(session, scale, "person")
    nw = (n + 31) // 32
    mid = torch.zeros(2 * nw, dtype=torch.int32, device="cuda")
    scratch = torch.zeros(nw, dtype=torch.int32, device="cuda")
    dstw = torch.zeros(nw, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    graph.two_hop_mark_mid(session, [rels], bm, bm, mid.data_ptr(), scratch.data_ptr())
    graph.two_hop_mark_dst(session, [rels], bm, bm, mid.data_ptr(), dstw.data_ptr())
    got = graph.words_popcount(session, dstw.data_ptr(), 0, nw)
    assert got == graph.two_hop_count_distinct(session, [rels], bm, bm, bm)


@pytest.mark.parametrize("scale", [8, 12])
def test_expand_filter_c2(session, scale):
    """C2: MATCH (a:Person)-[r]->(b:Person) WHERE a.age >= 18 AND a.age < 65 RETURN id(a), id(b)."""
    from capsmi import graph
    from capsmi.expr import Ands, BinOp, Col, Lit
    n = 1 << scale
    rels = _rels(session, scale)
    persons = graph.rmat_nodes(session, scale, graph.NODES_PERSON, 42)
    pred = Ands((BinOp(">=", Col("age"), Lit(18)), BinOp("<", Col("age"), Lit(65))))
    a_ok = graph.NodeBitmap(session, 0, n).add_scan(persons, "id", pred)
    b_ok = graph.NodeBitmap(session, 0, n).add_scan(persons, "id")
    out = graph.expand_filter(session, rels, a_ok, b_ok, ["source", "target"], ["a", "b"])
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    pm = cpu.person_mask(n)
    ids = np.arange(n)
    age = cpu.ages(ids)
    am = (pm.astype(bool) & (age >= 18) & (age < 65)).astype(np.uint8)
    assert out.fingerprint(["a", "b"]) == cpu.expand_filter(src, dst, am, pm)
    # device node table matches the oracle's label/age definition
    got_ids = persons.column("id").values
    np.testing.assert_array_equal(got_ids, np.nonzero(pm)[0])
    np.testing.assert_array_equal(persons.column("age").values, age[got_ids])


@pytest.mark.parametrize("layout", ["sorted", "shuffled", "dups_adjacent", "dups_far", "sparse"])
def test_bitmap_add_scan_stats(session, layout):
    """Wave-combined bitmap marking: set bits and the duplicate flag must not depend on lane layout."""
    from capsmi import ColumnData, I64, graph
    rng = np.random.default_rng(7)
    n = 5000
    if layout == "sorted":
        ids = np.arange(n)
    elif layout == "shuffled":
        ids = rng.permutation(n)
    elif layout == "dups_adjacent":
        ids = np.sort(np.concatenate([np.arange(n), [17, 4000]]))
    elif layout == "dups_far":
        ids = np.concatenate([np.arange(0, n, 2), [0, 64, 96, 127]])
        rng.shuffle(ids)
    else:
        ids = rng.choice(n, 300, replace=False) * 1
    nodes = session.table([ColumnData("id", I64, ids.astype(np.int64))])
    bm = graph.NodeBitmap(session, 0, n).add_scan(nodes)
    bits, uniq = bm.stats()
    assert bits == len(np.unique(ids))
    assert uniq == (len(np.unique(ids)) == len(ids))


@pytest.mark.parametrize("cols", [["target"], ["source", "target"], ["target", "source", "target"],
                                  ["source", "target", "source", "target"], ["id", "target"]])
@pytest.mark.parametrize("skip", [0, 1])
def test_expand_filter_projections(session, cols, skip):
    """Register-direct fast path (projections of source/target only) and the gathering path (other
    columns) against numpy, with rels outside the node domain and a misaligned (skipped) view."""
    from capsmi import ColumnData, I64, graph
    rng = np.random.default_rng(17 + skip)
    lo, hi, m = 1000, 1000 + (1 << 16), 300_000
    src = rng.integers(lo - 500, hi + 500, m).astype(np.int64)
    dst = rng.integers(lo - 500, hi + 500, m).astype(np.int64)
    rid = np.arange(m, dtype=np.int64) * 3
    rels = session.table([ColumnData("id", I64, rid), ColumnData("source", I64, src), ColumnData("target", I64, dst)])
    if skip:
        rels = rels.skip(skip)
        src, dst, rid = src[skip:], dst[skip:], rid[skip:]
    a_ids = np.nonzero(rng.random(hi - lo) < 0.4)[0] + lo
    b_ids = np.nonzero(rng.random(hi - lo) < 0.7)[0] + lo
    ta = session.table([ColumnData("id", I64, a_ids)])
    tb = session.table([ColumnData("id", I64, b_ids)])
    a_ok = graph.NodeBitmap(session, lo, hi).add_scan(ta)
    b_ok = graph.NodeBitmap(session, lo, hi).add_scan(tb)
    names = [f"c{k}" for k in range(len(cols))]
    out = graph.expand_filter(session, rels, a_ok, b_ok, cols, names)
    keep = np.isin(src, a_ids) & np.isin(dst, b_ids)
    full = {"id": rid, "source": src, "target": dst}
    want = np.stack([full[c][keep] for c in cols], axis=1)
    got = np.stack([out.column(nm).values for nm in names], axis=1)
    assert got.shape == want.shape
    order_w = np.lexsort(want.T[::-1])
    order_g = np.lexsort(got.T[::-1])
    np.testing.assert_array_equal(got[order_g], want[order_w])


@pytest.mark.parametrize("case", ["runs", "runs_overlap", "mixed", "skipped_view", "unaligned_runs"])
def test_bitmap_add_scan_bits(session, case):
    """The ascending-run fast path (256 consecutive ids per wave) and the generic path set exactly the
    scanned ids, across several scans into one bitmap; membership read back through expand_filter."""
    from capsmi import ColumnData, I64, graph
    rng = np.random.default_rng(23)
    lo, hi = 77, 77 + 20000
    if case == "runs":
        scans = [np.arange(lo + 5, lo + 9000), np.arange(lo + 12001, hi)]
    elif case == "runs_overlap":
        scans = [np.arange(lo + 3, lo + 4000), np.arange(lo + 3900, lo + 7777), np.arange(lo + 100, lo + 400)]
    elif case == "mixed":
        a = np.arange(lo + 31, lo + 10000)
        a[4000:4300] = rng.integers(lo, hi, 300)  # breaks some waves' runs
        scans = [a, rng.integers(lo, hi, 999)]
    elif case == "unaligned_runs":
        scans = [np.arange(lo + 1, lo + 300), np.arange(lo + 300, lo + 301), np.arange(lo + 301, lo + 9999)]
    else:
        scans = [np.arange(lo, lo + 7001)]
    bm = graph.NodeBitmap(session, lo, hi)
    for k, ids in enumerate(scans):
        t = session.table([ColumnData("id", I64, ids.astype(np.int64))])
        if case == "skipped_view":
            t = t.skip(3)  # misaligned 16-B loads -> generic loads
            ids = ids[3:]
        bm.add_scan(t)
    allids = np.unique(np.concatenate([s[3:] if case == "skipped_view" else s for s in scans]))
    total = sum(len(s) - (3 if case == "skipped_view" else 0) for s in scans)
    bits, uniq = bm.stats()
    assert bits == len(allids)
    assert uniq == (len(allids) == total)
    if not uniq:  # the fused expand refuses scans with repeated ids (ScanGraph.scala:72-76)
        return
    dom = np.arange(lo, hi, dtype=np.int64)
    rels = session.table([ColumnData("id", I64, dom), ColumnData("source", I64, dom),
                          ColumnData("target", I64, np.full(len(dom), lo, np.int64))])
    everyone = graph.NodeBitmap(session, lo, hi).add_scan(session.table([ColumnData("id", I64, dom)]))
    out = graph.expand_filter(session, rels, bm, everyone, ["source"], ["s"])
    np.testing.assert_array_equal(np.sort(out.column("s").values), allids)


@pytest.mark.parametrize("case", ["exact", "exact_wider_window", "dup_and_gap", "sparse"])
def test_bitmap_scan_of_exact_node_table(session, case):
    """A registered node table whose ids are exactly one window (checked at capsmi_node_table) scans
    into the bitmap as a range fill; the words and stats must equal a row-by-row scan of the same
    ids, and tables that only look exact (a duplicate plus a gap) take the row path."""
    import torch
    from capsmi import ColumnData, I64, graph
    rng = np.random.default_rng(5)
    lo = 1000
    ids = rng.permutation(np.arange(lo, lo + 70001)).astype(np.int64)
    if case == "dup_and_gap":
        ids[17] = ids[18]
    elif case == "sparse":
        ids = ids[::3].copy()
    wlo, whi = (lo - 45, lo + 70001 + 77) if case == "exact_wider_window" else (lo, lo + 70001)
    if case == "sparse":
        wlo, whi = int(ids.min()), int(ids.max()) + 1
    plain = session.table([ColumnData("id", I64, ids)])
    node = plain.as_node_table("id")
    nw = (whi - wlo + 31) // 32
    words = []
    for t in (node, plain):
        bm = graph.NodeBitmap(session, wlo, whi).add_scan(t, "id")
        w = torch.zeros(nw, dtype=torch.int32, device="cuda")
        bm.copy_words(0, nw, w.data_ptr(), to_bitmap=False)  # on the session's stream
        session.sync()
        words.append((w.cpu().numpy(), bm.stats()))
    np.testing.assert_array_equal(words[0][0], words[1][0])
    assert words[0][1] == words[1][1] == (len(np.unique(ids)), len(np.unique(ids)) == len(ids))


@pytest.mark.parametrize("case", ["sparse", "dup"])
def test_bitmap_scan_unique_table_with_predicate(session, case):
    """A registered node table without repeated ids scans with no count read back (the set-bit count of a
    filtered scan is computed when asked): words and stats equal a row-by-row scan of the unregistered
    table; a table with a repeated id keeps the counted path and reports it."""
    import torch
    from capsmi import ColumnData, I64, graph
    from capsmi.expr import BinOp, Col, Lit
    rng = np.random.default_rng(8)
    ids = rng.permutation(np.arange(5000, 95000))[::3].astype(np.int64)
    if case == "dup":
        ids[10] = ids[11]
    v = (ids % 7).astype(np.int64)
    plain = session.table([ColumnData("id", I64, ids), ColumnData("v", I64, v)])
    node = plain.as_node_table("id")
    pred = BinOp(">=", Col("v"), Lit(3))
    wlo, whi = 4000, 96000
    nw = (whi - wlo + 31) // 32
    got = []
    for t in (node, plain):
        bm = graph.NodeBitmap(session, wlo, whi).add_scan(t, "id", pred)
        w = torch.zeros(nw, dtype=torch.int32, device="cuda")
        bm.copy_words(0, nw, w.data_ptr(), to_bitmap=False)
        session.sync()
        got.append((w.cpu().numpy(), bm.stats()))
    np.testing.assert_array_equal(got[0][0], got[1][0])
    kept = ids[v >= 3]
    assert got[0][1] == got[1][1] == (len(np.unique(kept)), len(np.unique(kept)) == len(kept))
