"""2-D partitioned layout (k_part.hip) at sizes with several target/source slices.

The small-scale parity tests (test_gpu_graph.py) fit one 2^19-id slice, so the multi-cell walk,
the LDS pull of source slices (>= 8192 rels of one cell per workgroup) and coarse source slices
(domains > 2^26 ids) are exercised here.  The reference answer is a numpy restatement of the
X1/X2 frontier semantics (oracle/rmat.c orc_two_hop_closed), exact integer comparison.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _np_count_distinct(n, src, dst, a_ok, b_ok, c_ok):
    loop = src == dst
    sel = a_ok[src] & b_ok[dst]
    M = np.zeros(n, bool)
    M[dst[sel & ~loop]] = True
    selfc = np.bincount(dst[sel & loop], minlength=n)
    X1, X2 = M | (selfc >= 1), M | (selfc >= 2)
    hit = c_ok[dst] & np.where(loop, X2[src], X1[src])
    C = np.zeros(n, bool)
    C[dst[hit]] = True
    return int(C.sum())


def _mix64(x):
    z = x + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _check_layout(rp, lo, hi, src, dst):
    """Every relationship with both endpoints in [lo, hi) is stored exactly once, in its own cell:
    per-cell counts and wrapping sums of a 64-bit mix of the packed pair match a numpy grouping."""
    counts, sums, bad, (ns, sbits, tbits) = rp.digest()
    keep = (src >= lo) & (src < hi) & (dst >= lo) & (dst < hi)
    x, y = (src[keep] - lo).astype(np.uint64), (dst[keep] - lo).astype(np.uint64)
    cell = (y >> np.uint64(tbits)).astype(np.int64) * ns + (x >> np.uint64(sbits)).astype(np.int64)
    want_n = np.bincount(cell, minlength=len(counts))
    want_s = np.zeros(len(counts), np.uint64)
    with np.errstate(over="ignore"):
        np.add.at(want_s, cell, _mix64((x << np.uint64(32)) | y))
    assert bad == 0
    np.testing.assert_array_equal(counts, want_n)
    np.testing.assert_array_equal(sums, want_s)


def _bitmap(session, n, ids):
    from capsmi import ColumnData, I64, graph
    t = session.table([ColumnData("id", I64, np.asarray(ids, dtype=np.int64))])
    return graph.NodeBitmap(session, 0, n).add_scan(t)


@pytest.mark.parametrize("person_only", [False, True])
def test_rmat_multi_slice(session, person_only):
    from capsmi import graph
    scale = 21  # 4 x 4 cells of 2^19 ids; 16M rels -> every workgroup pulls source slices
    n = 1 << scale
    rels = graph.rmat_rels(session, scale, 0, 8 << scale)
    src = rels.column("source").values
    dst = rels.column("target").values
    rng = np.random.default_rng(3)
    ok = rng.random(n) < 0.8 if person_only else np.ones(n, bool)
    okc = rng.random(n) < 0.6 if person_only else ok
    a, c = _bitmap(session, n, np.nonzero(ok)[0]), _bitmap(session, n, np.nonzero(okc)[0])
    want = _np_count_distinct(n, src, dst, ok, ok, okc)
    rp = graph.RelPartition(session, [rels], 0, n)
    assert rp.size == len(src)
    assert rp.count_distinct(a, a, c) == want
    # one call builds its own layout
    assert graph.two_hop_count_distinct(session, [rels], a, a, c) == want
    rp.release()


def test_coarse_source_slices(session):
    """2^27-id domain: 256 target slices x 64 source slices of 2^21 ids (no LDS pull)."""
    from capsmi import ColumnData, I64, graph
    n = 1 << 27
    rng = np.random.default_rng(5)
    m = 1 << 20
    hubs = rng.integers(0, n, 4096)
    src = np.concatenate([rng.integers(0, n, m // 2), rng.choice(hubs, m // 2)]).astype(np.int64)
    dst = np.concatenate([rng.choice(hubs, m // 2), rng.integers(0, n, m // 2)]).astype(np.int64)
    src[:1000] = dst[:1000]  # self-loops
    src[1000:1500] = dst[:500]
    dst[1000:1500] = dst[:500]  # repeated self-loops
    rels = session.table([ColumnData("id", I64, np.arange(m)), ColumnData("source", I64, src),
                          ColumnData("target", I64, dst)])
    touched = np.unique(np.concatenate([src, dst]))
    keep = touched[rng.random(len(touched)) < 0.9]
    ok = np.zeros(n, bool)
    ok[keep] = True
    bm = _bitmap(session, n, keep)
    want = _np_count_distinct(n, src, dst, ok, ok, ok)
    assert graph.two_hop_count_distinct(session, [rels], bm, bm, bm) == want


def test_rels_outside_domain_are_dropped(session):
    from capsmi import ColumnData, I64, graph
    lo, hi = 1 << 20, 3 << 20
    rng = np.random.default_rng(9)
    m = 1 << 20
    src = rng.integers(0, 4 << 20, m).astype(np.int64)
    dst = rng.integers(0, 4 << 20, m).astype(np.int64)
    rels = session.table([ColumnData("id", I64, np.arange(m)), ColumnData("source", I64, src),
                          ColumnData("target", I64, dst)])
    ids = np.arange(lo, hi)
    t = session.table([ColumnData("id", I64, ids)])
    bm = graph.NodeBitmap(session, lo, hi).add_scan(t)
    inside = (src >= lo) & (src < hi) & (dst >= lo) & (dst < hi)
    rp = graph.RelPartition(session, [rels], lo, hi)
    assert rp.size == int(inside.sum())
    n = hi - lo
    s, d = src[inside] - lo, dst[inside] - lo
    allok = np.ones(n, bool)
    assert rp.count_distinct(bm, bm, bm) == _np_count_distinct(n, s, d, allok, allok, allok)
    rp.release()


def test_several_rel_tables(session):
    """Relationship types as separate tables (a union of rel scans): same answer as one table."""
    from capsmi import graph
    scale = 20
    n, m = 1 << scale, 8 << scale
    cut = [0, m // 3, m // 3 + 12345, m]
    parts = [graph.rmat_rels(session, scale, cut[k], cut[k + 1]) for k in range(3)]
    whole = graph.rmat_rels(session, scale, 0, m)
    src, dst = whole.column("source").values, whole.column("target").values
    ok = np.ones(n, bool)
    bm = _bitmap(session, n, np.arange(n))
    want = _np_count_distinct(n, src, dst, ok, ok, ok)
    rp = graph.RelPartition(session, parts, 0, n)
    assert rp.size == m
    assert rp.count_distinct(bm, bm, bm) == want
    rp.release()


def _mid_words(session, rp_factory, n, a, b):
    import torch
    nw = (n + 31) // 32
    mid = torch.zeros(2 * nw, dtype=torch.int32, device="cuda")
    scratch = torch.zeros(nw, dtype=torch.int32, device="cuda")
    rp = rp_factory(mid.data_ptr(), scratch.data_ptr())
    session.sync()
    return rp, mid.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("fused", [False, True])
def test_layout_digest_full_domain(session, fused):
    """2^26 ids = 128 x 128 cells (the whole-line pass-1 kernel and pass 2 with many segments per
    slice), uniform ids plus hub targets and sources: every pair stored once, in its own cell; with
    `fused` the layout comes from the build that runs hop 1 in pass 2."""
    import torch
    from capsmi import ColumnData, I64, graph
    n = 1 << 26
    rng = np.random.default_rng(31)
    m = 6 << 20
    hubs = rng.integers(0, n, 64)
    src = np.where(rng.random(m) < 0.2, rng.choice(hubs, m), rng.integers(0, n, m)).astype(np.int64)
    dst = np.where(rng.random(m) < 0.3, rng.choice(hubs, m), rng.integers(0, n, m)).astype(np.int64)
    src[::1001] = dst[::1001]  # self-loops
    rels = session.table([ColumnData("id", I64, np.arange(m)), ColumnData("source", I64, src),
                          ColumnData("target", I64, dst)])
    if fused:
        a = _bitmap(session, n, np.arange(n))
        nw = n // 32
        mid = torch.zeros(2 * nw, dtype=torch.int32, device="cuda")
        scratch = torch.zeros(nw, dtype=torch.int32, device="cuda")
        rp = graph.RelPartition.build_mark_mid(session, [rels], a, a, mid.data_ptr(), scratch.data_ptr())
        session.sync()
    else:
        rp = graph.RelPartition(session, [rels], 0, n)
    assert rp.size == m
    _check_layout(rp, 0, n, src, dst)
    rp.release()


@pytest.mark.parametrize("a_full", [True, False])
def test_build_mark_mid_matches_phased(session, a_full):
    """Hop 1 run inside the build's second pass (a_ok full) or after it (a_ok partial) gives the same
    X1 / X2 frontier words as the phased build + mark_mid, and the same final count."""
    from capsmi import graph
    scale = 21
    n = 1 << scale
    rels = graph.rmat_rels(session, scale, 0, 8 << scale)
    rng = np.random.default_rng(11)
    a = _bitmap(session, n, np.arange(n) if a_full else np.nonzero(rng.random(n) < 0.7)[0])
    b = _bitmap(session, n, np.nonzero(rng.random(n) < 0.8)[0])
    rp1 = graph.RelPartition(session, [rels], 0, n)
    _, want = _mid_words(session, lambda m, s: rp1.mark_mid(a, b, m, s), n, a, b)
    rp2, got = _mid_words(session, lambda m, s: graph.RelPartition.build_mark_mid(session, [rels], a, b, m, s),
                          n, a, b)
    assert np.array_equal(got, want)
    assert rp2.size == rp1.size == 8 << scale
    assert rp2.count_distinct(a, b, b) == rp1.count_distinct(a, b, b)
    rp1.release()
    rp2.release()


def test_skewed_slices_and_chunk_splits(session):
    """One target slice takes most relationships (its chunks split inside tiles), the others get a
    trickle (open chunks retired nearly empty); several input tables = several pass-1 launches."""
    from capsmi import ColumnData, I64, graph
    n = 1 << 23  # 16 target slices
    rng = np.random.default_rng(21)
    m = 3 << 20
    hot = rng.integers(0, 1 << 19, m)
    cold = rng.integers(0, n, m)
    dst = np.where(rng.random(m) < 0.9, hot, cold).astype(np.int64)
    src = rng.integers(0, n, m).astype(np.int64)
    src[::97] = dst[::97]  # self-loops, some repeated
    tabs = []
    cuts = [0, 5, 70000, m // 2, m]
    for k in range(4):
        sl = slice(cuts[k], cuts[k + 1])
        tabs.append(session.table([ColumnData("id", I64, np.arange(cuts[k], cuts[k + 1])),
                                   ColumnData("source", I64, src[sl]), ColumnData("target", I64, dst[sl])]))
    ok = np.ones(n, bool)
    okc = rng.random(n) < 0.5
    a, c = _bitmap(session, n, np.arange(n)), _bitmap(session, n, np.nonzero(okc)[0])
    want = _np_count_distinct(n, src, dst, ok, ok, okc)
    assert graph.two_hop_count_distinct(session, tabs, a, a, c) == want
    rp = graph.RelPartition(session, tabs, 0, n)
    assert rp.size == m
    _check_layout(rp, 0, n, src, dst)
    assert rp.count_distinct(a, a, c) == want
    rp.release()


def test_largest_domain(session):
    """2^30-id domain: 2048 target slices (the pass-1 LDS limit), coarse source slices."""
    from capsmi import ColumnData, I64, graph
    n = 1 << 30
    rng = np.random.default_rng(4)
    m = 1 << 18
    src = rng.integers(0, n, m).astype(np.int64)
    dst = np.where(rng.random(m) < 0.5, rng.integers(0, 1 << 12, m), rng.integers(0, n, m)).astype(np.int64)
    rels = session.table([ColumnData("id", I64, np.arange(m)), ColumnData("source", I64, src),
                          ColumnData("target", I64, dst)])
    ids = np.unique(np.concatenate([src, dst]))
    bm = _bitmap(session, n, ids)
    k = len(ids)  # the oracle on compacted ids (every endpoint is scanned)
    ok = np.ones(k, bool)
    want = _np_count_distinct(k, np.searchsorted(ids, src), np.searchsorted(ids, dst), ok, ok, ok)
    rp = graph.RelPartition(session, [rels], 0, n)
    assert rp.size == m
    _check_layout(rp, 0, n, src, dst)
    assert rp.count_distinct(bm, bm, bm) == want
    rp.release()


@pytest.mark.parametrize("nparts", [1, 2, 4])
def test_owner_partitioned_two_hop_with_torch_in_between(nparts):
    """The multi-GPU C3 step emulated on one device: per rank the owner(target) share, build + hop
    1, the owned frontier slices stitched by torch copies (the all-gather), hop 2 per rank, owned
    popcounts summed.  The session runs on torch's default stream (the null stream), so the torch
    copies between library calls are ordered after the library's kernels."""
    import torch
    from capsmi import Session, graph
    scale = 16
    n, m = 1 << scale, 16 << scale
    nw = (n + 31) // 32
    s = Session(0)
    s.set_stream(torch.cuda.current_stream().cuda_stream)
    persons = graph.rmat_nodes(s, scale, graph.NODES_ALL)
    full = graph.rmat_rels(s, scale, 0, m, graph.RMAT_GRAPH500, 7)
    p = graph.NodeBitmap(s, 0, n).add_scan(persons, "id")
    ref = graph.two_hop_count_distinct(s, [full], p, p, p)
    rels = [graph.rmat_rels(s, scale, 0, m, graph.RMAT_GRAPH500, 7, part_col=graph.PART_TARGET, part=r,
                            nparts=nparts) for r in range(nparts)]
    mids = [torch.zeros(2 * nw, dtype=torch.int32, device="cuda") for _ in range(nparts)]
    scratch = torch.zeros(nw, dtype=torch.int32, device="cuda")
    rps = [graph.RelPartition.build_mark_mid(s, [rels[r]], p, p, mids[r].data_ptr(), scratch.data_ptr())
           for r in range(nparts)]
    mid = torch.zeros(2 * nw, dtype=torch.int32, device="cuda")
    for r in range(nparts):
        wb, we = graph.owner_words(n, r, nparts)
        mid[wb:we] = mids[r][wb:we]
        mid[nw + wb:nw + we] = mids[r][nw + wb:nw + we]
    total = 0
    for r in range(nparts):
        wb, we = graph.owner_words(n, r, nparts)
        dst = torch.zeros(nw, dtype=torch.int32, device="cuda")
        rps[r].mark_dst(p, p, mid.data_ptr(), dst.data_ptr())
        total += graph.words_popcount(s, dst.data_ptr(), wb, we)
        rps[r].release()
    assert total == ref


@pytest.mark.parametrize("nparts", [2, 4])
def test_sharded_node_scan_assume_and_device_popcount(nparts):
    """The multi-GPU node scan and answer without host popcounts: every rank scans its owned
    :Person rows, the owned word slices are stitched (the all-gather), the summed owned set-bit
    counts are stated with capsmi_bitmap_assume, and each rank's owned hop-2 popcount goes into a
    device int64 (capsmi_words_popcount_device) that is summed on the device."""
    import torch
    from capsmi import Session, graph
    from capsmi.expr import Ands, BinOp, Col, Lit
    scale = 15
    n, m = 1 << scale, 16 << scale
    nw = (n + 31) // 32
    s = Session(0)
    s.set_stream(torch.cuda.current_stream().cuda_stream)
    persons = graph.rmat_nodes(s, scale, graph.NODES_PERSON, 3)
    full = graph.rmat_rels(s, scale, 0, m, graph.RMAT_GRAPH500, 5)
    p_ref = graph.NodeBitmap(s, 0, n).add_scan(persons, "id")
    ref = graph.two_hop_count_distinct(s, [full], p_ref, p_ref, p_ref)
    bits_ref, uniq_ref = p_ref.stats()
    words = torch.zeros(nw, dtype=torch.int32, device="cuda")
    total_bits = 0
    for r in range(nparts):
        wb, we = graph.owner_words(n, r, nparts)
        own = persons.filter(Ands((BinOp(">=", Col("id"), Lit(32 * wb)), BinOp("<", Col("id"), Lit(min(32 * we, n))))))
        q = graph.NodeBitmap(s, 0, n).add_scan(own, "id")
        total_bits += q.stats()[0]
        q.copy_words(wb, we, words[wb:we].data_ptr(), to_bitmap=False)
        q.release()
    p = graph.NodeBitmap(s, 0, n)
    p.copy_words(0, nw, words.data_ptr(), to_bitmap=True)
    p.assume(total_bits, True)
    assert p.stats() == (bits_ref, uniq_ref)
    rels = [graph.rmat_rels(s, scale, 0, m, graph.RMAT_GRAPH500, 5, part_col=graph.PART_TARGET, part=r, nparts=nparts)
            for r in range(nparts)]
    mids = [torch.zeros(2 * nw, dtype=torch.int32, device="cuda") for _ in range(nparts)]
    scratch = torch.zeros(nw, dtype=torch.int32, device="cuda")
    rps = [graph.RelPartition.build_mark_mid(s, [rels[r]], p, p, mids[r].data_ptr(), scratch.data_ptr())
           for r in range(nparts)]
    mid = torch.zeros(2 * nw, dtype=torch.int32, device="cuda")
    for r in range(nparts):
        wb, we = graph.owner_words(n, r, nparts)
        mid[wb:we] = mids[r][wb:we]
        mid[nw + wb:nw + we] = mids[r][nw + wb:nw + we]
    counts = torch.zeros(nparts, dtype=torch.int64, device="cuda")
    for r in range(nparts):
        wb, we = graph.owner_words(n, r, nparts)
        dst = torch.zeros(nw, dtype=torch.int32, device="cuda")
        rps[r].mark_dst(p, p, mid.data_ptr(), dst.data_ptr())
        graph.words_popcount_device(s, dst.data_ptr(), wb, we, counts[r:r + 1].data_ptr())
        rps[r].release()
    assert int(counts.sum().item()) == ref
    with pytest.raises(Exception):
        p.assume(n + 1, True)  # a count outside the domain is refused


@pytest.mark.parametrize("cached", [False, True])
def test_layout_build_is_deterministic(session, cached, knobs):
    """Run twice, the same layout: pass 2 writes at precomputed offsets (csrc/k_part.hip), so two builds of
    one relationship table give equal cell counts and per-cell digests, and the same 2-hop answer, unpacked
    (one query's layout) and packed (cached).  (Round 6 removed the 6-byte pass-1 pool this test used to
    compare against)"""
    from capsmi import graph
    scale = 21
    n = 1 << scale
    rels = graph.rmat_rels(session, scale, 0, 8 << scale)
    src, dst = rels.column("source").values, rels.column("target").values
    rng = np.random.default_rng(9)
    ok, okc = rng.random(n) < 0.8, rng.random(n) < 0.6
    a, c = _bitmap(session, n, np.nonzero(ok)[0]), _bitmap(session, n, np.nonzero(okc)[0])
    want = _np_count_distinct(n, src, dst, ok, ok, okc)
    knobs(session, CAPSMI_PAIRS="packed" if cached else "uint2")
    digests = []
    for run in range(2):
        rp = graph.RelPartition(session, [rels], 0, n)
        counts, sums, bad, geom = rp.digest()
        assert bad == 0, run
        digests.append((np.asarray(counts).tolist(), np.asarray(sums).tolist(), geom))
        assert rp.count_distinct(a, a, c) == want, run
        rp.release()
        assert graph.two_hop_count_distinct(session, [rels], a, a, c) == want, run
    assert digests[0] == digests[1]
