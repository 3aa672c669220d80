"""Fused var-length grouped count (C5 shape) vs edge-distinct path enumeration (oracle/rmat.c)."""
import numpy as np
import pytest

from oracle import cpu




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


@pytest.mark.gpu
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


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [8, 11])
def test_ldbc_shaped_rmat(session, scale):
    """C5 generator at small scale: R-MAT (0.45, 0.15, 0.15, 0.25), edge factor 32, all Person."""
    from capsmi import graph
    n, m = 1 << scale, 32 << scale
    rels = graph.rmat_rels(session, scale, 0, m, graph.RMAT_LDBC, 42)
    src, dst = cpu.rmat_edges(scale, 0, m, graph.RMAT_LDBC, 42)
    ones = np.ones(n, dtype=bool)
    _check(session, n, src, dst, ones, ones, 1, 3, rels=[rels])


@pytest.mark.gpu
def test_split_rel_tables_union(session):
    rng = np.random.default_rng(9)
    n, m = 100, 2000
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    t1, t2 = _table(session, src[:700], dst[:700]), _table(session, src[700:], dst[700:])
    ones = np.ones(n, dtype=bool)
    _check(session, n, src, dst, ones, ones, 1, 3, rels=[t1, t2])


@pytest.mark.gpu
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


@pytest.mark.gpu
def test_large_domain_atomic_path(session):
    """n > 2^24 ids takes the atomic passes; the answer is the same."""
    rng = np.random.default_rng(3)
    n, m = (1 << 24) + 77, 20_000
    nodes = rng.integers(0, n, 3000)
    src = rng.choice(nodes, m).astype(np.int64)
    dst = rng.choice(nodes, m).astype(np.int64)
    ones = np.ones(n, dtype=bool)
    _check(session, n, src, dst, ones, ones, 1, 3)


def _pair_paths(n, src, dst, a_mask, b_mask, lo, hi):
    """Edge-distinct path counts per start node from (pair, multiplicity): a path over node pairs
    p1..pk counts prod over uses of (m(p) - uses so far) -- parallel edges stay countable when one
    pair holds 10^5 relationships (the enumeration oracle would walk every path)."""
    from collections import Counter, defaultdict
    mult = Counter(zip(src.tolist(), dst.tolist()))
    out = defaultdict(list)
    for (u, v), c in mult.items():
        out[u].append((v, c))
    got = {}
    for a in range(n):
        if not a_mask[a]:
            continue
        total = 0
        stack = [(a, 0, 1, ())]
        while stack:
            v, depth, w, used = stack.pop()
            for x, c in out.get(v, ()):
                k = c - sum(1 for p in used if p == (v, x))
                if k <= 0:
                    continue
                ww = w * k
                if depth + 1 >= lo and b_mask[x]:
                    total += ww
                if depth + 1 < hi:
                    stack.append((x, depth + 1, ww, used + ((v, x),)))
        if total:
            got[a] = total
    return got


@pytest.mark.gpu
def test_pair_multiplicity_over_16_bits(session):
    """A (source, target) pair with more than 2^16 parallel relationships and its reverse: the
    candidate pair table's packed 16-bit count wraps into its overflow word."""
    from capsmi import ColumnData, I64, graph
    rng = np.random.default_rng(21)
    n = 40
    pairs = [(3, 7, 70_000), (7, 3, 5), (9, 9, 66_000), (3, 9, 2), (9, 3, 65_537)]
    src = [rng.integers(0, n, 400)]
    dst = [rng.integers(0, n, 400)]
    for u, v, c in pairs:
        src.append(np.full(c, u))
        dst.append(np.full(c, v))
    src, dst = np.concatenate(src).astype(np.int64), np.concatenate(dst).astype(np.int64)
    perm = rng.permutation(len(src))
    src, dst = src[perm], dst[perm]
    a_mask = np.ones(n, dtype=bool)
    b_mask = rng.random(n) < 0.8
    b_mask[[3, 7, 9]] = True
    for lo, hi in [(1, 3), (3, 3)]:
        rels = [_table(session, src, dst)]
        a_ok = graph.NodeBitmap(session, 0, n).add_scan(session.table([ColumnData("id", I64, np.arange(n))]))
        b_ok = graph.NodeBitmap(session, 0, n).add_scan(session.table([ColumnData("id", I64, np.nonzero(b_mask)[0])]))
        out = graph.var_length_count(session, rels, a_ok, b_ok, lo, hi, "a", "cnt")
        got = dict(zip(out.column("a").values.tolist(), out.column("cnt").values.tolist()))
        assert got == _pair_paths(n, src, dst, a_mask, b_mask, lo, hi)


def test_pair_paths_helper_matches_enumeration():
    """The multiplicity-aware helper above agrees with the enumeration oracle on small multigraphs."""
    rng = np.random.default_rng(5)
    n, m = 12, 60
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    src[:6] = dst[:6]
    a_mask = rng.random(n) < 0.8
    b_mask = rng.random(n) < 0.7
    for lo, hi in [(1, 1), (1, 3), (2, 3), (3, 3)]:
        _, g = cpu.var_length_count(n, src, dst, lo, hi, a_mask.astype(np.uint8), b_mask.astype(np.uint8))
        want = {int(i): int(g[i]) for i in np.nonzero(g)[0]}
        assert _pair_paths(n, src, dst, a_mask, b_mask, lo, hi) == want


@pytest.mark.gpu
def test_sliced_path_top_ids(session):
    """Domain of 2^24 - 1 ids (the largest the sliced passes take): ids near the top of the packed
    24-bit pair keys."""
    rng = np.random.default_rng(4)
    n, m = (1 << 24) - 1, 20_000
    nodes = np.concatenate([rng.integers(0, n, 2000), np.arange(n - 40, n)])
    src = rng.choice(nodes, m).astype(np.int64)
    dst = rng.choice(nodes, m).astype(np.int64)
    k = m // 4
    src[k:2 * k], dst[k:2 * k] = dst[:k].copy(), src[:k].copy()
    src[-50:] = dst[-50:] = n - 1
    ones = np.ones(n, dtype=bool)
    _check(session, n, src, dst, ones, ones, 1, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("sublog", [1, 3])
def test_filter_sub_regions(session, knobs, sublog):
    """Several filter regions per slice (one k_vl_bset pass each, partials ORed by k_vl_bmerge),
    forced through CAPSMI_VL_SUBLOG: same answer."""
    knobs(session, CAPSMI_VL_SUBLOG=str(sublog))
    test_many_source_slices(session, 0)


def _sharded(session, n, src, dst, a_mask, b_mask, lo, hi, nparts):
    """The multi-GPU C5 protocol emulated on one device: per rank the relationships it owns by
    source plus those into its owned ids from other ranks; od and Y summed over ranks by torch
    between the phases (the all-reduces); the ranks' rows concatenated."""
    import torch
    from capsmi import ColumnData, I64, Session, graph
    session = Session(0)  # on torch's stream: the torch sums between the phases are ordered with the kernels
    session.set_stream(torch.cuda.current_stream().cuda_stream)
    a_ok = graph.NodeBitmap(session, 0, n).add_scan(session.table([ColumnData("id", I64, np.nonzero(a_mask)[0])]))
    b_ok = graph.NodeBitmap(session, 0, n).add_scan(session.table([ColumnData("id", I64, np.nonzero(b_mask)[0])]))
    nw = (n + 31) // 32
    bounds = [(min(32 * (r * nw // nparts), n), min(32 * ((r + 1) * nw // nparts), n)) for r in range(nparts)]
    # garbage in the caller's buffers: begin() must zero od, mid() must write (or clear) every Y entry
    ods = [torch.full((n,), 7777, dtype=torch.int64, device="cuda") for _ in range(nparts)]
    ys = [torch.full((n,), -999, dtype=torch.int64, device="cuda") for _ in range(nparts)]
    shards = []
    for r, (ol, oh) in enumerate(bounds):
        own_s = (src >= ol) & (src < oh)
        own_t = (dst >= ol) & (dst < oh)
        out_t = _table(session, src[own_s], dst[own_s])
        in_t = _table(session, src[own_t & ~own_s], dst[own_t & ~own_s])
        shards.append(graph.VarlenShard(session, [out_t], [in_t], a_ok, b_ok, lo, hi, ol, oh, ods[r].data_ptr()))
    od = sum(ods)
    for r in range(nparts):
        ods[r].copy_(od)
        shards[r].mid(ys[r].data_ptr())
    y = sum(ys)
    got = {}
    for r in range(nparts):
        ys[r].copy_(y)
        out = shards[r].finish("a", "cnt")
        got.update(zip(out.column("a").values.tolist(), out.column("cnt").values.tolist()))
        shards[r].release()
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("nparts", [1, 2, 3, 4])
def test_sharded_matches_enumeration(session, nparts):
    """Owner-partitioned C5 (rows of each rank's own ids; reciprocal pairs across ranks; self-loops;
    multi-edges) against edge-distinct path enumeration."""
    rng = np.random.default_rng(40 + nparts)
    n, m = 3000, 30_000
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    k = m // 5
    src[k:2 * k], dst[k:2 * k] = dst[:k].copy(), src[:k].copy()
    src[-200:] = dst[-200:]
    a_mask = rng.random(n) < 0.8
    b_mask = rng.random(n) < 0.7
    for lo, hi in [(1, 3), (2, 3), (1, 2)]:
        got = _sharded(session, n, src, dst, a_mask, b_mask, lo, hi, nparts)
        _, g = cpu.var_length_count(n, src, dst, lo, hi, a_mask.astype(np.uint8), b_mask.astype(np.uint8))
        assert got == {int(i): int(g[i]) for i in np.nonzero(g)[0]}


@pytest.mark.gpu
def test_pack_misfit_hub(session):
    """A source with od >= 2^24 does not fit the 8-byte (od, Y) words: the misfit flag (zeroed with the
    accumulators, raised by k_vl_y / k_vl_pack) sends the T walk to the 16-byte (od, Y) pairs.  Single
    GPU and sharded over 2 owners, against the closed form."""
    rng = np.random.default_rng(11)
    n, hub, rest = 1000, (1 << 24) + 1000, 20_000
    src = np.concatenate([np.zeros(hub, np.int64), rng.integers(0, n, rest)]).astype(np.int64)
    dst = np.concatenate([rng.integers(0, n, hub), rng.integers(0, n, rest)]).astype(np.int64)
    ones = np.ones(n, dtype=np.uint8)
    _, g = cpu.var_length_closed_form(n, src, dst, 1, 3, ones, ones)
    want = {int(i): int(g[i]) for i in np.nonzero(g)[0]}
    from capsmi import ColumnData, I64, graph
    full = graph.NodeBitmap(session, 0, n).add_scan(session.table([ColumnData("id", I64, np.arange(n))]))
    out = graph.var_length_count(session, [_table(session, src, dst)], full, full, 1, 3, "a", "cnt")
    assert dict(zip(out.column("a").values.tolist(), out.column("cnt").values.tolist())) == want
    assert _sharded(session, n, src, dst, ones.astype(bool), ones.astype(bool), 1, 3, 2) == want


@pytest.mark.gpu
@pytest.mark.parametrize("f2", ["0", "1"])
def test_dense_reciprocal_candidates(session, knobs, f2):
    """Every relationship of a complete digraph (plus doubled pairs) has its reverse: every one is a
    reverse-count candidate, so a wave's step fills its LDS candidate buffer past capacity and the
    overflow goes straight to the list (k_vl_deg, list form); CAPSMI_VL_F2=1 runs the F2-filter form.
    Checked against the closed form (oracle/closed.c, pinned to enumeration by test_oracle_pins.py)."""
    from capsmi import ColumnData, I64, graph
    knobs(session, CAPSMI_VL_F2=f2)
    n = 180
    a, b = np.nonzero(~np.eye(n, dtype=bool))
    extra = np.arange(0, len(a), 7)  # doubled pairs: multiplicities 2
    src = np.concatenate([a, a[extra]]).astype(np.int64)
    dst = np.concatenate([b, b[extra]]).astype(np.int64)
    rng = np.random.default_rng(3)
    a_mask = rng.random(n) < 0.8
    b_mask = rng.random(n) < 0.7
    rels = [_table(session, src, dst)]
    a_nodes = session.table([ColumnData("id", I64, np.nonzero(a_mask)[0])])
    b_nodes = session.table([ColumnData("id", I64, np.nonzero(b_mask)[0])])
    a_ok = graph.NodeBitmap(session, 0, n).add_scan(a_nodes)
    b_ok = graph.NodeBitmap(session, 0, n).add_scan(b_nodes)
    for lo, hi in [(1, 3), (2, 3), (3, 3)]:
        out = graph.var_length_count(session, rels, a_ok, b_ok, lo, hi, "a", "cnt")
        _, g = cpu.var_length_closed_form(n, src, dst, lo, hi, a_mask.astype(np.uint8), b_mask.astype(np.uint8))
        want = {int(i): int(g[i]) for i in np.nonzero(g)[0]}
        got = dict(zip(out.column("a").values.tolist(), out.column("cnt").values.tolist()))
        assert got == want


# ---- four hops (var_length4, oracle/cpu.py var_length4_closed_form) ----------------

@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_four_hops_random_multigraphs(session, seed):
    """upper = 4: self-loops, reciprocal pairs, multi-edges and both node filters against enumeration."""
    rng = np.random.default_rng(40 + seed)
    n = int(rng.integers(5, 120))
    m = int(rng.integers(0, 1000))
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    src[: m // 6] = dst[: m // 6]  # self-loops
    k = m // 6
    src[k:2 * k], dst[k:2 * k] = dst[2 * k:3 * k].copy(), src[2 * k:3 * k].copy()  # reciprocal pairs
    a_mask = rng.random(n) < 0.7
    b_mask = rng.random(n) < 0.6
    for lo, hi in [(1, 4), (4, 4), (2, 4), (3, 4)]:
        _check(session, n, src, dst, a_mask, b_mask, lo, hi)


@pytest.mark.gpu
def test_four_hops_ldbc_shaped_rmat(session):
    from capsmi import graph
    scale = 7
    n, m = 1 << scale, 32 << scale
    rels = graph.rmat_rels(session, scale, 0, m, graph.RMAT_LDBC, 42)
    src, dst = cpu.rmat_edges(scale, 0, m, graph.RMAT_LDBC, 42)
    ones = np.ones(n, dtype=bool)
    _check(session, n, src, dst, ones, ones, 1, 4, rels=[rels])
    _check(session, n, src, dst, ones, ones, 4, 4, rels=[rels])


@pytest.mark.gpu
def test_four_hops_split_tables_and_source_slices(session):
    """Two relationship tables, a domain of several 8192-id source slices (the len <= 3 vectors from the sliced
    passes), hubs and reciprocal copies."""
    rng = np.random.default_rng(77)
    n, m = 20_000, 30_000
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    k = m // 5
    src[k:2 * k], dst[k:2 * k] = dst[:k].copy(), src[:k].copy()
    src[-200:] = dst[-200:]
    t1, t2 = _table(session, src[:9000], dst[:9000]), _table(session, src[9000:], dst[9000:])
    a_mask = rng.random(n) < 0.8
    b_mask = rng.random(n) < 0.7
    _check(session, n, src, dst, a_mask, b_mask, 1, 4, rels=[t1, t2])


@pytest.mark.gpu
def test_four_hops_pair_multiplicity_over_16_bits(session):
    """A pair of 70,000 relationships: multiplicities past 16 bits, and start 7's in-list longer than the LDS copy
    of a one-start wedge tile (those tiles search it in global memory)."""
    from capsmi import ColumnData, I64, graph
    rng = np.random.default_rng(23)
    n = 30
    pairs = [(3, 7, 70_000), (7, 3, 5), (3, 9, 2), (9, 3, 40), (9, 9, 3)]
    src = [rng.integers(0, n, 300)]
    dst = [rng.integers(0, n, 300)]
    for u, v, c in pairs:
        src.append(np.full(c, u))
        dst.append(np.full(c, v))
    src, dst = np.concatenate(src).astype(np.int64), np.concatenate(dst).astype(np.int64)
    perm = rng.permutation(len(src))
    src, dst = src[perm], dst[perm]
    a_mask = np.ones(n, dtype=bool)
    b_mask = rng.random(n) < 0.8
    b_mask[[3, 7, 9]] = True
    rels = [_table(session, src, dst)]
    a_ok = graph.NodeBitmap(session, 0, n).add_scan(session.table([ColumnData("id", I64, np.arange(n))]))
    b_ok = graph.NodeBitmap(session, 0, n).add_scan(session.table([ColumnData("id", I64, np.nonzero(b_mask)[0])]))
    out = graph.var_length_count(session, rels, a_ok, b_ok, 4, 4, "a", "cnt")
    got = dict(zip(out.column("a").values.tolist(), out.column("cnt").values.tolist()))
    assert got == _pair_paths(n, src, dst, a_mask, b_mask, 4, 4)


@pytest.mark.gpu
def test_four_hops_refused_above_2_24_ids(session):
    from capsmi import ColumnData, I64, graph
    from capsmi._lib import UnsupportedOperationException
    n = (1 << 24) + 77
    rels = [_table(session, np.array([0, 1], np.int64), np.array([1, 2], np.int64))]
    ok = graph.NodeBitmap(session, 0, n).add_scan(session.table([ColumnData("id", I64, np.arange(3))]))
    with pytest.raises(UnsupportedOperationException, match="2\\^24"):
        graph.var_length_count(session, rels, ok, ok, 1, 4, "a", "cnt")
