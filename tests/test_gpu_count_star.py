"""2-hop count(*) (capsmi_two_hop_count) in every form against the closed form of oracle/closed.c:
the two partitions of 2-byte records (default) and the per-relationship atomics (config CAPSMI_COUNT=atomic,
the form above 2^26 ids).  The closed form itself is pinned against binding enumeration in
tests/test_oracle*.py."""
import numpy as np
import pytest

from oracle import cpu

pytestmark = pytest.mark.gpu

MODES = ["rec", "atomic"]


def _mode(knobs, session, mode):
    knobs(session, CAPSMI_COUNT=mode)


def _bm(session, n, mask):
    from capsmi import ColumnData, I64, graph
    nodes = session.table([ColumnData("id", I64, np.nonzero(mask)[0].astype(np.int64))])
    return graph.NodeBitmap(session, 0, n).add_scan(nodes)


def _rels(session, src, dst):
    from capsmi import ColumnData, I64
    return session.table([ColumnData("id", I64, np.arange(len(src))), ColumnData("source", I64, src),
                          ColumnData("target", I64, dst)])


@pytest.mark.parametrize("mode", MODES)
def test_self_loops_and_distinct_masks(session, knobs, mode):
    from capsmi import graph
    _mode(knobs, session, mode)
    edges = [(0, 0), (1, 1), (1, 1), (3, 2), (2, 2), (4, 5), (5, 5), (5, 6), (2, 5), (6, 2), (3, 3)]
    src = np.array([e[0] for e in edges], dtype=np.int64)
    dst = np.array([e[1] for e in edges], dtype=np.int64)
    n = 8
    for am, bm_, cm in [([1] * 8, [1] * 8, [1] * 8), ([1, 1, 0, 1, 1, 1, 1, 1], [1, 1, 1, 0, 1, 1, 1, 1],
                                                      [0, 1, 1, 1, 1, 1, 1, 1])]:
        a, b, c = (np.array(x, dtype=np.uint8) for x in (am, bm_, cm))
        rows, _ = cpu.two_hop_closed_form(n, src, dst, a, b, c)
        assert graph.two_hop_count(session, [_rels(session, src, dst)], _bm(session, n, a), _bm(session, n, b),
                                   _bm(session, n, c)) == rows


@pytest.mark.parametrize("mode", MODES)
def test_hub_slices_and_split_walks(session, knobs, mode):
    """2^21 ids (64 slices of 2^15): hub slices far longer than one chunk, slices split between walk
    blocks, ids outside the domain, self-loops, two tables, distinct a/b/c filters."""
    from capsmi import graph
    _mode(knobs, session, mode)
    rng = np.random.default_rng(17)
    n = 1 << 21
    m = 400000
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    hubs = rng.integers(0, 1 << 14, 40)  # all in slice 0
    src[: m // 3] = hubs[rng.integers(0, 40, m // 3)]
    dst[m // 3: 2 * m // 3] = hubs[rng.integers(0, 40, m // 3)]
    src[:50] = dst[:50]
    outside = np.array([n + 5, -3, 7], dtype=np.int64)
    s_all = np.concatenate([src, outside]).astype(np.int64)
    d_all = np.concatenate([dst, [4, 5, n + 1]]).astype(np.int64)
    a = (rng.random(n) < 0.9).astype(np.uint8)
    b = (rng.random(n) < 0.8).astype(np.uint8)
    c = (rng.random(n) < 0.7).astype(np.uint8)
    keep = (s_all >= 0) & (s_all < n) & (d_all >= 0) & (d_all < n)
    rows, _ = cpu.two_hop_closed_form(n, s_all[keep], d_all[keep], a, b, c)
    h = len(s_all) // 2
    t1, t2 = _rels(session, s_all[:h], d_all[:h]), _rels(session, s_all[h:], d_all[h:])
    assert graph.two_hop_count(session, [t1, t2], _bm(session, n, a), _bm(session, n, b), _bm(session, n, c)) == rows


@pytest.mark.parametrize("mode", ["rec", "atomic"])
@pytest.mark.parametrize("scale,kind", [(12, "person"), (16, "all"), (17, "person")])
def test_rmat(session, knobs, mode, scale, kind):
    from capsmi import graph
    _mode(knobs, session, mode)
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    mask = np.ones(n, np.uint8) if kind == "all" else cpu.person_mask(n).astype(np.uint8)
    rows, _ = cpu.two_hop_closed_form(n, src, dst, mask, mask, mask)
    bm = _bm(session, n, mask)
    assert graph.two_hop_count(session, [_rels(session, src, dst)], bm, bm, bm) == rows


@pytest.mark.parametrize("mode", ["rec", "atomic"])
def test_dense_buckets_roll_chunks(session, knobs, mode):
    """3M relationships into three 2^16-id buckets: every partition block fills several chunks of one
    bucket (chunk rollover inside a tile, pieces split across chunks), plus a ragged tail and
    in-degrees far above 2^16 for a few ids."""
    from capsmi import graph
    _mode(knobs, session, mode)
    rng = np.random.default_rng(23)
    n = 1 << 20
    m = 3_000_001
    src = rng.integers(0, n, m)
    dst = rng.integers(0, 3 << 16, m)
    dst[: 300_000] = 12345  # one id with 300k in-edges
    src[300_000: 400_000] = 777  # and one with 100k out-edges
    a = (rng.random(n) < 0.95).astype(np.uint8)
    ones = np.ones(n, np.uint8)
    rows, _ = cpu.two_hop_closed_form(n, src.astype(np.int64), dst.astype(np.int64), a, ones, ones)
    got = graph.two_hop_count(session, [_rels(session, src.astype(np.int64), dst.astype(np.int64))], _bm(session, n, a),
                              _bm(session, n, ones), _bm(session, n, ones))
    assert got == rows


@pytest.mark.parametrize("seed", [0, 1])
def test_rec_counter_wraps_on_even_and_odd_ids(session, knobs, seed):
    """The IN walk counts two ids per 32-bit LDS word in 16-bit halves (even id low, odd id high).
    Pairs (x even, x + 1) with more than 2^16 in-relationships each exercise the low-half wrap (its
    carry reaches the high half), the high-half wrap, and a low-half carry into a high half sitting
    at 0xFFFF (x + 1 with 65535 mod 65536 in-relationships) -- each against the closed form."""
    from capsmi import graph
    _mode(knobs, session, "rec")
    rng = np.random.default_rng(100 + seed)
    n = 1 << 18
    counts = {2000: 200_001, 2001: 131_071, 4000: 65_536, 4001: 65_535, 6000: 70_000, 8000: 65_535, 8001: 196_607,
              65534: 131_072, 65535: 65_537}
    dst = np.concatenate([np.full(c, x, np.int64) for x, c in counts.items()] + [rng.integers(0, n, 400_000)])
    rng.shuffle(dst)
    src = rng.integers(0, n, len(dst)).astype(np.int64)
    src[:50] = dst[:50]  # a few self-loops
    a = (rng.random(n) < 0.9).astype(np.uint8)
    b = (rng.random(n) < 0.97).astype(np.uint8)
    for x in counts:
        b[x] = 1
    ones = np.ones(n, np.uint8)
    rows, _ = cpu.two_hop_closed_form(n, src, dst, a, b, ones)
    got = graph.two_hop_count(session, [_rels(session, src, dst)], _bm(session, n, a), _bm(session, n, b),
                              _bm(session, n, ones))
    assert got == rows


@pytest.mark.parametrize("mode", ["rec", "atomic"])
def test_offset_domain(session, knobs, mode):
    """Bitmaps over [lo, lo + n) with lo far from 0 and n not a multiple of the 2^16-id bucket:
    records are ids relative to lo, the last bucket is partial, and relationships leaving the domain
    on either side are dropped."""
    from capsmi import ColumnData, I64, graph
    _mode(knobs, session, mode)
    rng = np.random.default_rng(31)
    lo, n, m = 1 << 33, 200_003, 1_500_000
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    src[:1000] = dst[:1000]  # self-loops
    src[1000:1100] = n + 7  # outside the domain
    dst[1100:1200] = -5
    keep = (src >= 0) & (src < n) & (dst >= 0) & (dst < n)
    a = (rng.random(n) < 0.8).astype(np.uint8)
    b = (rng.random(n) < 0.9).astype(np.uint8)
    c = (rng.random(n) < 0.85).astype(np.uint8)
    rows, _ = cpu.two_hop_closed_form(n, src[keep].astype(np.int64), dst[keep].astype(np.int64), a, b, c)

    def bm(mask):
        nodes = session.table([ColumnData("id", I64, (np.nonzero(mask)[0] + lo).astype(np.int64))])
        return graph.NodeBitmap(session, lo, lo + n).add_scan(nodes)

    rels = _rels(session, (src + lo).astype(np.int64), (dst + lo).astype(np.int64))
    assert graph.two_hop_count(session, [rels], bm(a), bm(b), bm(c)) == rows


@pytest.mark.parametrize("nparts", [1, 3, 8])
def test_sharded_count(nparts):
    """The multi-GPU count(*) (capsmi_count_shard_*) with N owner(target) shards on one device: each
    shard holds the relationships into its owned id range (graph.owner_words: a ragged last range;
    plus, on rank 0, relationships whose target leaves the domain), writes its owned in-degrees, the
    slices are stitched into one array (the all-gather) and the shards' device parts sum to the
    closed form.  Self-loops, sources outside the domain and an in-degree above 2^16 included."""
    import torch
    from capsmi import Session, graph
    s = Session(0)
    s.set_stream(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(41 + nparts)
    n, m = 300_001, 2_000_000
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    dst[:200_000] = 4242
    src[200_000:201_000] = dst[200_000:201_000]
    src[201_000:201_100] = n + 3
    dst[201_100:201_200] = -1
    keep = (src >= 0) & (src < n) & (dst >= 0) & (dst < n)
    a = (rng.random(n) < 0.9).astype(np.uint8)
    b = (rng.random(n) < 0.8).astype(np.uint8)
    c = (rng.random(n) < 0.85).astype(np.uint8)
    rows, _ = cpu.two_hop_closed_form(n, src[keep].astype(np.int64), dst[keep].astype(np.int64), a, b, c)
    A, B, C = _bm(s, n, a), _bm(s, n, b), _bm(s, n, c)
    in_all = torch.zeros(n, dtype=torch.int32, device="cuda")
    parts = torch.zeros(nparts, dtype=torch.int64, device="cuda")
    shards = []
    for r in range(nparts):
        wb, we = graph.owner_words(n, r, nparts)
        own_lo, own_hi = 32 * wb, min(32 * we, n)
        sel = (dst >= own_lo) & (dst < own_hi)
        if r == 0:
            sel |= (dst < 0) | (dst >= n)
        rel = _rels(s, src[sel].astype(np.int64), dst[sel].astype(np.int64))
        owned = torch.full((max(own_hi - own_lo, 1),), 0x5eed, dtype=torch.int32, device="cuda")
        sh = graph.CountShard(s, [rel], A, B, C, own_lo, own_hi, owned.data_ptr())
        in_all[own_lo:own_hi] = owned[: own_hi - own_lo]
        shards.append((sh, rel, owned))
    for r, (sh, _, _) in enumerate(shards):
        sh.finish(in_all.data_ptr(), parts[r:r + 1].data_ptr())
        sh.close()
    assert int(parts.sum().item()) == rows
    assert graph.two_hop_count(s, [_rels(s, src.astype(np.int64), dst.astype(np.int64))], A, B, C) == rows


def test_sharded_count_refusals():
    """capsmi_count_shard_begin refuses what the phased count cannot answer: bitmaps over different
    id domains, an owned range outside the domain, a null owned buffer for a non-empty range."""
    import torch
    from capsmi import ColumnData, I64, Session, graph
    session = Session(0)
    session.set_stream(torch.cuda.current_stream().cuda_stream)
    n = 1000
    ones = np.ones(n, np.uint8)
    A = _bm(session, n, ones)
    rel = _rels(session, np.arange(10, dtype=np.int64), np.arange(1, 11, dtype=np.int64))
    other = graph.NodeBitmap(session, 0, n + 64).add_scan(session.table([ColumnData("id", I64, np.arange(5))]))
    buf = torch.zeros(n, dtype=torch.int32, device="cuda")
    with pytest.raises(Exception):
        graph.CountShard(session, [rel], A, other, A, 0, n, buf.data_ptr())
    with pytest.raises(Exception):
        graph.CountShard(session, [rel], A, A, A, 0, n + 32, buf.data_ptr())
    with pytest.raises(Exception):
        graph.CountShard(session, [rel], A, A, A, 0, 64, 0)
    with graph.CountShard(session, [rel], A, A, A, 0, n, buf.data_ptr()) as sh:  # and a valid one still works
        out = torch.zeros(1, dtype=torch.int64, device="cuda")
        sh.finish(buf.data_ptr(), out.data_ptr())
        assert int(out.item()) == 9  # chain 0->1->...->10: 9 two-hop pairs inside [0, 1000)
        from capsmi._lib import IllegalArgumentException
        with pytest.raises(IllegalArgumentException, match="twice"):  # one finish per handle
            sh.finish(buf.data_ptr(), out.data_ptr())
        assert int(out.item()) == 9
    # the handle keeps what it reads of b_ok: releasing the bitmaps between begin and finish is safe
    B = _bm(session, n, ones)
    sh = graph.CountShard(session, [rel], A, B, A, 0, n, buf.data_ptr())
    B.release()
    out = torch.zeros(1, dtype=torch.int64, device="cuda")
    sh.finish(buf.data_ptr(), out.data_ptr())
    sh.close()
    assert int(out.item()) == 9
