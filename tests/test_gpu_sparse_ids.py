"""Graphs whose Long ids do not fit one window of 2^30 ids -- edge-list ids near 2^40, tagged ids
(10 tag bits above 54 id bits, Tags.scala:36-55), dangling endpoints -- still reach the fused kernels
through the graph's dense id compaction (include/capsmi.h capsmi_graph_compact), with the original
ids in every result.  Expected values: the oracle on the same graph relabelled densely."""
import numpy as np
import pytest

from golden_util import same_rows

pytestmark = pytest.mark.gpu


def _sparse_graph(seed, n=3000, m=30000, base=1 << 40, spread=1 << 45, dangling=0):
    rng = np.random.default_rng(seed)
    ids = np.unique(rng.integers(base, base + spread, n))
    n = len(ids)
    w = rng.zipf(1.6, m) % n  # skewed endpoints (hubs)
    u = rng.integers(0, n, m)
    src, dst = ids[np.where(rng.random(m) < 0.5, w, u)], ids[rng.integers(0, n, m)]
    src[: m // 50] = dst[: m // 50]  # self-loops
    if dangling:  # endpoints that are in no node table
        extra = np.arange(dangling, dtype=np.int64) + base + spread + 7
        k = rng.integers(0, m, dangling)
        dst[k] = extra
    return ids, src.astype(np.int64), dst.astype(np.int64)


def _scan_graph(session, ids, src, dst, rtype="R"):
    from capsmi import ColumnData, I64
    from capsmi.planner import EntityTable, ScanGraph
    nodes = session.table([ColumnData("id", I64, ids)]).as_node_table("id")
    rels = session.table([ColumnData("id", I64, np.arange(len(src), dtype=np.int64) * 3 + (1 << 50)),
                          ColumnData("source", I64, src), ColumnData("target", I64, dst)]).as_rel_table(
        "id", "source", "target")
    assert session.compact_if_sparse([nodes], [rels])
    return ScanGraph(session, [EntityTable("node", frozenset({"N"}), {}, nodes, id_col="id")],
                     [EntityTable("rel", frozenset({rtype}), {}, rels, id_col="id", src_col="source", dst_col="target")])


def _dense(ids, src, dst):
    allv, inv = np.unique(np.concatenate([ids, src, dst]), return_inverse=True)
    node_mask = np.zeros(len(allv), np.uint8)
    node_mask[inv[: len(ids)]] = 1
    return len(allv), node_mask, inv[len(ids): len(ids) + len(src)], inv[len(ids) + len(src):], allv


def _run(session, sg, q):
    from capsmi.planner import Planner, result_rows
    t, outs = Planner(sg).run(q)
    return result_rows(t, outs, session.dictionary)


@pytest.mark.parametrize("seed", [0, 1])
def test_c3_on_ids_near_2_40(session, seed):
    from oracle import cpu
    ids, src, dst = _sparse_graph(seed)
    sg = _scan_graph(session, ids, src, dst)
    q = {"clauses": [{"match": "(a:N)-[:R]->(b:N)-[:R]->(c:N)"}],
         "return": {"items": [["d", ["count_distinct", ["id", "c"]]], ["n", ["count*"]]]}}
    before = session.route_count("two_hop")
    got = _run(session, sg, q)
    assert session.route_count("two_hop") == before + 1
    n, mask, ds, dd, _ = _dense(ids, src, dst)
    rows, dist = cpu.two_hop_enumerate(n, ds, dd, mask, mask, mask)
    assert got == [{"d": dist, "n": rows}]


def test_expand_projection_keeps_original_ids(session):
    ids, src, dst = _sparse_graph(3, dangling=40)
    sg = _scan_graph(session, ids, src, dst)
    q = {"clauses": [{"match": "(a:N)-[r:R]->(b:N)"}],
         "return": {"items": [["a", ["id", "a"]], ["r", ["id", "r"]], ["b", ["id", "b"]]]}}
    before = session.route_count("expand")
    got = _run(session, sg, q)
    assert session.route_count("expand") == before + 1
    node = set(ids.tolist())
    rid = np.arange(len(src), dtype=np.int64) * 3 + (1 << 50)
    want = [{"a": int(s), "r": int(r), "b": int(d)} for s, r, d in zip(src, rid, dst) if s in node and d in node]
    assert same_rows(got, want)


@pytest.mark.parametrize("dangling", [0, 25])
def test_var_length_with_dangling_intermediates(session, dangling):
    """Intermediate hops of a var-length path are not node-scanned: dangling endpoints take part."""
    from oracle import cpu
    ids, src, dst = _sparse_graph(5, n=800, m=6000, dangling=dangling)
    # some dangling targets also start relationships, so paths run through them
    if dangling:
        extra = dst[dst > ids.max()]
        src = np.concatenate([src, extra[:10]])
        dst = np.concatenate([dst, ids[:10]])
    sg = _scan_graph(session, ids, src, dst)
    q = {"clauses": [{"match": "(a:N)-[:R*1..3]->(b:N)"}], "return": {"items": [["a", ["id", "a"]], ["n", ["count*"]]]}}
    before = session.route_count("var_length")
    got = _run(session, sg, q)
    assert session.route_count("var_length") == before + 1
    n, mask, ds, dd, allv = _dense(ids, src, dst)
    _, per = cpu.var_length_count(n, ds, dd, 1, 3, mask, mask)
    want = [{"a": int(allv[i]), "n": int(per[i])} for i in np.nonzero(per)[0]]
    assert same_rows(got, want)


def test_triangles_on_tagged_ids(session):
    """Ids carrying a graph tag in the top 10 bits (Tags.scala: id | tag << 54)."""
    from oracle import cpu
    ids, src, dst = _sparse_graph(7, n=500, m=8000, base=0, spread=1 << 20)
    # two member graphs' ids: tag 0 and tag 3 (a union graph's retagged ids)
    tags = {int(v): (int(v) | (3 << 54)) if i % 2 else int(v) for i, v in enumerate(ids)}
    retag = np.vectorize(lambda v: tags[int(v)], otypes=[np.int64])
    sg = _scan_graph(session, retag(ids), retag(src), retag(dst))
    q = {"clauses": [{"match": "(a)-[:R]->(b)-[:R]->(c)-[:R]->(a)"}], "return": {"items": [["n", ["count*"]]]}}
    before = session.route_count("triangle")
    got = _run(session, sg, q)
    assert session.route_count("triangle") == before + 1
    n, mask, ds, dd, _ = _dense(ids, src, dst)
    keep = (mask[ds] != 0) & (mask[dd] != 0)
    assert got == [{"n": cpu.triangle_enumerate(n, ds[keep], dd[keep])}]


def test_edge_list_with_large_ids(session, tmp_path):
    """EdgeListDataSource ingest (EdgeListDataSource.scala:76-97) of Long ids near 2^40: compacted, fused."""
    from capsmi import io
    from capsmi.planner import EntityTable, Planner, ScanGraph, result_rows
    from oracle import cpu
    ids, src, dst = _sparse_graph(11, n=400, m=3000)
    f = tmp_path / "g.txt"
    f.write_text("# comment\n" + "".join(f"{s} {d}\n" for s, d in zip(src, dst)))
    nodes, rels = io.edge_list_graph(session, str(f))
    sg = ScanGraph(session, [EntityTable("node", frozenset({"V"}), {}, nodes, id_col="id")],
                   [EntityTable("rel", frozenset({"E"}), {}, rels, id_col="id", src_col="source", dst_col="target")])
    q = {"clauses": [{"match": "(a:V)-[:E]->(b:V)-[:E]->(c:V)"}],
         "return": {"items": [["d", ["count_distinct", ["id", "c"]]]]}}
    before = session.route_count("two_hop")
    t, outs = Planner(sg).run(q)
    got = result_rows(t, outs, session.dictionary)
    assert session.route_count("two_hop") == before + 1
    allv, inv = np.unique(np.concatenate([src, dst]), return_inverse=True)
    _, dist = cpu.two_hop_enumerate(len(allv), inv[: len(src)], inv[len(src):])
    assert got == [{"d": dist}]
