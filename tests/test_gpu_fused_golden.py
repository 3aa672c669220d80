"""The fused entry points (capsmi_two_hop_count(_distinct), _expand_filter, _triangle_count,
_var_length_count) on the reference's own test graphs, and against the committed full-size oracle
fixtures at sizes that run in seconds.

Expected values: (1) explicit numbers read off the reference's assertions (cited per case);
(2) for every golden graph and every label / type restriction, oracle/enumerate.py, which is pinned
by those same assertions (tests/test_golden_oracle.py)."""
import json
import os

import numpy as np
import pytest

from golden_util import all_cases, property_graph
from test_oracle_pins import _dense, _enum, _pat, _restrictions

pytestmark = pytest.mark.gpu

CASES = {c["name"]: c for _, c in all_cases()}


def _device(session, n, mask, src, dst, rel_ids=None):
    from capsmi import ColumnData, I64, graph
    ids = np.arange(len(src), dtype=np.int64) if rel_ids is None else np.asarray(rel_ids, np.int64)
    rels = session.table([ColumnData("id", I64, ids), ColumnData("source", I64, src), ColumnData("target", I64, dst)])
    nodes = session.table([ColumnData("id", I64, np.nonzero(mask)[0].astype(np.int64))])
    bm = graph.NodeBitmap(session, 0, n).add_scan(nodes)
    return rels, bm


def _fused(session, g, label, rtype):
    from capsmi import graph
    n, mask, src, dst = _dense(g, label, rtype)
    rels, bm = _device(session, n, mask, src, dst)
    out = {"rows": graph.two_hop_count(session, [rels], bm, bm, bm),
           "dist": graph.two_hop_count_distinct(session, [rels], bm, bm, bm),
           "tri": graph.triangle_count(session, [rels], bm),
           "expand": graph.expand_filter(session, rels, bm, bm, ["source", "target"], ["a", "b"]).size}
    for lo, hi in [(1, 1), (1, 2), (1, 3), (2, 3), (3, 3)]:
        t = graph.var_length_count(session, [rels], bm, bm, lo, hi, "a", "n")
        out[(lo, hi)] = dict(zip(t.column("a").values.tolist(), t.column("n").values.tolist()))
    return out


@pytest.mark.parametrize("name", list(CASES))
def test_fused_on_reference_graphs(session, name):
    _, g = property_graph(CASES[name])
    for label, rtype in _restrictions(g):
        lab, ty = _pat(label, rtype)
        got = _fused(session, g, label, rtype)
        two = _enum(g, f"(a{lab})-{ty}->(b{lab})-{ty}->(c{lab})",
                    [["rows", ["count*"]], ["dist", ["count_distinct", ["id", "c"]]]])[0]
        assert (got["rows"], got["dist"]) == (two["rows"], two["dist"]), (label, rtype)
        tri = _enum(g, f"(a{lab})-{ty}->(b{lab})-{ty}->(c{lab})-{ty}->(a)", [["n", ["count*"]]])[0]["n"]
        assert got["tri"] == tri, (label, rtype)
        one = _enum(g, f"(a{lab})-{ty}->(b{lab})", [["n", ["count*"]]])[0]["n"]
        assert got["expand"] == one, (label, rtype)
        for lo, hi in [(1, 1), (1, 2), (1, 3), (2, 3), (3, 3)]:
            rows = _enum(g, f"(a{lab})-{ty[:-1] if rtype else '['}*{lo}..{hi}]->(b{lab})",
                         [["a", ["id", "a"]], ["n", ["count*"]]])
            assert got[(lo, hi)] == {r["a"]: r["n"] for r in rows}, (label, rtype, lo, hi)


def test_reference_assertions(session):
    """Numbers read directly off the reference's assertions."""
    def fused(name, label, rtype):
        _, g = property_graph(CASES[name])
        return _fused(session, g, label, rtype)

    # MatchBehaviour.scala:97-125: (p1:Person)-[e1]->(p2:Person)-[e2]->(p3:Person) -> one row (Alice, Bob, Eve)
    r = fused("multiple match clauses", "Person", None)
    assert (r["rows"], r["dist"]) == (1, 1)
    # MatchBehaviour.scala:127-161: the 2-hop prefix of the asserted rows is (Bob, Alice, Bob), (Alice, Bob, Alice):
    # 2 bindings, 2 distinct p3 (cyphermorphism keeps e1 <> e2 on the reciprocal pair)
    r = fused("cyphermorphism and multiple match clauses", "Person", "KNOWS")
    assert (r["rows"], r["dist"]) == (2, 2)
    # AggregationBehaviour.scala:203-211: MATCH (n)-->(b:B) ... count(b) = 2
    _, g = property_graph(CASES["count after expand"])
    n, _, src, dst = _dense(g, None, None)
    _, bmask, _, _ = _dense(g, "B", None)
    all_nodes = _dense(g, None, None)[1]
    rels, a_ok = _device(session, n, all_nodes, src, dst)
    _, b_ok = _device(session, n, bmask, src, dst)
    from capsmi import graph
    assert graph.expand_filter(session, rels, a_ok, b_ok, ["target"], ["b"]).size == 2
    # BoundedVarExpandBehaviour.scala:91-110: a 3-cycle, (a)-[*..6]->(b) -> 9 paths, 3 per source (edge-distinct
    # paths on 3 edges have at most 3 hops, so *..6 = *1..3 here)
    r = fused("var expand with default lower and loop", "Node", "REL")
    assert r[(1, 3)] == {0: 3, 1: 3, 3: 3}
    # the same 3-cycle closes one directed triangle, bound once per start node
    assert r["tri"] == 3


FIXTURES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rmat_full.json")


def _fx(key):
    with open(FIXTURES) as f:
        return json.load(f)["cases"][key]


@pytest.mark.parametrize("scale", [16, 20])
def test_c3_vs_fixture(session, scale):
    from capsmi import graph
    fx = _fx(f"c3_s{scale}")
    rels = graph.rmat_rels(session, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
    p = graph.NodeBitmap(session, 0, 1 << scale).add_scan(graph.rmat_nodes(session, scale, graph.NODES_ALL))
    assert graph.two_hop_count_distinct(session, [rels], p, p, p) == fx["count_distinct_c"]
    assert graph.two_hop_count(session, [rels], p, p, p) == fx["count_star"]
    rp = graph.RelPartition(session, [rels], 0, 1 << scale)
    assert rp.count_distinct(p, p, p) == fx["count_distinct_c"]


def test_c2_vs_fixture(session):
    from capsmi import graph
    from capsmi.expr import Ands, BinOp, Col, Lit
    fx = _fx("c2_s16")
    scale = 16
    rels = graph.rmat_rels(session, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
    persons = graph.rmat_nodes(session, scale, graph.NODES_PERSON, 42)
    a = graph.NodeBitmap(session, 0, 1 << scale).add_scan(
        persons, "id", Ands((BinOp(">=", Col("age"), Lit(18)), BinOp("<", Col("age"), Lit(65)))))
    b = graph.NodeBitmap(session, 0, 1 << scale).add_scan(persons, "id")
    out = graph.expand_filter(session, rels, a, b, ["source", "target"], ["a", "b"])
    assert list(out.fingerprint(["a", "b"])) == [fx["fingerprint"][0], int(fx["fingerprint"][1]),
                                                 int(fx["fingerprint"][2])]


def test_c4_vs_fixture(session):
    from capsmi import graph
    scale = 14
    rels = graph.rmat_rels(session, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
    p = graph.NodeBitmap(session, 0, 1 << scale).add_scan(graph.rmat_nodes(session, scale, graph.NODES_ALL))
    assert graph.triangle_count(session, [rels], p) == _fx("c4_s14")["count_star"]


def test_c5_vs_fixture(session):
    from capsmi import graph
    fx = _fx("c5_s14")
    scale = 14
    rels = graph.rmat_rels(session, scale, 0, 32 << scale, graph.RMAT_LDBC, 42)
    p = graph.NodeBitmap(session, 0, 1 << scale).add_scan(graph.rmat_nodes(session, scale, graph.NODES_ALL))
    out = graph.var_length_count(session, [rels], p, p, 1, 3)
    assert int(out.column("count").values.sum()) == fx["sum_count"]
    assert list(out.fingerprint(["id", "count"])) == [fx["fingerprint"][0], int(fx["fingerprint"][1]),
                                                      int(fx["fingerprint"][2])]


def test_c5_four_hops_vs_fixture(session):
    """*1..4 at s = 14 against the oracle's full closed form (tests/golden/make_rmat_full.py c5u4_s14)."""
    from capsmi import graph
    fx = _fx("c5u4_s14")
    scale = 14
    rels = graph.rmat_rels(session, scale, 0, 32 << scale, graph.RMAT_LDBC, 42)
    p = graph.NodeBitmap(session, 0, 1 << scale).add_scan(graph.rmat_nodes(session, scale, graph.NODES_ALL))
    out = graph.var_length_count(session, [rels], p, p, 1, 4)
    assert int(out.column("count").values.sum()) == fx["sum_count"]
    assert list(out.fingerprint(["id", "count"])) == [fx["fingerprint"][0], int(fx["fingerprint"][1]),
                                                      int(fx["fingerprint"][2])]
