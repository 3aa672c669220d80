"""Undirected Expand patterns routed to the fused kernels (csrc/k_undirected.hip): the planner emits
each undirected hop as outgoing UNION incoming-without-self-loops (RelationalPlanner.scala:126-136), and
the recogniser takes the union of the 2^hops branches as one pattern.  Answers must equal binding
enumeration (oracle/enumerate.py on small multigraphs; oracle/rmat.c orc_two_hop_undirected_enumerate,
pinned to enumerate.py in tests/test_oracle_pins.py, on R-MAT), routed and operator by operator.
Also the route-miss counter and the unrouted-join size guard."""
import numpy as np
import pytest

from golden_util import same_rows

pytestmark = pytest.mark.gpu

QUERIES = [
    ("(a)-[r]-(b)", [["n", ["count*"]]]),
    ("(a)-[r]-(b)", [["n", ["count_distinct", ["id", "b"]]], ["m", ["count_distinct", ["id", "a"]]]]),
    ("(a:A)-[r:R]-(b)", [["n", ["count*"]], ["d", ["count_distinct", ["id", "b"]]]]),
    ("(a)-[r1]-(b)-[r2]-(c)", [["n", ["count*"]], ["dc", ["count_distinct", ["id", "c"]]],
                               ["da", ["count_distinct", ["id", "a"]]]]),
    ("(a:A)-[r1:R]-(b)-[r2:R]-(c:B)", [["n", ["count*"]], ["dc", ["count_distinct", ["id", "c"]]]]),
    ("(a)-[r1:R]-(b:A)-[r2:R]-(c)", [["dc", ["count_distinct", ["id", "c"]]], ["n", ["count*"]]]),
]


def _pg(g):
    from capsmi.planner import PGNode, PGRel, PropertyGraph
    return PropertyGraph([PGNode(x["id"], frozenset(x["labels"]), dict(x["props"])) for x in g["nodes"]],
                         [PGRel(r["id"], r["src"], r["dst"], r["type"], dict(r["props"])) for r in g["rels"]])


@pytest.mark.parametrize("seed", range(10))
def test_undirected_routed_vs_enumeration(session, seed):
    from capsmi.planner import Planner, ScanGraph, result_rows
    from capsmi.table import StringDictionary
    from oracle import enumerate as en
    from test_oracle_pins import _random_graph
    session.dictionary = StringDictionary()
    g = _random_graph(seed)
    graph = en.Graph(g)
    for pattern, items in QUERIES:
        q = {"clauses": [{"match": pattern}], "return": {"items": items}}
        want = en.project(graph, en.match(graph, q), q["return"])
        for fused in (True, False):
            session.set_fused(fused)
            before = session.route_count("undirected")
            try:
                sg = ScanGraph.from_property_graph(session, _pg(g))
                t, outs = Planner(sg).run(q)
                got = result_rows(t, outs, session.dictionary)
            finally:
                session.set_fused(True)
            assert same_rows(got, want), (pattern, fused, got, want)
            if fused and g["rels"]:
                assert session.route_count("undirected") == before + 1, pattern


@pytest.mark.parametrize("scale,kind", [(12, "all"), (12, "person"), (14, "all")])
def test_undirected_two_hop_on_rmat(session, scale, kind):
    """R-MAT (hubs, multi-edges, reciprocal pairs, self-loops) against the C enumeration."""
    from capsmi.planner import EntityTable, Planner, ScanGraph, result_rows
    from capsmi import graph
    from oracle import cpu
    n = 1 << scale
    rels = graph.rmat_rels(session, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
    nodes = graph.rmat_nodes(session, scale, graph.NODES_ALL if kind == "all" else graph.NODES_PERSON, 42)
    sg = ScanGraph(session, [EntityTable("node", frozenset({"Person"}), {"age": 0} if kind == "person" else {}, nodes,
                                         id_col="id")],
                   [EntityTable("rel", frozenset({"FRIEND_OF"}), {}, rels, id_col="id", src_col="source",
                                dst_col="target")])
    q = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]-(b:Person)-[:FRIEND_OF]-(c:Person)"}],
         "return": {"items": [["n", ["count*"]], ["dc", ["count_distinct", ["id", "c"]]],
                              ["da", ["count_distinct", ["id", "a"]]]]}}
    before = session.route_count("undirected")
    t, outs = Planner(sg).run(q)
    got = result_rows(t, outs, session.dictionary)[0]
    assert session.route_count("undirected") == before + 1
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    mask = np.ones(n, np.uint8) if kind == "all" else cpu.person_mask(n).astype(np.uint8)
    rows, dc, da = cpu.two_hop_undirected_enumerate(n, src, dst, mask, mask, mask)
    assert (got["n"], got["dc"], got["da"]) == (rows, dc, da)


def test_route_miss_counter_and_unrouted_guard(session):
    """A pattern no fused shape takes (node properties of both ends in the projection) runs operator
    by operator and counts as a route miss; with a session limit, an unrouted join whose estimate
    exceeds it is refused before any work."""
    from capsmi import _lib, graph
    from capsmi.planner import EntityTable, Planner, ScanGraph
    scale = 12
    rels = graph.rmat_rels(session, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
    nodes = graph.rmat_nodes(session, scale, graph.NODES_PERSON, 42)
    sg = ScanGraph(session, [EntityTable("node", frozenset({"Person"}), {"age": 0}, nodes, id_col="id")],
                   [EntityTable("rel", frozenset({"FRIEND_OF"}), {}, rels, id_col="id", src_col="source",
                                dst_col="target")])
    q = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]->(b:Person)"}],
         "return": {"items": [["x", ["prop", "a", "age"]], ["y", ["prop", "b", "age"]]]}}
    miss = session.route_count("miss")
    t, _ = Planner(sg).run(q)
    assert t.size > 0 and session.route_count("miss") == miss + 1
    four = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person)-[:FRIEND_OF]->"
                                  "(d:Person)-[:FRIEND_OF]->(e:Person)"}],
            "return": {"items": [["x", ["prop", "e", "age"]]]}}
    session.set_unrouted_limit(1 << 30)
    try:
        with pytest.raises(_lib.UnsupportedOperationException, match="estimated"):
            Planner(sg).run(four)[0].size
        assert Planner(sg).run(q)[0].size == t.size  # a small unrouted join still runs
    finally:
        session.set_unrouted_limit(0)


@pytest.mark.parametrize("scale", [16, 20])
@pytest.mark.parametrize("full_form", ["1", "0"])
def test_undirected_two_hop_vs_fixture(session, scale, full_form, knobs):
    """count(*) through the two-sided record partition with both arcs (k_count.hip k_rec_part<true>; with every
    node filter full, its full-filter form unless CAPSMI_REC_FULL=0), and the atomic form (CAPSMI_COUNT=atomic,
    A/B), and count(DISTINCT c), against the committed closed-form fixtures (tests/golden/rmat_full.json
    c3u_s16 / c3u_s20; oracle/closed.c orc_two_hop_undirected_closed_form)."""
    import json
    import os
    knobs(session, CAPSMI_REC_FULL=full_form)
    from capsmi.planner import EntityTable, Planner, ScanGraph, result_rows
    from capsmi import graph
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "tests", "golden", "rmat_full.json")) as f:
        fx = json.load(f)["cases"][f"c3u_s{scale}"]
    rels = graph.rmat_rels(session, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
    nodes = graph.rmat_nodes(session, scale, graph.NODES_ALL, 42)
    sg = ScanGraph(session, [EntityTable("node", frozenset({"Person"}), {}, nodes, id_col="id")],
                   [EntityTable("rel", frozenset({"FRIEND_OF"}), {}, rels, id_col="id", src_col="source",
                                dst_col="target")])
    q = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]-(b:Person)-[:FRIEND_OF]-(c:Person)"}],
         "return": {"items": [["n", ["count*"]], ["dc", ["count_distinct", ["id", "c"]]]]}}
    t, outs = Planner(sg).run(q)
    got = result_rows(t, outs, session.dictionary)[0]
    assert (got["n"], got["dc"]) == (fx["count_star"], fx["count_distinct_c"])
    with session.configured(CAPSMI_COUNT="atomic"):
        t, outs = Planner(sg).run({"clauses": q["clauses"], "return": {"items": [["n", ["count*"]]]}})
        assert result_rows(t, outs, session.dictionary)[0]["n"] == fx["count_star"]


@pytest.mark.parametrize("mode", ["layout", "stream"])
def test_undirected_distinct_layout_and_stream_forms(session, mode):
    """count(DISTINCT c) / count(DISTINCT a) of the undirected 2-hop over the 2-D cell layout (csrc/k_und_part.hip,
    the default up to 2^26 ids: both hops grouped by the slice the arcs go into, K(b) in LDS) and the streaming form
    (CAPSMI_UND=stream), with node filters at the ends or at the middle, against the closed form
    (oracle/closed.c orc_two_hop_undirected_closed_form, pinned to enumeration in tests/test_oracle_pins.py).
    R-MAT scale 21: 4 x 4 slices, so the walks cross slices and workgroups."""
    import os
    from capsmi.planner import EntityTable, Planner, ScanGraph, result_rows
    from capsmi import graph
    from oracle import cpu
    scale = 21
    n = 1 << scale
    rels = graph.rmat_rels(session, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
    sg = ScanGraph(session, [EntityTable("node", frozenset({"Person"}), {"age": 0},
                                         graph.rmat_nodes(session, scale, graph.NODES_PERSON, 42), id_col="id"),
                             EntityTable("node", frozenset({"Company"}), {},
                                         graph.rmat_nodes(session, scale, graph.NODES_COMPANY, 42), id_col="id")],
                   [EntityTable("rel", frozenset({"R"}), {}, rels, id_col="id", src_col="source", dst_col="target")])
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    person = cpu.person_mask(n).astype(np.uint8)
    every = np.ones(n, np.uint8)
    with session.configured(CAPSMI_UND="stream" if mode == "stream" else "part"):
        for pattern, (am, bm, cm) in (("(a:Person)-[:R]-(b)-[:R]-(c:Person)", (person, every, person)),
                                      ("(a)-[:R]-(b:Person)-[:R]-(c)", (every, person, every)),
                                      ("(a:Person)-[:R]-(b)-[:R]-(c)", (person, every, every))):
            q = {"clauses": [{"match": pattern}],
                 "return": {"items": [["dc", ["count_distinct", ["id", "c"]]], ["da", ["count_distinct", ["id", "a"]]]]}}
            before = session.route_count("undirected")
            t, outs = Planner(sg).run(q)
            got = result_rows(t, outs, session.dictionary)[0]
            assert session.route_count("undirected") == before + 1, pattern
            _, dc = cpu.two_hop_undirected_closed_form(n, src, dst, am, bm, cm)
            _, da = cpu.two_hop_undirected_closed_form(n, src, dst, cm, bm, am)
            assert (got["dc"], got["da"]) == (dc, da), (pattern, mode)
