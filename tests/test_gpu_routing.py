"""The relational planner's output routed to the fused kernels (include/capsmi.h: lazy Table[T] plans).

The planner mirror emits the Table[T] calls RelationalPlanner would (joins of node / relationship
scans, uniqueness filter, aggregate); libcapsmi recognises the Expand / ExpandInto / var-length
shapes at materialisation.  Each test runs a BASELINE query shape through ``Planner(sg).run`` on
R-MAT inputs, checks the answer against the CPU oracle (or enumeration), checks that the fused route
was taken (route counters, kernel timers), and that the same plan run operator by operator
(``set_fused(False)``) gives the same rows."""
import os

import numpy as np
import pytest

from golden_util import all_cases, run_planner, same_rows

pytestmark = pytest.mark.gpu


def _graph(session, scale, ef=16, probs=(57, 19, 19), kind="all", rtype="FRIEND_OF"):
    from capsmi import graph
    from capsmi.planner import EntityTable, ScanGraph
    rels = graph.rmat_rels(session, scale, 0, ef << scale, probs, 42)
    k = graph.NODES_ALL if kind == "all" else graph.NODES_PERSON
    nodes = graph.rmat_nodes(session, scale, k, 42)
    props = {"age": 0} if kind == "person" else {}
    sg = ScanGraph(session, [EntityTable("node", frozenset({"Person"}), props, nodes, id_col="id")],
                   [EntityTable("rel", frozenset({rtype}), {}, rels, id_col="id", src_col="source", dst_col="target")])
    return sg


def _run(session, sg, q, fused=True):
    from capsmi.planner import Planner, result_rows
    session.set_fused(fused)
    try:
        t, outs = Planner(sg).run(q)
        return result_rows(t, outs, session.dictionary)
    finally:
        session.set_fused(True)


def _routed(session, name, fn):
    before = session.route_count(name)
    out = fn()
    assert session.route_count(name) == before + 1, f"plan not routed to '{name}'"
    return out


C3 = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person)"}],
      "return": {"items": [["n", ["count_distinct", ["id", "c"]]]]}}


@pytest.mark.parametrize("scale", [10, 12])
def test_c3_count_distinct_routed(session, scale):
    import ctypes
    from capsmi import _lib
    from oracle import cpu
    sg = _graph(session, scale)
    _lib.call("capsmi_session_set_profiling", session.handle, 1)
    got = _routed(session, "two_hop", lambda: _run(session, sg, C3))
    cnt, ms = ctypes.c_int64(), ctypes.c_double()
    _lib.call("capsmi_session_kernel_time", session.handle, b"hop2", ctypes.byref(cnt), ctypes.byref(ms))
    _lib.call("capsmi_session_set_profiling", session.handle, 0)
    assert cnt.value > 0  # the fused hop-2 kernel ran
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    rows, dist = cpu.two_hop_enumerate(1 << scale, src, dst)
    assert got == [{"n": dist}]
    q = {"clauses": C3["clauses"], "return": {"items": [["n", ["count*"]], ["m", ["count", ["id", "b"]]],
                                                        ["d", ["count_distinct", ["id", "a"]]]]}}
    got = _routed(session, "two_hop", lambda: _run(session, sg, q))
    src_r, dst_r = dst, src  # distinct a = distinct c of the reversed walk
    _, dist_a = cpu.two_hop_enumerate(1 << scale, src_r, dst_r)
    assert got == [{"n": rows, "m": rows, "d": dist_a}]


def test_profiling_names_select_the_timers(session):
    """capsmi_session_set_profiling_names: only the named timers record; NULL restores every timer"""
    import ctypes
    from capsmi import _lib
    sg = _graph(session, 10)

    def launches(name):
        cnt, ms = ctypes.c_int64(), ctypes.c_double()
        _lib.call("capsmi_session_kernel_time", session.handle, name, ctypes.byref(cnt), ctypes.byref(ms))
        return cnt.value
    _lib.call("capsmi_session_set_profiling", session.handle, 1)
    try:
        launches(b"hop2"), launches(b"mid_combine")  # earlier tests' totals on the shared session
        _lib.call("capsmi_session_set_profiling_names", session.handle, b"hop2,no_such_timer")
        _run(session, sg, C3)
        assert launches(b"hop2") > 0 and launches(b"mid_combine") == 0
        _lib.call("capsmi_session_set_profiling_names", session.handle, None)
        _run(session, sg, C3)
        assert launches(b"hop2") > 0 and launches(b"mid_combine") > 0
    finally:
        _lib.call("capsmi_session_set_profiling", session.handle, 0)
        _lib.call("capsmi_session_set_profiling_names", session.handle, None)


@pytest.mark.parametrize("scale,kind", [(13, "all"), (16, "person")])
def test_c3_count_star_partitioned(session, scale, kind):
    """count(*) of C3 from the record partition (k_count.hip) equals the per-relationship atomic form and
    the oracle's closed form; at scale 16 a bucket's records span several blocks' chunk shares."""
    import os
    from oracle import cpu
    sg = _graph(session, scale, kind=kind)
    q = {"clauses": C3["clauses"], "return": {"items": [["n", ["count*"]]]}}
    got = _routed(session, "two_hop", lambda: _run(session, sg, q))
    with session.configured(CAPSMI_COUNT="atomic"):
        atomic = _run(session, sg, q)
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    pm = cpu.person_mask(n) if kind == "person" else np.ones(n, np.uint8)
    rows, _ = cpu.two_hop_closed_form_mt(n, src, dst, pm, pm, pm)
    assert got == atomic == [{"n": rows}]


def test_c3_unfused_equals_fused(session):
    sg = _graph(session, 8)
    assert _run(session, sg, C3, fused=False) == _run(session, sg, C3)


def test_c3_person_labels_routed(session):
    """Node scans of a label table with an id subset (Person = 3/4 of the ids)."""
    from oracle import cpu
    scale = 11
    sg = _graph(session, scale, kind="person")
    got = _routed(session, "two_hop", lambda: _run(session, sg, C3))
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    pm = cpu.person_mask(1 << scale)
    _, dist = cpu.two_hop_enumerate(1 << scale, src, dst, pm, pm, pm)
    assert got == [{"n": dist}]


def test_c2_projection_routed(session):
    """C2: MATCH (a:Person)-[r:FRIEND_OF]->(b:Person) WHERE a.age >= 18 AND a.age < 65 RETURN id(a), id(b)."""
    from capsmi.planner import Planner
    from oracle import cpu
    scale = 12
    sg = _graph(session, scale, kind="person")
    q = {"clauses": [{"match": "(a:Person)-[r:FRIEND_OF]->(b:Person)",
                      "where": ["and", [">=", ["prop", "a", "age"], ["lit", 18]], ["<", ["prop", "a", "age"], ["lit", 65]]]}],
         "return": {"items": [["a", ["id", "a"]], ["b", ["id", "b"]]]}}
    before = session.route_count("expand")
    t, outs = Planner(sg).run(q)
    fp = t.fingerprint([outs[0][2], outs[1][2]])
    assert session.route_count("expand") == before + 1
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    person, adult = cpu.c2_masks(n, 42)
    assert fp == cpu.expand_filter(src, dst, adult, person)
    session.set_fused(False)
    try:
        t2, outs2 = Planner(sg).run(q)
        assert t2.fingerprint([outs2[0][2], outs2[1][2]]) == fp
    finally:
        session.set_fused(True)


def test_c4_triangle_routed(session):
    from oracle import cpu
    scale = 9
    sg = _graph(session, scale)
    q = {"clauses": [{"match": "(a)-[r1:FRIEND_OF]->(b)-[r2:FRIEND_OF]->(c)-[r3:FRIEND_OF]->(a)"}],
         "return": {"items": [["n", ["count*"]]]}}
    got = _routed(session, "triangle", lambda: _run(session, sg, q))
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    assert got == [{"n": cpu.triangle_enumerate(1 << scale, src, dst)}]


@pytest.mark.parametrize("lo,hi", [(1, 3), (1, 1), (2, 3), (0, 3), (0, 1)])
def test_c5_var_length_routed(session, lo, hi):
    """lower = 0 adds the zero-length path of every start node (VarLengthExpandPlanner.scala:146-153)."""
    from oracle import cpu
    scale = 8
    sg = _graph(session, scale, ef=32, probs=(45, 15, 15), rtype="KNOWS")
    q = {"clauses": [{"match": f"(a:Person)-[:KNOWS*{lo}..{hi}]->(b:Person)"}],
         "return": {"items": [["a", ["id", "a"]], ["n", ["count*"]]]}}
    got = _routed(session, "var_length", lambda: _run(session, sg, q))
    src, dst = cpu.rmat_edges(scale, 0, 32 << scale, (45, 15, 15), 42)
    _, per_a = cpu.var_length_count(1 << scale, src, dst, max(lo, 1), hi)
    if lo == 0:
        per_a = per_a + 1
    want = [{"a": int(i), "n": int(per_a[i])} for i in np.nonzero(per_a)[0]]
    assert same_rows(got, want)
    if (lo, hi) in ((1, 3), (0, 3)) and scale <= 8:
        assert same_rows(_run(session, sg, q, fused=False), want)


@pytest.mark.parametrize("lo,hi", [(1, 4), (0, 4), (4, 4)])
def test_c5_four_hops_routed(session, lo, hi):
    """upper = 4 routes to the fused count on one device (var_length4) and equals enumeration."""
    from oracle import cpu
    scale = 6
    sg = _graph(session, scale, ef=32, probs=(45, 15, 15), rtype="KNOWS")
    q = {"clauses": [{"match": f"(a:Person)-[:KNOWS*{lo}..{hi}]->(b:Person)"}],
         "return": {"items": [["a", ["id", "a"]], ["n", ["count*"]]]}}
    got = _routed(session, "var_length", lambda: _run(session, sg, q))
    src, dst = cpu.rmat_edges(scale, 0, 32 << scale, (45, 15, 15), 42)
    _, per_a = cpu.var_length_count(1 << scale, src, dst, max(lo, 1), hi)
    if lo == 0:
        per_a = per_a + 1
    want = [{"a": int(i), "n": int(per_a[i])} for i in np.nonzero(per_a)[0]]
    assert same_rows(got, want)


def test_expand_count_routed(session):
    from oracle import cpu
    scale = 10
    sg = _graph(session, scale, kind="person")
    q = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]->(b:Person)"}], "return": {"items": [["n", ["count*"]]]}}
    got = _routed(session, "expand_count", lambda: _run(session, sg, q))
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    pm = cpu.person_mask(1 << scale).astype(bool)
    assert got == [{"n": int((pm[src] & pm[dst]).sum())}]


GOLDEN = all_cases()


@pytest.mark.parametrize("fname,case", GOLDEN, ids=[c["name"] for _, c in GOLDEN])
def test_golden_fused_and_unfused(session, fname, case):
    """Every golden vector through the lazy device plans, routed (default) and operator by operator."""
    from capsmi.table import StringDictionary
    session.dictionary = StringDictionary()
    got = run_planner(session, case)
    assert same_rows(got, case["expected"], case.get("ordered", False)), (got, case["expected"])
    session.set_fused(False)
    try:
        session.dictionary = StringDictionary()
        got2 = run_planner(session, case)
    finally:
        session.set_fused(True)
    assert same_rows(got2, case["expected"], case.get("ordered", False)), (got2, case["expected"])


def test_entity_table_contract(session):
    """EntityTable.verify at the boundary: Long non-null ids, canonical column order; Int ids widened
    to Long at ingest (DataFrameOps.withCypherCompatibleTypes); relType flattening."""
    import ctypes
    from capsmi import ColumnData, _lib
    from capsmi.expr import BOOL, I64, STR
    bad = session.table([ColumnData("id", I64, np.arange(3)), ColumnData("name", I64, np.arange(3)),
                         ColumnData("age", I64, np.arange(3))])
    with pytest.raises(_lib.IllegalArgumentException, match="Columns"):
        bad.as_node_table("id")  # properties not sorted
    assert bad.select("id", "age", "name").as_node_table("id").entity() == (1, 0, 3)
    nul = session.table([ColumnData("id", I64, np.arange(3), np.array([1, 0, 1], bool))])
    with pytest.raises(_lib.IllegalArgumentException, match="non-nullable"):
        nul.as_node_table("id")
    flt = session.table([ColumnData("id", 2, np.arange(3, dtype=np.float64))])
    with pytest.raises(_lib.IllegalArgumentException, match="CTInteger"):
        flt.as_node_table("id")
    t = session.table([ColumnData("id", I64, np.array([5, 9, 7])), ColumnData("age", I64, np.arange(3))])
    assert t.as_node_table("id").entity() == (1, 5, 10)
    # int32 ids arrive as Long
    ids32 = np.array([3, -4, 2**31 - 1], dtype=np.int32)
    descs = (_lib.ColDesc * 1)()
    descs[0].name, descs[0].type, descs[0].data, descs[0].valid = b"id", 16, ids32.ctypes.data, None
    out = ctypes.c_void_p()
    _lib.call("capsmi_table_from_host", session.handle, 1, descs, 3, ctypes.byref(out))
    from capsmi.table import GpuTable
    w = GpuTable(session, out)
    assert w.columnType == {"id": I64}
    np.testing.assert_array_equal(w.column("id").values, ids32.astype(np.int64))
    assert w.as_node_table("id").entity() == (1, -4, 2**31)
    # relationship type String column -> Boolean flags
    session.dictionary.extend(["KNOWS", "LIKES"])
    codes = [session.encode_str(x) for x in ["KNOWS", "LIKES", "KNOWS"]]
    r = session.table([ColumnData("id", I64, np.arange(3)), ColumnData("source", I64, np.zeros(3, np.int64)),
                       ColumnData("target", I64, np.ones(3, np.int64)), ColumnData("type", STR, np.array(codes))])
    f = r.flatten_rel_types("type", ["KNOWS", "LIKES"], ["KNOWS", "LIKES"])
    assert f.physicalColumns == ["id", "source", "target", "KNOWS", "LIKES"]
    assert f.columnType["KNOWS"] == BOOL
    np.testing.assert_array_equal(f.column("KNOWS").values, [1, 0, 1])
    assert f.as_rel_table("id", "source", "target", ["KNOWS", "LIKES"]).entity() == (2, 0, 2)


def test_lazy_schema_errors_at_call(session):
    """Operators stay lazy, but argument errors surface at the call (DataFrame analysis)."""
    from capsmi import ColumnData, _lib
    from capsmi.expr import I64
    t = session.table([ColumnData("a", I64, np.arange(5))])
    u = t.withColumnRenamed("a", "b").select("b")
    with pytest.raises(_lib.IllegalArgumentException):
        u.select("a")
    with pytest.raises(_lib.IllegalArgumentException):
        u.join(u, "inner", ("b", "b"))
    assert u.size == 5


@pytest.mark.parametrize("scale,kind", [(12, "all"), (14, "all"), (12, "person"), (16, "person"), (20, "all")])
def test_c3_grouped_routed(session, scale, kind):
    """C3's grouped form (RETURN id(a), count(DISTINCT c), the parity variant at s <= 14) and
    the grouped count(*), routed to the grouped 2-hop kernels (csrc/k_grouped.hip), against per-a
    enumeration (oracle/rmat.c orc_two_hop_enumerate), and the same plan operator by operator."""
    from oracle import cpu
    sg = _graph(session, scale, kind=kind)
    q = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person)"}],
         "return": {"items": [["a", ["id", "a"]], ["dc", ["count_distinct", ["id", "c"]]], ["n", ["count*"]]]}}
    got = _routed(session, "two_hop_grouped", lambda: _run(session, sg, q))
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    mask = np.ones(n, np.uint8) if kind == "all" else cpu.person_mask(n).astype(np.uint8)
    _, _, grows, gdist = cpu.two_hop_enumerate(n, src, dst, mask, mask, mask, grouped=True)
    want = [{"a": int(a), "dc": int(gdist[a]), "n": int(grows[a])} for a in np.nonzero(grows)[0]]
    assert same_rows(got, want)
    if scale == 12:
        assert same_rows(_run(session, sg, q, fused=False), want)
        with session.configured(CAPSMI_GROUPED="keys"):  # the per-binding key sort: the same rows
            assert same_rows(_run(session, sg, q), want)
