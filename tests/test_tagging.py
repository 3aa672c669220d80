"""Multi-graph id tagging: Tags / TagSupport restatement, the tag expressions
on both backends, and UNION ALL graph scans.  Golden values from
spark-cypher-testing/src/test/scala/org/opencypher/spark/{api/TagsTest.scala,
impl/util/TagSupportTest.scala, impl/SparkSQLExprMapperTest.scala:59-72, impl/UnionGraphTest.scala,
impl/ScanGraphTest.scala:44-109}."""
import numpy as np
import pytest

from capsmi import tagging as tg
from capsmi.expr import Col, Lit
from capsmi.planner import PGNode, PGRel, PropertyGraph, ScanGraph, UnionGraph

BACKENDS = ["numpy", pytest.param("gpu", marks=pytest.mark.gpu)]


@pytest.fixture
def backend(request):
    from capsmi.table import StringDictionary
    if request.param == "numpy":
        from oracle.relational import NumpyBackend
        return NumpyBackend(StringDictionary())
    s = request.getfixturevalue("session")
    s.dictionary = StringDictionary()
    return s


def test_pick_free_tag():  # TagsTest.scala:35-45
    assert tg.pick_free_tag(set()) == 0
    assert tg.pick_free_tag({0}) == 1
    assert tg.pick_free_tag(set(range(tg.MAX_TAG))) == tg.MAX_TAG
    assert tg.pick_free_tag(set(range(1, tg.MAX_TAG + 1))) == 0
    with pytest.raises(tg.TagSpaceExhausted):
        tg.pick_free_tag(set(range(tg.MAX_TAG + 1)))


def test_replacements_for():  # TagSupportTest.scala:33-41
    assert tg.replacements_for({0}, {0}) == {0: 1}
    assert tg.replacements_for({0}, {1}) == {1: 1}
    assert tg.replacements_for({0, 1, 2}, {1}) == {1: 3}
    assert tg.replacements_for(set(), set()) == {}
    assert tg.replacements_for(set(), {1, 2, 3}) == {1: 1, 2: 2, 3: 3}
    assert tg.replacements_for({1, 2, 3}, {1, 2, 3}) == {1: 4, 2: 5, 3: 6}
    assert tg.replacements_for({1, 2, 3}, {0, 1}) == {0: 0, 1: 4}


def test_compute_retaggings():
    r = tg.compute_retaggings({"g1": {0}, "g2": {0}, "g3": {0, 1}})
    assert r == {"g1": {0: 0}, "g2": {0: 1}, "g3": {0: 2, 1: 3}}
    r = tg.compute_retaggings({"a": {0}, "b": {0}}, fixed={"a": {0: 5}})
    assert r == {"a": {0: 5}, "b": {0: 0}}


def test_long_tagging_roundtrip():
    rng = np.random.default_rng(1)
    for _ in range(200):
        i = int(rng.integers(0, 1 << 54))
        t = int(rng.integers(0, tg.MAX_TAG + 1))
        x = tg.set_tag(i, t)
        assert tg.get_tag(x) == t and (x & tg.INVERTED_TAG_MASK) == i
        assert tg.replace_tag(x, t, 7) == tg.set_tag(i, 7)
        assert tg.replace_tag(x, (t + 1) % 1024, 7) == x
    assert tg.set_tag(5, 1023) < 0  # the top tag bit is the Long sign bit


def _eval(backend, e, values):
    from capsmi.expr import I64
    from capsmi.table import ColumnData
    t = backend.table([ColumnData("x", I64, np.asarray(values, dtype=np.int64))])
    out = t.withColumns((e, "y")).column("y")
    return [None if (out.valid is not None and not out.valid[i]) else int(out.values[i]) for i in range(len(values))]


@pytest.mark.parametrize("backend", BACKENDS, indirect=True)
def test_tag_expressions(backend):
    # SparkSQLExprMapperTest.scala:59-72
    assert _eval(backend, tg.expr_get_tag(tg.expr_replace_tag(Lit(0), 0, 1)), [0]) == [1]
    assert _eval(backend, tg.expr_get_tag(tg.expr_replace_tags(tg.expr_set_tag(Lit(0), 1), {0: 1, 1: 2})), [0]) == [2]
    rng = np.random.default_rng(2)
    ids = [tg.set_tag(int(rng.integers(0, 1 << 54)), int(t)) for t in rng.integers(0, 6, 300)] + [-1, 0]
    rep = {0: 3, 2: 1023, 5: 0}
    got = _eval(backend, tg.expr_replace_tags(Col("x"), rep), ids)
    assert got == [tg.replace_tags(i, rep) for i in ids]
    assert _eval(backend, tg.expr_get_tag(Col("x")), ids) == [tg.get_tag(i) for i in ids]
    assert _eval(backend, tg.expr_set_tag(Col("x"), 9), ids) == [tg.set_tag(i, 9) for i in ids]


def _pg(nodes, rels):
    return PropertyGraph([PGNode(i, frozenset(l), p) for i, l, p in nodes],
                         [PGRel(i, s, d, t, p) for i, s, d, t, p in rels])


PERSONS = [(1, {"Person", "Swedish"}, {"name": "Mats", "luckyNumber": 23}),
           (2, {"Person"}, {"name": "Martin", "luckyNumber": 42}),
           (3, {"Person"}, {"name": "Max", "luckyNumber": 1337}),
           (4, {"Person"}, {"name": "Stefan", "luckyNumber": 9})]
KNOWS = [(1, 1, 2, "KNOWS", {"since": 2017}), (2, 1, 3, "KNOWS", {"since": 2016}), (3, 1, 4, "KNOWS", {"since": 2015}),
         (4, 2, 3, "KNOWS", {"since": 2016}), (5, 2, 4, "KNOWS", {"since": 2013}), (6, 3, 4, "KNOWS", {"since": 2016})]
BOOKS = [(10, {"Book"}, {"title": "1984", "year": 1949}), (20, {"Book"}, {"title": "Cryptonomicon", "year": 1999}),
         (30, {"Book"}, {"title": "The Eye of the World", "year": 1990}),
         (40, {"Book"}, {"title": "The Circle", "year": 2013})]
PROGRAMMERS = [(100, {"Person", "Programmer"}, {"name": "Alice", "luckyNumber": 42, "language": "C"}),
               (200, {"Person", "Programmer"}, {"name": "Bob", "luckyNumber": 23, "language": "D"}),
               (300, {"Person", "Programmer"}, {"name": "Eve", "luckyNumber": 84, "language": "F"}),
               (400, {"Person", "Programmer"}, {"name": "Carl", "luckyNumber": 49, "language": "R"})]
READS = [(100, 100, 10, "READS", {"recommends": True}), (200, 200, 40, "READS", {"recommends": True}),
         (300, 300, 30, "READS", {"recommends": True}), (400, 400, 20, "READS", {"recommends": False})]


def _rows(backend, table, header):
    from capsmi.expr import BOOL, F64, STR
    cols = {c.name: c for c in table.to_columns()}
    out = []
    for r in range(table.size):
        row = []
        for h in header:
            c = cols[h]
            if c.valid is not None and not c.valid[r]:
                row.append(None)
                continue
            v = c.values[r]
            row.append(bool(v) if c.type == BOOL else backend.dictionary.decode(int(v)) if c.type == STR
                       else float(v) if c.type == F64 else int(v))
        out.append(tuple(row))
    return sorted(out, key=repr)


@pytest.mark.parametrize("backend", BACKENDS, indirect=True)
def test_union_all_scans(backend):
    """ScanGraphTest "executes union": graph2's ids move to tag 1; labels and properties aligned."""
    p1, p2 = _pg(PERSONS, KNOWS), _pg(PROGRAMMERS + BOOKS, READS)
    # graphs loaded one after the other: graph 2's strings interleave graph 1's (stable codes)
    g1 = ScanGraph.from_property_graph(backend, p1)
    g2 = ScanGraph.from_property_graph(backend, p2)
    u = UnionGraph.union_all(backend, g1, g2)
    assert u.tags == {0, 1}
    t1 = lambda i: tg.set_tag(i, 1)  # noqa: E731
    nodes, header = u.node_scan("n", [])
    assert header == ["n", "n:Book", "n:Person", "n:Programmer", "n:Swedish", "n.language", "n.luckyNumber",
                      "n.name", "n.title", "n.year"]
    want = [(1, False, True, False, True, None, 23, "Mats", None, None),
            (2, False, True, False, False, None, 42, "Martin", None, None),
            (3, False, True, False, False, None, 1337, "Max", None, None),
            (4, False, True, False, False, None, 9, "Stefan", None, None),
            (t1(10), True, False, False, False, None, None, None, "1984", 1949),
            (t1(20), True, False, False, False, None, None, None, "Cryptonomicon", 1999),
            (t1(30), True, False, False, False, None, None, None, "The Eye of the World", 1990),
            (t1(40), True, False, False, False, None, None, None, "The Circle", 2013),
            (t1(100), False, True, True, False, "C", 42, "Alice", None, None),
            (t1(200), False, True, True, False, "D", 23, "Bob", None, None),
            (t1(300), False, True, True, False, "F", 84, "Eve", None, None),
            (t1(400), False, True, True, False, "R", 49, "Carl", None, None)]
    assert _rows(backend, nodes, header) == sorted(want, key=repr)
    rels, rh = u.rel_scan("r", [])
    cols = ["r.__src", "r", "r.__type", "r.__dst", "r.recommends", "r.since"]
    want = [(1, 1, "KNOWS", 2, None, 2017), (1, 2, "KNOWS", 3, None, 2016), (1, 3, "KNOWS", 4, None, 2015),
            (2, 4, "KNOWS", 3, None, 2016), (2, 5, "KNOWS", 4, None, 2013), (3, 6, "KNOWS", 4, None, 2016),
            (t1(100), t1(100), "READS", t1(10), True, None), (t1(200), t1(200), "READS", t1(40), True, None),
            (t1(300), t1(300), "READS", t1(30), True, None), (t1(400), t1(400), "READS", t1(20), False, None)]
    assert _rows(backend, rels, cols) == sorted(want, key=repr)


@pytest.mark.parametrize("backend", BACKENDS, indirect=True)
def test_union_of_a_graph_with_itself(backend):
    """UnionGraphTest "Returns only distinct results" / "supports UNION ALL": the second copy is
    retagged, so both copies survive the union's Distinct; a MATCH over the union sees both."""
    from capsmi.planner import Planner, result_rows
    g = ScanGraph.from_property_graph(backend, _pg(PERSONS, KNOWS))
    u = UnionGraph.union_all(backend, g, g)
    nodes, header = u.node_scan("n", ["Person"])
    ids = sorted(r[0] for r in _rows(backend, nodes, header))
    assert ids == sorted([1, 2, 3, 4] + [tg.set_tag(i, 1) for i in (1, 2, 3, 4)])
    q = {"clauses": [{"match": "(a:Person)-[r:KNOWS]->(b:Person)"}], "return": {"items": [["n", ["count*"]]]}}
    table, outs = Planner(u).run(q)
    assert result_rows(table, outs, backend.dictionary) == [{"n": 12}]
    # a union of unions: tags {0, 1} and {0, 1} -> the second member moves to {2, 3}
    uu = UnionGraph.union_all(backend, u, u)
    assert uu.tags == {0, 1, 2, 3}
    nodes, header = uu.node_scan("n", [])
    assert len(_rows(backend, nodes, header)) == 16


@pytest.mark.parametrize("backend", BACKENDS, indirect=True)
def test_union_deduplicates_within_a_member(backend):
    """The union's Distinct (UnionGraph.scala:77) removes a node listed twice in one member graph,
    which a plain scan keeps (ScanGraph.scala:72-76)."""
    dup = _pg([(1, {"A"}, {"v": 1}), (1, {"A"}, {"v": 1}), (2, {"A"}, {"v": 2})], [])
    g = ScanGraph.from_property_graph(backend, dup)
    plain, h = g.node_scan("n", ["A"])
    assert plain.size == 3
    u = UnionGraph.union_all(backend, g)
    nodes, h = u.node_scan("n", ["A"])
    assert _rows(backend, nodes, h) == [(1, True, 1), (2, True, 2)]
