"""StringDictionary: order-preserving AND stable codes (a string keeps its code when later graphs,
driving tables or literals add strings).  CPU only."""
import random

import pytest


def test_codes_stable_and_ordered_under_insertion():
    from capsmi.table import StringDictionary
    d = StringDictionary(["Bob", "Dave"])
    before = {s: d.encode(s) for s in ("Bob", "Dave")}
    rnd = random.Random(3)
    words = ["".join(rnd.choice("abcBDE") for _ in range(rnd.randint(1, 6))) for _ in range(400)]
    for k in range(0, len(words), 37):  # many batches, interleaving the known strings
        d.extend(words[k:k + 37])
        assert {s: d.encode(s) for s in before} == before
    allw = sorted(set(words) | set(before))
    codes = [d.encode(w) for w in allw]
    assert codes == sorted(codes) and len(set(codes)) == len(codes)
    assert all(d.decode(d.encode(w)) == w for w in allw)


def test_unknown_literals_get_distinct_codes():
    """'Bob' and 'Bobby' between the same neighbours must not share a code."""
    from capsmi.table import StringDictionary
    d = StringDictionary(["Alice", "Carol"])
    a, b = d.encode("Bob"), d.encode("Bobby")
    assert a != b and d.encode("Alice") < a < b < d.encode("Carol")
    assert d.decode(a) == "Bob" and d.decode(b) == "Bobby"


def test_gap_exhaustion_raises_instead_of_renumbering():
    from capsmi.table import StringDictionary
    d = StringDictionary(["a", "b"])
    s = "a"
    with pytest.raises(OverflowError):
        for _ in range(200):  # each new string sits between "a..." and the previous one: halving gaps
            s = s + "a"
            d.extend([s])
            d.extend([s[:-1] + "0"])


def test_two_graphs_loaded_one_after_the_other():
    """Load g1, then g2 whose strings interleave g1's; g1's queries still decode and compare right."""
    from capsmi.planner import PGNode, PGRel, Planner, PropertyGraph, ScanGraph, result_rows
    from capsmi.table import StringDictionary
    from oracle.relational import NumpyBackend
    be = NumpyBackend(StringDictionary())
    g1 = PropertyGraph([PGNode(0, frozenset({"P"}), {"name": "Bob"}), PGNode(1, frozenset({"P"}), {"name": "Dave"})],
                       [PGRel(2, 0, 1, "K")])
    s1 = ScanGraph.from_property_graph(be, g1)
    g2 = PropertyGraph([PGNode(0, frozenset({"P"}), {"name": "Carol"}), PGNode(1, frozenset({"P"}), {"name": "Ann"})],
                       [PGRel(2, 1, 0, "K")])
    ScanGraph.from_property_graph(be, g2)
    q = {"clauses": [{"match": "(a:P)-[:K]->(b:P)", "where": ["<", ["prop", "a", "name"], ["lit", "Carl"]]}],
         "return": {"items": [["a", ["prop", "a", "name"]], ["b", ["prop", "b", "name"]]],
                    "order_by": [["a", "asc"]]}}
    t, outs = Planner(s1).run(q)
    assert result_rows(t, outs, be.dictionary) == [{"a": "Bob", "b": "Dave"}]
    q2 = {"clauses": [{"match": "(a:P)"}], "return": {"items": [["n", ["prop", "a", "name"]]],
                                                       "order_by": [["n", "desc"]]}}
    t, outs = Planner(s1).run(q2)
    assert [r["n"] for r in result_rows(t, outs, be.dictionary)] == ["Dave", "Bob"]


def test_driving_table_strings_are_registered():
    """strings of a driving table that the graph does not hold still compare and decode."""
    from capsmi.planner import PGNode, Planner, PropertyGraph, ScanGraph, result_rows
    from capsmi.table import StringDictionary
    from oracle.relational import NumpyBackend
    be = NumpyBackend(StringDictionary())
    sg = ScanGraph.from_property_graph(be, PropertyGraph([PGNode(0, frozenset({"P"}), {"name": "Bob"})], []))
    q = {"driving": {"x": ["Bobby", "Bo"]}, "clauses": [{"match": "(a:P)", "where": ["<", ["var", "x"], ["prop", "a", "name"]]}],
         "return": {"items": [["x", ["var", "x"]]]}}
    t, outs = Planner(sg).run(q)
    assert result_rows(t, outs, be.dictionary) == [{"x": "Bo"}]


def test_driving_table_floats_keep_their_type():
    """A driving-table column with a float is Double, not truncated to Long."""
    from capsmi.planner import PGNode, Planner, PropertyGraph, ScanGraph, result_rows
    from capsmi.table import StringDictionary
    from oracle.relational import NumpyBackend
    be = NumpyBackend(StringDictionary())
    sg = ScanGraph.from_property_graph(be, PropertyGraph([PGNode(0, frozenset({"P"}), {"v": 2})], []))
    q = {"driving": {"x": [1.5, 2]}, "clauses": [{"match": "(a:P)", "where": ["<", ["var", "x"], ["prop", "a", "v"]]}],
         "return": {"items": [["x", ["var", "x"]]]}}
    t, outs = Planner(sg).run(q)
    assert result_rows(t, outs, be.dictionary) == [{"x": 1.5}]
