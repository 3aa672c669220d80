"""The relational lowering (capsmi.planner over a Table backend) against the brute-force enumerator
(oracle/enumerate.py) on random small multigraphs with labels, types, null properties and
self-loops: expand, undirected expand, expand-into, var-length, OPTIONAL MATCH and EXISTS.  The
numpy restatement of the Table operators runs on CPU; the device operators behind the GPU mark."""
import numpy as np
import pytest

from golden_util import same_rows

BACKENDS = ["numpy", pytest.param("gpu", marks=pytest.mark.gpu)]

ID = lambda v: ["id", v]  # noqa: E731
V = lambda v: ["prop", v, "v"]  # noqa: E731

QUERIES = [
    {"clauses": [{"match": "(a)-[r]->(b)"}], "return": {"items": [["a", ID("a")], ["r", ID("r")], ["b", ID("b")]]}},
    {"clauses": [{"match": "(a:A)-[:R]->(b)-[:S]->(c)", "where": ["<", V("a"), V("c")]}],
     "return": {"items": [["a", ID("a")], ["b", ID("b")], ["c", ID("c")]]}},
    {"clauses": [{"match": "(a)-[r]-(b)"}], "return": {"items": [["a", ID("a")], ["r", ID("r")], ["b", ID("b")]]}},
    {"clauses": [{"match": "(a)-->(b)-->(c)-->(a)"}], "return": {"items": [["n", ["count*"]]]}},
    {"clauses": [{"match": "(a:A)-[*1..3]->(b)"}], "return": {"items": [["a", ID("a")], ["n", ["count*"]]]}},
    {"clauses": [{"match": "(a:A)"}, {"optional_match": "(a)-[:R]->(b:B)"}],
     "return": {"items": [["a", ID("a")], ["b", ID("b")]]}},
    {"clauses": [{"match": "(a)-->(b)", "where": ["exists", "(a)-->()-->(b)"]}],
     "return": {"items": [["a", ID("a")], ["b", ID("b")]]}},
    {"clauses": [{"match": "(a)"}],
     "return": {"items": [["a", ID("a")], ["e", ["exists", "(a)-[:S]->(x:B)", [">", V("x"), V("a")]]]]}},
    {"clauses": [{"match": "(a)-[r:R]->(b)", "where": ["not", ["exists", "(b)-[*1..2]->(a)"]]}],
     "return": {"items": [["a", ID("a")], ["r", ID("r")]]}},
    {"clauses": [{"match": "(a)-->(b)"}, {"match": "(b)-->(c)", "where": ["<>", ID("a"), ID("c")]}],
     "return": {"items": [["b", ID("b")], ["n", ["count*"]]]}},
    {"clauses": [{"match": "(a:A), (b:B)", "where": ["=", V("a"), V("b")]}],  # ValueJoin
     "return": {"items": [["a", ID("a")], ["b", ID("b")]]}},
    {"clauses": [{"match": "(a)-[r]->(c), (b)-->(d)", "where": ["and", ["=", V("b"), V("c")], ["<", V("a"), V("d")]]}],
     "return": {"items": [["a", ID("a")], ["r", ID("r")], ["b", ID("b")], ["d", ID("d")]]}},
    # entity values; grouping by an entity variable groups by every column it owns
    # (SparkTable.scala:128-133 header.ownedBy) -- and collect / collect(DISTINCT) (:169-177)
    {"clauses": [{"match": "(a)-[r]->(b)"}],
     "return": {"items": [["a", ["entity", "a"]], ["n", ["count*"]], ["bs", ["collect", ID("b")]]]}},
    {"clauses": [{"match": "(a:A)-[r:R]-(b)"}],
     "return": {"items": [["r", ["entity", "r"]], ["vs", ["collect_distinct", V("b")]], ["m", ["max", V("a")]]]}},
    {"clauses": [{"match": "(a:A)"}, {"optional_match": "(a)-[s:S]->(b)"}],
     "return": {"items": [["a", ["entity", "a"]], ["s", ["entity", "s"]], ["b", ["entity", "b"]]]}},
    {"clauses": [{"match": "(a)-->(b)-->(c)"}],
     "return": {"items": [["b", ["entity", "b"]], ["cs", ["collect_distinct", ID("c")]], ["vs", ["collect", V("a")]]]}},
]


def _graph(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(3, 9))
    nodes = []
    for i in range(n):
        labels = [l for l in ("A", "B") if rng.random() < 0.5]
        props = {} if rng.random() < 0.2 else {"v": int(rng.integers(0, 5))}
        nodes.append({"id": i, "labels": labels, "props": props})
    m = int(rng.integers(0, 3 * n))
    rels = []
    for j in range(m):
        s, d = int(rng.integers(0, n)), int(rng.integers(0, n))
        if rng.random() < 0.15:
            d = s  # self-loop
        rels.append({"id": n + j, "src": s, "dst": d, "type": "R" if rng.random() < 0.6 else "S", "props": {}})
    return {"nodes": nodes, "rels": rels}


@pytest.fixture
def backend(request):
    from capsmi.table import StringDictionary
    if request.param == "numpy":
        from oracle.relational import NumpyBackend
        return NumpyBackend(StringDictionary())
    s = request.getfixturevalue("session")
    s.dictionary = StringDictionary()
    return s


@pytest.mark.parametrize("backend", BACKENDS, indirect=True)
@pytest.mark.parametrize("seed", range(12))
def test_planner_matches_enumeration(backend, seed):
    from capsmi.planner import PGNode, PGRel, Planner, PropertyGraph, ScanGraph, result_rows
    from oracle import enumerate as en
    g = _graph(seed)
    pg = PropertyGraph([PGNode(x["id"], frozenset(x["labels"]), dict(x["props"])) for x in g["nodes"]],
                       [PGRel(r["id"], r["src"], r["dst"], r["type"], dict(r["props"])) for r in g["rels"]])
    graph = en.Graph(g)
    for q in QUERIES:
        sg = ScanGraph.from_property_graph(backend, pg)
        table, outs = Planner(sg).run(q)
        got = result_rows(table, outs, backend.dictionary)
        want = en.project(graph, en.match(graph, q), q["return"])
        assert same_rows(got, want), (q, got, want)


@pytest.mark.parametrize("backend", BACKENDS, indirect=True)
def test_entity_grouping_keeps_owned_columns(backend):
    """Node id 0 sits in two node tables (labels {A} and {B}, different `v`): a label-free node scan
    yields it twice (ScanGraph.scala:72-76), and grouping by the variable groups by every column it
    owns -- id, label flags, properties (SparkTable.scala:128-133) -- so the two rows stay two groups
    (grouping by the id column alone would merge them into one group of 2)."""
    from capsmi.expr import BOOL, I64
    from capsmi.planner import ID as IDC, EntityTable, Planner, ScanGraph, result_rows
    from capsmi.table import ColumnData
    A = backend.table([ColumnData(IDC, I64, np.array([0, 1])), ColumnData("v", I64, np.array([10, 11]))])
    B = backend.table([ColumnData(IDC, I64, np.array([0])), ColumnData("v", I64, np.array([20]))])
    nodes = [EntityTable("node", frozenset({"A"}), {"v": I64}, A.as_node_table(IDC)),
             EntityTable("node", frozenset({"B"}), {"v": I64}, B.as_node_table(IDC))]
    sg = ScanGraph(backend, nodes, [])
    q = {"clauses": [{"match": "(a)"}], "return": {"items": [["a", ["entity", "a"]], ["n", ["count*"]]]}}
    table, outs = Planner(sg).run(q)
    got = result_rows(table, outs, backend.dictionary)
    want = [{"a": {"id": 0, "labels": ["A"], "props": {"v": 10}}, "n": 1},
            {"a": {"id": 0, "labels": ["B"], "props": {"v": 20}}, "n": 1},
            {"a": {"id": 1, "labels": ["A"], "props": {"v": 11}}, "n": 1}]
    assert same_rows(got, want), got
    q2 = {"clauses": [{"match": "(a)"}], "return": {"items": [["a", ID("a")], ["n", ["count*"]]]}}
    table, outs = Planner(sg).run(q2)  # grouping by id(a), an expression: one group per id
    assert same_rows(result_rows(table, outs, backend.dictionary), [{"a": 0, "n": 2}, {"a": 1, "n": 1}])
