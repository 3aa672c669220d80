"""File-system CSV graph source (capsmi/fs.py) on the reference's own example graph
(spark-cypher-examples/src/main/resources/csv/products, copied as a fixture under tests/golden/fs),
checked against CypherSQLRoundtripExample's recorded output
(spark-cypher-examples/src/main/resources/example_outputs/CypherSQLRoundtripExample.out)."""
import os

import pytest

from golden_util import same_rows

HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCTS = os.path.join(HERE, "golden", "fs", "products")

# CypherSQLRoundtripExample.scala:50-71: persons (CaseClassExample.scala:67-71) as the driving table
# `SELECT age, name FROM people`, then
#   MATCH (c:Customer {name: name})-->(p:Product) RETURN c.name, age, p.title
QUERY = {"driving": {"age": [10, 20, 15], "name": ["Alice", "Bob", "Carol"]},
         "clauses": [{"match": "(c:Customer)-->(p:Product)", "where": ["=", ["prop", "c", "name"], ["var", "name"]]}],
         "return": {"items": [["c.name", ["prop", "c", "name"]], ["age", ["var", "age"]],
                              ["p.title", ["prop", "p", "title"]]]}}
EXPECTED = [{"c.name": "Carol", "age": 15, "p.title": "Jurassic Park"},
            {"c.name": "Alice", "age": 10, "p.title": "1984"},
            {"c.name": "Carol", "age": 15, "p.title": "Shakira"},
            {"c.name": "Alice", "age": 10, "p.title": "Terminator 2"}]


def _run(backend):
    from capsmi.fs import fs_graph
    from capsmi.planner import Planner, result_rows
    sg = fs_graph(backend, PRODUCTS, extra_strings=QUERY["driving"]["name"])
    table, outs = Planner(sg).run(QUERY)
    return sg, result_rows(table, outs, backend.dictionary)


def test_schema_and_tables_cpu():
    from capsmi.fs import fs_graph, read_schema
    from capsmi.expr import I64, STR
    from capsmi.table import StringDictionary
    from oracle.relational import NumpyBackend
    nodes, rels = read_schema(PRODUCTS)
    assert dict(nodes)[frozenset(["Product"])] == {"title": STR, "rank": I64, "category": STR}
    assert dict(rels)["BOUGHT"] == {"rating": I64, "helpful": I64, "votes": I64}
    sg = fs_graph(NumpyBackend(StringDictionary()), PRODUCTS)
    sizes = {tuple(sorted(t.labels)): t.table.size for t in sg.nodes + sg.rels}
    assert sizes == {("Customer",): 12, ("Product",): 16, ("BOUGHT",): 8}


def test_roundtrip_example_cpu_oracle():
    from capsmi.table import StringDictionary
    from oracle.relational import NumpyBackend
    _, got = _run(NumpyBackend(StringDictionary()))
    assert same_rows(got, EXPECTED), got


@pytest.mark.gpu
def test_roundtrip_example_gpu(session):
    _, got = _run(session)
    assert same_rows(got, EXPECTED), got
