"""Shared helpers: build a CAPS-style scan graph from a golden case and compare result bags."""
import json
import math
import os
from collections import Counter

HERE = os.path.dirname(os.path.abspath(__file__))


def load_cases(name):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)["cases"]


def all_cases():
    return [(f, c) for f in ("acceptance.json", "predicates.json") for c in load_cases(f)]


def property_graph(case):
    """PropertyGraph of a golden case (CREATE text + optional explicit relationships)."""
    from capsmi.planner import PGNode, PGRel, PropertyGraph
    from oracle.create_graph import create_graph
    g = create_graph(case["create"])
    rels = case.get("rels", g["rels"])
    return PropertyGraph([PGNode(n["id"], frozenset(n["labels"]), dict(n["props"])) for n in g["nodes"]],
                         [PGRel(r["id"], r["src"], r["dst"], r["type"], dict(r["props"])) for r in rels]), \
        {"nodes": g["nodes"], "rels": rels}


def _norm(v):
    if isinstance(v, float):
        return ("f", round(v, 9))
    if isinstance(v, bool):
        return ("b", v)
    if isinstance(v, list):
        return ("l", tuple(_norm(x) for x in v))
    if isinstance(v, dict):  # node / relationship values
        return ("d", tuple(sorted((k, _norm(x)) for k, x in v.items())))
    return ("v", v)


def bag(rows):
    return Counter(tuple(sorted((k, _norm(v)) for k, v in r.items())) for r in rows)


def same_rows(got, expected, ordered=False):
    if ordered:
        return [bag([g]) for g in got] == [bag([e]) for e in expected]
    return bag(got) == bag(expected)


def run_planner(backend, case):
    from capsmi.planner import Planner, ScanGraph, result_rows
    pg, _ = property_graph(case)
    sg = ScanGraph.from_property_graph(backend, pg)
    table, outs = Planner(sg).run(case["query"])
    return result_rows(table, outs, backend.dictionary)


def approx_equal(a, b):
    if isinstance(a, float) or isinstance(b, float):
        return a is not None and b is not None and math.isclose(a, b, rel_tol=1e-9)
    return a == b
