"""Run twice, same answer (SURVEY.md §5 determinism checks: two runs -> identical fingerprints).

Every query shape of the hot path runs twice on one session -- through the planner route and operator by
operator -- and the two results' order-insensitive fingerprints (capsmi_table_fingerprint: row count, sum and
xor of the row hashes) must be equal, and equal to the oracle where one is cheap.  The kernels use atomics
(slot order of hash inserts, chunk order of the partitions), so row ORDER may differ between runs; the row
multiset may not."""
import numpy as np
import pytest

from test_gpu_routing import _graph

pytestmark = pytest.mark.gpu

C2 = {"clauses": [{"match": "(a:Person)-[r:FRIEND_OF]->(b:Person)",
                   "where": ["and", [">=", ["prop", "a", "age"], ["lit", 18]], ["<", ["prop", "a", "age"], ["lit", 65]]]}],
      "return": {"items": [["a", ["id", "a"]], ["b", ["id", "b"]]]}}
C3 = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person)"}],
      "return": {"items": [["n", ["count*"]], ["dc", ["count_distinct", ["id", "c"]]]]}}
C3G = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person)"}],
       "return": {"items": [["a", ["id", "a"]], ["dc", ["count_distinct", ["id", "c"]]], ["n", ["count*"]]]}}
C4 = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person)-[:FRIEND_OF]->(a)"}],
      "return": {"items": [["n", ["count*"]]]}}
C5 = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF*1..3]->(b:Person)"}],
      "return": {"items": [["id", ["id", "a"]], ["count", ["count*"]]]}}


def _fp(session, sg, q, fused):
    from capsmi.planner import Planner
    session.set_fused(fused)
    try:
        t, outs = Planner(sg).run(q)
        return t.fingerprint([o[2] for o in outs]), t.size
    finally:
        session.set_fused(True)


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("name,q,kind,scale", [("c2", C2, "person", 13), ("c3", C3, "all", 11), ("c3g", C3G, "all", 10),
                                                ("c4", C4, "all", 10), ("c5", C5, "all", 9)])
def test_query_twice_same_fingerprint(session, name, q, kind, scale, fused):
    sg = _graph(session, scale, kind=kind)
    first = _fp(session, sg, q, fused)
    second = _fp(session, sg, q, fused)
    assert first == second, (name, first, second)
    if name == "c2" and fused:
        from oracle import cpu
        n = 1 << scale
        src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
        pm = cpu.person_mask(n)
        age = cpu.ages(np.arange(n))
        am = (pm.astype(bool) & (age >= 18) & (age < 65)).astype(np.uint8)
        assert first[0] == cpu.expand_filter(src, dst, am, pm)


def test_fused_and_unfused_agree_on_fingerprints(session):
    """The routed C2 expand and the same plan through the generic joins: one row multiset."""
    sg = _graph(session, 13, kind="person")
    assert _fp(session, sg, C2, True) == _fp(session, sg, C2, False)


def test_four_hops_twice_same_fingerprint(session):
    """The fused *1..4 count (the four-hop wedge tiles' atomics land in any order): one answer per run."""
    q = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF*1..4]->(b:Person)"}],
         "return": {"items": [["id", ["id", "a"]], ["count", ["count*"]]]}}
    sg = _graph(session, 10, kind="all")
    first = _fp(session, sg, q, True)
    assert first == _fp(session, sg, q, True)
    assert first[1] > 0
