"""Pin the fused path's checker (oracle/rmat.c enumeration, oracle/closed.c closed forms) to the
golden-pinned enumerator (oracle/enumerate.py, itself pinned by the reference's own assertions in
tests/test_golden_oracle.py).  CPU only.

For every graph -- the CREATE graph of every golden case (the reference's own test graphs) and
random multigraphs with self-loops, multi-edges and labels -- and for every relationship-type
restriction and node label, the C checker must equal enumerate.py on:
  C3 shape  MATCH (a:L)-[:T]->(b:L)-[:T]->(c:L) RETURN count(*), count(DISTINCT c)
            MATCH (a:L)-[:T]-(b:L)-[:T]-(c:L) RETURN count(*), count(DISTINCT c), count(DISTINCT a)
  C4 shape  MATCH (a:L)-[:T]->(b:L)-[:T]->(c:L)-[:T]->(a) RETURN count(*)
  C5 shape  MATCH (a:L)-[:T*lo..hi]->(b:L) RETURN id(a), count(*)
"""
import numpy as np
import pytest

from golden_util import all_cases, property_graph

CASES = [c for _, c in all_cases()]


def _random_graph(seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(2, 14))
    nodes = [{"id": i, "labels": [l for l in ("A", "B") if rng.random() < 0.6], "props": {}} for i in range(n)]
    m = int(rng.integers(0, 4 * n))
    rels = []
    for j in range(m):
        s, d = int(rng.integers(0, n)), int(rng.integers(0, n))
        if rng.random() < 0.2:
            d = s  # self-loop
        rels.append({"id": n + j, "src": s, "dst": d, "type": "R" if rng.random() < 0.7 else "S", "props": {}})
    if m and rng.random() < 0.5:  # multi-edges and reciprocal pairs
        for r in list(rels[: m // 3]):
            rels.append({"id": n + len(rels), "src": r["src"], "dst": r["dst"], "type": r["type"], "props": {}})
            rels.append({"id": n + len(rels), "src": r["dst"], "dst": r["src"], "type": r["type"], "props": {}})
    return {"nodes": nodes, "rels": rels}


def _dense(g, label, rtype):
    """rmat.c inputs: dense id domain [0, max id], a node mask (node exists and carries `label`), the
    relationship columns of type `rtype` (all when None)."""
    ids = [x["id"] for x in g["nodes"]] + [r["id"] for r in g["rels"]] + [0]
    n = max(ids) + 1
    mask = np.zeros(n, dtype=np.uint8)
    for x in g["nodes"]:
        if label is None or label in x["labels"]:
            mask[x["id"]] = 1
    rs = [r for r in g["rels"] if rtype is None or r["type"] == rtype]
    src = np.array([r["src"] for r in rs], dtype=np.int64)
    dst = np.array([r["dst"] for r in rs], dtype=np.int64)
    return n, mask, src, dst


def _enum(g, pattern, items):
    from oracle import enumerate as en
    graph = en.Graph(g)
    q = {"clauses": [{"match": pattern}], "return": {"items": items}}
    return en.project(graph, en.match(graph, q), q["return"])


def _restrictions(g):
    labels = sorted({l for x in g["nodes"] for l in x["labels"]})[:3]
    types = sorted({r["type"] for r in g["rels"]})[:3]
    return [(l, t) for l in [None] + labels for t in [None] + types]


def _pat(label, rtype):
    lab = f":{label}" if label else ""
    ty = f"[:{rtype}]" if rtype else "[]"
    return lab, ty


def _check_graph(g):
    from oracle import cpu
    for label, rtype in _restrictions(g):
        n, mask, src, dst = _dense(g, label, rtype)
        lab, ty = _pat(label, rtype)
        # C3
        want = _enum(g, f"(a{lab})-{ty}->(b{lab})-{ty}->(c{lab})",
                     [["rows", ["count*"]], ["dist", ["count_distinct", ["id", "c"]]]])[0]
        expect = (want["rows"], want["dist"])
        assert cpu.two_hop_enumerate(n, src, dst, mask, mask, mask) == expect, (label, rtype)
        assert cpu.two_hop_closed_form(n, src, dst, mask, mask, mask) == expect, (label, rtype)
        assert cpu.two_hop_closed_form_mt(n, src, dst, mask, mask, mask, threads=2) == expect, (label, rtype)
        # C3 undirected: outgoing + incoming-without-self-loops per hop, r1 <> r2
        want = _enum(g, f"(a{lab})-{ty}-(b{lab})-{ty}-(c{lab})",
                     [["rows", ["count*"]], ["dc", ["count_distinct", ["id", "c"]]],
                      ["da", ["count_distinct", ["id", "a"]]]])[0]
        assert cpu.two_hop_undirected_enumerate(n, src, dst, mask, mask, mask) == (want["rows"], want["dc"], want["da"]), \
            (label, rtype)
        assert cpu.two_hop_undirected_closed_form(n, src, dst, mask, mask, mask, threads=2) == \
            (want["rows"], want["dc"]), (label, rtype)
        # C4 (rmat.c enumeration has no node mask: keep the relationships with both ends in the scan)
        want = _enum(g, f"(a{lab})-{ty}->(b{lab})-{ty}->(c{lab})-{ty}->(a)", [["rows", ["count*"]]])[0]["rows"]
        keep = (mask[src] != 0) & (mask[dst] != 0) if len(src) else np.zeros(0, bool)
        assert cpu.triangle_enumerate(n, src[keep], dst[keep]) == want, (label, rtype)
        assert cpu.triangle_closed_form(n, src, dst, mask) == want, (label, rtype)
        # C5
        for lo, hi in [(1, 1), (1, 2), (1, 3), (2, 3), (3, 3), (2, 2)]:
            rows = _enum(g, f"(a{lab})-{ty[:-1] if rtype else '['}*{lo}..{hi}]->(b{lab})",
                         [["a", ["id", "a"]], ["n", ["count*"]]])
            want = {r["a"]: r["n"] for r in rows}
            tot, per_a = cpu.var_length_count(n, src, dst, lo, hi, mask, mask)
            got = {int(i): int(per_a[i]) for i in np.nonzero(per_a)[0]}
            assert got == want and tot == sum(want.values()), (label, rtype, lo, hi)
            tot2, per_a2 = cpu.var_length_closed_form(n, src, dst, lo, hi, mask, mask)
            np.testing.assert_array_equal(per_a2, per_a)
            assert tot2 == tot


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_checker_on_reference_graphs(case):
    """The reference's own test graphs (ids as CreateQueryParser assigns them)."""
    _, g = property_graph(case)
    _check_graph(g)


@pytest.mark.parametrize("seed", range(16))
def test_checker_on_random_multigraphs(seed):
    _check_graph(_random_graph(seed))


@pytest.mark.parametrize("seed", range(12))
def test_checker_on_planner_random_graphs(seed):
    """The 12 random multigraphs of tests/test_planner_random.py."""
    from test_planner_random import _graph
    _check_graph(_graph(seed))


@pytest.mark.parametrize("scale,probs,ef", [(9, (57, 19, 19), 16), (8, (45, 15, 15), 32)])
def test_closed_forms_equal_enumeration_on_rmat(scale, probs, ef):
    """R-MAT inputs (hubs, many multi-edges and reciprocal pairs): closed forms = enumeration."""
    from oracle import cpu
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, ef << scale, probs, 7)
    person, adult = cpu.c2_masks(n, 42)
    for a_ok, b_ok in [(None, None), (person, person), (adult, person)]:
        assert cpu.two_hop_closed_form_mt(n, src, dst, a_ok, b_ok, b_ok) == \
            cpu.two_hop_enumerate(n, src, dst, a_ok, b_ok, b_ok)
        assert cpu.two_hop_undirected_closed_form(n, src, dst, a_ok, b_ok, b_ok) == \
            cpu.two_hop_undirected_enumerate(n, src, dst, a_ok, b_ok, b_ok)[:2]
        assert cpu.two_hop_undirected_closed_form(n, src, dst, b_ok, a_ok, person) == \
            cpu.two_hop_undirected_enumerate(n, src, dst, b_ok, a_ok, person)[:2]
        tot, g = cpu.var_length_count(n, src, dst, 1, 3, a_ok, b_ok)
        tot2, g2 = cpu.var_length_closed_form(n, src, dst, 1, 3, a_ok, b_ok)
        assert tot == tot2
        np.testing.assert_array_equal(g, g2)
    keep = (person[src] != 0) & (person[dst] != 0)
    assert cpu.triangle_closed_form(n, src, dst) == cpu.triangle_enumerate(n, src, dst)
    assert cpu.triangle_closed_form(n, src, dst, person) == cpu.triangle_enumerate(n, src[keep], dst[keep])


@pytest.mark.parametrize("seed", range(24))
def test_var_length4_closed_form_equals_enumeration(seed):
    """The 4-hop relationship-distinct path count per start node (inclusion-exclusion, oracle/cpu.py) equals
    path enumeration on random multigraphs with self-loops, reciprocal pairs and node filters -- and *1..4 is
    the closed forms for 1..3 plus it (the count-only form's first step)."""
    from oracle import cpu
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 14))
    m = int(rng.integers(0, 45))
    src = rng.integers(0, n, m).astype(np.int64)
    dst = rng.integers(0, n, m).astype(np.int64)
    src[: m // 5] = dst[: m // 5]
    if m >= 12:  # three relationships reversed: reciprocal pairs
        k = m // 5
        src[-3:], dst[-3:] = dst[k:k + 3].copy(), src[k:k + 3].copy()
    a_ok = None if seed % 3 == 0 else (rng.random(n) < 0.8).astype(np.uint8)
    b_ok = None if seed % 4 == 0 else (rng.random(n) < 0.7).astype(np.uint8)
    tot, per = cpu.var_length_count(n, src, dst, 4, 4, a_ok, b_ok)
    tot4, per4 = cpu.var_length4_closed_form(n, src, dst, a_ok, b_ok)
    np.testing.assert_array_equal(per4, per)
    assert tot4 == tot
    tot14, per14 = cpu.var_length_count(n, src, dst, 1, 4, a_ok, b_ok)
    tot13, per13 = cpu.var_length_closed_form(n, src, dst, 1, 3, a_ok, b_ok)
    np.testing.assert_array_equal(per13 + per4, per14)


@pytest.mark.parametrize("scale,probs,ef", [(7, (57, 19, 19), 16), (6, (45, 15, 15), 32)])
def test_var_length4_closed_form_on_rmat(scale, probs, ef):
    from oracle import cpu
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, ef << scale, probs, 7)
    person, adult = cpu.c2_masks(n, 42)
    for a_ok, b_ok in [(None, None), (adult, person)]:
        tot, per = cpu.var_length_count(n, src, dst, 4, 4, a_ok, b_ok)
        tot4, per4 = cpu.var_length4_closed_form(n, src, dst, a_ok, b_ok)
        np.testing.assert_array_equal(per4, per)


def test_c2_masks_match_scalar_definition():
    from oracle import cpu
    n = 4096
    person, adult = cpu.c2_masks(n, 42)
    np.testing.assert_array_equal(person, cpu.person_mask(n))
    age = cpu.ages(np.arange(n))
    np.testing.assert_array_equal(adult, (person.astype(bool) & (age >= 18) & (age < 65)).astype(np.uint8))
