"""Brute-force MATCH enumeration over an in-memory property graph -- TEST INFRASTRUCTURE ONLY.

An independent restatement of the bindings CAPS produces for a MATCH, written as nested loops over
nodes and relationships instead of relational joins.  It is used to cross-check the relational
lowering (capsmi.planner + device Table operators) on random graphs.  Semantics, each pinned by
the reference:
  - node scan rows = nodes carrying all required labels (ScanGraph.scala:61-96)
  - directed hop: one binding per relationship (multigraph, self-loops kept)
  - undirected hop to a new node: outgoing + incoming with self-loops only once
    (RelationalPlanner.scala:126-136)
  - hop between two bound nodes (ExpandInto): directed join on both ends; undirected: both
    orientations; a cyclic (a)--(a) hop is directed (RelationalPlanner.scala:139-154,
    LogicalPlanner.scala:509-514)
  - directed var-length: edge-distinct paths of length lower..upper; the first hop also differs
    from every relationship bound before the expand (VarLengthExpandPlanner.scala:83-136)
  - uniqueness: NOT(r_i = r_j) for single-length relationships of one MATCH with overlapping types
  - WHERE: three-valued logic, a row survives only if TRUE
  - EXISTS(pattern): some extension of the row's binding matches the pattern (its var-length first
    hop, like any, avoids the relationships already bound) (RelationalPlanner.scala:181-202)
"""
from __future__ import annotations

from typing import Dict, List, Optional

from capsmi.planner import NodePat, RelPat, _Names, parse_pattern  # pattern text parser (front-end stand-in)


class Graph:
    def __init__(self, g: dict):
        self.nodes = {n["id"]: n for n in g["nodes"]}
        self.rels = {r["id"]: r for r in g["rels"]}
        self.out: Dict[int, List[dict]] = {i: [] for i in self.nodes}
        self.inc: Dict[int, List[dict]] = {i: [] for i in self.nodes}
        for r in g["rels"]:
            self.out.setdefault(r["src"], []).append(r)
            self.inc.setdefault(r["dst"], []).append(r)


def _type_ok(r, types):
    return not types or r["type"] in types


def _labels_ok(g: Graph, nid, labels):
    return set(labels) <= set(g.nodes[nid]["labels"])


def _cmp(a, b):
    if a is None or b is None:
        return None
    num = lambda x: isinstance(x, (int, float)) and not isinstance(x, bool)  # noqa: E731
    if num(a) and num(b):
        return (a > b) - (a < b)
    if type(a) is not type(b):
        return None
    return (a > b) - (a < b)


def eval_expr(spec, b: dict, g: Graph):
    op = spec[0]
    if op == "prop":
        v = b.get(spec[1])
        if v is None:
            return None
        ent = g.rels.get(v) if isinstance(b.get("__kind_" + spec[1]), str) and b["__kind_" + spec[1]] == "rel" \
            else g.nodes.get(v)
        return ent["props"].get(spec[2]) if ent else None
    if op in ("var", "id"):
        return b.get(spec[1])
    if op == "entity":  # CAPSNode / CAPSRelationship value (null properties left out)
        v = b.get(spec[1])
        if v is None:
            return None
        if b.get("__kind_" + spec[1]) == "rel":
            r = g.rels[v]
            return {"id": v, "src": r["src"], "dst": r["dst"], "type": r["type"],
                    "props": {k: x for k, x in sorted(r["props"].items()) if x is not None}}
        n = g.nodes[v]
        return {"id": v, "labels": sorted(n["labels"]),
                "props": {k: x for k, x in sorted(n["props"].items()) if x is not None}}
    if op == "type":
        v = b.get(spec[1])
        return None if v is None else g.rels[v]["type"]
    if op == "lit":
        return spec[1]
    if op == "haslabel":
        v = b.get(spec[1])
        return None if v is None else spec[2] in g.nodes[v]["labels"]
    if op in ("=", "<>", "<", "<=", ">", ">="):
        c = _cmp(eval_expr(spec[1], b, g), eval_expr(spec[2], b, g))
        if c is None:
            return None
        return {"=": c == 0, "<>": c != 0, "<": c < 0, "<=": c <= 0, ">": c > 0, ">=": c >= 0}[op]
    if op == "not":
        v = eval_expr(spec[1], b, g)
        return None if v is None else not v
    if op in ("and", "or"):
        vals = [eval_expr(s, b, g) for s in spec[1:]]
        if op == "and":
            return False if any(v is False for v in vals) else (None if any(v is None for v in vals) else True)
        return True if any(v is True for v in vals) else (None if any(v is None for v in vals) else False)
    if op == "isnull":
        return eval_expr(spec[1], b, g) is None
    if op == "isnotnull":
        return eval_expr(spec[1], b, g) is not None
    if op == "in":
        x = eval_expr(spec[1], b, g)
        if x is None:
            return None
        hits = [_cmp(x, v) for v in spec[2]]
        if any(h == 0 for h in hits):
            return True
        return None if any(h is None for h in hits) else False
    if op == "exists":  # some extension of b matches the pattern (and its WHERE)
        sub = {"clauses": [{"match": spec[1], "where": spec[2] if len(spec) > 2 else None, "unique": False}]}
        return bool(match(g, sub, rows=[b], names=_SubNames()))
    if op in ("+", "-", "*"):
        a, c = eval_expr(spec[1], b, g), eval_expr(spec[2], b, g)
        if a is None or c is None:
            return None
        return a + c if op == "+" else (a - c if op == "-" else a * c)
    raise ValueError(f"expression {spec!r}")


class _SubNames(_Names):
    """fresh names of an EXISTS pattern, apart from the outer query's"""
    _n = 0

    def fresh(self, kind: str) -> str:
        _SubNames._n += 1
        return f"_x{kind}{_SubNames._n}"


def match(g: Graph, query: dict, rows: Optional[List[dict]] = None, names: Optional[_Names] = None) -> List[dict]:
    names = names or _Names()
    rows = rows if rows is not None else [dict()]
    bound_rels_order: List[str] = [v for v in (rows[0] if rows else {}) if rows[0].get("__kind_" + v) == "rel"]
    for clause in query["clauses"]:
        optional = "optional_match" in clause
        pattern = clause["optional_match"] if optional else clause["match"]
        paths = parse_pattern(pattern, names)
        clause_rels: List[RelPat] = []
        per_row = [_clause(g, b, list(paths), clause_rels, bound_rels_order) for b in rows]
        # uniqueness (single-length, overlapping types)
        singles = []
        seen = set()
        for r in (clause_rels if clause.get("unique", True) else []):  # no uniqueness inside EXISTS
            if r.var_length is None and r.var not in seen:
                seen.add(r.var)
                singles.append(r)

        def keep(b):
            for i in range(len(singles)):
                for j in range(i + 1, len(singles)):
                    x, y = singles[i], singles[j]
                    if x.types and y.types and not (set(x.types) & set(y.types)):
                        continue
                    if b[x.var] == b[y.var]:
                        return False
            return clause.get("where") is None or eval_expr(clause["where"], b, g) is True

        out = []
        has_fields = any(k for b in rows for k in b if not k.startswith("__"))
        pattern_vars = [e.var for p in paths for e in p]
        for b, ext in zip(rows, per_row):
            ext = [e for e in ext if keep(e)]
            if optional and has_fields and not ext:  # OPTIONAL MATCH keeps the row, new variables null
                nb = dict(b)
                for v in pattern_vars:
                    nb.setdefault(v, None)
                out.append(nb)
            else:
                out.extend(ext)
        rows = out
        for r in clause_rels:
            if r.var not in bound_rels_order:
                bound_rels_order.append(r.var)
    return rows


def _clause(g: Graph, b: dict, pending: list, clause_rels: list, bound_rels_order: list):
    # same component order as the planner: a path touching a bound node first
    if not pending:
        return [b]
    idx = next((i for i, p in enumerate(pending) if any(isinstance(e, NodePat) and e.var in b for e in p)), 0)
    path = pending[idx]
    rest = pending[:idx] + pending[idx + 1:]
    for e in path:
        if isinstance(e, RelPat) and all(e.var != r.var for r in clause_rels):
            clause_rels.append(e)
    out = []
    for b2 in _path(g, b, path, 0, bound_rels_order):
        out.extend(_clause(g, b2, rest, clause_rels, bound_rels_order))
    return out


def _path(g: Graph, b: dict, path: list, k: int, bound_rels_order: list):
    if k == 0:
        first: NodePat = path[0]
        if first.var in b:
            if _labels_ok(g, b[first.var], first.labels):
                yield from _path(g, b, path, 1, bound_rels_order)
            return
        for nid in g.nodes:
            if _labels_ok(g, nid, first.labels):
                b2 = dict(b)
                b2[first.var] = nid
                yield from _path(g, b2, path, 1, bound_rels_order)
        return
    if k >= len(path):
        yield b
        return
    rel: RelPat = path[k]
    x: NodePat = path[k - 1]
    y: NodePat = path[k + 1]
    xv = b[x.var]
    if rel.var_length is not None:
        lower, upper = rel.var_length
        if rel.direction != "out" and rel.direction != "in":
            raise NotImplementedError("undirected var-length is checked by the golden vectors only")
        prior = [b[v] for v in _rel_vars(b)]
        for edges, end in _var_paths(g, xv, rel, lower, upper, prior):
            if y.var in b:
                if b[y.var] != end:
                    continue
                b2 = dict(b)
            else:
                if not _labels_ok(g, end, y.labels):
                    continue
                b2 = dict(b)
                b2[y.var] = end
            b2["__list_" + rel.var] = edges
            for i in range(1, upper + 1):
                b2[f"{rel.var}#{i}"] = edges[i - 1] if i <= len(edges) else None
                b2["__kind_" + f"{rel.var}#{i}"] = "rel"
            yield from _path(g, b2, path, k + 2, bound_rels_order)
        return
    cands = []  # (rel, other end)
    if y.var in b:  # ExpandInto
        yv = b[y.var]
        if x.var == y.var or rel.direction == "out":
            cands = [(r, yv) for r in g.out[xv] if r["dst"] == yv]
        elif rel.direction == "in":
            cands = [(r, yv) for r in g.inc[xv] if r["src"] == yv]
        else:
            cands = [(r, yv) for r in g.out[xv] if r["dst"] == yv] + [(r, yv) for r in g.inc[xv] if r["src"] == yv]
    else:
        if rel.direction in ("out", "both"):
            cands += [(r, r["dst"]) for r in g.out[xv]]
        if rel.direction in ("in", "both"):
            cands += [(r, r["src"]) for r in g.inc[xv] if not (rel.direction == "both" and r["src"] == r["dst"])]
    for r, other in cands:
        if not _type_ok(r, rel.types):
            continue
        if rel.var in b and b[rel.var] != r["id"]:
            continue
        if y.var not in b and not _labels_ok(g, other, y.labels):
            continue
        b2 = dict(b)
        b2[rel.var] = r["id"]
        b2["__kind_" + rel.var] = "rel"
        b2[y.var] = other
        yield from _path(g, b2, path, k + 2, bound_rels_order)


def _rel_vars(b: dict):
    """relationship variables bound so far (fixed-length and var-length hops), non-null"""
    return [k[7:] for k, v in b.items() if k.startswith("__kind_") and v == "rel" and b.get(k[7:]) is not None]


def _var_paths(g: Graph, start: int, rel: RelPat, lower: int, upper: int, prior: list):
    out = []

    def step(node, edges):
        if len(edges) >= lower and len(edges) >= 1:
            out.append((list(edges), node))
        if len(edges) == upper:
            return
        nxt = g.out[node] if rel.direction == "out" else g.inc[node]
        for r in nxt:
            if not _type_ok(r, rel.types) or r["id"] in edges:
                continue
            if not edges and r["id"] in prior:
                continue
            edges.append(r["id"])
            step(r["dst"] if rel.direction == "out" else r["src"], edges)
            edges.pop()

    step(start, [])
    if lower == 0:
        out.append(([], start))
    return out


def project(g: Graph, rows: List[dict], ret: dict) -> List[dict]:
    items = ret["items"]
    aggs = [(a, s) for a, s in items
            if s[0] in ("count*", "count", "count_distinct", "min", "max", "sum", "avg", "collect", "collect_distinct")]
    plain = [(a, s) for a, s in items if (a, s) not in aggs]

    def plain_val(s, b):
        if s[0] == "rels":
            lst = b.get("__list_" + s[1], [])
            return [[e, g.rels[e]["src"], g.rels[e]["dst"], g.rels[e]["type"]] for e in lst]
        return eval_expr(s, b, g)

    if not aggs:
        out = [{a: plain_val(s, b) for a, s in plain} for b in rows]
        if ret.get("distinct"):
            seen, uniq = set(), []
            for r in out:
                key = repr(sorted(r.items()))
                if key not in seen:
                    seen.add(key)
                    uniq.append(r)
            out = uniq
        return _order_skip_limit(out, ret)
    groups: Dict[str, list] = {}
    keys: Dict[str, dict] = {}
    for b in rows:
        kv = {a: plain_val(s, b) for a, s in plain}
        k = repr(sorted(kv.items()))
        groups.setdefault(k, []).append(b)
        keys[k] = kv
    if not plain and not groups:
        groups[""] = []
        keys[""] = {}
    out = []
    for k, members in groups.items():
        row = dict(keys[k])
        for a, s in aggs:
            if s[0] == "count*":
                row[a] = len(members)
                continue
            vals = [eval_expr(s[1], b, g) for b in members]
            vals = [v for v in vals if v is not None]
            if s[0] == "count":
                row[a] = len(vals)
            elif s[0] == "count_distinct":
                row[a] = len(set(vals))
            elif s[0] == "collect":  # sort_array(collect_list), SparkTable.scala:169-177
                row[a] = sorted(vals)
            elif s[0] == "collect_distinct":  # sort_array(collect_set)
                row[a] = sorted(set(vals))
            elif s[0] == "min":
                row[a] = min(vals) if vals else None
            elif s[0] == "max":
                row[a] = max(vals) if vals else None
            elif s[0] == "sum":
                row[a] = sum(vals) if vals else None
            elif s[0] == "avg":  # avg(..).cast(cypherType): integer input -> Long (truncated)
                if not vals:
                    row[a] = None
                elif all(isinstance(v, int) and not isinstance(v, bool) for v in vals):
                    row[a] = int(sum(vals) / len(vals))
                else:
                    row[a] = sum(vals) / len(vals)
        out.append(row)
    return _order_skip_limit(out, ret)


def _order_skip_limit(out: List[dict], ret: dict) -> List[dict]:
    """ORDER BY (Spark asc / desc: nulls first ascending, last descending; SparkTable.scala:94-104),
    then SKIP and LIMIT."""
    for alias, direction in reversed(ret.get("order_by") or []):
        desc = direction.lower().startswith("desc")
        out = sorted(out, key=lambda r: (r[alias] is not None, r[alias] if r[alias] is not None else 0), reverse=desc)
    if ret.get("skip"):
        out = out[int(ret["skip"]):]
    if ret.get("limit") is not None:
        out = out[:int(ret["limit"])]
    return out
