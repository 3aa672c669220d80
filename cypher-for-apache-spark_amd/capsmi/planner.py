"""Pattern -> Table operator sequence, mirroring okapi-relational's planner.

In a CAPS deployment this layer stays in Scala, unchanged: RelationalPlanner emits joins, filters,
unions and aggregates against ``Table[T]`` and the backend only sees those calls.  This module
re-states the lowering for the MATCH shapes on the hot path so that the backend can be driven
(and checked) without a JVM.  It is backend-agnostic: anything with the ``Table`` methods of
capsmi.table.GpuTable works (the device tables, or the test oracle's CPU tables).

Followed code (okapi-relational/src/main/scala/org/opencypher/okapi/relational/impl/planning/):
  - Expand            RelationalPlanner.scala:113-137 (undirected incoming branch drops self-loops)
  - ExpandInto        RelationalPlanner.scala:139-154 (undirected keeps both orientations)
  - var-length        VarLengthExpandPlanner.scala:46-310 (init/expand/finalize/isomorphismFilter/
                      copyEntity/addTargetOps; Directed :247-260, Undirected :278-308)
  - scans             RelationalPlanner.planScan :220-238, ScanGraph.scanOperator (impl/graph/ScanGraph.scala:61-96)
  - choice of operator okapi-logical/.../LogicalPlanner.scala:474-526 (bound target -> ExpandInto,
                      cyclic (a)--(a) -> directed ExpandInto :509-514)
  - uniqueness        front-end rewrite (CypherParser.scala:64-76): NOT(r_i = r_j) for every pair of
                      single-length relationship variables of one MATCH whose type sets may overlap
Column naming: node var v -> "v" (id), "v:Label" (Boolean), "v.key"; rel var r -> "r" (id),
"r.__src", "r.__dst", "r.__type", "r.key"; var-length hop i -> "r#i", "r#i.__src", ...
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, FrozenSet, List, Optional, Sequence, Tuple

import numpy as np

from .expr import (BOOL, F64, I64, STR, Ands, BinOp, Col, Expr, In, IsNotNull, IsNull, Lit, Not, Ors, ands, eq)
from .table import ColumnData, decode_value


class PlanningError(RuntimeError):
    pass


# ---------------------------------------------------------------------------------------------
# property graph input (what CAPSScanGraphFactory turns into entity tables)
# ---------------------------------------------------------------------------------------------
@dataclass
class PGNode:
    id: int
    labels: FrozenSet[str]
    props: Dict[str, object] = field(default_factory=dict)


@dataclass
class PGRel:
    id: int
    src: int
    dst: int
    type: str
    props: Dict[str, object] = field(default_factory=dict)


@dataclass
class PropertyGraph:
    nodes: List[PGNode]
    rels: List[PGRel]

    def strings(self) -> List[str]:
        out = set()
        for n in self.nodes:
            out |= set(n.labels)
            out |= {v for v in n.props.values() if isinstance(v, str)}
        for r in self.rels:
            out.add(r.type)
            out |= {v for v in r.props.values() if isinstance(v, str)}
        return sorted(out)


def _value_type(v) -> int:
    if isinstance(v, bool):
        return BOOL
    if isinstance(v, int):
        return I64
    if isinstance(v, float):
        return F64
    if isinstance(v, str):
        return STR
    raise PlanningError(f"unsupported property value {v!r}")


def _prop_types(entities) -> Dict[str, int]:
    """Property key -> physical type; Int/Float mixes widen to Float, other conflicts are errors
    (schema conflict, MatchBehaviour 'type conflicts on expressions')."""
    out: Dict[str, int] = {}
    for e in entities:
        for k, v in e.props.items():
            if v is None:
                continue
            t = _value_type(v)
            if k in out and out[k] != t:
                if {out[k], t} == {I64, F64}:
                    t = F64
                else:
                    raise PlanningError(f"property '{k}' has conflicting types")
            out[k] = t
    return out


def _column(name: str, ty: int, values: Sequence, encode) -> ColumnData:
    n = len(values)
    valid = np.array([v is not None for v in values], dtype=bool)
    if ty == F64:
        arr = np.array([float(v) if v is not None else 0.0 for v in values], dtype=np.float64)
    elif ty == STR:
        arr = np.array([encode(v) if v is not None else 0 for v in values], dtype=np.int64)
    else:
        arr = np.array([int(v) if v is not None else 0 for v in values], dtype=np.int64)
    return ColumnData(name, ty, arr.reshape(n), None if valid.all() else valid)


# physical column names of the entity keys (CAPS keeps them apart from property columns too:
# EntityMapping.allSourceKeys = idKeys ++ labels ++ relType ++ properties, EntityMapping.scala:50)
ID, SRC, DST = "__id", "__source", "__target"


@dataclass
class EntityTable:
    """A node or relationship table plus its mapping (NodeMapping / RelationshipMapping analogue,
    okapi-api/.../io/conversion/{Node,Relationship}Mapping.scala)."""
    kind: str                   # "node" | "rel"
    labels: FrozenSet[str]      # node: implied labels; rel: {type}
    props: Dict[str, int]       # property key -> type (column name = key)
    table: object               # backend table
    id_col: str = ID
    src_col: str = SRC
    dst_col: str = DST


class ScanGraph:
    """Entity tables of one graph: one node table per label combination, one rel table per type
    (CAPSScanGraphFactory.scala:52-103), scanned like ScanGraph.scanOperator."""

    def __init__(self, backend, nodes: List[EntityTable], rels: List[EntityTable], tags=frozenset({0})):
        self.backend = backend
        self.nodes = nodes
        self.rels = rels
        self.tags = frozenset(tags)  # graph tags its ids carry (RelationalCypherGraph.tags)

    def entity_tables(self):
        return self.nodes, self.rels

    @staticmethod
    def from_property_graph(backend, pg: PropertyGraph) -> "ScanGraph":
        backend.dictionary.extend(pg.strings())
        enc = backend.dictionary.encode
        combos: Dict[FrozenSet[str], List[PGNode]] = {}
        for n in pg.nodes:
            combos.setdefault(frozenset(n.labels), []).append(n)
        nodes = []
        for labels in sorted(combos, key=lambda s: sorted(s)):
            ns = combos[labels]
            pt = _prop_types(ns)
            cols = [_column(ID, I64, [n.id for n in ns], enc)]
            for k in sorted(pt):
                cols.append(_column(k, pt[k], [n.props.get(k) for n in ns], enc))
            nodes.append(EntityTable("node", labels, pt, backend.table(cols).as_node_table(ID)))
        types: Dict[str, List[PGRel]] = {}
        for r in pg.rels:
            types.setdefault(r.type, []).append(r)
        rels = []
        for t in sorted(types):
            rs = types[t]
            pt = _prop_types(rs)
            cols = [_column(ID, I64, [r.id for r in rs], enc), _column(SRC, I64, [r.src for r in rs], enc),
                    _column(DST, I64, [r.dst for r in rs], enc)]
            for k in sorted(pt):
                cols.append(_column(k, pt[k], [r.props.get(k) for r in rs], enc))
            rels.append(EntityTable("rel", frozenset([t]), pt, backend.table(cols).as_rel_table(ID, SRC, DST)))
        backend.compact_if_sparse([e.table for e in nodes], [e.table for e in rels])
        return ScanGraph(backend, nodes, rels)

    # ---- scans --------------------------------------------------------------------------
    def node_scan(self, var: str, labels: Sequence[str]):
        req = set(labels)
        sel = [t for t in self.nodes if req <= t.labels]
        all_labels = sorted(set().union(*[t.labels for t in sel])) if sel else sorted(req)
        props: Dict[str, int] = {}
        for t in sel:
            for k, ty in t.props.items():
                if k in props and props[k] != ty:
                    raise PlanningError(f"property '{k}' has conflicting types across scanned tables")
                props[k] = ty
        header = [var] + [f"{var}:{l}" for l in all_labels] + [f"{var}.{k}" for k in sorted(props)]
        if not sel:
            return self._empty([(var, I64)] + [(f"{var}:{l}", BOOL) for l in all_labels]), header
        ops = []
        for t in sel:
            cols = [(Col(t.id_col), var)]
            cols += [(Lit(l in t.labels), f"{var}:{l}") for l in all_labels]
            cols += [(Col(k) if k in t.props else Lit(None, props[k]), f"{var}.{k}") for k in sorted(props)]
            ops.append(t.table.withColumns(*cols).select(*header))
        out = ops[0]
        for o in ops[1:]:
            out = out.unionAll(o)
        return out, header

    def rel_scan(self, var: str, types: Sequence[str]):
        sel = [t for t in self.rels if not types or (t.labels & set(types))]
        props: Dict[str, int] = {}
        for t in sel:
            for k, ty in t.props.items():
                if k in props and props[k] != ty:
                    raise PlanningError(f"property '{k}' has conflicting types across scanned tables")
                props[k] = ty
        header = [var, f"{var}.__src", f"{var}.__dst", f"{var}.__type"] + [f"{var}.{k}" for k in sorted(props)]
        if not sel:
            return self._empty([(var, I64), (f"{var}.__src", I64), (f"{var}.__dst", I64), (f"{var}.__type", STR)]
                               + [(f"{var}.{k}", ty) for k, ty in sorted(props.items())]), header
        ops = []
        for t in sel:
            (ty_name,) = tuple(t.labels)
            cols = [(Col(t.id_col), var), (Col(t.src_col), f"{var}.__src"), (Col(t.dst_col), f"{var}.__dst"),
                    (Lit(ty_name), f"{var}.__type")]
            cols += [(Col(k) if k in t.props else Lit(None, props[k]), f"{var}.{k}") for k in sorted(props)]
            ops.append(t.table.withColumns(*cols).select(*header))
        out = ops[0]
        for o in ops[1:]:
            out = out.unionAll(o)
        return out, header

    def _empty(self, schema):
        return self.backend.table([ColumnData(n, ty, np.zeros(0, dtype=np.float64 if ty == F64 else np.int64))
                                   for n, ty in schema])


class UnionGraph:
    """UNION ALL of graphs (okapi-relational/.../impl/graph/UnionGraph.scala:41-80): each member's
    ids (node id; relationship id, source and target -- RecordHeader.idExpressions) are retagged by
    its replacement map so the members' ids are disjoint, the scans are aligned and union'ed, and
    the union is deduplicated on the scanned entity (``Distinct(..., Set(targetEntity))``, :77).
    The retagging is a device ``withColumns`` of Tags.ExprTagging's CaseExpr, as retagVariable
    (RelationalPlanner.scala:332-335) plans it."""

    def __init__(self, backend, graphs_to_replacements):
        if not graphs_to_replacements:
            raise PlanningError("Union requires at least one graph")
        self.backend = backend
        self.members = list(graphs_to_replacements)  # [(graph, {from: to})]
        self.tags = frozenset(t for _, rep in self.members for t in rep.values())

    @staticmethod
    def union_all(backend, *graphs) -> "UnionGraph":
        """RelationalCypherGraphFactory.unionGraph(graphs*) (RelationalCypherGraph.scala:52-55)."""
        from .tagging import compute_retaggings
        keyed = {i: g.tags for i, g in enumerate(graphs)}
        rep = compute_retaggings(keyed)
        return UnionGraph(backend, [(g, rep[i]) for i, g in enumerate(graphs)])

    def entity_tables(self):
        from .tagging import expr_replace_tags
        nodes, rels = [], []
        for g, rep in self.members:
            moves = {f: t for f, t in rep.items() if f != t}
            gn, gr = g.entity_tables()
            for et in gn + gr:
                keys = [et.id_col] + ([et.src_col, et.dst_col] if et.kind == "rel" else [])
                tab = et.table if not moves else et.table.withColumns(
                    *[(expr_replace_tags(Col(c), rep), c) for c in keys])
                (nodes if et.kind == "node" else rels).append(
                    EntityTable(et.kind, et.labels, et.props, tab, et.id_col, et.src_col, et.dst_col))
        return nodes, rels

    def _flat(self) -> ScanGraph:
        nodes, rels = self.entity_tables()
        return ScanGraph(self.backend, nodes, rels, self.tags)

    def node_scan(self, var: str, labels: Sequence[str]):
        out, header = self._flat().node_scan(var, labels)
        return out.distinct(*header), header

    def rel_scan(self, var: str, types: Sequence[str]):
        out, header = self._flat().rel_scan(var, types)
        return out.distinct(*header), header


# ---------------------------------------------------------------------------------------------
# pattern text: a small parser for MATCH patterns (the openCypher front-end stays in Scala)
# ---------------------------------------------------------------------------------------------
@dataclass
class NodePat:
    var: str
    labels: Tuple[str, ...]
    anon: bool = False


@dataclass
class RelPat:
    var: str
    types: Tuple[str, ...]
    direction: str            # "out" (left->right), "in" (right->left), "both"
    var_length: Optional[Tuple[int, int]] = None
    anon: bool = False


_NODE_RE = re.compile(r"\(\s*([A-Za-z_][A-Za-z_0-9]*)?\s*((?::\s*[A-Za-z_][A-Za-z_0-9]*\s*)*)\)")
_REL_RE = re.compile(r"(<)?-\s*(?:\[\s*([A-Za-z_][A-Za-z_0-9]*)?\s*((?::\s*[A-Za-z_][A-Za-z_0-9]*(?:\s*\|\s*:?\s*[A-Za-z_][A-Za-z_0-9]*)*)?)"
                     r"\s*(\*\s*(\d*)\s*(?:\.\.\s*(\d*))?)?\s*\])?\s*-(>)?")


class _Names:
    def __init__(self):
        self.n = 0

    def fresh(self, kind: str) -> str:
        self.n += 1
        return f"_{kind}{self.n}"


def parse_pattern(text: str, names: _Names) -> List[List[object]]:
    """'(a:A)-[r:T]->(b), (c)' -> [[NodePat, RelPat, NodePat], [NodePat]]"""
    paths = []
    pos = 0
    text = text.strip()
    while pos < len(text):
        elems: List[object] = []
        m = _NODE_RE.match(text, pos)
        if not m:
            raise PlanningError(f"cannot parse pattern at: {text[pos:]!r}")
        elems.append(_node(m, names))
        pos = m.end()
        while True:
            rest = text[pos:].lstrip()
            pos = len(text) - len(rest)
            r = _REL_RE.match(text, pos) if rest[:1] in ("-", "<") else None
            if not r:
                break
            elems.append(_rel(r, names))
            pos = r.end()
            rest = text[pos:].lstrip()
            pos = len(text) - len(rest)
            m = _NODE_RE.match(text, pos)
            if not m:
                raise PlanningError(f"cannot parse node at: {text[pos:]!r}")
            elems.append(_node(m, names))
            pos = m.end()
        paths.append(elems)
        rest = text[pos:].lstrip()
        pos = len(text) - len(rest)
        if rest.startswith(","):
            pos += 1
            rest = text[pos:].lstrip()
            pos = len(text) - len(rest)
        elif rest:
            raise PlanningError(f"unexpected pattern text: {rest!r}")
    return paths


def _node(m, names) -> NodePat:
    var = m.group(1)
    labels = tuple(l.strip() for l in m.group(2).split(":") if l.strip()) if m.group(2) else ()
    if var:
        return NodePat(var, labels)
    return NodePat(names.fresh("n"), labels, anon=True)


def _rel(m, names) -> RelPat:
    left, var, types, star, lo, hi, right = m.group(1), m.group(2), m.group(3), m.group(4), m.group(5), m.group(6), m.group(7)
    if left and right:
        raise PlanningError("relationship cannot point both ways")
    direction = "in" if left else ("out" if right else "both")
    ts = tuple(t.strip().lstrip(":").strip() for t in re.split(r"[|]", types.replace(":", "|", 1))) if types else ()
    ts = tuple(t for t in ts if t)
    vl = None
    if star:
        if lo is None and hi is None and ".." not in star:
            raise PlanningError("unbounded var-length is not supported (PatternConverter.scala:134-136)")
        if ".." in star:
            lower = int(lo) if lo else 1
            if not hi:
                raise PlanningError("unbounded var-length is not supported (PatternConverter.scala:134-136)")
            upper = int(hi)
        else:
            lower = upper = int(lo)
        vl = (lower, upper)
    if var:
        return RelPat(var, ts, direction, vl)
    return RelPat(names.fresh("r"), ts, direction, vl, anon=True)


# ---------------------------------------------------------------------------------------------
# expression DSL (JSON prefix lists) -> Expr over the current header
# ---------------------------------------------------------------------------------------------
_CMP = {"=", "<>", "<", "<=", ">", ">=", "+", "-", "*"}


def to_expr(spec, header: Sequence[str]) -> Expr:
    cols = set(header)
    op = spec[0]
    if op == "prop":
        name = f"{spec[1]}.{spec[2]}"
        return Col(name) if name in cols else Lit(None)  # missing property -> null (SparkSQLExprMapper.scala:94)
    if op in ("var", "id"):
        return Col(spec[1])
    if op == "type":
        return Col(f"{spec[1]}.__type")
    if op == "lit":
        return Lit(spec[1])
    if op == "haslabel":
        name = f"{spec[1]}:{spec[2]}"
        return Col(name) if name in cols else Lit(False)
    if op in _CMP:
        return BinOp(op, to_expr(spec[1], header), to_expr(spec[2], header))
    if op == "not":
        return Not(to_expr(spec[1], header))
    if op == "and":
        return Ands(tuple(to_expr(s, header) for s in spec[1:]))
    if op == "or":
        return Ors(tuple(to_expr(s, header) for s in spec[1:]))
    if op == "isnull":
        return IsNull(to_expr(spec[1], header))
    if op == "isnotnull":
        return IsNotNull(to_expr(spec[1], header))
    if op == "in":
        return In(to_expr(spec[1], header), tuple(Lit(v) for v in spec[2]))
    raise PlanningError(f"unknown expression {spec!r}")


AGGS = {"count*": "count_star", "count": "count", "count_distinct": "count", "min": "min", "max": "max",
        "sum": "sum", "avg": "avg", "collect": "collect", "collect_distinct": "collect"}
DISTINCT_AGGS = ("count_distinct", "collect_distinct")


# ---------------------------------------------------------------------------------------------
# the planner
# ---------------------------------------------------------------------------------------------
class _Op:
    """A backend table plus its header bookkeeping."""

    def __init__(self, table, header: List[str], node_vars: set, rel_vars: List[str]):
        self.table = table
        self.header = header
        self.node_vars = node_vars
        self.rel_vars = rel_vars      # relationship id columns in the header (incl. var-length hops)


class Planner:
    def __init__(self, graph: ScanGraph):
        self.g = graph
        self.names = _Names()

    # ---- query ------------------------------------------------------------------------------
    def run(self, query: dict):
        """Execute ``{"clauses": [{"match": str, "where": expr?}], "return": {...}}``; returns
        (table, output spec) ready for :func:`result_rows`."""
        cur: Optional[_Op] = None
        varlen: Dict[str, int] = {}
        if query.get("driving"):  # driving table: its columns are value variables (planStartWithDrivingTable)
            d = query["driving"]
            cols = []
            dictionary = self.g.backend.dictionary
            for name, values in d.items():
                if any(isinstance(v, str) for v in values):
                    ty = STR
                    # codes are stable under insertion, so new strings are added, never guessed at
                    dictionary.extend(v for v in values if v is not None)
                else:
                    ty = F64 if any(isinstance(v, float) for v in values) else I64
                cols.append(_column(name, ty, values, dictionary.encode))
            cur = _Op(self.g.backend.table(cols), list(d), set(), [])
        for clause in query["clauses"]:
            if "optional_match" in clause:
                cur = self._optional(cur, clause["optional_match"], clause.get("where"), varlen)
            else:
                cur = self._match(cur, clause["match"], clause.get("where"), varlen)
        return self._return(cur, query["return"], varlen)

    def _optional(self, cur: Optional[_Op], pattern: str, where, varlen: Dict[str, int]) -> _Op:
        """OPTIONAL MATCH: the pattern is planned on top of the input (LogicalPlanner.scala:115-128);
        planOptional (RelationalPlanner.scala:241-276) then left-outer-joins the input with that plan
        on every variable they share, after dropping the right side's copies of the shared
        variables' other columns and renaming its join columns apart."""
        if cur is None or not (cur.node_vars or cur.rel_vars):  # `lhs.fields.isEmpty` -> rhs
            return self._match(cur, pattern, where, varlen)
        lhs = cur
        rhs = self._match(_Op(cur.table, list(cur.header), set(cur.node_vars), list(cur.rel_vars)), pattern, where,
                          varlen)
        join_vars = [v for v in lhs.header if v in lhs.node_vars or v in lhs.rel_vars]
        new_cols = [c for c in rhs.header if c not in lhs.header]
        renames = [(v, self.names.fresh("opt")) for v in join_vars]
        right = rhs.table.select(*(join_vars + new_cols))
        for v, tmp in renames:
            right = right.withColumnRenamed(v, tmp)
        joined = lhs.table.join(right, "left_outer", *renames)
        t = joined.select(*(lhs.header + new_cols))
        return _Op(t, lhs.header + new_cols, rhs.node_vars, rhs.rel_vars)

    def _match(self, cur: Optional[_Op], pattern: str, where, varlen: Dict[str, int], unique: bool = True) -> _Op:
        paths = parse_pattern(pattern, self.names)
        clause_rels: List[RelPat] = []
        pending = list(paths)
        # connect components: plan paths that touch bound variables first (in text order)
        while pending:
            bound = cur.node_vars if cur else set()
            idx = next((i for i, p in enumerate(pending) if any(isinstance(e, NodePat) and e.var in bound for e in p)), 0)
            path = pending.pop(idx)
            cur = self._path(cur, path, clause_rels, varlen, where)
        # uniqueness among single-length relationships of this clause (a MATCH clause only: the
        # front-end's rewrite does not reach pattern predicates / EXISTS)
        preds = []
        singles = [r for r in clause_rels if r.var_length is None] if unique else []
        for i in range(len(singles)):
            for j in range(i + 1, len(singles)):
                a, b = singles[i], singles[j]
                if a.var == b.var:
                    continue
                if a.types and b.types and not (set(a.types) & set(b.types)):
                    continue  # the front-end skips pairs that can never be equal
                preds.append(Not(eq(Col(a.var), Col(b.var))))
        for a in singles:
            for b in (clause_rels if unique else []):
                if b.var_length is not None and not (a.types and b.types and not (set(a.types) & set(b.types))):
                    raise PlanningError("uniqueness between a single and a var-length relationship is "
                                        "not supported by CAPS (NotImplementedException)")
        helper: List[str] = []
        if where is not None:
            cur, where = self._lower_exists(cur, where, varlen, helper)
            preds.append(to_expr(where, cur.header))
        pred = ands(*preds)
        if not (isinstance(pred, Lit) and pred.value is True):
            cur.table = cur.table.filter(pred)
        if helper:
            cur.table = cur.table.drop(*helper)
            cur.header = [h for h in cur.header if h not in helper]
        return cur

    def _lower_exists(self, cur: _Op, spec, varlen: Dict[str, int], helper: List[str]):
        """Replace every ``["exists", pattern, where?]`` in an expression spec by a BOOL column
        planned as an ExistsSubQuery; returns (op, spec)."""
        if not isinstance(spec, list) or not spec:
            return cur, spec
        if spec[0] == "exists":
            cur, col = self._exists(cur, spec[1], spec[2] if len(spec) > 2 else None, varlen)
            helper.append(col)
            return cur, ["var", col]
        out = [spec[0]]
        for s in spec[1:]:
            cur, s = self._lower_exists(cur, s, varlen, helper)
            out.append(s)
        return cur, out

    def _exists(self, cur: Optional[_Op], pattern: str, where, varlen: Dict[str, int]):
        """EXISTS(pattern) / a pattern predicate (RelationalPlanner.scala:181-202): the pattern is
        planned on top of the input, its rows are reduced to the distinct bindings of the variables
        the input already has (renamed apart), left-outer-joined back, and IsNotNull of a join
        column is the predicate."""
        if cur is None:
            raise PlanningError("EXISTS needs bound variables")
        lhs = cur
        rhs = self._match(_Op(cur.table, list(cur.header), set(cur.node_vars), list(cur.rel_vars)), pattern, where,
                          dict(varlen), unique=False)
        join_vars = [h for h in lhs.header
                     if h in lhs.node_vars or h in lhs.rel_vars or not any(c in h for c in ".:#")]
        if not join_vars:
            raise PlanningError("EXISTS needs bound variables")
        renames = [(v, self.names.fresh("ex")) for v in join_vars]
        right = rhs.table.select(*join_vars)
        for v, tmp in renames:
            right = right.withColumnRenamed(v, tmp)
        right = right.distinct()
        col = self.names.fresh("exists")
        joined = lhs.table.join(right, "left_outer", *renames)
        t = joined.withColumns((IsNotNull(Col(renames[0][1])), col)).select(*(lhs.header + [col]))
        return _Op(t, lhs.header + [col], lhs.node_vars, lhs.rel_vars), col

    def _path(self, cur: Optional[_Op], path: List[object], clause_rels: List[RelPat],
              varlen: Dict[str, int], where=None) -> _Op:
        first: NodePat = path[0]
        if cur is None or first.var not in cur.node_vars:
            scan, header = self.g.node_scan(first.var, first.labels)
            op = _Op(scan, header, {first.var}, [])
            if cur is None:
                cur = op
            else:  # disconnected component: cartesian product (RelationalPlanner.scala:56-57) ...
                vj = self._value_join_keys(cur, op, where)
                if vj is None:
                    t = cur.table.join(op.table, "cross")
                else:  # ... or an equi-join on a WHERE equality across it (ValueJoin)
                    (le, lk), (re_, rk) = vj
                    t = cur.table.withColumns((le, lk)).join(op.table.withColumns((re_, rk)), "inner", (lk, rk))
                    t = t.drop(lk, rk)
                cur = _Op(t, cur.header + op.header, cur.node_vars | op.node_vars, cur.rel_vars)
        else:
            cur = self._bound_labels(cur, first)
        for k in range(1, len(path), 2):
            rel: RelPat = path[k]
            left: NodePat = path[k - 1]
            right: NodePat = path[k + 1]
            clause_rels.append(rel)
            if rel.var_length is not None:
                cur = self._var_expand(cur, left, rel, right, varlen)
            elif right.var in cur.node_vars:
                cur = self._expand_into(cur, left, rel, right)
                cur = self._bound_labels(cur, right)
            else:
                cur = self._expand(cur, left, rel, right)
        return cur

    def _value_join_keys(self, lhs: _Op, rhs: _Op, where):
        """LogicalOptimizer.replaceCartesianWithValueJoin (LogicalOptimizer.scala:58-76): a WHERE
        conjunct ``x = y`` whose sides are each a variable or a variable's property, one solved by
        the product's left input and one by its right, turns the product into an equi-join on the
        two expressions.  The conjunct stays in the filter (always true on the joined rows).  Only
        key pairs the join can compare (same type, or both numeric) are taken."""
        if where is None:
            return None
        conj = where[1:] if where[0] == "and" else [where]

        def side(spec, op):
            if not isinstance(spec, list) or not spec or spec[0] not in ("prop", "var", "id"):
                return None
            col = f"{spec[1]}.{spec[2]}" if spec[0] == "prop" else spec[1]
            return col if spec[1] in op.header and col in op.header else None

        ltypes, rtypes = lhs.table.columnType, rhs.table.columnType
        for c in conj:
            if not isinstance(c, list) or not c or c[0] != "=":
                continue
            for a, b in ((c[1], c[2]), (c[2], c[1])):
                lc, rc = side(a, lhs), side(b, rhs)
                if lc is None or rc is None:
                    continue
                lt, rt = ltypes[lc], rtypes[rc]
                if lt == rt or (lt in (I64, F64) and rt in (I64, F64)):
                    return (Col(lc), self.names.fresh("vjl")), (Col(rc), self.names.fresh("vjr"))
        return None

    def _bound_labels(self, cur: _Op, n: NodePat) -> _Op:
        if not n.labels:
            return cur
        pred = ands(*[Col(f"{n.var}:{l}") if f"{n.var}:{l}" in cur.header else Lit(False) for l in n.labels])
        cur.table = cur.table.filter(pred)
        return cur

    # Expand: RelationalPlanner.scala:113-137
    def _expand(self, cur: _Op, x: NodePat, r: RelPat, y: NodePat) -> _Op:
        rs, rh = self.g.rel_scan(r.var, r.types)
        ns, nh = self.g.node_scan(y.var, y.labels)
        src, dst = f"{r.var}.__src", f"{r.var}.__dst"
        if r.direction in ("out", "in"):
            start, end = (src, dst) if r.direction == "out" else (dst, src)
            t = cur.table.join(rs, "inner", (x.var, start)).join(ns, "inner", (end, y.var))
        else:
            out = cur.table.join(rs, "inner", (x.var, src)).join(ns, "inner", (dst, y.var))
            no_loops = rs.filter(Not(eq(Col(src), Col(dst))))
            inc = cur.table.join(no_loops, "inner", (x.var, dst)).join(ns, "inner", (src, y.var))
            t = out.unionAll(inc)
        return _Op(t, cur.header + rh + nh, cur.node_vars | {y.var}, cur.rel_vars + [r.var])

    # ExpandInto: RelationalPlanner.scala:139-154; cyclic (a)--(a) is directed (LogicalPlanner.scala:509-514)
    def _expand_into(self, cur: _Op, x: NodePat, r: RelPat, y: NodePat) -> _Op:
        rs, rh = self.g.rel_scan(r.var, r.types)
        src, dst = f"{r.var}.__src", f"{r.var}.__dst"
        if x.var == y.var or r.direction == "out":
            t = cur.table.join(rs, "inner", (x.var, src), (y.var, dst))
        elif r.direction == "in":
            t = cur.table.join(rs, "inner", (x.var, dst), (y.var, src))
        else:
            t = cur.table.join(rs, "inner", (x.var, src), (y.var, dst)).unionAll(
                cur.table.join(rs, "inner", (y.var, src), (x.var, dst)))
        return _Op(t, cur.header + rh, cur.node_vars, cur.rel_vars + [r.var])

    # BoundedVarLengthExpand: VarLengthExpandPlanner.scala
    def _var_expand(self, cur: _Op, x: NodePat, r: RelPat, y: NodePat, varlen: Dict[str, int]) -> _Op:
        lower, upper = r.var_length
        varlen[r.var] = upper
        into = y.var in cur.node_vars
        if lower == 0 and into:
            raise PlanningError("zero-length var-length ExpandInto is not supported")
        seg = lambda i: f"{r.var}#{i}"  # noqa: E731

        def scan(i):
            t, _ = self.g.rel_scan(seg(i), r.types)
            return t.select(seg(i), f"{seg(i)}.__src", f"{seg(i)}.__dst", f"{seg(i)}.__type")

        def seg_cols(i):
            return [seg(i), f"{seg(i)}.__src", f"{seg(i)}.__dst", f"{seg(i)}.__type"]

        def iso(i, candidates):
            return ands(*[Not(eq(Col(c), Col(seg(i)))) for c in candidates])

        def filt(t, e):
            return t if (isinstance(e, Lit) and e.value is True) else t.filter(e)

        base_rels = list(cur.rel_vars)
        end_of = lambda i: f"{seg(i)}.__dst"    # noqa: E731
        start_of = lambda i: f"{seg(i)}.__src"  # noqa: E731

        def init(direction):
            key = start_of(1) if direction == "out" else end_of(1)
            return filt(cur.table.join(scan(1), "inner", (x.var, key)), iso(1, base_rels))

        def expand(i, t, d_prev, d_next):
            left = end_of(i - 1) if d_prev == "out" else start_of(i - 1)
            right = start_of(i) if d_next == "out" else end_of(i)
            return filt(t.join(scan(i), "inner", (left, right)), iso(i, [seg(j) for j in range(1, i)]))

        ns = nh = None
        if not into:
            ns, nh = self.g.node_scan(y.var, y.labels)

        def add_target(t, i, direction):
            endpoint = end_of(i) if direction == "out" else start_of(i)
            if into:
                return t.filter(eq(Col(y.var), Col(endpoint)))
            return t.join(ns, "inner", (endpoint, y.var))

        paths = []  # (table, length)
        if r.direction in ("out", "in"):
            d = r.direction
            last = init(d)
            levels = [(last, 1)]
            for i in range(2, upper + 1):
                last = expand(i, last, d, d)
                levels.append((last, i))
            for t, k in levels:
                if k >= lower:
                    paths.append((add_target(t, k, d), k))
        else:  # Undirected plan, VarLengthExpandPlanner.scala:278-308 (orientation pairing as written there)
            out_t, in_t = init("out"), init("in")
            levels = [(out_t, in_t, 1)]
            for i in range(2, upper + 1):
                o_o = expand(i, out_t, "out", "out")
                o_i = expand(i, out_t, "out", "in")
                i_o = expand(i, in_t, "in", "out")
                i_i = expand(i, in_t, "in", "in")
                out_t, in_t = o_o.unionAll(i_o), o_i.unionAll(i_i)
                levels.append((out_t, in_t, i))
            for o, n_, k in levels:
                if k >= lower and upper >= 1:
                    paths.append((add_target(o, k, "out").unionAll(add_target(n_, k, "in")), k))

        if upper == 0:  # `*0`: only the zero-length copy (VarLengthExpandPlanner.scala:150-152)
            paths = []
        target_header = cur.header + [c for i in range(1, upper + 1) for c in seg_cols(i)] + ([] if into else nh)
        aligned = []
        for t, k in paths:
            pad = [(Lit(None, I64), c) for i in range(k + 1, upper + 1) for c in seg_cols(i)[:3]]
            pad += [(Lit(None, STR), seg_cols(i)[3]) for i in range(k + 1, upper + 1)]
            if pad:
                t = t.withColumns(*pad)
            aligned.append(t.select(*target_header))
        if lower == 0:  # copyEntity(source -> target) plus all-null hops, VarLengthExpandPlanner.scala:146-153,190-210
            z = cur.table
            cols = [(Col(x.var), y.var)]
            for c in nh[1:]:
                suffix = c[len(y.var):]
                src_col = x.var + suffix
                if src_col in cur.header:
                    cols.append((Col(src_col), c))
                else:
                    cols.append((Lit(False) if suffix.startswith(":") else self._null_like(ns, c), c))
            cols += [(Lit(None, I64), c) for i in range(1, upper + 1) for c in seg_cols(i)[:3]]
            cols += [(Lit(None, STR), seg_cols(i)[3]) for i in range(1, upper + 1)]
            z = z.withColumns(*cols).select(*target_header)
            aligned.append(z)
        if not aligned:
            raise PlanningError("empty var-length range")
        t = aligned[0]
        for o in aligned[1:]:
            t = t.unionAll(o)
        return _Op(t, target_header, cur.node_vars | {y.var}, cur.rel_vars + [seg(i) for i in range(1, upper + 1)])

    @staticmethod
    def _null_like(table, col: str) -> Lit:
        return Lit(None, table.columnType[col])

    # ---- RETURN ---------------------------------------------------------------------------------
    def _return(self, cur: _Op, ret: dict, varlen: Dict[str, int]):
        items = []
        for alias, spec in ret["items"]:
            if spec and spec[0] not in AGGS and spec[0] != "rels":
                cur, spec = self._lower_exists(cur, spec, varlen, [])
            items.append((alias, spec))
        t = cur.table
        plain, aggs, outs = [], [], []
        computed = []
        for i, (alias, spec) in enumerate(items):
            kind = spec[0]
            if kind == "entity":
                # a node / relationship variable: every column it owns (RecordHeader.ownedBy,
                # RecordHeader.scala:96-104) -- when aggregating these are all grouping keys, as
                # DataFrameTable.group groups by header.ownedBy(var) (SparkTable.scala:128-133)
                v = spec[1]
                owned = [h for h in cur.header if h == v or h.startswith(v + ".") or h.startswith(v + ":")]
                if v not in cur.header or not (v in cur.node_vars or v in cur.rel_vars):
                    raise PlanningError(f"{v} is not a node or relationship variable")
                parts = []
                for h in owned:
                    new = f"__ret{i}{h[len(v):]}"
                    computed.append((Col(h), new))
                    plain.append(new)
                    parts.append((h[len(v):], new))
                outs.append(("entity", alias, (v in cur.rel_vars, parts)))
            elif kind == "rels":  # var-length list: keep the hop columns, assembled on the host
                upper = varlen[spec[1]]
                cols = []
                for h in range(1, upper + 1):
                    for suf in ("", ".__src", ".__dst", ".__type"):
                        c = f"{spec[1]}#{h}{suf}"
                        new = f"__ret{i}_{h}{suf}"
                        computed.append((Col(c), new))
                        cols.append(new)
                plain.extend(cols)
                outs.append(("rels", alias, cols))
            elif kind in AGGS:
                name = f"__agg{i}"
                inp = None
                if kind != "count*":
                    inp = f"__aggin{i}"
                    computed.append((to_expr(spec[1], cur.header), inp))
                aggs.append((AGGS[kind], inp, kind in DISTINCT_AGGS, name))
                outs.append(("col", alias, name))
            else:
                name = f"__ret{i}"
                computed.append((to_expr(spec, cur.header), name))
                plain.append(name)
                outs.append(("col", alias, name))
        if computed:
            t = t.withColumns(*computed)
        if aggs:
            t = t.group(plain, aggs)
        else:
            t = t.select(*plain)
            if ret.get("distinct"):
                t = t.distinct()
        if ret.get("order_by"):
            names = {alias: col for k, alias, col in outs if k == "col"}
            t = t.orderBy(*[(names[a], o) for a, o in ret["order_by"]])
        if ret.get("skip"):
            t = t.skip(int(ret["skip"]))
        if ret.get("limit") is not None:
            t = t.limit(int(ret["limit"]))
        return t, outs


def result_rows(table, outs, dictionary) -> List[dict]:
    """Decode a RETURN table to Cypher-like values (strings decoded, var-length lists assembled as
    [id, source, target, type] per relationship, entities as CAPSNode / CAPSRelationship-like dicts:
    {"id", "labels", "props"} / {"id", "src", "dst", "type", "props"}, null properties left out as
    CAPSNode's property map leaves them out)."""
    cols = {c.name: c for c in table.to_columns()}
    n = table.size

    def val(c: ColumnData, r: int):
        if c.valid is not None and not c.valid[r]:
            return None
        return decode_value(c.type, c.values[r], dictionary)

    rows = []
    for r in range(n):
        row = {}
        for kind, alias, spec in outs:
            if kind == "col":
                row[alias] = val(cols[spec], r)
            elif kind == "entity":
                row[alias] = _entity_value(spec, {suf: val(cols[c], r) for suf, c in spec[1]})
            else:
                lst = []
                for h in range(0, len(spec), 4):
                    rid = val(cols[spec[h]], r)
                    if rid is None:
                        continue
                    lst.append([rid, val(cols[spec[h + 1]], r), val(cols[spec[h + 2]], r), val(cols[spec[h + 3]], r)])
                row[alias] = lst
        rows.append(row)
    return rows


def _entity_value(spec, vals: dict):
    is_rel, _ = spec
    if vals[""] is None:  # an OPTIONAL MATCH miss
        return None
    if is_rel:
        props = {k[1:]: v for k, v in vals.items() if k.startswith(".") and not k.startswith(".__") and v is not None}
        return {"id": vals[""], "src": vals[".__src"], "dst": vals[".__dst"], "type": vals[".__type"], "props": props}
    labels = sorted(k[1:] for k, v in vals.items() if k.startswith(":") and v)
    props = {k[1:]: v for k, v in vals.items() if k.startswith(".") and v is not None}
    return {"id": vals[""], "labels": labels, "props": props}
