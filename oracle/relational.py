"""CPU restatement of DataFrameTable semantics -- TEST INFRASTRUCTURE ONLY.

Only tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() may use this module, and only
as the checker.  The product (libcapsmi.so and the capsmi package) never imports it.

It restates, with numpy, the semantics Spark SQL 2.2.1 gives each operator of
    spark-cypher/src/main/scala/org/opencypher/spark/impl/table/SparkTable.scala
(Spark itself is third-party and absent here; the semantics below are Spark's
documented behaviour as CAPS relies on it):
  select / drop / withColumnRenamed                      SparkTable.scala:61-63, 90-92, 237-238
  filter: keep rows whose predicate is TRUE (3VL)        SparkTable.scala:65-67, SparkSQLExprMapper.scala:81-312
  withColumns: replace in place, append new              SparkTable.scala:69-88
  join: inner/outer/cross, `===` never matches null      SparkTable.scala:205-229
  unionAll: positional, types must match                 SparkTable.scala:190-203
  distinct / dropDuplicates: nulls group together        SparkTable.scala:231-235
  group: count(lit 0), count, countDistinct (nulls ignored), min, max, sum, avg,
         collect / collect(DISTINCT) as sorted lists     SparkTable.scala:121-188
  orderBy: ASC nulls first, DESC nulls last              SparkTable.scala:94-103
Tables here are plain numpy columns; the implementation deliberately shares nothing with the
device code (sort/searchsorted joins instead of hash tables, np.unique instead of hashing).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Sequence, Tuple

import numpy as np

I64, BOOL, F64, STR = 0, 1, 2, 3
LIST = 8  # list of element type t: LIST + t (Collect results; one numpy array per row)


class OracleError(RuntimeError):
    pass


class Col_:
    __slots__ = ("type", "values", "valid")

    def __init__(self, ty: int, values: np.ndarray, valid: np.ndarray):
        self.type = ty
        self.values = values
        self.valid = valid


class ColumnOut:
    """Exported column (same shape as capsmi.table.ColumnData)."""

    def __init__(self, name, ty, values, valid):
        self.name, self.type, self.values, self.valid = name, ty, values, valid


def _empty_like(ty: int, n: int) -> np.ndarray:
    return np.zeros(n, dtype=np.float64 if ty == F64 else np.int64)


class NumpyBackend:
    def __init__(self, dictionary):
        self.dictionary = dictionary

    def compact_if_sparse(self, nodes, rels):  # dense-id compaction is a device-path concern
        return False

    def table(self, columns) -> "NumpyTable":
        cols = OrderedDict()
        n = None
        for c in columns:
            vals = np.asarray(c.values)
            vals = vals.astype(np.float64 if c.type == F64 else np.int64)
            if n is None:
                n = len(vals)
            if len(vals) != n:
                raise OracleError("ragged columns")
            valid = np.ones(len(vals), dtype=bool) if c.valid is None else np.asarray(c.valid, dtype=bool)
            if c.name in cols:
                raise OracleError(f"duplicate column {c.name}")
            cols[c.name] = Col_(c.type, vals, valid)
        return NumpyTable(self, cols, n or 0)


class NumpyTable:
    def __init__(self, backend: NumpyBackend, cols: "OrderedDict[str, Col_]", n: int):
        self.backend = backend
        self.cols = cols
        self.n = n

    # ---- CypherTable ------------------------------------------------------------------
    @property
    def size(self) -> int:
        return self.n

    @property
    def physicalColumns(self) -> List[str]:
        return list(self.cols)

    @property
    def columnType(self) -> dict:
        return {k: c.type for k, c in self.cols.items()}

    def to_columns(self):
        return [ColumnOut(k, c.type, c.values, None if c.valid.all() else c.valid) for k, c in self.cols.items()]

    def column(self, name):
        c = self.cols[name]
        return ColumnOut(name, c.type, c.values, None if c.valid.all() else c.valid)

    def _new(self, cols, n) -> "NumpyTable":
        return NumpyTable(self.backend, cols, n)

    def _take(self, idx: np.ndarray, missing: np.ndarray = None) -> "OrderedDict[str, Col_]":
        out = OrderedDict()
        for k, c in self.cols.items():
            safe = np.where(idx < 0, 0, idx) if len(c.values) else np.zeros(len(idx), dtype=np.int64)
            vals = c.values[safe] if len(c.values) else _empty_like(c.type, len(idx))
            valid = (c.valid[safe] if len(c.values) else np.zeros(len(idx), dtype=bool)) & (idx >= 0)
            out[k] = Col_(c.type, vals, valid)
        return out

    # ---- entity tables: EntityTable.verify (okapi-relational/.../api/io/EntityTable.scala:59-65, 105-164) --
    def as_node_table(self, id_col, label_cols=()):
        _verify_entity(self, [(id_col, "id key", I64)], [(c, "optional label", BOOL) for c in label_cols])
        return self

    def as_rel_table(self, id_col, src_col, dst_col, type_cols=()):
        _verify_entity(self, [(id_col, "id key", I64), (src_col, "start node", I64), (dst_col, "end node", I64)],
                       [(c, "relationship type", BOOL) for c in type_cols])
        return self

    def flatten_rel_types(self, type_col, types, out_cols):
        """CAPSRelationshipTable.fromMapping's type flattening (CAPSTable.scala:189-204)."""
        c = self.cols[type_col]
        if c.type != STR:
            raise OracleError(f"relationship type column `{type_col}` of type CTString")
        out = OrderedDict((k, v) for k, v in self.cols.items() if k != type_col)
        for t, name in zip(types, out_cols):
            code = self.backend.dictionary.encode(t)
            out[name] = Col_(BOOL, (c.valid & (c.values == code)).astype(np.int64), np.ones(self.n, dtype=bool))
        return self._new(out, self.n)

    # ---- operators -------------------------------------------------------------------------
    def cache(self):
        return self

    def select(self, *cols):
        for c in cols:
            if c not in self.cols:
                raise OracleError(f"no column {c}")
        return self._new(OrderedDict((c, self.cols[c]) for c in cols), self.n)

    def drop(self, *cols):
        return self._new(OrderedDict((k, v) for k, v in self.cols.items() if k not in cols), self.n)

    def withColumnRenamed(self, old, new):
        if old not in self.cols:
            raise OracleError(f"no column {old}")
        return self._new(OrderedDict(((new if k == old else k), v) for k, v in self.cols.items()), self.n)

    def filter(self, expr):
        ty, vals, valid = evaluate(expr, self)
        keep = valid & (vals != 0) if ty == BOOL else np.zeros(self.n, dtype=bool)
        idx = np.nonzero(keep)[0]
        return self._new(self._take(idx), len(idx))

    def withColumns(self, *columns):
        out = OrderedDict(self.cols)
        for e, name in columns:
            ty, vals, valid = evaluate(e, self)
            if ty < 0:
                ty = getattr(e, "type", -1)
                ty = ty if ty is not None and ty >= 0 else I64
            if ty < LIST:  # a list column is only ever aliased
                vals = vals.astype(np.float64 if ty == F64 else np.int64)
            out[name] = Col_(ty, vals, valid)
        return self._new(out, self.n)

    def join(self, other: "NumpyTable", join_type: str, *pairs):
        for k in self.cols:
            if k in other.cols:
                raise OracleError(f"join inputs share column {k}")
        if join_type == "cross":
            li = np.repeat(np.arange(self.n), other.n)
            ri = np.tile(np.arange(other.n), self.n)
        else:
            lk = [self.cols[a] for a, _ in pairs]
            rk = [other.cols[b] for _, b in pairs]
            li, ri = _equi_join(lk, rk, self.n, other.n, join_type)
        cols = self._take(li)
        for k, v in other._take(ri).items():
            cols[k] = v
        return self._new(cols, len(li))

    def unionAll(self, other: "NumpyTable"):
        if len(self.cols) != len(other.cols):
            raise OracleError("union: column counts differ")
        out = OrderedDict()
        for (k, a), b in zip(self.cols.items(), other.cols.values()):
            if a.type != b.type:
                raise OracleError(f"union: type mismatch on {k}")
            out[k] = Col_(a.type, np.concatenate([a.values, b.values]), np.concatenate([a.valid, b.valid]))
        return self._new(out, self.n + other.n)

    def orderBy(self, *items):
        keys = []
        for name, order in reversed(items):  # np.lexsort: last key is primary
            c = self.cols[name]
            desc = order.lower().startswith("desc")
            v = c.values
            keys.append(-v if desc and c.type == F64 else (~v if desc else v))
            # ASC: nulls first (null flag 0 sorts first); DESC: nulls last
            keys.append(np.where(c.valid, 0, 1) if desc else np.where(c.valid, 1, 0))
        idx = np.lexsort(keys) if keys else np.arange(self.n)
        return self._new(self._take(idx), self.n)

    def skip(self, n):
        idx = np.arange(min(n, self.n), self.n)
        return self._new(self._take(idx), len(idx))

    def limit(self, n):
        idx = np.arange(min(n, self.n))
        return self._new(self._take(idx), len(idx))

    def distinct(self, *cols):
        names = list(cols) if cols else list(self.cols)
        gid, first = _factorize([self.cols[c] for c in names], self.n)
        return self._new(self._take(first), len(first))

    def group(self, by, aggregations):
        if by:
            gid, first = _factorize([self.cols[c] for c in by], self.n)
            ng = len(first)
            out = self.select(*by)._take(first)
        else:
            gid = np.zeros(self.n, dtype=np.int64)
            ng = 1
            out = OrderedDict()
        for kind, inp, distinct, name in aggregations:
            if kind == "count_star":
                out[name] = Col_(I64, np.bincount(gid, minlength=ng).astype(np.int64), np.ones(ng, dtype=bool))
                continue
            c = self.cols[inp]
            m = c.valid
            if kind == "collect":  # sort_array(collect_list / collect_set), SparkTable.scala:169-177
                lists = np.empty(ng, dtype=object)
                for k in range(ng):
                    v = c.values[m & (gid == k)]
                    if distinct:  # collect_set: equal 64-bit words are one value
                        v = np.unique(v.view(np.int64)).view(v.dtype) if len(v) else v
                    lists[k] = np.sort(v, kind="stable")
                out[name] = Col_(LIST + c.type, lists, np.ones(ng, dtype=bool))
                continue
            if c.type >= LIST:
                raise OracleError(f"aggregate {kind} over a list column")
            if kind == "count":
                if distinct:
                    sel = np.nonzero(m)[0]
                    pair = np.stack([gid[sel], c.values[sel].view(np.int64)], axis=1) if len(sel) else np.zeros((0, 2), np.int64)
                    upairs = np.unique(pair, axis=0) if len(sel) else pair
                    cnt = np.bincount(upairs[:, 0], minlength=ng) if len(upairs) else np.zeros(ng, np.int64)
                else:
                    cnt = np.bincount(gid[m], minlength=ng)
                out[name] = Col_(I64, cnt.astype(np.int64), np.ones(ng, dtype=bool))
            elif kind in ("min", "max", "sum", "avg"):
                seen = np.bincount(gid[m], minlength=ng) > 0
                vals = c.values[m]
                g = gid[m]
                if kind == "sum":
                    if c.type == F64:
                        acc = np.zeros(ng, dtype=np.float64)
                        np.add.at(acc, g, vals)
                    else:
                        acc = np.zeros(ng, dtype=np.int64)
                        np.add.at(acc, g, vals)  # wraps like Spark Long sums
                    out[name] = Col_(c.type, acc, seen)
                elif kind == "avg":
                    acc = np.zeros(ng, dtype=np.float64)
                    np.add.at(acc, g, vals.astype(np.float64))
                    cnt = np.bincount(g, minlength=ng)
                    with np.errstate(invalid="ignore", divide="ignore"):
                        res = np.where(cnt > 0, acc / np.maximum(cnt, 1), 0.0)
                    if c.type == I64:  # avg(..).cast(cypherType): an integer average is cast back to Long
                        out[name] = Col_(I64, np.trunc(res).astype(np.int64), seen)
                    else:
                        out[name] = Col_(F64, res, seen)
                else:
                    if c.type == F64:
                        acc = np.full(ng, np.inf if kind == "min" else -np.inf)
                    else:
                        acc = np.full(ng, np.iinfo(np.int64).max if kind == "min" else np.iinfo(np.int64).min,
                                      dtype=np.int64)
                    (np.minimum if kind == "min" else np.maximum).at(acc, g, vals)
                    out[name] = Col_(c.type, np.where(seen, acc, 0).astype(acc.dtype), seen)
            else:
                raise OracleError(f"aggregate {kind}")
        return self._new(out, ng)


# ---- helpers ---------------------------------------------------------------------------------
def _verify_entity(t: NumpyTable, keys, flags):
    """EntityTable.verify: key columns non-nullable of the stated type, canonical column order
    keys ++ flags ++ sorted properties (EntityMapping.allSourceKeys, EntityMapping.scala:50)."""
    for name, what, ty in keys + flags:
        if name not in t.cols:
            raise OracleError(f"table with column key {name}")
        c = t.cols[name]
        if c.type != ty:
            raise OracleError(f"{what} column `{name}` of type {'CTInteger' if ty == I64 else 'CTBoolean'}")
        if not c.valid.all():
            raise OracleError(f"non-nullable type for {what} column `{name}`")
    fixed = [n for n, _, _ in keys + flags]
    want = fixed + sorted(k for k in t.cols if k not in fixed)
    if list(t.cols) != want:
        raise OracleError(f"Columns: {', '.join(want)} expected, got Columns: {', '.join(t.cols)}")


def _key_matrix(cols: Sequence[Col_], n: int, with_nulls: bool) -> np.ndarray:
    parts = []
    for c in cols:
        if c.type >= LIST:
            raise OracleError("list column as a key")
        v = c.values.view(np.int64) if c.values.dtype == np.float64 else c.values
        if with_nulls:
            parts.append(np.where(c.valid, v, 0))
            parts.append((~c.valid).astype(np.int64))
        else:
            parts.append(v)
    return np.stack(parts, axis=1) if parts else np.zeros((n, 0), dtype=np.int64)


def _factorize(cols: Sequence[Col_], n: int):
    """group id per row (nulls group together) and the first row of each group"""
    if n == 0:
        return np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.int64)
    km = _key_matrix(cols, n, with_nulls=True)
    if km.shape[1] == 0:
        return np.zeros(n, dtype=np.int64), np.zeros(1, dtype=np.int64)
    _, first, inv = np.unique(km, axis=0, return_index=True, return_inverse=True)
    return inv.reshape(-1).astype(np.int64), first.astype(np.int64)


def _promote(lc: Col_, rc: Col_) -> Tuple[np.ndarray, np.ndarray]:
    if (lc.type == F64) != (rc.type == F64):
        a = lc.values.astype(np.float64)
        b = rc.values.astype(np.float64)
        return a.view(np.int64), b.view(np.int64)
    a = lc.values.view(np.int64) if lc.values.dtype == np.float64 else lc.values
    b = rc.values.view(np.int64) if rc.values.dtype == np.float64 else rc.values
    return a, b


def _equi_join(lk: List[Col_], rk: List[Col_], nl: int, nr: int, join_type: str):
    lvalid = np.ones(nl, dtype=bool)
    rvalid = np.ones(nr, dtype=bool)
    la, ra = [], []
    for a, b in zip(lk, rk):
        x, y = _promote(a, b)
        la.append(x)
        ra.append(y)
        lvalid &= a.valid
        rvalid &= b.valid
    # joint factorisation of the key tuples of both sides
    L = np.stack(la, axis=1) if la else np.zeros((nl, 0), np.int64)
    R = np.stack(ra, axis=1) if ra else np.zeros((nr, 0), np.int64)
    both = np.concatenate([L, R], axis=0)
    if len(both):
        _, inv = np.unique(both, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
    else:
        inv = np.zeros(0, dtype=np.int64)
    lid = np.where(lvalid, inv[:nl], -1)
    rid = np.where(rvalid, inv[nl:], -2)
    order = np.argsort(rid, kind="stable")
    rs = rid[order]
    lo = np.searchsorted(rs, lid, side="left")
    hi = np.searchsorted(rs, lid, side="right")
    cnt = np.where(lid >= 0, hi - lo, 0)
    li = np.repeat(np.arange(nl), cnt)
    starts = np.repeat(lo, cnt)
    within = np.arange(len(li)) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    ri = order[starts + within] if len(li) else np.zeros(0, dtype=np.int64)
    if join_type in ("left_outer", "full_outer"):
        miss = np.nonzero(cnt == 0)[0]
        li = np.concatenate([li, miss])
        ri = np.concatenate([ri, -np.ones(len(miss), dtype=np.int64)])
    if join_type in ("right_outer", "full_outer"):
        matched = np.zeros(nr, dtype=bool)
        matched[ri[ri >= 0]] = True
        miss = np.nonzero(~matched)[0]
        li = np.concatenate([li, -np.ones(len(miss), dtype=np.int64)])
        ri = np.concatenate([ri, miss])
    return li.astype(np.int64), ri.astype(np.int64)


# ---- expression evaluation (3VL) --------------------------------------------------------------
def evaluate(e, t: NumpyTable):
    """-> (type, values, valid); type -1 = NULL literal of unknown type"""
    n = t.n
    name = type(e).__name__
    if name == "Col":
        c = t.cols[e.name]
        return c.type, c.values, c.valid
    if name == "Lit":
        v = e.value
        if v is None:
            ty = e.type if e.type >= 0 else -1
            return ty, _empty_like(ty, n), np.zeros(n, dtype=bool)
        ty = e.resolved_type()
        if ty == STR:
            code = t.backend.dictionary.encode(v)
            return STR, np.full(n, code, dtype=np.int64), np.ones(n, dtype=bool)
        if ty == F64:
            return F64, np.full(n, float(v)), np.ones(n, dtype=bool)
        return ty, np.full(n, int(v), dtype=np.int64), np.ones(n, dtype=bool)
    if name == "BinOp":
        lt, lv, lm = evaluate(e.left, t)
        rt, rv, rm = evaluate(e.right, t)
        m = lm & rm
        if e.op in ("+", "-", "*"):
            if lt not in (I64, F64) or rt not in (I64, F64):
                return I64, np.zeros(n, np.int64), np.zeros(n, bool)
            if lt == F64 or rt == F64:
                a, b = lv.astype(np.float64), rv.astype(np.float64)
                res = a + b if e.op == "+" else (a - b if e.op == "-" else a * b)
                return F64, res, m
            with np.errstate(over="ignore"):
                a, b = lv.astype(np.int64), rv.astype(np.int64)
                res = a + b if e.op == "+" else (a - b if e.op == "-" else a * b)
            return I64, res, m
        if e.op in ("&", "|", "<<", ">>>"):  # Long only (SparkSQLExprMapper.scala:264-274)
            if lt != I64 or rt != I64:
                return I64, np.zeros(n, np.int64), np.zeros(n, bool)
            a, b = lv.astype(np.int64).view(np.uint64), rv.astype(np.int64).view(np.uint64)
            sh = b & np.uint64(63)  # Java long shift count
            res = {"&": lambda: a & b, "|": lambda: a | b, "<<": lambda: a << sh, ">>>": lambda: a >> sh}[e.op]()
            return I64, res.view(np.int64), m
        numeric = lt in (I64, F64) and rt in (I64, F64)
        if not numeric and lt != rt:
            return BOOL, np.zeros(n, np.int64), np.zeros(n, bool)
        if numeric and (lt == F64 or rt == F64):
            a, b = lv.astype(np.float64), rv.astype(np.float64)
            m = m & ~np.isnan(a) & ~np.isnan(b)
        else:
            a, b = lv, rv
        op = {"=": np.equal, "<>": np.not_equal, "<": np.less, "<=": np.less_equal, ">": np.greater,
              ">=": np.greater_equal}[e.op]
        return BOOL, op(a, b).astype(np.int64), m
    if name == "Not":
        ty, v, m = evaluate(e.arg, t)
        return BOOL, (v == 0).astype(np.int64), m
    if name in ("Ands", "Ors"):
        is_and = name == "Ands"
        decided = np.zeros(n, dtype=bool)
        any_null = np.zeros(n, dtype=bool)
        for a in e.args:
            ty, v, m = evaluate(a, t)
            any_null |= ~m
            decided |= m & ((v == 0) if is_and else (v != 0))
        val = np.where(decided, not is_and, is_and).astype(np.int64)
        return BOOL, val, decided | ~any_null
    if name == "IsNull":
        _, _, m = evaluate(e.arg, t)
        return BOOL, (~m).astype(np.int64), np.ones(n, dtype=bool)
    if name == "IsNotNull":
        _, _, m = evaluate(e.arg, t)
        return BOOL, m.astype(np.int64), np.ones(n, dtype=bool)
    if name == "In":
        xt, xv, xm = evaluate(e.arg, t)
        hit = np.zeros(n, dtype=bool)
        unknown = ~xm
        for v in e.values:
            vt, vv, vm = evaluate(v, t)
            if xt in (I64, F64) and vt in (I64, F64):
                same = xv.astype(np.float64) == vv.astype(np.float64)
            elif xt == vt:
                same = xv == vv
            else:
                unknown |= np.ones(n, dtype=bool)
                continue
            hit |= xm & vm & same
            unknown |= ~vm
        return BOOL, hit.astype(np.int64), hit | ~unknown
    if name == "Coalesce":
        ty_out, vals, valid = -1, None, np.zeros(n, dtype=bool)
        for a in e.args:
            ty, v, m = evaluate(a, t)
            if vals is None:
                vals = v.copy()
            take = ~valid & m
            vals = np.where(take, v, vals)
            valid |= m
            if ty >= 0:
                ty_out = ty
        return ty_out, vals, valid
    if name == "Case":  # first TRUE alternative, else default (SparkSQLExprMapper.scala:283-298)
        if e.default is not None:
            ty_out, vals, valid = evaluate(e.default, t)
            vals, valid = vals.copy(), valid.copy()
        else:
            ty_out, vals, valid = -1, np.zeros(n, np.int64), np.zeros(n, dtype=bool)
        for p, v in reversed(e.alternatives):
            _, pv, pm = evaluate(p, t)
            vt, vv, vm = evaluate(v, t)
            take = pm & (pv != 0)
            if vals.dtype != vv.dtype:
                vals = vals.astype(vv.dtype)
            vals = np.where(take, vv, vals)
            valid = np.where(take, vm, valid)
            if vt >= 0:
                ty_out = vt
        return ty_out, vals, valid
    if name == "Neg":
        ty, v, m = evaluate(e.arg, t)
        return ty, -v, m
    raise OracleError(f"expression {e!r}")
