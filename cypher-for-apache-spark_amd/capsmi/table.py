"""Host mirror of CAPS's backend table interface over the C ABI.

``GpuTable`` follows the member names, argument meaning and error behaviour of
    trait Table[T <: Table[T]] extends CypherTable
    okapi-relational/src/main/scala/org/opencypher/okapi/relational/api/table/Table.scala:43-176
as implemented for Spark by DataFrameTable (spark-cypher/.../impl/table/SparkTable.scala:47-257),
so that a relational plan written against ``Table`` runs unchanged on the device.
Every operator executes in libcapsmi.so (HIP, gfx950); Python only marshals handles.
"""
from __future__ import annotations

import bisect
import contextlib
import ctypes
import threading
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .expr import BOOL, F64, I64, LIST, STR, CapsmiExpr, Col, Expr, Lit, compile_program, to_ctypes

_TLS = threading.local()

_EXPR_PTR = ctypes.POINTER(CapsmiExpr)
_LIT_PROGS = {}  # (python type, value, declared type) -> one-node program of a Boolean / Long / null literal

JOIN_TYPES = {"inner": 0, "left_outer": 1, "right_outer": 2, "full_outer": 3, "cross": 4}
AGG_KINDS = {"count_star": 0, "count": 1, "min": 2, "max": 3, "sum": 4, "avg": 5, "collect": 6}


@dataclass
class ColumnData:
    """Host column: ``values`` int64 (I64/BOOL/STR codes) or float64 (F64); ``valid`` bool mask or None.
    A list column (type LIST + element type) holds one numpy array of element words per row (object
    array; float64 elements for F64 lists)."""
    name: str
    type: int
    values: np.ndarray
    valid: Optional[np.ndarray] = None

    def words(self) -> np.ndarray:
        v = np.asarray(self.values)
        if self.type == F64:
            return np.ascontiguousarray(v.astype(np.float64)).view(np.int64)
        return np.ascontiguousarray(v.astype(np.int64))


def decode_value(ty: int, v, dictionary):
    """One exported value as a Python value (CypherValue analogue); lists element by element."""
    if ty >= LIST:
        return [decode_value(ty - LIST, x, dictionary) for x in v]
    if ty == BOOL:
        return bool(v)
    if ty == STR:
        return dictionary.decode(int(v))
    if ty == F64:
        return float(v)
    return int(v)


class StringDictionary:
    """Order-preserving dictionary for CTString values (include/capsmi.h: STR columns are codes).

    Codes are stable: once a string has a code it keeps it for the life of the dictionary, so device
    columns encoded earlier (a first graph, a driving table) stay valid when later graphs or
    literals bring new strings.  Order is preserved by allocating codes from gaps: a batch of new
    strings that falls between two known neighbours is spread evenly over the open interval between
    their codes (the first batch over [-2^62, 2^62]).  Equality and ordering on codes therefore equal
    equality and ordering on strings.  Every string that is encoded -- query literals included --
    is inserted, so two distinct strings never share a code.  A gap only runs out after ~60 nested
    insertions at one spot; that raises instead of renumbering codes already on the device."""

    LO, HI = -(1 << 62), 1 << 62

    def __init__(self, strings: Iterable[str] = ()):
        self._sorted: List[str] = []
        self._codes: List[int] = []
        self._by_code = {}
        self.extend(strings)

    def extend(self, strings: Iterable[str]) -> None:
        new = sorted(set(strings) - set(self._by_code.values()))
        if not new:
            return
        # group the new strings by the gap (insertion point) they fall into
        groups = {}
        for x in new:
            groups.setdefault(bisect.bisect_left(self._sorted, x), []).append(x)
        placed = []
        for i, xs in groups.items():
            lo = self._codes[i - 1] if i > 0 else self.LO
            hi = self._codes[i] if i < len(self._codes) else self.HI
            step = (hi - lo) // (len(xs) + 1)
            if step < 1:
                raise OverflowError("string dictionary: no code left between "
                                    f"{self._sorted[i - 1] if i > 0 else None!r} and "
                                    f"{self._sorted[i] if i < len(self._sorted) else None!r}")
            placed += [(lo + (k + 1) * step, x) for k, x in enumerate(xs)]
        for c, x in placed:
            self._by_code[c] = x
        merged = sorted(list(zip(self._codes, self._sorted)) + placed)
        self._codes = [c for c, _ in merged]
        self._sorted = [x for _, x in merged]

    def encode(self, s: str) -> int:
        i = bisect.bisect_left(self._sorted, s)
        if i < len(self._sorted) and self._sorted[i] == s:
            return self._codes[i]
        self.extend([s])
        return self._codes[bisect.bisect_left(self._sorted, s)]

    def decode(self, code: int) -> str:
        try:
            return self._by_code[int(code)]
        except KeyError:
            raise KeyError(f"code {code} is not a dictionary string") from None

    def __len__(self) -> int:
        return len(self._sorted)


class Session:
    """One device, one HIP stream (CAPSSession.local analogue, spark-cypher/.../api/CAPSSession.scala:110-131)."""

    def __init__(self, device: int = 0, dictionary: Optional[StringDictionary] = None):
        self._h = ctypes.c_void_p()
        _lib.call("capsmi_session_create", device, ctypes.byref(self._h))
        self.device = device
        self.dictionary = dictionary or StringDictionary()

    @property
    def handle(self):
        return self._h

    def set_stream(self, hip_stream: Optional[int]) -> None:
        """Run on `hip_stream` (an int handle, e.g. ``torch.cuda.current_stream().cuda_stream``;
        0 is the null stream, torch's default), or on the session's own stream for None."""
        if hip_stream is None:
            _lib.call("capsmi_session_set_stream", self._h, ctypes.c_void_p(0))
        else:
            _lib.call("capsmi_session_use_stream", self._h, ctypes.c_void_p(hip_stream))

    def sync(self) -> None:
        _lib.call("capsmi_session_sync", self._h)

    def set_config(self, name: str, value: Optional[str]) -> None:
        """One CAPSMI_* knob for this session (include/capsmi.h capsmi_session_set_config); the environment is
        read only when the session is created.  None = back to the environment's value or the default."""
        _lib.call("capsmi_session_set_config", self._h, name.encode(),
                  None if value is None else str(value).encode())

    @contextlib.contextmanager
    def configured(self, **knobs):
        """``with session.configured(CAPSMI_COUNT="atomic"): ...`` -- the knobs for the block, then back to the
        environment's values (or the defaults)."""
        for k, v in knobs.items():
            self.set_config(k, v)
        try:
            yield self
        finally:
            for k in knobs:
                self.set_config(k, None)

    def close(self) -> None:
        if self._h:
            _lib.call("capsmi_session_destroy", self._h)
            self._h = ctypes.c_void_p()

    def table(self, columns: Sequence[ColumnData]) -> "GpuTable":
        """CAPSNodeTable / CAPSRelationshipTable ingest: copies host columns to the device."""
        n = len(columns[0].values) if columns else 0
        descs = (_lib.ColDesc * max(1, len(columns)))()
        keep = []
        for i, c in enumerate(columns):
            if len(c.values) != n:
                raise _lib.IllegalArgumentException(f"column {c.name} has {len(c.values)} rows, expected {n}")
            w = c.words()
            keep.append(w)
            descs[i].name = c.name.encode()
            descs[i].type = c.type
            descs[i].data = w.ctypes.data if n else None
            if c.valid is not None:
                vb = np.ascontiguousarray(np.asarray(c.valid, dtype=np.uint8))
                keep.append(vb)
                descs[i].valid = vb.ctypes.data if n else None
            else:
                descs[i].valid = None
        out = ctypes.c_void_p()
        _lib.call("capsmi_table_from_host", self._h, len(columns), descs, n, ctypes.byref(out))
        return GpuTable(self, out)

    def encode_str(self, s: str) -> int:
        return self.dictionary.encode(s)

    def read_csv(self, paths: Sequence[str], names: Sequence[str], types: Sequence[int], delimiter: Optional[str] = ",",
                 comment: Optional[str] = None, row_id_col: Optional[str] = None) -> "GpuTable":
        """DataFrameReader.csv with an explicit schema, parsed natively by host threads into a device
        table (include/capsmi.h capsmi_read_csv).  ``delimiter`` is Spark's one-character ``sep``;
        None opts in to whitespace splitting (runs of blanks).  String fields are encoded with this
        session's dictionary."""
        def intern(_ctx, ptr, n):
            return self.dictionary.encode(ctypes.string_at(ptr, n).decode("utf-8"))

        cb = _lib.INTERN_FN(intern)
        tys = (ctypes.c_int32 * max(1, len(types)))(*types)
        out = ctypes.c_void_p()
        _lib.call("capsmi_read_csv", self._h, len(paths), _lib.strs(list(paths)),
                  b"\0" if delimiter is None else delimiter.encode()[:1],
                  (comment or "\0").encode()[:1], len(names), _lib.strs(list(names)), tys, cb, None,
                  row_id_col.encode() if row_id_col else None, ctypes.byref(out))
        return GpuTable(self, out)

    def compact_graph(self, nodes: Sequence["GpuTable"], rels: Sequence["GpuTable"]) -> int:
        """Dense ids for one graph's registered node / relationship tables (include/capsmi.h
        capsmi_graph_compact); returns the number of dense ids."""
        na = (ctypes.c_void_p * max(1, len(nodes)))(*[t.handle for t in nodes])
        ra = (ctypes.c_void_p * max(1, len(rels)))(*[t.handle for t in rels])
        n = ctypes.c_int64()
        _lib.call("capsmi_graph_compact", self._h, len(nodes), na, len(rels), ra, ctypes.byref(n))
        return n.value

    def compact_if_sparse(self, nodes: Sequence["GpuTable"], rels: Sequence["GpuTable"]) -> bool:
        """Compact when the tables' ids do not fit the fused kernels' window of 2^30 ids."""
        spans = [t.entity() for t in list(nodes) + list(rels)]
        spans = [(lo, hi) for k, lo, hi in spans if k and hi > lo]
        if not spans or max(h for _, h in spans) - min(l for l, _ in spans) <= (1 << 30):
            return False
        self.compact_graph(nodes, rels)
        return True

    def set_params(self, values: Sequence[object]) -> None:
        """Query parameters for ``expr.Param(i)`` (the CypherMap of SparkSQLExprMapper.scala:86-92):
        ``values[i]`` is a Python scalar (int, float, bool, str, None) or a list of them (usable as the
        element list of ``In``).  Strings are dictionary-encoded; an int list with a float is Double."""
        from .expr import BOOL, F64, I64, STR, _lit_bits

        def type_of(v):
            return BOOL if isinstance(v, bool) else I64 if isinstance(v, int) else F64 if isinstance(v, float) \
                else STR if isinstance(v, str) else None

        keep, arr = [], (_lib.Param * max(1, len(values)))()
        for i, v in enumerate(values):
            items = list(v) if isinstance(v, (list, tuple)) else [v]
            tys = {type_of(x) for x in items} - {None}
            if tys == {I64, F64}:
                tys = {F64}
            if len(tys) > 1:
                raise _lib.IllegalArgumentException(f"parameter {i}: mixed value types")
            ty = tys.pop() if tys else I64
            vals = (_lib.Value * max(1, len(items)))()
            for k, x in enumerate(items):
                vals[k].is_null = 1 if x is None else 0
                vals[k].ival = 0 if x is None else _lit_bits(x, ty, self.encode_str)
            keep.append(vals)
            arr[i].type, arr[i].is_list, arr[i].count, arr[i].values = ty, int(isinstance(v, (list, tuple))), \
                len(items), ctypes.cast(vals, ctypes.c_void_p)
        _lib.call("capsmi_session_set_params", self._h, len(values), arr)

    def set_fused(self, enabled: bool) -> None:
        """Route lazy plans of the Expand shapes to the fused kernels (default) or run them operator
        by operator (include/capsmi.h capsmi_session_set_fused)."""
        _lib.call("capsmi_session_set_fused", self._h, 1 if enabled else 0)

    def set_unrouted_limit(self, max_bytes: int) -> None:
        """Refuse unrouted joins whose estimated output exceeds `max_bytes` (0: no limit;
        include/capsmi.h capsmi_session_set_unrouted_limit)."""
        _lib.call("capsmi_session_set_unrouted_limit", self._h, int(max_bytes))

    def set_csv_partitioning(self, default_parallelism: int, max_partition_bytes: int = 128 << 20,
                             open_cost_bytes: int = 4 << 20) -> None:
        """read_csv row ids as Spark's monotonically_increasing_id over its file-scan partitions
        (include/capsmi.h capsmi_session_set_csv_partitioning); 0 = one partition (row numbers)."""
        _lib.call("capsmi_session_set_csv_partitioning", self._h, int(default_parallelism), int(max_partition_bytes),
                  int(open_cost_bytes))

    def set_ranks(self, rank: int, world: int, collective=None) -> None:
        """This process is rank `rank` of `world`; `collective(op, send_ptr, recv_ptr, count, dtype)`
        runs the exchange on this session's stream (capsmi.dist.TorchCollective; include/capsmi.h
        capsmi_session_set_ranks)."""
        if collective is None:
            self._coll = None
            _lib.call("capsmi_session_set_ranks", self._h, rank, world, _lib.COLLECTIVE_FN(), None)
            return

        def fn(_ctx, op, send, recv, count, dtype):
            try:
                collective(op, send, recv, count, dtype)
                return 0
            except Exception as e:  # reported as CAPSMI_ERR_DEVICE by the library
                self.collective_error = e
                return 1

        self._coll = _lib.COLLECTIVE_FN(fn)  # kept alive with the session
        _lib.call("capsmi_session_set_ranks", self._h, rank, world, self._coll, None)

    def route_count(self, name: str) -> int:
        """Plans routed to fused entry point `name` ("expand", "expand_count", "two_hop", "triangle",
        "var_length") so far; "miss" counts materialisations where a pattern ran unrouted."""
        v = ctypes.c_int64()
        _lib.call("capsmi_session_route_count", self._h, name.encode(), ctypes.byref(v))
        return v.value


class GpuTable:
    """A device-resident, immutable table; each operator returns a new GpuTable."""

    def __init__(self, session: Session, handle: ctypes.c_void_p):
        self.session = session
        self._h = handle
        self._schema = None  # (names, types): tables are immutable, so the schema is read once
        self._index = None  # name -> position (expression compilation)
        self._leaf = None  # column name -> its one-node program (the planner's scans project columns)
        self._wcols = None  # withColumns argument arrays of column / literal projections, by structure

    # ---- lifetime ------------------------------------------------------------------------
    @property
    def handle(self):
        return self._h

    def release(self) -> None:
        if self._h:
            _lib.call("capsmi_table_release", self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            if self._h and _lib._lib is not None:
                _lib._lib.capsmi_table_release(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass

    def _wrap(self, h) -> "GpuTable":
        return GpuTable(self.session, h)

    # ---- CypherTable (okapi-api/.../api/table/CypherTable.scala:41-68) -------------------
    @property
    def size(self) -> int:
        v = ctypes.c_int64()
        _lib.call("capsmi_table_size", self._h, ctypes.byref(v))
        return v.value

    _MAXC = 256

    def _read_schema(self):
        if self._schema is None:  # one call for names and types (include/capsmi.h capsmi_table_schema)
            n = ctypes.c_int32()
            buf = getattr(_TLS, "names", None)  # a reusable name buffer per thread (ctypes drops the GIL)
            if buf is None:
                buf = _TLS.names = ctypes.create_string_buffer(16384)
            types = (ctypes.c_int32 * self._MAXC)()
            _lib.call("capsmi_table_schema", self._h, ctypes.byref(n), buf, len(buf), types, None, self._MAXC)
            if n.value > self._MAXC:
                raise _lib.NotImplementedException(f"table with {n.value} columns")
            raw, names, pos = buf.raw, [], 0  # n NUL-terminated names (not a split of the whole buffer)
            for _ in range(n.value):
                end = raw.index(b"\0", pos)
                names.append(raw[pos:end].decode())
                pos = end + 1
            self._schema = (names, list(types[:n.value]))
        return self._schema

    @property
    def physicalColumns(self) -> List[str]:
        return list(self._read_schema()[0])

    @property
    def columnType(self) -> dict:
        names, types = self._read_schema()
        return dict(zip(names, types))

    # ---- entity tables (include/capsmi.h capsmi_node_table / capsmi_rel_table) -----------------
    def as_node_table(self, id_col: str, label_cols: Sequence[str] = ()) -> "GpuTable":
        """CAPSNodeTable + EntityTable.verify (EntityTable.scala:59-65, 105-131)."""
        out = ctypes.c_void_p()
        _lib.call("capsmi_node_table", self._h, id_col.encode(), len(label_cols), _lib.strs(label_cols),
                  ctypes.byref(out))
        return self._wrap(out)

    def as_rel_table(self, id_col: str, src_col: str, dst_col: str, type_cols: Sequence[str] = ()) -> "GpuTable":
        """CAPSRelationshipTable + EntityTable.verify (EntityTable.scala:59-65, 137-164)."""
        out = ctypes.c_void_p()
        _lib.call("capsmi_rel_table", self._h, id_col.encode(), src_col.encode(), dst_col.encode(), len(type_cols),
                  _lib.strs(type_cols), ctypes.byref(out))
        return self._wrap(out)

    @property
    def partitioned(self) -> bool:
        """Whether the rows are this rank's partition of a distributed result."""
        v = ctypes.c_int32()
        _lib.call("capsmi_table_partitioned", self._h, ctypes.byref(v))
        return bool(v.value)

    def owned_rows(self, col: str, id_lo: int, id_hi: int) -> "GpuTable":
        """The rows whose Long column `col` holds an id this rank owns (include/capsmi.h capsmi_owned_rows)."""
        out = ctypes.c_void_p()
        _lib.call("capsmi_owned_rows", self.session.handle, self._h, col.encode(), id_lo, id_hi, ctypes.byref(out))
        return self._wrap(out)

    def entity(self) -> Tuple[int, int, int]:
        """(kind: 0 plain / 1 node / 2 relationship, id_lo, id_hi)"""
        k, lo, hi = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
        _lib.call("capsmi_table_entity", self._h, ctypes.byref(k), ctypes.byref(lo), ctypes.byref(hi))
        return k.value, lo.value, hi.value

    def flatten_rel_types(self, type_col: str, types: Sequence[str], out_cols: Sequence[str]) -> "GpuTable":
        """CAPSRelationshipTable.fromMapping's String type column -> Boolean flags (CAPSTable.scala:189-204)."""
        codes = (ctypes.c_int64 * max(1, len(types)))(*[self.session.encode_str(t) for t in types])
        out = ctypes.c_void_p()
        _lib.call("capsmi_flatten_rel_types", self._h, type_col.encode(), len(types), codes, _lib.strs(out_cols),
                  ctypes.byref(out))
        return self._wrap(out)

    def column_index(self, name: str) -> int:
        v = ctypes.c_int32()
        _lib.call("capsmi_table_column_index", self._h, name.encode(), ctypes.byref(v))
        if v.value < 0:
            raise _lib.IllegalArgumentException(f"no column named '{name}'")
        return v.value

    def column(self, name: str, offset: int = 0, n: Optional[int] = None) -> ColumnData:
        idx = self.column_index(name)
        size = self.size
        if n is None:
            n = size - offset
        ty = self.columnType[name]
        if ty >= LIST:
            return self._list_column(name, idx, ty, offset, n)
        vals = np.empty(n, dtype=np.int64)
        valid = np.empty(n, dtype=np.uint8)
        _lib.call("capsmi_table_export", self._h, idx, vals.ctypes.data if n else None,
                  valid.ctypes.data if n else None, offset, n)
        nullable = ctypes.c_int32()
        _lib.call("capsmi_table_column_nullable", self._h, idx, ctypes.byref(nullable))
        if ty == F64:
            vals = vals.view(np.float64)
        return ColumnData(name, ty, vals, valid.astype(bool) if nullable.value else None)

    def _list_column(self, name: str, idx: int, ty: int, offset: int, n: int) -> ColumnData:
        """A list column's rows (include/capsmi.h capsmi_table_export_list)."""
        total = ctypes.c_int64()
        _lib.call("capsmi_table_export_list", self._h, idx, offset, n, None, None, None, 0, ctypes.byref(total))
        offs = np.empty(n + 1, dtype=np.int64)
        valid = np.empty(max(1, n), dtype=np.uint8)
        vals = np.empty(max(1, total.value), dtype=np.int64)
        _lib.call("capsmi_table_export_list", self._h, idx, offset, n, offs.ctypes.data, valid.ctypes.data,
                  vals.ctypes.data, len(vals), ctypes.byref(total))
        if ty - LIST == F64:
            vals = vals.view(np.float64)
        rows = np.empty(n, dtype=object)
        for i in range(n):
            rows[i] = vals[offs[i]:offs[i + 1]]
        nullable = ctypes.c_int32()
        _lib.call("capsmi_table_column_nullable", self._h, idx, ctypes.byref(nullable))
        return ColumnData(name, ty, rows, valid[:n].astype(bool) if nullable.value else None)

    def to_columns(self) -> List[ColumnData]:
        return [self.column(c) for c in self.physicalColumns]

    def rows(self) -> List[dict]:
        """CypherTable.rows: host rows with strings decoded."""
        cols = self.to_columns()
        n = self.size
        out = []
        for r in range(n):
            row = {}
            for c in cols:
                if c.valid is not None and not c.valid[r]:
                    row[c.name] = None
                    continue
                row[c.name] = decode_value(c.type, c.values[r], self.session.dictionary)
            out.append(row)
        return out

    def fingerprint(self, cols: Sequence[str]) -> Tuple[int, int, int]:
        cnt, s, x = ctypes.c_int64(), ctypes.c_uint64(), ctypes.c_uint64()
        _lib.call("capsmi_table_fingerprint", self._h, len(cols), _lib.strs(cols), ctypes.byref(cnt),
                  ctypes.byref(s), ctypes.byref(x))
        return cnt.value, s.value, x.value

    # ---- Table[T] operators ----------------------------------------------------------------
    def cache(self) -> "GpuTable":
        out = ctypes.c_void_p()
        _lib.call("capsmi_cache", self._h, ctypes.byref(out))
        return self._wrap(out)

    def select(self, *cols: str) -> "GpuTable":
        out = ctypes.c_void_p()
        _lib.call("capsmi_select", self._h, len(cols), _lib.strs(cols), ctypes.byref(out))
        return self._wrap(out)

    def _column_index(self) -> dict:
        if self._index is None:  # name -> position, built once per table (expressions are compiled per column)
            self._index = {n: i for i, n in enumerate(self._read_schema()[0])}
        return self._index

    def _program(self, e: Expr):
        if type(e) is Col:  # the common leaf: one program per (table, column), reused (C copies it)
            if self._leaf is None:
                self._leaf = {}
            hit = self._leaf.get(e.name)
            if hit is not None:
                return 1, hit
        elif type(e) is Lit and (e.value is None or type(e.value) in (bool, int)):  # label flags, nulls
            key = (type(e.value), e.value, e.type)
            hit = _LIT_PROGS.get(key)
            if hit is None:
                hit = _LIT_PROGS[key] = to_ctypes(compile_program(e, None, None))
            return 1, hit
        index = self._column_index()

        def col(name: str) -> int:
            if name not in index:
                raise _lib.IllegalArgumentException(f"expression references unknown column '{name}'")
            return index[name]

        prog = compile_program(e, col, self.session.encode_str)
        arr = to_ctypes(prog)
        if type(e) is Col:
            self._leaf[e.name] = arr
        return len(prog), arr

    def filter(self, expr: Expr) -> "GpuTable":
        n, prog = self._program(expr)
        out = ctypes.c_void_p()
        _lib.call("capsmi_filter", self._h, n, prog, ctypes.byref(out))
        return self._wrap(out)

    def drop(self, *cols: str) -> "GpuTable":
        out = ctypes.c_void_p()
        _lib.call("capsmi_drop", self._h, len(cols), _lib.strs(cols), ctypes.byref(out))
        return self._wrap(out)

    def join(self, other: "GpuTable", join_type: str, *join_cols: Tuple[str, str]) -> "GpuTable":
        if join_type not in JOIN_TYPES:
            raise _lib.IllegalArgumentException(f"join type {join_type}")
        out = ctypes.c_void_p()
        lc = [a for a, _ in join_cols]
        rc = [b for _, b in join_cols]
        _lib.call("capsmi_join", self._h, other._h, JOIN_TYPES[join_type], len(join_cols), _lib.strs(lc),
                  _lib.strs(rc), ctypes.byref(out))
        return self._wrap(out)

    def unionAll(self, other: "GpuTable") -> "GpuTable":
        out = ctypes.c_void_p()
        _lib.call("capsmi_union_all", self._h, other._h, ctypes.byref(out))
        return self._wrap(out)

    def orderBy(self, *items: Tuple[str, str]) -> "GpuTable":
        cols = [c for c, _ in items]
        desc = (ctypes.c_int32 * max(1, len(items)))(*[1 if o.lower().startswith("desc") else 0 for _, o in items])
        out = ctypes.c_void_p()
        _lib.call("capsmi_order_by", self._h, len(items), _lib.strs(cols), desc, ctypes.byref(out))
        return self._wrap(out)

    def skip(self, n: int) -> "GpuTable":
        out = ctypes.c_void_p()
        _lib.call("capsmi_skip", self._h, n, ctypes.byref(out))
        return self._wrap(out)

    def limit(self, n: int) -> "GpuTable":
        out = ctypes.c_void_p()
        _lib.call("capsmi_limit", self._h, n, ctypes.byref(out))
        return self._wrap(out)

    def distinct(self, *cols: str) -> "GpuTable":
        out = ctypes.c_void_p()
        if cols:  # DataFrameTable.distinct(cols) = dropDuplicates(cols), SparkTable.scala:234-235
            _lib.call("capsmi_distinct_on", self._h, len(cols), _lib.strs(cols), ctypes.byref(out))
        else:
            _lib.call("capsmi_distinct", self._h, ctypes.byref(out))
        return self._wrap(out)

    def group(self, by: Sequence[str], aggregations: Sequence[Tuple[str, Optional[str], bool, str]]) -> "GpuTable":
        """``aggregations``: (kind, input column, distinct, output column); kind in AGG_KINDS."""
        aggs = (_lib.Agg * max(1, len(aggregations)))()
        for i, (kind, inp, distinct, outname) in enumerate(aggregations):
            aggs[i].kind = AGG_KINDS[kind]
            aggs[i].distinct = 1 if distinct else 0
            aggs[i].input = inp.encode() if inp else None
            aggs[i].output = outname.encode()
        out = ctypes.c_void_p()
        _lib.call("capsmi_group", self._h, len(by), _lib.strs(by), len(aggregations), aggs, ctypes.byref(out))
        return self._wrap(out)

    def withColumns(self, *columns: Tuple[Expr, str]) -> "GpuTable":
        # the scans' projections (columns and label / null literals) repeat on the same entity tables
        # query after query: their argument arrays are kept per table, keyed by their structure
        key = []
        for e, name in columns:
            if type(e) is Col:
                key.append((name, e.name))
            elif type(e) is Lit and (e.value is None or type(e.value) in (bool, int)):
                key.append((name, type(e.value), e.value, e.type))
            else:
                key = None
                break
        if key is not None:
            key = tuple(key)
            hit = self._wcols.get(key) if self._wcols is not None else None
            if hit is not None:
                out = ctypes.c_void_p()
                _lib.call("capsmi_with_columns", self._h, len(columns), hit[0], ctypes.byref(out))
                return self._wrap(out)
        arr = (_lib.ExprColumn * max(1, len(columns)))()
        keep = []
        for i, (e, name) in enumerate(columns):
            n, prog = self._program(e)
            keep.append(prog)
            arr[i].name = name.encode()
            arr[i].nnodes = n
            arr[i].prog = ctypes.cast(prog, _EXPR_PTR)
        if key is not None:
            if self._wcols is None or len(self._wcols) > 256:
                self._wcols = {}
            self._wcols[key] = (arr, keep)  # keep: the programs the array points into
        out = ctypes.c_void_p()
        _lib.call("capsmi_with_columns", self._h, len(columns), arr, ctypes.byref(out))
        return self._wrap(out)

    def withColumnRenamed(self, old: str, new: str) -> "GpuTable":
        out = ctypes.c_void_p()
        _lib.call("capsmi_with_column_renamed", self._h, old.encode(), new.encode(), ctypes.byref(out))
        return self._wrap(out)

    def show(self, rows: int = 20) -> None:
        for r in self.limit(rows).rows():
            print(r)
