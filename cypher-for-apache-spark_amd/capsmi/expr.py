"""Expression trees handed to ``Table.filter`` / ``Table.withColumns``.

The analogue of okapi's ``Expr`` hierarchy (okapi-ir/src/main/scala/org/opencypher/okapi/ir/api/expr/Expr.scala)
restricted to what SparkSQLExprMapper maps for the pattern-matching path
(spark-cypher/src/main/scala/org/opencypher/spark/impl/SparkSQLExprMapper.scala:81-312):
column references (a Var / Property / HasLabel / HasType resolves to a physical column of the
RecordHeader, :97-105), literals and parameters (:86-92, :111-117), Equals (:120), Not (:121),
IsNull / IsNotNull (:122-123), Ands / Ors (:132-136), In (:138-145), < <= > >= (:147-150),
Add / Subtract / Multiply, and the id-tag vocabulary BitwiseAnd / BitwiseOr / ShiftLeft /
ShiftRightUnsigned (:264-274) and CaseExpr (:283-298).

``compile_program`` lowers a tree to the postfix ``capsmi_expr`` program of include/capsmi.h.
"""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass
from typing import Callable, Sequence, Tuple, Union

# physical types (include/capsmi.h)
I64, BOOL, F64, STR = 0, 1, 2, 3
LIST = 8  # list column of element type t: LIST + t (include/capsmi.h CAPSMI_LIST_*; Collect results)
TYPE_NAMES = {I64: "I64", BOOL: "BOOL", F64: "F64", STR: "STR"}

# expression opcodes (include/capsmi.h CAPSMI_X_*)
X_COL, X_LIT, X_NULL, X_EQ, X_NEQ, X_LT, X_LE, X_GT, X_GE, X_NOT, X_AND, X_OR = range(12)
X_ISNULL, X_ISNOTNULL, X_IN, X_ADD, X_SUB, X_MUL, X_NEG, X_COALESCE = range(12, 20)
X_BITAND, X_BITOR, X_SHL, X_SHRU, X_CASE, X_PARAM = range(20, 26)

BIN_OPS = {"=": X_EQ, "<>": X_NEQ, "<": X_LT, "<=": X_LE, ">": X_GT, ">=": X_GE, "+": X_ADD, "-": X_SUB, "*": X_MUL,
           "&": X_BITAND, "|": X_BITOR, "<<": X_SHL, ">>>": X_SHRU}


class Expr:
    """Base class; trees are immutable value objects."""

    # small builder conveniences so planner code reads like Cypher
    def __eq__(self, other):  # type: ignore[override]
        return type(self) is type(other) and self.__dict__ == other.__dict__

    def __hash__(self):
        return hash((type(self).__name__, repr(self)))


@dataclass(frozen=True, eq=False)
class Col(Expr):
    name: str


@dataclass(frozen=True, eq=False)
class Lit(Expr):
    """A literal.  ``value`` is a Python int / bool / float / str (strings are dictionary-encoded
    by the session before reaching the device) or None for NULL."""
    value: object
    type: int = -1

    def resolved_type(self) -> int:
        if self.type >= 0:
            return self.type
        v = self.value
        if isinstance(v, bool):
            return BOOL
        if isinstance(v, int):
            return I64
        if isinstance(v, float):
            return F64
        if isinstance(v, str):
            return STR
        return -1


@dataclass(frozen=True, eq=False)
class BinOp(Expr):
    op: str
    left: Expr
    right: Expr


@dataclass(frozen=True, eq=False)
class Not(Expr):
    arg: Expr


@dataclass(frozen=True, eq=False)
class Neg(Expr):
    arg: Expr


@dataclass(frozen=True, eq=False)
class Ands(Expr):
    args: Tuple[Expr, ...]


@dataclass(frozen=True, eq=False)
class Ors(Expr):
    args: Tuple[Expr, ...]


@dataclass(frozen=True, eq=False)
class IsNull(Expr):
    arg: Expr


@dataclass(frozen=True, eq=False)
class IsNotNull(Expr):
    arg: Expr


@dataclass(frozen=True, eq=False)
class In(Expr):
    arg: Expr
    values: Tuple[Expr, ...]


@dataclass(frozen=True, eq=False)
class Coalesce(Expr):
    args: Tuple[Expr, ...]


@dataclass(frozen=True, eq=False)
class Case(Expr):
    """CaseExpr (okapi-ir Expr.scala; SparkSQLExprMapper.scala:283-298): the value of the first
    alternative whose predicate is TRUE, else ``default`` (NULL when None)."""
    alternatives: Tuple[Tuple[Expr, Expr], ...]
    default: object = None


@dataclass(frozen=True, eq=False)
class Param(Expr):
    """Param(name) (okapi-ir Expr.scala): query parameter ``index`` of the session's parameter table
    (``Session.set_params``), bound to a literal by the library when the program is handed over, as
    SparkSQLExprMapper.scala:86-92 turns it into ``functions.lit``.  A list parameter may only be an
    element of ``In``, where it stands for its values."""
    index: int


TRUE = Lit(True)
FALSE = Lit(False)
NULL = Lit(None)


def eq(a: Expr, b: Expr) -> Expr:
    return BinOp("=", a, b)


def ands(*args: Expr) -> Expr:
    flat = []
    for a in args:
        if isinstance(a, Ands):
            flat.extend(a.args)
        elif not (isinstance(a, Lit) and a.value is True):
            flat.append(a)
    if not flat:
        return TRUE
    return flat[0] if len(flat) == 1 else Ands(tuple(flat))


def columns_of(e: Expr) -> set:
    """Physical columns an expression reads."""
    if isinstance(e, Col):
        return {e.name}
    out = set()
    for v in e.__dict__.values():
        if isinstance(v, Expr):
            out |= columns_of(v)
        elif isinstance(v, tuple):
            for x in v:
                if isinstance(x, Expr):
                    out |= columns_of(x)
                elif isinstance(x, tuple):  # Case alternatives
                    for y in x:
                        out |= columns_of(y)
    return out


class CapsmiExpr(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("arg", ctypes.c_int32), ("type", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("ival", ctypes.c_int64)]


def _lit_bits(value, ty: int, encode_str: Callable[[str], int]) -> int:
    if ty == BOOL:
        return 1 if value else 0
    if ty == I64:
        v = int(value)
        if not -(1 << 63) <= v < (1 << 63):
            raise OverflowError("integer literal outside Long range")
        return v
    if ty == F64:
        return struct.unpack("<q", struct.pack("<d", float(value)))[0]
    if ty == STR:
        return encode_str(value)
    raise ValueError(f"literal type {ty}")


def compile_program(e: Expr, column_index: Callable[[str], int], encode_str: Callable[[str], int]):
    """Postfix program (list of (op, arg, type, ival)) for ``e``."""
    out = []

    def go(x: Expr):
        if isinstance(x, Col):
            out.append((X_COL, column_index(x.name), 0, 0))
        elif isinstance(x, Lit):
            ty = x.resolved_type()
            if x.value is None or ty < 0:
                out.append((X_NULL, x.type + 1 if x.type >= 0 else 0, 0, 0))
            else:
                out.append((X_LIT, 0, ty, _lit_bits(x.value, ty, encode_str)))
        elif isinstance(x, Param):
            out.append((X_PARAM, x.index, 0, 0))
        elif isinstance(x, BinOp):
            go(x.left)
            go(x.right)
            out.append((BIN_OPS[x.op], 0, 0, 0))
        elif isinstance(x, Not):
            go(x.arg)
            out.append((X_NOT, 0, 0, 0))
        elif isinstance(x, Neg):
            go(x.arg)
            out.append((X_NEG, 0, 0, 0))
        elif isinstance(x, (Ands, Ors)):
            if not x.args:
                out.append((X_LIT, 0, BOOL, 1 if isinstance(x, Ands) else 0))
                return
            for a in x.args:
                go(a)
            out.append((X_AND if isinstance(x, Ands) else X_OR, len(x.args), 0, 0))
        elif isinstance(x, IsNull):
            go(x.arg)
            out.append((X_ISNULL, 0, 0, 0))
        elif isinstance(x, IsNotNull):
            go(x.arg)
            out.append((X_ISNOTNULL, 0, 0, 0))
        elif isinstance(x, In):
            go(x.arg)
            for v in x.values:
                go(v)
            out.append((X_IN, len(x.values), 0, 0))
        elif isinstance(x, Coalesce):
            for a in x.args:
                go(a)
            out.append((X_COALESCE, len(x.args), 0, 0))
        elif isinstance(x, Case):
            if not x.alternatives:
                go(x.default if x.default is not None else NULL)
                return
            for p, v in x.alternatives:
                go(p)
                go(v)
            go(x.default if x.default is not None else NULL)
            out.append((X_CASE, len(x.alternatives), 0, 0))
        else:
            raise NotImplementedError(f"expression {x!r}")

    go(e)
    return out


def to_ctypes(prog: Sequence[Tuple[int, int, int, int]]):
    arr = (CapsmiExpr * max(1, len(prog)))()
    for i, (op, arg, ty, ival) in enumerate(prog):
        arr[i].op, arr[i].arg, arr[i].type, arr[i].ival = op, arg, ty, ival
    return arr


ExprLike = Union[Expr, str]
