"""Collect / collect(DISTINCT) (SparkTable.scala:169-177: sort_array(collect_list / collect_set)) on the
device against the numpy restatement, and list columns travelling through the other Table operators.
Exact equality: lists compare element word by element word."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _tables(session, rng, n, null_frac=0.2, key_range=6):
    from capsmi import ColumnData
    from capsmi.expr import BOOL, F64, I64, STR
    from oracle.relational import NumpyBackend
    strings = [f"s{i:03d}" for i in range(40)]
    session.dictionary.extend(strings)
    codes = np.array([session.dictionary.encode(x) for x in strings], dtype=np.int64)
    cols = [
        ColumnData("k", I64, rng.integers(0, key_range, n), rng.random(n) >= null_frac),
        ColumnData("b", BOOL, rng.integers(0, 2, n), rng.random(n) >= null_frac),
        ColumnData("v", I64, rng.integers(-20, 20, n), rng.random(n) >= null_frac),
        # repeated values (collect_set keeps one of each).  No -0.0: sort_array orders it equal to 0.0
        # (Spark's nanSafeCompareDoubles) in collect order, which Spark does not fix
        ColumnData("f", F64, np.round(rng.standard_normal(n), 1) + 0.0, rng.random(n) >= null_frac),
        ColumnData("s", STR, codes[rng.integers(0, 40, n)], rng.random(n) >= null_frac),
    ]
    return session.table(cols), NumpyBackend(session.dictionary).table(cols)


def _cell(c, r):
    from capsmi.expr import F64, LIST
    if c.valid is not None and not c.valid[r]:
        return None
    v = c.values[r]
    if c.type >= LIST:
        return ("list",) + tuple(np.asarray(v).view(np.int64).tolist())
    if c.type == F64:
        return ("f", int(np.float64(v).view(np.int64)))
    return int(v)


def _rows(t):
    cols = t.to_columns()
    return sorted((tuple(_cell(c, r) for c in cols) for r in range(t.size)), key=repr)


def _same(g, o):
    assert g.physicalColumns == o.physicalColumns
    assert g.columnType == o.columnType
    assert g.size == o.size
    a, b = _rows(g), _rows(o)
    for name, i in zip(g.physicalColumns, range(len(g.physicalColumns))):
        assert [r[i] for r in a] == [r[i] for r in b], name
    assert a == b


AGGS = [("collect", "v", False, "lv"), ("collect", "v", True, "sv"), ("collect", "f", False, "lf"),
        ("collect", "f", True, "sf"), ("collect", "s", True, "ss"), ("collect", "b", False, "lb"),
        ("count_star", None, False, "n")]


@pytest.mark.parametrize("by", [[], ["k"], ["k", "b"], ["s"]])
def test_collect_vs_oracle(session, by):
    rng = np.random.default_rng(5 + len(by))
    g, o = _tables(session, rng, 3000)
    _same(g.group(by, AGGS), o.group(by, AGGS))


def test_collect_large_groups(session):
    """Many groups and long lists: the (group, value) sort spans several radix passes."""
    from capsmi import ColumnData
    from capsmi.expr import I64
    from oracle.relational import NumpyBackend
    rng = np.random.default_rng(17)
    n = 200_000
    cols = [ColumnData("k", I64, rng.integers(0, 3000, n)), ColumnData("v", I64, rng.integers(-(1 << 40), 1 << 40, n)),
            ColumnData("w", I64, rng.integers(0, 50, n), rng.random(n) >= 0.3)]
    g, o = session.table(cols), NumpyBackend(session.dictionary).table(cols)
    aggs = [("collect", "v", False, "lv"), ("collect", "w", True, "sw")]
    _same(g.group(["k"], aggs), o.group(["k"], aggs))


def test_collect_empty_input(session):
    from capsmi import ColumnData
    from capsmi.expr import I64
    from oracle.relational import NumpyBackend
    cols = [ColumnData("k", I64, np.zeros(0, np.int64)), ColumnData("v", I64, np.zeros(0, np.int64))]
    g, o = session.table(cols), NumpyBackend(session.dictionary).table(cols)
    aggs = [("collect", "v", False, "l"), ("collect", "v", True, "s")]
    glob = g.group([], aggs)
    _same(glob, o.group([], aggs))  # global: one row of empty lists
    assert glob.rows() == [{"l": [], "s": []}]
    _same(g.group(["k"], aggs), o.group(["k"], aggs))  # grouped: no rows


def test_list_columns_through_operators(session):
    """A list column is a payload of filter / order / skip / limit / join / union / rename / alias, as a
    Spark array column would be; its rows keep their lists."""
    from capsmi.expr import BinOp, Col, Lit
    rng = np.random.default_rng(23)
    g, o = _tables(session, rng, 2000, key_range=30)
    gg, og = g.group(["k"], AGGS[:3]), o.group(["k"], AGGS[:3])
    steps = [
        lambda t: t.filter(BinOp("<", Col("k"), Lit(12))),
        lambda t: t.withColumnRenamed("lv", "renamed").select("k", "renamed"),
        lambda t: t.withColumns((Col("sv"), "alias")),
        lambda t: t.drop("lf"),
    ]
    for f in steps:
        _same(f(gg), f(og))
    _same(gg.orderBy(("k", "desc")).skip(3).limit(10), og.orderBy(("k", "desc")).skip(3).limit(10))
    # union: two different list stores, and a store with itself
    g2, o2 = _tables(session, np.random.default_rng(24), 1500, key_range=30)
    gg2, og2 = g2.group(["k"], AGGS[:3]), o2.group(["k"], AGGS[:3])
    _same(gg.unionAll(gg2), og.unionAll(og2))
    _same(gg.unionAll(gg), og.unionAll(og))
    # join payload, both sides, with a null-padding outer join
    right_g = gg2.withColumnRenamed("k", "k2").withColumnRenamed("lv", "lv2").withColumnRenamed("sv", "sv2") \
        .withColumnRenamed("lf", "lf2")
    right_o = og2.withColumnRenamed("k", "k2").withColumnRenamed("lv", "lv2").withColumnRenamed("sv", "sv2") \
        .withColumnRenamed("lf", "lf2")
    for jt in ("inner", "left_outer", "full_outer"):
        _same(gg.join(right_g, jt, ("k", "k2")), og.join(right_o, jt, ("k", "k2")))


def test_list_column_as_key_is_not_implemented(session):
    from capsmi._lib import NotImplementedException
    from capsmi.expr import BinOp, Col, Lit
    rng = np.random.default_rng(3)
    g, _ = _tables(session, rng, 200)
    lists = g.group(["k"], [("collect", "v", False, "lv")])
    with pytest.raises(NotImplementedException):
        lists.group(["lv"], [("count_star", None, False, "n")])
    with pytest.raises(NotImplementedException):
        lists.distinct()
    with pytest.raises(NotImplementedException):
        lists.orderBy(("lv", "asc"))
    with pytest.raises(NotImplementedException):
        lists.join(lists.withColumnRenamed("lv", "lv2").withColumnRenamed("k", "k2"), "inner", ("lv", "lv2"))
    with pytest.raises(NotImplementedException):
        lists.filter(BinOp("=", Col("lv"), Lit(1)))
    with pytest.raises(NotImplementedException):
        lists.group([], [("collect", "lv", False, "ll")])
