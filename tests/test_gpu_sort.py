"""The device radix sort (k_sort.hip) through ORDER BY: the output order must equal numpy's stable
argsort exactly -- ties keep their input order (LSD passes rely on that), on ragged sizes around the
4096-key tile, skewed digits (many equal bytes) and negative / Double keys (per-pass histograms; round 6
removed the measured-slower onesweep form)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _order(session, values, ty, desc=False):
    from capsmi import ColumnData
    from capsmi.expr import I64
    n = len(values)
    t = session.table([ColumnData("k", ty, values, None), ColumnData("i", I64, np.arange(n, dtype=np.int64), None)])
    return np.asarray(t.orderBy(("k", "desc" if desc else "asc")).column("i").values, dtype=np.int64)


@pytest.mark.parametrize("n", [1, 7, 4095, 4096, 4097, 100_003, 1 << 20, 1024 * 12288 + 12289])  # last: 12288-key tiles
def test_order_by_is_stable_argsort(session, n):
    from capsmi.expr import I64
    rng = np.random.default_rng(n)
    k = rng.integers(-50, 50, n).astype(np.int64)  # few distinct keys: long runs of ties
    np.testing.assert_array_equal(_order(session, k, I64), np.argsort(k, kind="stable"))


def test_order_by_skewed_and_wide_keys(session):
    from capsmi.expr import I64
    rng = np.random.default_rng(5)
    n = 3 * 4096 + 17
    k = np.where(rng.random(n) < 0.9, 0, rng.integers(-(1 << 62), 1 << 62, n)).astype(np.int64)  # one hot digit
    np.testing.assert_array_equal(_order(session, k, I64), np.argsort(k, kind="stable"))
    desc = _order(session, k, I64, desc=True)
    np.testing.assert_array_equal(desc, np.argsort(-k, kind="stable"))


def test_order_by_doubles(session):
    from capsmi.expr import F64
    rng = np.random.default_rng(9)
    n = 50_000
    k = np.round(rng.standard_normal(n), 2)
    k[k == 0] = 0.0  # -0.0 sorts below 0.0 by its bits (Double.compare); numpy ties them
    np.testing.assert_array_equal(_order(session, k, F64), np.argsort(k, kind="stable"))
