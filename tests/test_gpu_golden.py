"""Golden vectors from the reference's acceptance tests, executed with the device Table operators
(libcapsmi.so) through the relational planner mirror.  Exact row-multiset equality."""
import pytest

from golden_util import all_cases, run_planner, same_rows

pytestmark = pytest.mark.gpu

CASES = all_cases()


@pytest.mark.parametrize("fname,case", CASES, ids=[c["name"] for _, c in CASES])
def test_device_matches_golden(session, fname, case):
    from capsmi.table import StringDictionary
    session.dictionary = StringDictionary()
    got = run_planner(session, case)
    assert same_rows(got, case["expected"], case.get("ordered", False)), (got, case["expected"])
