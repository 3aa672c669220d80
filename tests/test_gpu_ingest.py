"""Native CSV ingest (include/capsmi.h capsmi_read_csv): DataFrameReader.csv with an explicit schema,
as EdgeListDataSource (EdgeListDataSource.scala:76-97) and the FS graph source use it.  Checked
against pandas' C parser on the same files."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_edge_list_formats(session, tmp_path):
    from capsmi import io
    p = tmp_path / "e.txt"
    p.write_text("# header comment\n1 2\n  3   4\r\n\n# mid comment\n1099511627776 -5\n7\t8\n")
    nodes, rels = io.edge_list_graph(session, str(p), delimiter=None)  # whitespace-separated (opt-in)
    assert rels.column("id").values.tolist() == [0, 1, 2, 3]
    assert rels.column("source").values.tolist() == [1, 3, 1099511627776, 7]
    assert rels.column("target").values.tolist() == [2, 4, -5, 8]
    assert sorted(nodes.column("id").values.tolist()) == sorted({1, 2, 3, 4, 1099511627776, -5, 7, 8})
    s, d = io.read_edge_list(str(p), delimiter=None)
    np.testing.assert_array_equal(s, rels.column("source").values)


def test_csv_fields(session, tmp_path):
    from capsmi.expr import BOOL, F64, I64, STR
    p = tmp_path / "t.csv"
    p.write_text('1,"Alice, A.",2.5,true\n'
                 '2,"say ""hi""",,false\n'
                 '3,,-1e3,TRUE\n'
                 '4,plain\n'                      # missing trailing fields -> null (PERMISSIVE)
                 '5,x,0.25,false,extra,tokens\n'  # extra tokens dropped
                 '6,"",7,\n')                     # "" is the empty string, not null
    t = session.read_csv([str(p)], ["id", "name", "score", "ok"], [I64, STR, F64, BOOL])
    assert t.size == 6
    assert t.column("id").values.tolist() == [1, 2, 3, 4, 5, 6]
    names = t.column("name")
    dec = [None if names.valid is not None and not names.valid[i] else session.dictionary.decode(int(v))
           for i, v in enumerate(names.values)]
    assert dec == ["Alice, A.", 'say "hi"', None, "plain", "x", ""]
    sc = t.column("score")
    assert [None if not sc.valid[i] else float(v) for i, v in enumerate(sc.values)] == [2.5, None, -1000.0, None,
                                                                                        0.25, 7.0]
    ok = t.column("ok")
    assert [None if not ok.valid[i] else bool(v) for i, v in enumerate(ok.values)] == [True, False, True, None,
                                                                                      False, None]


def test_csv_errors(session, tmp_path):
    from capsmi import _lib
    from capsmi.expr import BOOL, I64
    p = tmp_path / "bad.csv"
    p.write_text("1,2\n3,x4\n")
    with pytest.raises(_lib.IllegalArgumentException, match="not a Long"):
        session.read_csv([str(p)], ["a", "b"], [I64, I64])
    for token in ("flase", "1", "yes", "t"):  # Spark's CSV Boolean takes true / false only
        p.write_text(f"1,true\n2,FALSE\n3,{token}\n")
        with pytest.raises(_lib.IllegalArgumentException, match="not a Boolean"):
            session.read_csv([str(p)], ["a", "b"], [I64, BOOL])
    with pytest.raises(_lib.IllegalArgumentException, match="cannot open"):
        session.read_csv([str(tmp_path / "missing.csv")], ["a"], [I64])


def test_csv_delimiter_and_comment_lines(session, tmp_path):
    """Spark's `sep` is one character: with ' ', two spaces hold an empty (null) field, and a leading
    space starts with an empty field; a comment is a line whose FIRST character is the comment
    character; lines of blanks hold no record.  Whitespace splitting is the opt-in delimiter None."""
    from capsmi.expr import I64
    p = tmp_path / "e.txt"
    p.write_text("# header\n1 2\n3  4\n 5 6\n  # not a comment\n   \n7 8\n")
    t = session.read_csv([str(p)], ["a", "b"], [I64, I64], delimiter=" ", comment="#")
    a, b = t.column("a"), t.column("b")
    got = [(None if not a.valid[i] else int(a.values[i]), None if not b.valid[i] else int(b.values[i]))
           for i in range(t.size)]
    assert got[:3] == [(1, 2), (3, None), (None, 5)]
    assert got[-1] == (7, 8) and len(got) == 5  # '  # not...' is a record: (null, null) -> fields '', ''
    assert got[3] == (None, None)
    p.write_text("# header\n1 2\n3   4\n\t5\t 6\n")
    t = session.read_csv([str(p)], ["a", "b"], [I64, I64], delimiter=None, comment="#")
    assert list(zip(t.column("a").values.tolist(), t.column("b").values.tolist())) == [(1, 2), (3, 4), (5, 6)]


def test_many_files_and_chunks(session, tmp_path):
    """Several files in order, each large enough to be split over all parser threads."""
    from capsmi.expr import I64
    rng = np.random.default_rng(3)
    paths, want = [], []
    for f in range(3):
        a = rng.integers(-(1 << 62), 1 << 62, (300_000, 2))
        p = tmp_path / f"part-{f}.csv"
        np.savetxt(p, a, fmt="%d", delimiter=",")
        paths.append(str(p))
        want.append(a)
    want = np.concatenate(want)
    t = session.read_csv(paths, ["s", "t"], [I64, I64], row_id_col="rid")
    assert t.physicalColumns == ["rid", "s", "t"]
    np.testing.assert_array_equal(t.column("s").values, want[:, 0])
    np.testing.assert_array_equal(t.column("t").values, want[:, 1])
    np.testing.assert_array_equal(t.column("rid").values, np.arange(len(want)))


def test_ingest_rate(session, tmp_path):
    """8M-edge file: the native parser's rate (reported; the round-1 Python loop took minutes)."""
    from capsmi import io
    rng = np.random.default_rng(1)
    a = rng.integers(0, 1 << 26, (8_000_000, 2))
    p = tmp_path / "big.txt"
    np.savetxt(p, a, fmt="%d", delimiter=" ")
    t0 = time.perf_counter()
    nodes, rels = io.edge_list_graph(session, str(p))
    n = rels.size
    dt = time.perf_counter() - t0
    print(f"edge-list ingest: {n} edges in {dt:.2f} s = {n / dt / 1e6:.1f} M edges/s (incl. node distinct)")
    assert n == len(a)
    np.testing.assert_array_equal(rels.column("target").values[-5:], a[-5:, 1])


@pytest.mark.parametrize("par,maxp,cost", [(4, 4096, 512), (3, 1 << 20, 1 << 12), (16, 700, 0), (8, 128 << 20, 4 << 20)])
def test_spark_partition_row_ids(session, tmp_path, par, maxp, cost):
    """capsmi_session_set_csv_partitioning: read_csv's row ids are Spark's monotonically_increasing_id over
    its file-scan partitions (EdgeListDataSource.scala:86), checked against the independent restatement
    tests/spark_ids.py (parity unpinned: no reference fixture holds a multi-partition read)."""
    from capsmi.expr import I64
    from spark_ids import spark_row_ids
    rng = np.random.default_rng(par)
    paths, blobs = [], []
    for f, n in enumerate([2000, 37, 900, 1]):
        lines = [f"{a} {b}" for a, b in rng.integers(0, 1 << 40, (n, 2))]
        if f == 2:
            lines.insert(5, "# a comment")
            lines.insert(9, "")
        text = ("\n".join(lines) + ("\n" if f != 1 else "")).encode()
        p = tmp_path / f"part-{f}.txt"
        p.write_bytes(text)
        paths.append(str(p))
        blobs.append(text)
    session.set_csv_partitioning(par, maxp, cost)
    try:
        t = session.read_csv(paths, ["source", "target"], [I64, I64], delimiter=" ", comment="#", row_id_col="id")
    finally:
        session.set_csv_partitioning(0)
    want = spark_row_ids(blobs, par, maxp, cost, comment=b"#")
    assert t.column("id").values.tolist() == want
    assert len(set(want)) == len(want)
