"""The restatement of Spark's multi-partition monotonically_increasing_id (tests/spark_ids.py, the checker
of capsmi_session_set_csv_partitioning) on a hand-worked case.  CPU only."""
from spark_ids import spark_row_ids


def test_hand_worked_splits():
    # maxSplitBytes = min(10, max(0, 35 / 1)) = 10.  Splits: f0 [0,10) (10 B); f1 [0,10), [10,20), [20,25).
    # Sorted by length (stable): f0k0, f1k0, f1k1, f1k2; next fit with cap 10 puts each in its own partition.
    f0 = b"1 2\n3 4\n5\n"                 # lines at 0, 4, 8: all split 0 -> partition 0
    f1 = b"10 20\n30 40\n50 60\n7 8\n9 9"  # lines at 0, 6 (split 0), 12, 18 (split 1), 22 (split 2)
    ids = spark_row_ids([f0, f1], parallelism=1, max_partition_bytes=10, open_cost=0)
    P = 1 << 33
    assert ids == [0, 1, 2, P + 0, P + 1, 2 * P + 0, 2 * P + 1, 3 * P + 0]


def test_small_files_get_a_partition_each():
    # Spark's defaults: maxSplitBytes = max(openCost 4 MiB, total / 8) = 4 MiB; every small file is one
    # split, and a split's open cost (4 MiB) fills a partition, so each file is its own partition, numbered
    # by descending length: f2 (10 B) -> 0, f0 (8 B) -> 1, f1 (4 B) -> 2; one file alone: row numbers
    files = [b"1 2\n3 4\n", b"5 6\n", b"# c\n\n7 8\n"]
    P = 1 << 33
    assert spark_row_ids(files, parallelism=8, comment=b"#") == [P + 0, P + 1, 2 * P, 0]
    assert spark_row_ids([b"1 2\n3 4\n5 6\n"], parallelism=8) == [0, 1, 2]


def test_line_starting_at_a_split_boundary_belongs_to_the_previous_split():
    # split = 4: "abc\n" ends at 4, the line starting at byte 4 is read by split 0 (it reads one line past
    # its end), the line at 8 by split 1
    f = b"1 2\n3 4\n5 6\n"
    ids = spark_row_ids([f], parallelism=1, max_partition_bytes=4, open_cost=0)
    P = 1 << 33
    assert ids == [0, 1, P + 0]
