"""Test infrastructure: Spark 2.2.1's monotonically_increasing_id for a CSV file scan, restated in Python
(EdgeListDataSource.scala:86 numbers the relationships with it; the partitioning is Spark's
FileSourceScanExec.createNonBucketedReadRDD, third-party and not vendored, so this restatement is parity
unpinned: no reference fixture covers a multi-partition read).  An independent second statement of
csrc/ingest.hip spark_row_ids, used as its checker."""


def spark_row_ids(files, parallelism, max_partition_bytes=128 << 20, open_cost=4 << 20, comment=None):
    """files: the file contents (bytes) in read order; returns the ids of the records, in file / line
    order (a record is a line that is neither blank nor a comment line)."""
    total = sum(len(b) + open_cost for b in files)
    split = max(1, min(max_partition_bytes, max(open_cost, total // parallelism)))
    splits = []  # [file, k, length, rows]
    first = []
    for f, b in enumerate(files):
        first.append(len(splits))
        o = k = 0
        while o < len(b):
            splits.append([f, k, min(split, len(b) - o), 0])
            o += split
            k += 1
    recs = []  # (split index) per record
    for f, b in enumerate(files):
        pos = 0
        for line in b.split(b"\n"):
            start = pos
            pos += len(line) + 1
            body = line.rstrip(b"\r")
            if not body.strip(b" \t") or (comment is not None and body[:1] == comment):
                continue
            k = 0 if start == 0 else (start - 1) // split  # Hadoop LineRecordReader: split (o, o + len]
            recs.append(first[f] + k)
            splits[first[f] + k][3] += 1
    order = sorted(range(len(splits)), key=lambda i: -splits[i][2])  # stable, descending length
    part_of, base_of = {}, {}
    part, cur, base, opened = 0, 0, 0, False
    for i in order:  # next fit decreasing
        if opened and cur + splits[i][2] > split:
            part, cur, base = part + 1, 0, 0
        part_of[i], base_of[i] = part, base
        base += splits[i][3]
        cur += splits[i][2] + open_cost
        opened = True
    seen = {}
    ids = []
    for i in recs:
        ids.append((part_of[i] << 33) | (base_of[i] + seen.get(i, 0)))
        seen[i] = seen.get(i, 0) + 1
    return ids
