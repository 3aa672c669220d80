"""Ingest: edge-list data source.

Restates EdgeListDataSource.graph
(spark-cypher/src/main/scala/org/opencypher/spark/api/io/edgelist/EdgeListDataSource.scala:76-97):
  - the file holds one `source target` pair of Longs per line (Spark CSV reader options, e.g. the
    delimiter, are honoured for the delimiter and comment prefix);
  - relationships get `id = monotonically_increasing_id()`, which for a single input partition is
    the row number 0, 1, 2, ...;
  - nodes = distinct(source UNION target), label "V"; relationship type "E" (:45-53).
Parsing is host work (file IO); the node table's distinct runs on the device.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from .expr import I64
from .table import ColumnData, GpuTable, Session

NODE_LABEL = "V"
REL_TYPE = "E"


def read_edge_list(path: str, delimiter: str = " ", comment: str = "#") -> Tuple[np.ndarray, np.ndarray]:
    src, dst = [], []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or (comment and line.startswith(comment)):
                continue
            parts = [p for p in line.split(delimiter) if p != ""] if delimiter != " " else line.split()
            if len(parts) < 2:
                raise ValueError(f"malformed edge-list line: {line!r}")
            src.append(int(parts[0]))
            dst.append(int(parts[1]))
    return np.asarray(src, dtype=np.int64), np.asarray(dst, dtype=np.int64)


def edge_list_tables(session: Session, src: np.ndarray, dst: np.ndarray) -> Tuple[GpuTable, GpuTable]:
    """(node table [id], relationship table [id, source, target]) of an edge list."""
    m = len(src)
    rels = session.table([ColumnData("id", I64, np.arange(m, dtype=np.int64)), ColumnData("source", I64, src),
                          ColumnData("target", I64, dst)])
    s = rels.select("source").withColumnRenamed("source", "id")
    t = rels.select("target").withColumnRenamed("target", "id")
    nodes = s.unionAll(t).distinct().as_node_table("id")
    rels = rels.as_rel_table("id", "source", "target")
    session.compact_if_sparse([nodes], [rels])  # edge-list ids are arbitrary Longs
    return nodes, rels


def edge_list_graph(session: Session, path: str, delimiter: str = " ") -> Tuple[GpuTable, GpuTable]:
    src, dst = read_edge_list(path, delimiter)
    return edge_list_tables(session, src, dst)
