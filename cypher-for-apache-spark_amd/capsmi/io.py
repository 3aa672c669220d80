"""Ingest: edge-list data source.

Restates EdgeListDataSource.graph
(spark-cypher/src/main/scala/org/opencypher/spark/api/io/edgelist/EdgeListDataSource.scala:76-97):
  - the file holds one `source target` pair of Longs per line (Spark CSV reader options, e.g. the
    delimiter, are honoured for the delimiter and comment prefix);
  - relationships get `id = monotonically_increasing_id()`, which for a single input partition is
    the row number 0, 1, 2, ...;
  - nodes = distinct(source UNION target), label "V"; relationship type "E" (:45-53).
Parsing runs in libcapsmi's native CSV reader (host threads); the node table's distinct runs on the
device.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from .expr import I64
from .table import ColumnData, GpuTable, Session

NODE_LABEL = "V"
REL_TYPE = "E"


def read_edge_list(path: str, delimiter: Optional[str] = " ", comment: str = "#") -> Tuple[np.ndarray, np.ndarray]:
    """Host arrays of an edge-list file (vectorised C parser; the device path is edge_list_graph).
    ``delimiter`` None: whitespace-separated."""
    import pandas as pd
    sep = r"\s+" if delimiter is None else delimiter
    df = pd.read_csv(path, sep=sep, comment=comment or None, header=None, usecols=[0, 1], dtype=np.int64,
                     engine="c")
    return df[0].to_numpy(np.int64), df[1].to_numpy(np.int64)


def edge_list_tables(session: Session, src: np.ndarray, dst: np.ndarray) -> Tuple[GpuTable, GpuTable]:
    """(node table [id], relationship table [id, source, target]) of an edge list."""
    m = len(src)
    rels = session.table([ColumnData("id", I64, np.arange(m, dtype=np.int64)), ColumnData("source", I64, src),
                          ColumnData("target", I64, dst)])
    return _graph_of(session, rels)


def _graph_of(session: Session, rels: GpuTable) -> Tuple[GpuTable, GpuTable]:
    s = rels.select("source").withColumnRenamed("source", "id")
    t = rels.select("target").withColumnRenamed("target", "id")
    nodes = s.unionAll(t).distinct().as_node_table("id")
    rels = rels.as_rel_table("id", "source", "target")
    session.compact_if_sparse([nodes], [rels])  # edge-list ids are arbitrary Longs
    return nodes, rels


def edge_list_graph(session: Session, path: str, delimiter: Optional[str] = " ",
                    comment: str = "#") -> Tuple[GpuTable, GpuTable]:
    """EdgeListDataSource.graph: the file parsed by libcapsmi's native CSV reader (host threads), rel ids
    = row numbers, nodes = distinct endpoints on the device."""
    rels = session.read_csv([path], ["source", "target"], [I64, I64], delimiter, comment, row_id_col="id")
    return _graph_of(session, rels)
