"""File-system property-graph source, CSV format: one directory per graph.

Restates the reference's FS layout and table schemas:
  - DefaultGraphDirectoryStructure (spark-cypher/.../api/io/fs/GraphDirectoryStructure.scala:55-99):
    <graph>/propertyGraphSchema.json, <graph>/capsGraphMetaData.json,
    <graph>/nodes/<sorted labels joined by '_'>/, <graph>/relationships/<type>/
  - canonical column order (spark-cypher/.../api/io/util/CAPSGraphExport.scala:45-64):
    node tables [id, properties sorted by name]; relationship tables [id, source, target,
    properties sorted by name]; ids Long
  - AbstractPropertyGraphDataSource.graph (AbstractPropertyGraphDataSource.scala:95-121): one node
    table per label combination of the schema, one relationship table per type
  - Spark's CSV reader with an explicit schema: no header line, ',' separated, '"' quoted, an
    empty field is null.
On a device session the tables are parsed by libcapsmi's native CSV reader (host threads) straight
into device entity tables; the CPU oracle backend parses them in Python.
"""
from __future__ import annotations

import csv
import glob
import json
import os
from typing import Dict, List, Tuple

import numpy as np

from .expr import BOOL, F64, I64, STR
from .planner import DST, ID, SRC, EntityTable, PlanningError, ScanGraph, _column

_TYPES = {"STRING": STR, "INTEGER": I64, "FLOAT": F64, "BOOLEAN": BOOL}


def _cypher_type(t: str) -> int:
    base = t.rstrip("?").upper()
    if base not in _TYPES:
        raise PlanningError(f"unsupported property type {t!r} in propertyGraphSchema.json")
    return _TYPES[base]


def _parse(ty: int, field: str):
    if field == "":
        return None
    if ty == I64:
        return int(field)
    if ty == F64:
        return float(field)
    if ty == BOOL:
        return field.strip().lower() == "true"
    return field


def _read_rows(table_dir: str, ncols: int) -> List[List[str]]:
    rows = []
    for f in sorted(glob.glob(os.path.join(table_dir, "*.csv"))):
        with open(f, newline="") as fh:
            for r in csv.reader(fh):
                if not r:
                    continue
                if len(r) != ncols:
                    raise PlanningError(f"{f}: expected {ncols} columns, got {len(r)}")
                rows.append(r)
    return rows


def read_schema(graph_dir: str) -> Tuple[List[Tuple[frozenset, Dict[str, int]]], List[Tuple[str, Dict[str, int]]]]:
    with open(os.path.join(graph_dir, "propertyGraphSchema.json")) as f:
        s = json.load(f)
    nodes = [(frozenset(e["labels"]), {k: _cypher_type(v) for k, v in e["properties"].items()})
             for e in s.get("labelPropertyMap", [])]
    rels = [(e["relType"], {k: _cypher_type(v) for k, v in e["properties"].items()})
            for e in s.get("relTypePropertyMap", [])]
    return nodes, rels


def _native_tables(session, graph_dir, node_schemas, rel_schemas):
    """Device path: every table directory parsed by libcapsmi's native CSV reader (capsmi_read_csv)."""
    nodes, rels = [], []
    for labels, props in node_schemas:
        d = os.path.join(graph_dir, "nodes", "_".join(sorted(labels)))
        keys = sorted(props)
        t = session.read_csv(sorted(glob.glob(os.path.join(d, "*.csv"))), [ID] + keys, [I64] + [props[k] for k in keys])
        nodes.append(EntityTable("node", labels, dict(props), t.as_node_table(ID)))
    for rtype, props in rel_schemas:
        d = os.path.join(graph_dir, "relationships", rtype)
        keys = sorted(props)
        t = session.read_csv(sorted(glob.glob(os.path.join(d, "*.csv"))), [ID, SRC, DST] + keys,
                             [I64, I64, I64] + [props[k] for k in keys])
        rels.append(EntityTable("rel", frozenset([rtype]), dict(props), t.as_rel_table(ID, SRC, DST)))
    return nodes, rels


def fs_graph(backend, graph_dir: str, extra_strings=()) -> ScanGraph:
    """ScanGraph of a CSV graph directory; `backend` is a capsmi Session (GPU) or the oracle's backend.
    `extra_strings`: strings to register up front (codes are stable, so later strings may also be added)."""
    node_schemas, rel_schemas = read_schema(graph_dir)
    if hasattr(backend, "read_csv"):  # a device session
        backend.dictionary.extend(extra_strings)
        nodes, rels = _native_tables(backend, graph_dir, node_schemas, rel_schemas)
        backend.compact_if_sparse([e.table for e in nodes], [e.table for e in rels])
        return ScanGraph(backend, nodes, rels)
    parsed = []
    strings = set()
    for labels, props in node_schemas:
        d = os.path.join(graph_dir, "nodes", "_".join(sorted(labels)))
        keys = sorted(props)
        rows = _read_rows(d, 1 + len(keys))
        cols = {ID: [int(r[0]) for r in rows]}
        for i, k in enumerate(keys):
            cols[k] = [_parse(props[k], r[1 + i]) for r in rows]
            if props[k] == STR:
                strings |= {v for v in cols[k] if v is not None}
        parsed.append(("node", labels, props, keys, cols))
        strings |= set(labels)
    for rtype, props in rel_schemas:
        d = os.path.join(graph_dir, "relationships", rtype)
        keys = sorted(props)
        rows = _read_rows(d, 3 + len(keys))
        cols = {ID: [int(r[0]) for r in rows], SRC: [int(r[1]) for r in rows], DST: [int(r[2]) for r in rows]}
        for i, k in enumerate(keys):
            cols[k] = [_parse(props[k], r[3 + i]) for r in rows]
            if props[k] == STR:
                strings |= {v for v in cols[k] if v is not None}
        parsed.append(("rel", frozenset([rtype]), props, keys, cols))
        strings.add(rtype)
    backend.dictionary.extend(sorted(strings | set(extra_strings)))
    enc = backend.dictionary.encode
    nodes, rels = [], []
    for kind, labels, props, keys, cols in parsed:
        ids = [ID] if kind == "node" else [ID, SRC, DST]
        data = [_column(c, I64, cols[c], enc) for c in ids] + [_column(k, props[k], cols[k], enc) for k in keys]
        t = backend.table(data)
        t = t.as_node_table(ID) if kind == "node" else t.as_rel_table(ID, SRC, DST)
        et = EntityTable(kind, labels, dict(props), t)
        (nodes if kind == "node" else rels).append(et)
    backend.compact_if_sparse([e.table for e in nodes], [e.table for e in rels])
    return ScanGraph(backend, nodes, rels)
