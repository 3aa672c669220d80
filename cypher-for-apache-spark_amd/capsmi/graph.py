"""Graph fast path over the C ABI: node-scan bitmaps and fused Expand kernels.

The relational planner lowers ``(a)-[r]->(b)`` to two joins
(okapi-relational/.../planning/RelationalPlanner.scala:113-137); when the joined scans are base
entity tables with dense Long ids these entry points compute the same row multisets in one
streaming pass per hop (see include/capsmi.h, "graph fast path").
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

from . import _lib
from .expr import Expr, compile_program, to_ctypes
from .table import GpuTable, Session

RMAT_GRAPH500 = (57, 19, 19)  # (A, B, C) percent, D = 5  -- SURVEY.md §8d
RMAT_LDBC = (45, 15, 15)      # C5 "LDBC-shaped" proposal


class NodeBitmap:
    """Node scan (+ label/property predicate) collapsed to one bit per id in [lo, hi)."""

    def __init__(self, session: Session, lo: int, hi: int):
        self.session = session
        self.lo, self.hi = lo, hi
        self._h = ctypes.c_void_p()
        _lib.call("capsmi_bitmap_create", session.handle, lo, hi, ctypes.byref(self._h))

    @property
    def handle(self):
        return self._h

    @property
    def nwords(self) -> int:
        return (self.hi - self.lo + 31) // 32

    def add_scan(self, nodes: GpuTable, id_col: str = "id", predicate: Optional[Expr] = None) -> "NodeBitmap":
        if predicate is None:
            _lib.call("capsmi_bitmap_add_scan", self._h, nodes.handle, id_col.encode(), 0, None)
        else:
            names = nodes.physicalColumns
            index = {n: i for i, n in enumerate(names)}
            prog = compile_program(predicate, lambda c: index[c], self.session.encode_str)
            _lib.call("capsmi_bitmap_add_scan", self._h, nodes.handle, id_col.encode(), len(prog), to_ctypes(prog))
        return self

    def stats(self) -> Tuple[int, bool]:
        bits, uniq = ctypes.c_int64(), ctypes.c_int32()
        _lib.call("capsmi_bitmap_stats", self._h, ctypes.byref(bits), ctypes.byref(uniq))
        return bits.value, bool(uniq.value)

    def words_ptr(self) -> int:
        """Device address of the bitmap's uint32 words (include/capsmi.h capsmi_bitmap_words)."""
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        _lib.call("capsmi_bitmap_words", self._h, ctypes.byref(p), ctypes.byref(n))
        return p.value or 0

    def copy_words(self, w_begin: int, w_end: int, ext_ptr: int, to_bitmap: bool) -> None:
        """Device copy of words [w_begin, w_end) between the bitmap and a caller buffer (e.g. a torch
        tensor's data_ptr), ordered on the session stream."""
        _lib.call("capsmi_bitmap_copy_words", self._h, w_begin, w_end, ctypes.c_void_p(ext_ptr), 1 if to_bitmap else 0)

    def refresh(self, unique_rows: bool = True) -> "NodeBitmap":
        """Re-derive the set-bit count after the words were written (e.g. all-gathered)."""
        _lib.call("capsmi_bitmap_refresh", self._h, 1 if unique_rows else 0)
        return self

    def assume(self, set_bits: int, unique_rows: bool = True) -> "NodeBitmap":
        """State the set-bit count after the words were written (no device popcount, no sync)."""
        _lib.call("capsmi_bitmap_assume", self._h, set_bits, 1 if unique_rows else 0)
        return self

    def release(self) -> None:
        if self._h:
            _lib.call("capsmi_bitmap_release", self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            if self._h and _lib._lib is not None:
                _lib._lib.capsmi_bitmap_release(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


def _handles(rels: Sequence[GpuTable]):
    arr = (ctypes.c_void_p * max(1, len(rels)))()
    for i, t in enumerate(rels):
        arr[i] = t.handle
    return arr


def expand_filter(session: Session, rels: GpuTable, src_ok: NodeBitmap, dst_ok: NodeBitmap,
                  out_cols: Sequence[str], out_names: Optional[Sequence[str]] = None,
                  src_col: str = "source", dst_col: str = "target") -> GpuTable:
    """``MATCH (a)-[r]->(b) WHERE src_ok(a) AND dst_ok(b)`` -> the surviving rel rows, projected."""
    out = ctypes.c_void_p()
    _lib.call("capsmi_expand_filter", session.handle, rels.handle, src_col.encode(), dst_col.encode(),
              src_ok.handle, dst_ok.handle, len(out_cols), _lib.strs(out_cols),
              _lib.strs(out_names) if out_names else None, ctypes.byref(out))
    return GpuTable(session, out)


def two_hop_count_distinct(session: Session, rels: Sequence[GpuTable], a_ok: NodeBitmap, b_ok: NodeBitmap,
                           c_ok: NodeBitmap, src_col: str = "source", dst_col: str = "target") -> int:
    """``MATCH (a)-[r1]->(b)-[r2]->(c) RETURN count(DISTINCT c)`` (r1 <> r2 implied)."""
    v = ctypes.c_int64()
    _lib.call("capsmi_two_hop_count_distinct", session.handle, len(rels), _handles(rels), src_col.encode(),
              dst_col.encode(), a_ok.handle, b_ok.handle, c_ok.handle, ctypes.byref(v))
    return v.value


def two_hop_count(session: Session, rels: Sequence[GpuTable], a_ok: NodeBitmap, b_ok: NodeBitmap, c_ok: NodeBitmap,
                  src_col: str = "source", dst_col: str = "target") -> int:
    """count(*) of the same 2-hop MATCH, closed form (sum_b inA(b) outC(b) - eligible self-loops)."""
    v = ctypes.c_int64()
    _lib.call("capsmi_two_hop_count", session.handle, len(rels), _handles(rels), src_col.encode(), dst_col.encode(),
              a_ok.handle, b_ok.handle, c_ok.handle, ctypes.byref(v))
    return v.value


class CountShard:
    """count(*) of the 2-hop chain on one rank of an owner(target) partition (capsmi_count_shard_*).

    ``begin`` writes the in-degrees of the owned ids [own_lo, own_hi) (domain-relative) to the device
    buffer at ``owned_ptr`` (uint32); the caller all-gathers those slices into one array of every
    id's in-degree and ``finish`` writes this rank's part of the count to the device int64 at
    ``out_ptr``.  The ranks' parts sum to the count.  Both calls are stream-ordered.
    """

    def __init__(self, session: Session, rels: Sequence[GpuTable], a_ok: NodeBitmap, b_ok: NodeBitmap,
                 c_ok: NodeBitmap, own_lo: int, own_hi: int, owned_ptr: int, src_col: str = "source",
                 dst_col: str = "target"):
        h = ctypes.c_void_p()
        _lib.call("capsmi_count_shard_begin", session.handle, len(rels), _handles(rels), src_col.encode(),
                  dst_col.encode(), a_ok.handle, b_ok.handle, c_ok.handle, own_lo, own_hi,
                  ctypes.c_void_p(owned_ptr), ctypes.byref(h))
        self.handle = h
        self._keep = (session, list(rels), a_ok, b_ok, c_ok)

    def finish(self, in_all_ptr: int, out_ptr: int) -> None:
        _lib.call("capsmi_count_shard_finish", self.handle, ctypes.c_void_p(in_all_ptr), ctypes.c_void_p(out_ptr))

    def close(self) -> None:
        if self.handle:
            _lib.call("capsmi_count_shard_release", self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def two_hop_mark_mid(session: Session, rels: Sequence[GpuTable], a_ok: NodeBitmap, b_ok: NodeBitmap,
                     mid_ptr: int, scratch_ptr: int, src_col: str = "source", dst_col: str = "target") -> None:
    _lib.call("capsmi_two_hop_mark_mid", session.handle, len(rels), _handles(rels), src_col.encode(),
              dst_col.encode(), a_ok.handle, b_ok.handle, ctypes.c_void_p(mid_ptr), ctypes.c_void_p(scratch_ptr))


def two_hop_mark_dst(session: Session, rels: Sequence[GpuTable], b_ok: NodeBitmap, c_ok: NodeBitmap, mid_ptr: int,
                     dst_ptr: int, src_col: str = "source", dst_col: str = "target") -> None:
    _lib.call("capsmi_two_hop_mark_dst", session.handle, len(rels), _handles(rels), src_col.encode(),
              dst_col.encode(), b_ok.handle, c_ok.handle, ctypes.c_void_p(mid_ptr), ctypes.c_void_p(dst_ptr))


def var_length_count(session: Session, rels: Sequence[GpuTable], a_ok: NodeBitmap, b_ok: NodeBitmap, lower: int,
                     upper: int, id_name: str = "id", count_name: str = "count", src_col: str = "source",
                     dst_col: str = "target") -> GpuTable:
    """``MATCH (a)-[*lower..upper]->(b) WHERE a_ok(a) AND b_ok(b) RETURN id(a), count(*)`` (0 <= lower <= upper <= 4)."""
    out = ctypes.c_void_p()
    _lib.call("capsmi_var_length_count", session.handle, len(rels), _handles(rels), src_col.encode(), dst_col.encode(),
              a_ok.handle, b_ok.handle, lower, upper, id_name.encode(), count_name.encode(), ctypes.byref(out))
    return GpuTable(session, out)


class VarlenShard:
    """One rank's share of the var-length grouped count (multi-GPU C5; include/capsmi.h
    capsmi_varlen_shard_*).  The rank owns source ids [own_lo, own_hi); `out_rels` are the
    relationships it owns by source, `in_rels` those from other ranks into its owned ids.  `od_ptr`
    and (in mid) `y_ptr` are device int64 buffers over the id domain that the caller sums over
    ranks between the phases:  begin -> sum od -> mid -> sum y -> finish."""

    def __init__(self, session: Session, out_rels: Sequence[GpuTable], in_rels: Sequence[GpuTable], a_ok: NodeBitmap,
                 b_ok: NodeBitmap, lower: int, upper: int, own_lo: int, own_hi: int, od_ptr: int,
                 src_col: str = "source", dst_col: str = "target"):
        self.session = session
        self._h = ctypes.c_void_p()
        self._keep = (list(out_rels), list(in_rels), a_ok, b_ok)  # inputs stay alive until finish
        _lib.call("capsmi_varlen_shard_begin", session.handle, len(out_rels), _handles(out_rels), len(in_rels),
                  _handles(in_rels), src_col.encode(), dst_col.encode(), a_ok.handle, b_ok.handle, lower, upper,
                  own_lo, own_hi, ctypes.c_void_p(od_ptr), ctypes.byref(self._h))

    def mid(self, y_ptr: int) -> None:
        _lib.call("capsmi_varlen_shard_mid", self._h, ctypes.c_void_p(y_ptr))

    def finish(self, id_name: str = "id", count_name: str = "count") -> GpuTable:
        out = ctypes.c_void_p()
        _lib.call("capsmi_varlen_shard_finish", self._h, id_name.encode(), count_name.encode(), ctypes.byref(out))
        return GpuTable(self.session, out)

    def release(self) -> None:
        if self._h:
            _lib.call("capsmi_varlen_shard_release", self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            if self._h and _lib._lib is not None:
                _lib._lib.capsmi_varlen_shard_release(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


class TriGraph:
    """Oriented simple graph with directed multiplicities for the cyclic triangle count (C4)."""

    def __init__(self, session: Session, rels: Sequence[GpuTable], n_ok: NodeBitmap, src_col: str = "source",
                 dst_col: str = "target"):
        self.session = session
        self._h = ctypes.c_void_p()
        _lib.call("capsmi_trigraph_build", session.handle, len(rels), _handles(rels), src_col.encode(),
                  dst_col.encode(), n_ok.handle, ctypes.byref(self._h))

    def count(self, part: int = 0, nparts: int = 1) -> int:
        v = ctypes.c_int64()
        _lib.call("capsmi_trigraph_count", self.session.handle, self._h, part, nparts, ctypes.byref(v))
        return v.value

    def stats(self):
        """(id-domain size, oriented simple edges)"""
        n, ne = ctypes.c_int64(), ctypes.c_int64()
        _lib.call("capsmi_trigraph_stats", self._h, ctypes.byref(n), ctypes.byref(ne))
        return n.value, ne.value

    def release(self) -> None:
        if self._h:
            _lib.call("capsmi_trigraph_release", self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            if self._h and _lib._lib is not None:
                _lib._lib.capsmi_trigraph_release(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


def triangle_count(session: Session, rels: Sequence[GpuTable], n_ok: NodeBitmap, src_col: str = "source",
                   dst_col: str = "target") -> int:
    """``MATCH (a)-[r1]->(b)-[r2]->(c)-[r3]->(a) RETURN count(*)`` (pairwise-distinct relationships)."""
    v = ctypes.c_int64()
    _lib.call("capsmi_triangle_count", session.handle, len(rels), _handles(rels), src_col.encode(), dst_col.encode(),
              n_ok.handle, ctypes.byref(v))
    return v.value


class RelPartition:
    """Radix-partitioned relationship layout (include/capsmi.h capsmi_relpart_*): built per query
    on the cold path, or kept across queries as the Cache analogue."""

    def __init__(self, session: Session, rels: Sequence[GpuTable], lo: int, hi: int, src_col: str = "source",
                 dst_col: str = "target", _handle=None):
        self.session = session
        self._h = ctypes.c_void_p() if _handle is None else _handle
        if _handle is None:
            _lib.call("capsmi_relpart_build", session.handle, len(rels), _handles(rels), src_col.encode(),
                      dst_col.encode(), lo, hi, ctypes.byref(self._h))

    @classmethod
    def build_mark_mid(cls, session: Session, rels: Sequence[GpuTable], a_ok: "NodeBitmap", b_ok: "NodeBitmap",
                       mid_ptr: int, scratch_ptr: int, src_col: str = "source",
                       dst_col: str = "target") -> "RelPartition":
        """Cold 2-hop: build the layout over b_ok's id domain and run hop 1 (RelPartition.mark_mid) in
        the same pass when a_ok is full (include/capsmi.h capsmi_relpart_build_mark_mid)."""
        h = ctypes.c_void_p()
        _lib.call("capsmi_relpart_build_mark_mid", session.handle, len(rels), _handles(rels), src_col.encode(),
                  dst_col.encode(), a_ok.handle, b_ok.handle, ctypes.c_void_p(mid_ptr), ctypes.c_void_p(scratch_ptr),
                  ctypes.byref(h))
        return cls(session, rels, 0, 0, _handle=h)

    @property
    def handle(self):
        return self._h

    @property
    def size(self) -> int:
        v = ctypes.c_int64()
        _lib.call("capsmi_relpart_size", self._h, ctypes.byref(v))
        return v.value

    def digest(self):
        """Layout check (include/capsmi.h capsmi_relpart_digest): per-cell pair counts, per-cell wrapping
        sums of mix64(source << 32 | target) (ids relative to the domain), the number of misplaced pairs,
        and the geometry (ns, sbits, tbits)."""
        import numpy as np
        nc, ns, sb, tb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32()
        _lib.call("capsmi_relpart_digest", self._h, ctypes.byref(nc), ctypes.byref(ns), ctypes.byref(sb),
                  ctypes.byref(tb), None, None, None)
        counts = np.zeros(nc.value, np.int64)
        sums = np.zeros(nc.value, np.uint64)
        bad = ctypes.c_int64()
        _lib.call("capsmi_relpart_digest", self._h, ctypes.byref(nc), ctypes.byref(ns), ctypes.byref(sb),
                  ctypes.byref(tb), ctypes.c_void_p(counts.ctypes.data), ctypes.c_void_p(sums.ctypes.data),
                  ctypes.byref(bad))
        return counts, sums, bad.value, (ns.value, sb.value, tb.value)

    def release(self) -> None:
        if self._h:
            _lib.call("capsmi_relpart_release", self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            if self._h and _lib._lib is not None:
                _lib._lib.capsmi_relpart_release(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass

    def count_distinct(self, a_ok: NodeBitmap, b_ok: NodeBitmap, c_ok: NodeBitmap) -> int:
        v = ctypes.c_int64()
        _lib.call("capsmi_two_hop_count_distinct_part", self.session.handle, self._h, a_ok.handle, b_ok.handle,
                  c_ok.handle, ctypes.byref(v))
        return v.value

    def mark_mid(self, a_ok: NodeBitmap, b_ok: NodeBitmap, mid_ptr: int, scratch_ptr: int) -> None:
        _lib.call("capsmi_two_hop_mark_mid_part", self.session.handle, self._h, a_ok.handle, b_ok.handle,
                  ctypes.c_void_p(mid_ptr), ctypes.c_void_p(scratch_ptr))

    def mark_dst(self, b_ok: NodeBitmap, c_ok: NodeBitmap, mid_ptr: int, dst_ptr: int) -> None:
        _lib.call("capsmi_two_hop_mark_dst_part", self.session.handle, self._h, b_ok.handle, c_ok.handle,
                  ctypes.c_void_p(mid_ptr), ctypes.c_void_p(dst_ptr))


def words_popcount(session: Session, words_ptr: int, w_begin: int, w_end: int) -> int:
    v = ctypes.c_int64()
    _lib.call("capsmi_words_popcount", session.handle, ctypes.c_void_p(words_ptr), w_begin, w_end, ctypes.byref(v))
    return v.value


def words_popcount_device(session: Session, words_ptr: int, w_begin: int, w_end: int, out_ptr: int) -> None:
    """The popcount into a device int64 at `out_ptr` (e.g. a torch tensor's data_ptr), no host sync."""
    _lib.call("capsmi_words_popcount_device", session.handle, ctypes.c_void_p(words_ptr), w_begin, w_end,
              ctypes.c_void_p(out_ptr))


def cluster_by(rels: GpuTable, key_col: str, lo: int, hi: int) -> GpuTable:
    out = ctypes.c_void_p()
    _lib.call("capsmi_cluster_by", rels.handle, key_col.encode(), lo, hi, ctypes.byref(out))
    return GpuTable(rels.session, out)


def owner_words(nbits: int, part: int, nparts: int) -> Tuple[int, int]:
    b, e = ctypes.c_int64(), ctypes.c_int64()
    _lib.call("capsmi_owner_words", nbits, part, nparts, ctypes.byref(b), ctypes.byref(e))
    return b.value, e.value


PART_NONE, PART_SOURCE, PART_TARGET = -1, 0, 1


def rmat_rels(session: Session, scale: int, e_begin: int, e_end: int, probs=RMAT_GRAPH500, seed: int = 42,
              part_col: int = PART_NONE, part: int = 0, nparts: int = 1) -> GpuTable:
    """R-MAT relationship table [id, source, target] (definition: oracle/rmat.c)."""
    out = ctypes.c_void_p()
    pa, pb, pc = probs
    _lib.call("capsmi_rmat_rels", session.handle, scale, e_begin, e_end, pa, pb, pc, seed, part_col, part, nparts,
              ctypes.byref(out))
    return GpuTable(session, out)


NODES_ALL, NODES_PERSON, NODES_COMPANY = 0, 1, 2


def rmat_nodes(session: Session, scale: int, kind: int = NODES_ALL, seed: int = 42) -> GpuTable:
    out = ctypes.c_void_p()
    _lib.call("capsmi_rmat_nodes", session.handle, scale, kind, seed, ctypes.byref(out))
    return GpuTable(session, out)
