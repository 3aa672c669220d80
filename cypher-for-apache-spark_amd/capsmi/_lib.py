"""ctypes binding of libcapsmi.so (include/capsmi.h).

The library is built in-tree (``make -C cypher-for-apache-spark_amd``).  There is no fallback:
if the shared object is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int32, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

from .expr import CapsmiExpr

# CAPSMI_LIB: an alternative build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("CAPSMI_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcapsmi.so")

OK = 0
ERR_ILLEGAL_ARGUMENT = 1
ERR_NOT_IMPLEMENTED = 2
ERR_UNSUPPORTED = 3
ERR_DEVICE = 4
ERR_OUT_OF_MEMORY = 5
ERR_INTERNAL = 6


class CapsmiError(RuntimeError):
    """Base error; subclasses mirror okapi's exception classes
    (okapi-api/src/main/scala/org/opencypher/okapi/impl/exception/InternalException.scala:34-59)."""
    code = ERR_INTERNAL


class IllegalArgumentException(CapsmiError):
    code = ERR_ILLEGAL_ARGUMENT


class NotImplementedException(CapsmiError):
    code = ERR_NOT_IMPLEMENTED


class UnsupportedOperationException(CapsmiError):
    code = ERR_UNSUPPORTED


class DeviceError(CapsmiError):
    code = ERR_DEVICE


class OutOfMemoryError(CapsmiError):
    code = ERR_OUT_OF_MEMORY


class InternalException(CapsmiError):
    code = ERR_INTERNAL


_BY_CODE = {c.code: c for c in (IllegalArgumentException, NotImplementedException, UnsupportedOperationException,
                                DeviceError, OutOfMemoryError, InternalException)}


class ColDesc(ctypes.Structure):
    _fields_ = [("name", c_char_p), ("type", c_int32), ("data", c_void_p), ("valid", c_void_p)]


class Value(ctypes.Structure):  # capsmi_value
    _fields_ = [("ival", ctypes.c_int64), ("is_null", c_int32), ("reserved", c_int32)]


class Param(ctypes.Structure):  # capsmi_param
    _fields_ = [("type", c_int32), ("is_list", c_int32), ("count", c_int32), ("reserved", c_int32),
                ("values", c_void_p)]


class ExprColumn(ctypes.Structure):
    _fields_ = [("name", c_char_p), ("nnodes", c_int32), ("prog", POINTER(CapsmiExpr))]


class Agg(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("distinct", c_int32), ("input", c_char_p), ("output", c_char_p)]


P = c_void_p  # opaque handles
PP = POINTER(c_void_p)
STRS = POINTER(c_char_p)

INTERN_FN = ctypes.CFUNCTYPE(c_int64, c_void_p, ctypes.POINTER(ctypes.c_char), c_size_t)
# capsmi_collective_fn(ctx, op, send, recv, count, dtype) -> 0 on success
COLLECTIVE_FN = ctypes.CFUNCTYPE(c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_int64, c_int32)
COLL_ALL_GATHER, COLL_ALL_REDUCE_SUM, COLL_ALL_REDUCE_MAX, COLL_ALL_TO_ALL_V, COLL_U32 = 0, 1, 2, 3, 100


class CollVec(ctypes.Structure):
    """capsmi_coll_vec: one side of an ALL_TO_ALL_V (device data, host counts per rank)."""
    _fields_ = [("data", c_void_p), ("counts", POINTER(c_int64))]

NODES_REPLICATED, NODES_OWNED = 0, 1
RELS_BY_SOURCE, RELS_BY_TARGET = 0, 1

# name -> (restype-is-status, argtypes)
_SIGS = {
    "capsmi_last_error": (c_size_t, [c_char_p, c_size_t]),
    "capsmi_version": (c_char_p, []),
    "capsmi_session_create": (c_int32, [c_int32, PP]),
    "capsmi_session_destroy": (c_int32, [P]),
    "capsmi_session_set_stream": (c_int32, [P, c_void_p]),
    "capsmi_session_use_stream": (c_int32, [P, c_void_p]),
    "capsmi_session_sync": (c_int32, [P]),
    "capsmi_session_set_config": (c_int32, [P, c_char_p, c_char_p]),
    "capsmi_config_check": (c_int32, [c_char_p, c_char_p]),
    "capsmi_session_set_profiling": (c_int32, [P, c_int32]),
    "capsmi_session_set_profiling_names": (c_int32, [P, c_char_p]),
    "capsmi_session_kernel_time": (c_int32, [P, c_char_p, POINTER(c_int64), POINTER(ctypes.c_double)]),
    "capsmi_session_kernel_bytes": (c_int32, [P, c_char_p, POINTER(ctypes.c_double)]),
    "capsmi_session_set_params": (c_int32, [P, c_int32, P]),
    "capsmi_table_from_host": (c_int32, [P, c_int32, POINTER(ColDesc), c_int64, PP]),
    "capsmi_table_from_device": (c_int32, [P, c_int32, POINTER(ColDesc), c_int64, PP]),
    "capsmi_table_retain": (c_int32, [P]),
    "capsmi_table_release": (c_int32, [P]),
    "capsmi_table_size": (c_int32, [P, POINTER(c_int64)]),
    "capsmi_table_num_columns": (c_int32, [P, POINTER(c_int32)]),
    "capsmi_table_column_name": (c_int32, [P, c_int32, c_char_p, c_size_t]),
    "capsmi_table_column_type": (c_int32, [P, c_int32, POINTER(c_int32)]),
    "capsmi_table_column_index": (c_int32, [P, c_char_p, POINTER(c_int32)]),
    "capsmi_table_column_nullable": (c_int32, [P, c_int32, POINTER(c_int32)]),
    "capsmi_table_schema": (c_int32, [P, POINTER(c_int32), c_char_p, c_size_t, POINTER(c_int32), POINTER(c_int32),
                                      c_int32]),
    "capsmi_table_export": (c_int32, [P, c_int32, c_void_p, c_void_p, c_int64, c_int64]),
    "capsmi_table_export_list": (c_int32, [P, c_int32, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_int64,
                                           POINTER(c_int64)]),
    "capsmi_table_column_device_ptr": (c_int32, [P, c_int32, PP, PP]),
    "capsmi_cache": (c_int32, [P, PP]),
    "capsmi_select": (c_int32, [P, c_int32, STRS, PP]),
    "capsmi_filter": (c_int32, [P, c_int32, POINTER(CapsmiExpr), PP]),
    "capsmi_drop": (c_int32, [P, c_int32, STRS, PP]),
    "capsmi_join": (c_int32, [P, P, c_int32, c_int32, STRS, STRS, PP]),
    "capsmi_union_all": (c_int32, [P, P, PP]),
    "capsmi_order_by": (c_int32, [P, c_int32, STRS, POINTER(c_int32), PP]),
    "capsmi_skip": (c_int32, [P, c_int64, PP]),
    "capsmi_limit": (c_int32, [P, c_int64, PP]),
    "capsmi_distinct": (c_int32, [P, PP]),
    "capsmi_distinct_on": (c_int32, [P, c_int32, STRS, PP]),
    "capsmi_group": (c_int32, [P, c_int32, STRS, c_int32, POINTER(Agg), PP]),
    "capsmi_with_columns": (c_int32, [P, c_int32, POINTER(ExprColumn), PP]),
    "capsmi_with_column_renamed": (c_int32, [P, c_char_p, c_char_p, PP]),
    "capsmi_bitmap_create": (c_int32, [P, c_int64, c_int64, PP]),
    "capsmi_bitmap_add_scan": (c_int32, [P, P, c_char_p, c_int32, POINTER(CapsmiExpr)]),
    "capsmi_bitmap_stats": (c_int32, [P, POINTER(c_int64), POINTER(c_int32)]),
    "capsmi_bitmap_release": (c_int32, [P]),
    "capsmi_bitmap_words": (c_int32, [P, PP, POINTER(c_int64)]),
    "capsmi_bitmap_refresh": (c_int32, [P, c_int32]),
    "capsmi_bitmap_assume": (c_int32, [P, c_int64, c_int32]),
    "capsmi_bitmap_copy_words": (c_int32, [P, c_int64, c_int64, c_void_p, c_int32]),
    "capsmi_expand_filter": (c_int32, [P, P, c_char_p, c_char_p, P, P, c_int32, STRS, STRS, PP]),
    "capsmi_two_hop_count_distinct": (c_int32, [P, c_int32, PP, c_char_p, c_char_p, P, P, P, POINTER(c_int64)]),
    "capsmi_two_hop_count": (c_int32, [P, c_int32, PP, c_char_p, c_char_p, P, P, P, POINTER(c_int64)]),
    "capsmi_two_hop_mark_mid": (c_int32, [P, c_int32, PP, c_char_p, c_char_p, P, P, c_void_p, c_void_p]),
    "capsmi_two_hop_mark_dst": (c_int32, [P, c_int32, PP, c_char_p, c_char_p, P, P, c_void_p, c_void_p]),
    "capsmi_words_popcount": (c_int32, [P, c_void_p, c_int64, c_int64, POINTER(c_int64)]),
    "capsmi_words_popcount_device": (c_int32, [P, c_void_p, c_int64, c_int64, c_void_p]),
    "capsmi_count_shard_begin": (c_int32, [P, c_int32, c_void_p, c_char_p, c_char_p, P, P, P, c_int64, c_int64, c_void_p,
                                           POINTER(c_void_p)]),
    "capsmi_count_shard_finish": (c_int32, [P, c_void_p, c_void_p]),
    "capsmi_count_shard_release": (c_int32, [P]),
    "capsmi_relpart_build": (c_int32, [P, c_int32, PP, c_char_p, c_char_p, c_int64, c_int64, PP]),
    "capsmi_relpart_build_mark_mid": (c_int32, [P, c_int32, PP, c_char_p, c_char_p, P, P, P, P, PP]),
    "capsmi_relpart_size": (c_int32, [P, POINTER(c_int64)]),
    "capsmi_relpart_digest": (c_int32, [P, POINTER(c_int64), POINTER(c_int64), POINTER(c_int32), POINTER(c_int32), P, P,
                                        POINTER(c_int64)]),
    "capsmi_trigraph_build": (c_int32, [P, c_int32, PP, c_char_p, c_char_p, P, PP]),
    "capsmi_trigraph_count": (c_int32, [P, P, c_int32, c_int32, POINTER(c_int64)]),
    "capsmi_trigraph_release": (c_int32, [P]),
    "capsmi_trigraph_stats": (c_int32, [P, POINTER(c_int64), POINTER(c_int64)]),
    "capsmi_triangle_count": (c_int32, [P, c_int32, PP, c_char_p, c_char_p, P, POINTER(c_int64)]),
    "capsmi_undirected_count": (c_int32, [P, c_int32, PP, c_char_p, c_char_p, c_int32, P, P, P, c_int32,
                                          POINTER(c_int64)]),
    "capsmi_var_length_count": (c_int32, [P, c_int32, PP, c_char_p, c_char_p, P, P, c_int32, c_int32, c_char_p,
                                          c_char_p, PP]),
    "capsmi_varlen_shard_begin": (c_int32, [P, c_int32, PP, c_int32, PP, c_char_p, c_char_p, P, P, c_int32, c_int32,
                                            c_int64, c_int64, c_void_p, PP]),
    "capsmi_varlen_shard_mid": (c_int32, [P, c_void_p]),
    "capsmi_varlen_shard_finish": (c_int32, [P, c_char_p, c_char_p, PP]),
    "capsmi_varlen_shard_release": (c_int32, [P]),
    "capsmi_relpart_release": (c_int32, [P]),
    "capsmi_two_hop_mark_mid_part": (c_int32, [P, P, P, P, c_void_p, c_void_p]),
    "capsmi_two_hop_mark_dst_part": (c_int32, [P, P, P, P, c_void_p, c_void_p]),
    "capsmi_two_hop_count_distinct_part": (c_int32, [P, P, P, P, P, POINTER(c_int64)]),
    "capsmi_cluster_by": (c_int32, [P, c_char_p, c_int64, c_int64, PP]),
    "capsmi_rmat_rels": (c_int32, [P, c_int32, c_int64, c_int64, c_int32, c_int32, c_int32, c_uint64, c_int32,
                                   c_int32, c_int32, PP]),
    "capsmi_owner_words": (c_int32, [c_int64, c_int32, c_int32, POINTER(c_int64), POINTER(c_int64)]),
    "capsmi_rmat_nodes": (c_int32, [P, c_int32, c_int32, c_uint64, PP]),
    "capsmi_table_fingerprint": (c_int32, [P, c_int32, STRS, POINTER(c_int64), POINTER(c_uint64), POINTER(c_uint64)]),
    "capsmi_node_table": (c_int32, [P, c_char_p, c_int32, STRS, PP]),
    "capsmi_rel_table": (c_int32, [P, c_char_p, c_char_p, c_char_p, c_int32, STRS, PP]),
    "capsmi_table_entity": (c_int32, [P, POINTER(c_int32), POINTER(c_int64), POINTER(c_int64)]),
    "capsmi_flatten_rel_types": (c_int32, [P, c_char_p, c_int32, POINTER(c_int64), STRS, PP]),
    "capsmi_session_set_fused": (c_int32, [P, c_int32]),
    "capsmi_graph_compact": (c_int32, [P, c_int32, PP, c_int32, PP, POINTER(c_int64)]),
    "capsmi_read_csv": (c_int32, [P, c_int32, STRS, ctypes.c_char, ctypes.c_char, c_int32, STRS, POINTER(c_int32),
                                  INTERN_FN, c_void_p, c_char_p, PP]),
    "capsmi_session_route_count": (c_int32, [P, c_char_p, POINTER(c_int64)]),
    "capsmi_session_set_unrouted_limit": (c_int32, [P, c_int64]),
    "capsmi_session_set_csv_partitioning": (c_int32, [P, c_int64, c_int64, c_int64]),
    "capsmi_session_set_ranks": (c_int32, [P, c_int32, c_int32, COLLECTIVE_FN, c_void_p]),
    "capsmi_graph_distribute": (c_int32, [P, c_int64, c_int64, c_int32, PP, c_int32, c_int32, PP, c_int32]),
    "capsmi_owned_rows": (c_int32, [P, P, c_char_p, c_int64, c_int64, PP]),
    "capsmi_table_partitioned": (c_int32, [P, POINTER(c_int32)]),
    "capsmi_id_owner": (c_int32, [c_int64, c_int64, c_int32, c_int64, POINTER(c_int32), POINTER(c_int64)]),
}

EXPORTED = tuple(_SIGS)

_lib = None


def load():
    """Load libcapsmi.so (raises if it was not built: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built; run `make -C cypher-for-apache-spark_amd`")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7).
    # Loading torch first makes libcapsmi's NEEDED entry resolve to that same runtime, so device
    # pointers, streams and RCCL collectives from torch and from libcapsmi live in one context.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    lib = load()
    buf = ctypes.create_string_buffer(4096)
    lib.capsmi_last_error(buf, 4096)
    return buf.value.decode("utf-8", "replace")


def check(status: int, what: str = "") -> None:
    if status != OK:
        cls = _BY_CODE.get(status, CapsmiError)
        raise cls(f"{what}: {last_error()}" if what else last_error())


_FN = {}  # name -> bound foreign function (skips the CDLL attribute lookup per call)


def call(name: str, *args) -> None:
    fn = _FN.get(name)
    if fn is None:
        fn = _FN[name] = getattr(load(), name)
    status = fn(*args)
    if status != OK:
        check(status, name)


_STRS = {}  # tuple of names -> its char* array (column-name lists repeat across a query's calls)


def strs(names):
    key = tuple(names)
    arr = _STRS.get(key)
    if arr is None:
        arr = (c_char_p * max(1, len(key)))(*[n.encode() for n in key])
        if len(_STRS) > 4096:
            _STRS.clear()
        _STRS[key] = arr
    return arr


__all__ = ["load", "call", "check", "strs", "last_error", "EXPORTED", "ColDesc", "ExprColumn", "Agg", "CapsmiError",
           "IllegalArgumentException", "NotImplementedException", "UnsupportedOperationException", "DeviceError",
           "OutOfMemoryError", "InternalException", "c_int64", "c_int32", "c_uint64", "c_uint32", "c_void_p"]
