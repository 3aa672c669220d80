"""Multi-GPU host side: the collective libcapsmi calls at the exchange points of its fused routes
(include/capsmi.h capsmi_session_set_ranks), and the registration of a rank's shard of a graph
(capsmi_graph_distribute).

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  The library hands device
pointers on the session's stream; they are wrapped as torch tensors (``__cuda_array_interface__``,
zero-copy) and the collective runs on torch's current stream -- the session runs on that same stream
(``Session.set_stream``), so kernels and collectives stay in one order.  With the gloo backend (a
rehearsal of several ranks on one GPU) the stream is drained around each collective, and the
all-to-all goes through host copies (gloo's all-to-all takes host tensors).

The ALL_TO_ALL_V is Spark's Exchange hashpartitioning (SparkTable.scala:133, 226): the library has
exchanged the per-rank counts already (an ALL_GATHER), so both count lists arrive with the call.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

from . import _lib
from .table import GpuTable, Session

_DT = {0: "<i8", _lib.COLL_U32: "<i4"}


class _DevPtr:
    """A device buffer as a ``__cuda_array_interface__`` exporter (no copy)."""

    def __init__(self, ptr: int, count: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (int(count),), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 2}


def device_view(ptr: int, count: int, dtype: int):
    import torch
    if count == 0 or not ptr:
        return torch.empty(0, dtype=torch.int64 if dtype == 0 else torch.int32, device="cuda")
    return torch.as_tensor(_DevPtr(ptr, count, _DT[dtype]), device="cuda")


def host_view(ptr: int, count: int, dtype: int):
    """A host buffer as a tensor (no copy): the collective over host memory (CPU rehearsals / tests)."""
    import torch
    tdt = torch.int64 if dtype == 0 else torch.int32
    if count == 0 or not ptr:
        return torch.empty(0, dtype=tdt)
    ct = ctypes.c_int64 if dtype == 0 else ctypes.c_int32
    return torch.frombuffer((ct * int(count)).from_address(int(ptr)), dtype=tdt)


def a2av_lists(send: int, recv: int, world: int):
    """(send data, send counts, recv data, recv counts) of an ALL_TO_ALL_V call's descriptors."""
    sv = _lib.CollVec.from_address(int(send))
    rv = _lib.CollVec.from_address(int(recv))
    return sv.data or 0, [int(sv.counts[q]) for q in range(world)], rv.data or 0, [int(rv.counts[q]) for q in range(world)]


class SerialGate:
    """A rehearsal of N ranks on one GPU with their GPU work serialised (gloo ranks, CAPSMI_SERIAL_LOCK=
    <file>): a rank holds an inter-process lock while it runs between collectives and gives it up inside
    every collective, so no two ranks' kernels overlap and a rank's busy time (lock held) is what its
    share of the step takes on a device of its own -- the collectives' own time excluded (SURVEY.md 8e
    per-rank diagnostic; the multi-GPU scaling itself is measured by the driver on an 8-GPU node)."""

    def __init__(self, path: str):
        import os
        self.fd = os.open(path, os.O_CREAT | os.O_RDWR, 0o600)
        self.busy = 0.0
        self.t0 = None

    def acquire(self) -> None:
        import fcntl
        import time
        fcntl.flock(self.fd, fcntl.LOCK_EX)
        self.t0 = time.perf_counter()

    def release(self) -> None:
        import fcntl
        import time
        import torch
        torch.cuda.synchronize()
        self.busy += time.perf_counter() - self.t0
        self.t0 = None
        fcntl.flock(self.fd, fcntl.LOCK_UN)


def serial_gate():
    """The SerialGate of this process when CAPSMI_SERIAL_LOCK is set, else None."""
    import os
    global _GATE
    path = os.environ.get("CAPSMI_SERIAL_LOCK")
    if path and _GATE is None:
        _GATE = SerialGate(path)
    return _GATE


_GATE = None


class TorchCollective:
    """capsmi_collective_fn over torch.distributed (RCCL or, for rehearsals, gloo).  `device="cpu"`
    takes host pointers (the gloo CPU tests of the exchange logic).  One call of the library is one
    torch.distributed call: libcapsmi itself cuts every collective to at most CAPSMI_COLL_CHUNK elements
    (csrc/k_dist.hip collective / collective_a2av), so no adapter splits anything."""

    def __init__(self, group=None, device: str = "cuda"):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.device = device
        self.drain = device == "cuda" and dist.get_backend(group) != "nccl"
        self._make_view = device_view if device == "cuda" else host_view
        self._views = {}  # (ptr, count, dtype) -> tensor: the library's block cache hands back the same
        # buffers query after query, so their views are built once (a view costs tens of microseconds)
        self.gate = serial_gate() if self.drain else None

    def view(self, ptr: int, count: int, dtype: int):
        key = (int(ptr or 0), int(count), int(dtype))
        t = self._views.get(key)
        if t is None:
            t = self._make_view(ptr, count, dtype)
            if len(self._views) >= 256:
                self._views.clear()
            self._views[key] = t
        return t

    def __call__(self, op: int, send: int, recv: int, count: int, dtype: int) -> None:
        import torch
        if self.drain:
            torch.cuda.current_stream().synchronize()
        gated = self.gate is not None and self.gate.t0 is not None
        if gated:  # the serialised rehearsal: another rank runs while this one waits in the collective
            self.gate.release()
        try:
            self._run(op, send, recv, count, dtype)
        finally:
            if gated:
                self.gate.acquire()

    def _run(self, op: int, send: int, recv: int, count: int, dtype: int) -> None:
        import torch
        dist = self.dist
        W = self.world
        if op == _lib.COLL_ALL_GATHER:
            dist.all_gather_into_tensor(self.view(recv, count * W, dtype), self.view(send, count, dtype),
                                        group=self.group)
        elif op in (_lib.COLL_ALL_REDUCE_SUM, _lib.COLL_ALL_REDUCE_MAX):
            r = self.view(recv, count, dtype)
            if send != recv:
                r.copy_(self.view(send, count, dtype))
            rop = dist.ReduceOp.SUM if op == _lib.COLL_ALL_REDUCE_SUM else dist.ReduceOp.MAX
            dist.all_reduce(r, op=rop, group=self.group)
        elif op == _lib.COLL_ALL_TO_ALL_V:
            assert count == W, (count, W)
            sd, sc, rd, rc = a2av_lists(send, recv, W)
            inp, out = self.view(sd, sum(sc), dtype), self.view(rd, sum(rc), dtype)
            if self.drain:  # gloo: host tensors
                host = torch.empty(sum(rc), dtype=out.dtype)
                dist.all_to_all_single(host, inp.cpu(), output_split_sizes=rc, input_split_sizes=sc, group=self.group)
                out.copy_(host)
            else:
                dist.all_to_all_single(out, inp, output_split_sizes=rc, input_split_sizes=sc, group=self.group)
        else:
            raise ValueError(f"collective op {op}")
        if self.drain:
            torch.cuda.current_stream().synchronize()


def join_ranks(session: Session, group=None) -> None:
    """Give the session its rank view over the torch.distributed process group."""
    import torch.distributed as dist
    session.set_ranks(dist.get_rank(group), dist.get_world_size(group), TorchCollective(group))


def distribute(session: Session, id_lo: int, id_hi: int, nodes: Sequence[GpuTable], rels: Sequence[GpuTable],
               nodes_owned: bool = True, rels_by: str = "target") -> None:
    """Register this rank's entity tables as its shard of a graph over ids [id_lo, id_hi)
    (include/capsmi.h capsmi_graph_distribute).  rels_by="source" also exchanges the relationships into
    this rank's owned ids from other ranks' sources (the shard's in-relationships)."""
    na = (_lib.c_void_p * max(1, len(nodes)))(*[t.handle for t in nodes])
    ra = (_lib.c_void_p * max(1, len(rels)))(*[t.handle for t in rels])
    _lib.call("capsmi_graph_distribute", session.handle, id_lo, id_hi, len(nodes), na,
              _lib.NODES_OWNED if nodes_owned else _lib.NODES_REPLICATED, len(rels), ra,
              _lib.RELS_BY_TARGET if rels_by == "target" else _lib.RELS_BY_SOURCE)
