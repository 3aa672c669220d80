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
COLL_CHUNK_ELEMS = 1 << 26  # words one collective call moves in all (512 MiB of int64)


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
    takes host pointers (the gloo CPU tests of the exchange logic)."""

    def __init__(self, group=None, device: str = "cuda", chunk_elems: int | None = None):
        import os

        import torch.distributed as dist
        self.dist = dist
        # elements one collective call moves in all (CAPSMI_COLL_CHUNK): the C4 build's exchanges and
        # all-gathers carry up to 2^28 words (2 GiB), which go out in calls of at most this many
        self.chunk = max(1, int(chunk_elems or os.environ.get("CAPSMI_COLL_CHUNK", COLL_CHUNK_ELEMS)))
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
        dist = self.dist
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
            out, inp = self.view(recv, count * W, dtype), self.view(send, count, dtype)
            per = max(1, self.chunk // W)
            if count <= per:
                dist.all_gather_into_tensor(out, inp, group=self.group)
            else:  # rank-major slices of at most `per` words per rank, placed into the rank-major output
                o2 = out.view(W, count)
                for off in range(0, count, per):
                    c = min(per, count - off)
                    tmp = torch.empty(W * c, dtype=out.dtype, device=out.device)
                    dist.all_gather_into_tensor(tmp, inp[off:off + c], group=self.group)
                    o2[:, off:off + c].copy_(tmp.view(W, c))
        elif op in (_lib.COLL_ALL_REDUCE_SUM, _lib.COLL_ALL_REDUCE_MAX):
            r = self.view(recv, count, dtype)
            if send != recv:
                r.copy_(self.view(send, count, dtype))
            rop = dist.ReduceOp.SUM if op == _lib.COLL_ALL_REDUCE_SUM else dist.ReduceOp.MAX
            for off in range(0, max(count, 1), self.chunk):
                dist.all_reduce(r[off:off + self.chunk], op=rop, group=self.group)
        elif op == _lib.COLL_ALL_TO_ALL_V:
            assert count == W, (count, W)
            sd, sc, rd, rc = a2av_lists(send, recv, W)
            inp, out = self.view(sd, sum(sc), dtype), self.view(rd, sum(rc), dtype)
            if self.drain:  # gloo: host tensors
                host = torch.empty(sum(rc), dtype=out.dtype)
                self._a2av(host, inp.cpu(), sc, rc)
                out.copy_(host)
            else:
                self._a2av(out, inp, sc, rc)
        else:
            raise ValueError(f"collective op {op}")
        if self.drain:
            torch.cuda.current_stream().synchronize()

    def _a2av(self, dst, src, sc, rc) -> None:
        """all_to_all_single in rounds of at most `chunk / world` words per (source, destination) pair; the
        ranks agree on the number of rounds by one MAX all-reduce when any rank needs more than one."""
        import torch
        dist = self.dist
        W = self.world
        per = max(1, self.chunk // W)
        local = max(1, -(-max(max(sc), max(rc)) // per))
        rounds = local
        if W > 1:
            t = torch.tensor([local], dtype=torch.int64, device=src.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            rounds = int(t.item())
        if rounds == 1:
            dist.all_to_all_single(dst, src, output_split_sizes=rc, input_split_sizes=sc, group=self.group)
            return
        so, ro = [0] * W, [0] * W
        for q in range(1, W):
            so[q] = so[q - 1] + sc[q - 1]
            ro[q] = ro[q - 1] + rc[q - 1]
        for k in range(rounds):
            ss = [min(per, max(0, sc[q] - k * per)) for q in range(W)]
            rr = [min(per, max(0, rc[q] - k * per)) for q in range(W)]
            parts = [src[so[q] + k * per:so[q] + k * per + ss[q]] for q in range(W) if ss[q]]
            tin = torch.cat(parts) if parts else src.new_empty(0)
            tout = dst.new_empty(sum(rr))
            dist.all_to_all_single(tout, tin, output_split_sizes=rr, input_split_sizes=ss, group=self.group)
            pos = 0
            for q in range(W):
                if rr[q]:
                    dst[ro[q] + k * per:ro[q] + k * per + rr[q]].copy_(tout[pos:pos + rr[q]])
                    pos += rr[q]


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
