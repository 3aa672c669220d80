"""Multi-GPU host side: the collective libcapsmi calls at the exchange points of its fused routes
(include/capsmi.h capsmi_session_set_ranks), and the registration of a rank's shard of a graph
(capsmi_graph_distribute).

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  The library hands device
pointers on the session's stream; they are wrapped as torch tensors (``__cuda_array_interface__``,
zero-copy) and the collective runs on torch's current stream -- the session runs on that same stream
(``Session.set_stream``), so kernels and collectives stay in one order.  With the gloo backend (a
rehearsal of several ranks on one GPU) the stream is drained around each collective.
"""
from __future__ import annotations

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
    return torch.as_tensor(_DevPtr(ptr, count, _DT[dtype]), device="cuda")


class TorchCollective:
    """capsmi_collective_fn over torch.distributed (RCCL or, for rehearsals, gloo)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.drain = dist.get_backend(group) != "nccl"

    def __call__(self, op: int, send: int, recv: int, count: int, dtype: int) -> None:
        import torch
        dist = self.dist
        if self.drain:
            torch.cuda.current_stream().synchronize()
        if op == _lib.COLL_ALL_GATHER:
            dist.all_gather_into_tensor(device_view(recv, count * self.world, dtype), device_view(send, count, dtype),
                                        group=self.group)
        elif op in (_lib.COLL_ALL_REDUCE_SUM, _lib.COLL_ALL_REDUCE_MAX):
            r = device_view(recv, count, dtype)
            if send != recv:
                r.copy_(device_view(send, count, dtype))
            dist.all_reduce(r, op=dist.ReduceOp.SUM if op == _lib.COLL_ALL_REDUCE_SUM else dist.ReduceOp.MAX,
                            group=self.group)
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
    (include/capsmi.h capsmi_graph_distribute)."""
    na = (_lib.c_void_p * max(1, len(nodes)))(*[t.handle for t in nodes])
    ra = (_lib.c_void_p * max(1, len(rels)))(*[t.handle for t in rels])
    _lib.call("capsmi_graph_distribute", session.handle, id_lo, id_hi, len(nodes), na,
              _lib.NODES_OWNED if nodes_owned else _lib.NODES_REPLICATED, len(rels), ra,
              _lib.RELS_BY_TARGET if rels_by == "target" else _lib.RELS_BY_SOURCE)
