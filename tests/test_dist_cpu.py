"""Multi-GPU decomposition of C3, rehearsed on CPU with the gloo backend (world size 2 and 4).

Each rank keeps the relationships whose target id it owns (capsmi_owner_words slices), computes
hop 1 for its owned middle nodes, all-gathers the owned frontier slices (the one exchange of
bench.py), computes hop 2 for its owned end nodes, and all-reduces the popcount.  The per-rank
hop logic here is the numpy statement of the device kernels' rules; the result must equal the
single-process oracle enumeration."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _owner_ranges(n, world):
    import ctypes
    from capsmi import _lib
    lib = _lib.load()
    out = []
    for r in range(world):
        b, e = ctypes.c_int64(), ctypes.c_int64()
        assert lib.capsmi_owner_words(n, r, world, ctypes.byref(b), ctypes.byref(e)) == 0
        out.append((b.value * 32, min(e.value * 32, n)))
    return out


def _rank_main(rank, world, port, scale, result_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "cypher-for-apache-spark_amd")]
    import torch
    from oracle import cpu
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << scale
    lo, hi = _owner_ranges(n, world)[rank]
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    mine = (dst >= lo) & (dst < hi)          # partition by owner(target)
    s, t = src[mine], dst[mine]
    # hop 1 (all nodes Person): M = owned targets of non-loop rels; S1/S2 = 1 / 2+ self-loops
    M = np.zeros(n, dtype=np.uint8)
    M[t[s != t]] = 1
    loops = np.bincount(t[s == t], minlength=n)
    X1 = (M | (loops >= 1)).astype(np.uint8)
    X2 = (M | (loops >= 2)).astype(np.uint8)
    assert not X1[:lo].any() and not X1[hi:].any()   # hop 1 only marks owned middle nodes
    # the exchange: all-gather of owned slices
    for X in (X1, X2):
        parts = [torch.zeros(h - l, dtype=torch.uint8) for (l, h) in _owner_ranges(n, world)]
        dist.all_gather(parts, torch.from_numpy(X[lo:hi].copy()))
        X[:] = torch.cat(parts).numpy()
    # hop 2 on owned end nodes
    hit = np.where(s != t, X1[s], X2[s]).astype(bool)
    C = np.zeros(n, dtype=np.uint8)
    C[t[hit]] = 1
    cnt = torch.tensor([int(C[lo:hi].sum())], dtype=torch.int64)
    dist.all_reduce(cnt)
    if rank == 0:
        result_q.put(int(cnt.item()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_partitioned_two_hop_gloo(world):
    from oracle import cpu
    scale = 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, scale, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    _, want = cpu.two_hop_enumerate(1 << scale, src, dst)
    assert got == want


def test_owner_ranges_tile_the_domain():
    for n, world in [(1 << 10, 2), (1 << 26, 8), (1000, 3)]:
        r = _owner_ranges(n, world)
        assert r[0][0] == 0 and r[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
        assert all(l % 32 == 0 for l, _ in r)


def _count_rank_main(rank, world, port, scale, result_q):
    """count(*) over ranks (bench.py step_count_shards): owned in-degrees of a-ok sources into b-ok
    owned targets, one all-gather of the owned slices, each rank's sum of inA(source) over its
    relationships into c-ok targets less its a/b/c-ok self-loops, one all-reduce."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "cypher-for-apache-spark_amd")]
    import torch
    from oracle import cpu
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << scale
    lo, hi = _owner_ranges(n, world)[rank]
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    a, b, c = _count_masks(n)
    mine = (dst >= lo) & (dst < hi)
    s, t = src[mine], dst[mine]
    own = np.bincount(t[a[s] == 1] - lo, minlength=hi - lo).astype(np.int32) * b[lo:hi]
    parts = [torch.zeros(h - l, dtype=torch.int32) for (l, h) in _owner_ranges(n, world)]
    dist.all_gather(parts, torch.from_numpy(own.astype(np.int32)))
    in_all = torch.cat(parts).numpy().astype(np.int64)
    keep = c[t] == 1
    part = int(in_all[s[keep]].sum()) - int(((s == t) & (a[s] == 1) & (b[s] == 1) & (c[s] == 1)).sum())
    tot = torch.tensor([part], dtype=torch.int64)
    dist.all_reduce(tot)
    if rank == 0:
        result_q.put(int(tot.item()))
    dist.destroy_process_group()


def _count_masks(n):
    rng = np.random.default_rng(5)
    return tuple((rng.random(n) < p).astype(np.int64) for p in (0.9, 0.8, 0.85))


@pytest.mark.parametrize("world", [2, 4])  # gloo all_gather needs equal owned slices
def test_partitioned_count_star_gloo(world):
    from oracle import cpu
    scale = 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_count_rank_main, args=(r, world, port, scale, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale)
    a, b, c = _count_masks(n)
    want, _ = cpu.two_hop_closed_form(n, src, dst, a.astype(np.uint8), b.astype(np.uint8), c.astype(np.uint8))
    assert got == want
