#!/usr/bin/env python3
"""Benchmark: 2-hop friend-of-friend count(DISTINCT c) on R-MAT (BASELINE.json configs[2], "C3").

    MATCH (a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person) RETURN count(DISTINCT c)

Workload: R-MAT scale 26 (2^26 nodes, all Person), edge factor 16 (2^30
relationships), (A,B,C,D) = (.57,.19,.19,.05), seed 42, self-loops and multi-edges kept.  The
relationship table [id, source, target] (int64) is generated on the device; with N ranks each rank
holds the relationships whose target falls in its owner range (one rank per GPU, strong scaling:
the graph is fixed).  A step = the whole query from resident entity tables: node-scan bitmap
build, hop 1, the RCCL all-gather of the hop-1 frontier (N > 1), hop 2, popcount, all-reduce.

metric value = matched rows / s, where matched rows = count(*) of the same MATCH, i.e. the bindings
CAPS's joins would emit.  It is computed once in closed form (sum_b in(b)*out(b) - self-loops) on
the device outside the timed region -- the query never enumerates them.
Run: python bench.py [--gpus N --steps K --warmup W]  (torchrun for N > 1)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cypher-for-apache-spark_amd"))
sys.path.insert(0, ROOT)

METRIC = "matched rows/sec for 2-hop MATCH on R-MAT 2^30 edges; % HBM roofline @1/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--scale", type=int, default=26)
    p.add_argument("--edge-factor", type=int, default=16)
    p.add_argument("--layout", choices=["ingest", "clustered"], default="ingest",
                   help="ingest: rel rows in generation order; clustered: Cache-analogue copy sorted by target")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-scale", type=int, default=20)
    return p.parse_args()


def cpu_baseline(scale, ef):
    """The oracle (CPU restatement) on a bounded sample: the same query on R-MAT scale `scale`,
    computed the way CAPS's joins compute it -- every (a, r1, b, r2, c) binding enumerated."""
    from oracle import cpu
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    src, dst = cpu.rmat_edges(scale, 0, ef << scale)
    t0 = time.perf_counter()
    rows, dist = cpu.two_hop_enumerate(1 << scale, src, dst, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": rows / dt, "unit": "matched rows/s", "cores": threads, "kind": "port",
            "sample": f"R-MAT scale {scale} (2^{scale} nodes, {ef << scale} rels), full C3 query by binding "
                      f"enumeration (oracle/rmat.c orc_two_hop_enumerate): {rows} bindings, "
                      f"count(DISTINCT c)={dist}, {dt:.2f} s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("run with torch.distributed.run for --gpus > 1")
    distributed = world > 1
    torch.cuda.set_device(local)
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from capsmi import Session, graph

    sess = Session(local)
    stream = torch.cuda.current_stream()
    sess.set_stream(stream.cuda_stream)  # library kernels and RCCL collectives share one stream

    scale, ef = args.scale, args.edge_factor
    n = 1 << scale
    m_total = ef << scale
    nw = (n + 31) // 32
    assert nw % world == 0, "owner slices must be equal for all-gather"
    wb, we = graph.owner_words(n, rank, world)

    # ---- ingest (untimed): partitioned relationship table + replicated Person node table ----------
    t0 = time.perf_counter()
    rels = graph.rmat_rels(sess, scale, 0, m_total, graph.RMAT_GRAPH500, 42,
                           part_col=graph.PART_TARGET if distributed else graph.PART_NONE, part=rank, nparts=world)
    if args.layout == "clustered":
        rels = graph.cluster_by(rels, "target", 0, n)
    persons = graph.rmat_nodes(sess, scale, graph.NODES_ALL)
    m_local = rels.size
    sess.sync()
    ingest_s = time.perf_counter() - t0

    mid = torch.zeros(2 * nw, dtype=torch.int32, device="cuda")
    scratch = torch.zeros(nw, dtype=torch.int32, device="cuda")
    dstw = torch.zeros(nw, dtype=torch.int32, device="cuda")
    x1, x2 = mid[:nw], mid[nw:]
    sl = slice(wb, we)

    def step():
        p = graph.NodeBitmap(sess, 0, n).add_scan(persons, "id")  # node scan of :Person (a, b, c)
        graph.two_hop_mark_mid(sess, [rels], p, p, mid.data_ptr(), scratch.data_ptr())
        if distributed:  # frontier exchange: every rank needs X1/X2 of every middle node b
            dist.all_gather_into_tensor(x1, x1[sl].clone())
            dist.all_gather_into_tensor(x2, x2[sl].clone())
        graph.two_hop_mark_dst(sess, [rels], p, p, mid.data_ptr(), dstw.data_ptr())
        local_cnt = graph.words_popcount(sess, dstw.data_ptr(), wb, we)
        if distributed:
            t = torch.tensor([local_cnt], dtype=torch.int64, device="cuda")
            dist.all_reduce(t)
            return int(t.item())
        return local_cnt

    for _ in range(args.warmup):
        result = step()

    # ---- timed region --------------------------------------------------------------------------
    from capsmi import _lib
    import ctypes
    _lib.call("capsmi_session_set_profiling", sess.handle, 1)
    for k in ("hop1", "hop2", "mid_combine", "bitmap_add"):
        _lib.call("capsmi_session_kernel_time", sess.handle, k.encode(), ctypes.byref(ctypes.c_int64()),
                  ctypes.byref(ctypes.c_double()))
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        result = step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kt = {}
    for k in ("hop1", "hop2", "mid_combine", "bitmap_add"):
        cnt, ms = ctypes.c_int64(), ctypes.c_double()
        _lib.call("capsmi_session_kernel_time", sess.handle, k.encode(), ctypes.byref(cnt), ctypes.byref(ms))
        kt[k] = (cnt.value, ms.value)
    _lib.call("capsmi_session_set_profiling", sess.handle, 0)
    if distributed:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # ---- untimed checks: matched rows (closed form) and the unpartitioned answer on rank 0 -------
    matched = None
    check = None
    if rank == 0:
        if distributed:
            full = graph.rmat_rels(sess, scale, 0, m_total, graph.RMAT_GRAPH500, 42)
        else:
            full = rels
        p = graph.NodeBitmap(sess, 0, n).add_scan(persons, "id")
        matched = graph.two_hop_count(sess, [full], p, p, p)
        ref_distinct = graph.two_hop_count_distinct(sess, [full], p, p, p)
        check = "ok" if ref_distinct == result else f"MISMATCH partitioned={result} full={ref_distinct}"
        del full

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        hop2_n, hop2_ms = kt["hop2"]
        hop1_n, hop1_ms = kt["hop1"]
        avg2 = hop2_ms / max(hop2_n, 1)
        avg1 = hop1_ms / max(hop1_n, 1)
        # algorithmic bytes: a rel scan = E * (16 + 8 [rel id referenced by r1 <> r2]),
        # a node scan = N * 8.  hop2 processes rel scan r2 + node scan c on this rank's rels.
        alg2 = m_local * 24 + n * 8
        alg1 = m_local * 24 + 2 * n * 8
        dom, avg, alg = ("hop2", avg2, alg2) if avg2 >= avg1 else ("hop1", avg1, alg1)
        achieved = alg / (avg * 1e-3) / 1e9
        query_alg = 2 * 24 * m_total + 3 * 8 * n
        line = {
            "metric": METRIC,
            "value": matched / (elapsed / args.steps),
            "unit": "matched rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic R-MAT (on-device counter-based generator, oracle/rmat.c definition)",
            "config": {"workload": "C3: MATCH (a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person) "
                                   "RETURN count(DISTINCT c)",
                       "scale": scale, "nodes": n, "relationships": m_total, "rmat": [0.57, 0.19, 0.19, 0.05],
                       "seed": 42, "layout": args.layout,
                       "parallelism": f"rels partitioned by owner(target) over {world} GPU(s); "
                                      "hop-1 frontier all-gather + count all-reduce over RCCL"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": f"k_{dom}",
                         "kernel_ms": avg, "alg_bytes_per_launch": alg},
            "query": {"count_distinct_c": result, "matched_rows": matched, "check_vs_unpartitioned": check,
                      "hop1_ms": avg1, "hop2_ms": avg2,
                      "alg_bytes_query": query_alg,
                      "alg_GBs_query_per_gpu": query_alg / world / (ms_per_step * 1e-3) / 1e9,
                      "rels_local_rank0": m_local, "ingest_s": ingest_s},
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(args.cpu_scale, ef)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    sess.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
