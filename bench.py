#!/usr/bin/env python3
"""Benchmark: 2-hop friend-of-friend count(DISTINCT c) on R-MAT (BASELINE.json configs[2], "C3").

    MATCH (a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person) RETURN count(DISTINCT c)

Workload: R-MAT scale 26 (2^26 nodes, all Person), edge factor 16 (2^30
relationships), (A,B,C,D) = (.57,.19,.19,.05), seed 42, self-loops and multi-edges kept.  The
relationship table [id, source, target] (int64, generation order) is generated on the device; with N
ranks each rank holds the relationships whose target falls in its owner range (one rank per GPU,
strong scaling: the graph is fixed).

A step = the whole query from the resident entity tables, issued as the Table[T] calls the relational
planner emits (Planner(sg).run) and routed by libcapsmi to the fused kernels:
  cold (the reported value): node-scan bitmap, radix partition of the relationship table, hop 1, hop 2,
       popcount.  N > 1: every rank runs the same query over its shard of the distributed graph
       (relationships by a hash of their target, node rows by a hash of their id:
       capsmi_graph_distribute); the route all-gathers the owned node-scan and hop-1 frontier bitmap
       slices and all-reduces the count over RCCL (capsmi_session_set_ranks);
  warm: the same with the partition kept from an earlier query (Cache analogue);
  count: count(*) of the same match through the route;
  direct / direct_warm / stream (N = 1): the same kernels called explicitly (comparison).

metric value = matched rows / s, where matched rows = count(*) of the same MATCH, i.e. the bindings
CAPS's joins would emit.  It is computed once in closed form (sum_b in(b)*out(b) - self-loops) on the
device outside the timed region; the query itself never enumerates bindings.
Run: python bench.py [--gpus N --steps K --warmup W]  (torch.distributed.run for N > 1)
"""
import argparse
import ctypes
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cypher-for-apache-spark_amd"))
sys.path.insert(0, ROOT)

METRIC = "matched rows/sec for 2-hop MATCH on R-MAT 2^30 edges; % HBM roofline @1/8 GPU"
C2_QUERY = {"clauses": [{"match": "(a:Person)-[r:FRIEND_OF]->(b:Person)",
                          "where": ["and", [">=", ["prop", "a", "age"], ["lit", 18]],
                                    ["<", ["prop", "a", "age"], ["lit", 65]]]}],
            "return": {"items": [["a", ["id", "a"]], ["b", ["id", "b"]]]}}
C3_COUNT_QUERY = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person)"}],
                  "return": {"items": [["n", ["count*"]]]}}
C3_QUERY = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person)"}],
            "return": {"items": [["count(DISTINCT c)", ["count_distinct", ["id", "c"]]]]}}
# the undirected 2-hop (RelationalPlanner.scala:126-136: out ∪ in-without-loops per hop), bench modes und_count /
# und_distinct, checked against tests/golden/rmat_full.json c3u_s<scale>
C3U_COUNT_QUERY = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]-(b:Person)-[:FRIEND_OF]-(c:Person)"}],
                   "return": {"items": [["n", ["count*"]]]}}
C3U_QUERY = {"clauses": [{"match": "(a:Person)-[:FRIEND_OF]-(b:Person)-[:FRIEND_OF]-(c:Person)"}],
             "return": {"items": [["count(DISTINCT c)", ["count_distinct", ["id", "c"]]]]}}
C4_QUERY = {"clauses": [{"match": "(a:Person)-[r1:FRIEND_OF]->(b:Person)-[r2:FRIEND_OF]->(c:Person)-[r3:FRIEND_OF]->(a)"}],
            "return": {"items": [["n", ["count*"]]]}}
C5_QUERY = {"clauses": [{"match": "(a:Person)-[:KNOWS*1..3]->(b:Person)"}],
            "return": {"items": [["id", ["id", "a"]], ["count", ["count*"]]]}}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PROFILED_STEPS = 3  # untimed steps with every kernel timer (the per-kernel breakdown)
PAR_SOURCE = ("dp{w}: relationships hash-partitioned by source over {w} GPUs (capsmi_graph_distribute, north_star's "
              "owner(source)); hop-1 frontier slices exchanged by ALL_TO_ALL_V and ORed on their owner, end-bitmap "
              "slices the same, count all-reduce, over RCCL inside the route")
PAR_TARGET = ("dp{w}: relationships hash-partitioned by target over {w} GPUs (capsmi_graph_distribute); hop-1 "
              "frontier bitmap all-gather + count all-reduce over RCCL inside the route")
# what each C3-line mode runs (config.workload of a line headed by that mode), and the key of its answer
MODE_QUERY = {
    "und_count": ("C3 undirected: MATCH (a:Person)-[:FRIEND_OF]-(b:Person)-[:FRIEND_OF]-(c:Person) RETURN count(*)",
                  "und_count_star"),
    "und_distinct": ("C3 undirected: MATCH (a:Person)-[:FRIEND_OF]-(b:Person)-[:FRIEND_OF]-(c:Person) "
                     "RETURN count(DISTINCT c)", "und_count_distinct_c"),
    "count": ("C3: MATCH (a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person) RETURN count(*)", "count_star"),
    "count_atomic": ("C3: MATCH (a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person) RETURN count(*)",
                     "count_star"),
}
C3_WORKLOAD = "C3: MATCH (a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person) RETURN count(DISTINCT c)"
KERNELS = ("part_scatter1", "part_scatter2_hop1", "part_scatter2", "hop1", "hop2", "mid_combine", "bitmap_add",
           "bitmap_range",
           "count_part", "count_in", "count_out", "degrees", "und_count_part",
           "und_count", "und_distinct", "und_hop1", "und_hop2")
# timer name -> kernel name as rocprofv3 reports it (hop1 and hop2 are two instances of k_hop_2d)
KERNEL_SYMBOL = {"part_scatter1": "k_scatter_l", "part_scatter2_hop1": "k_scatter_s2", "part_scatter2": "k_scatter_s2",
                 "hop1": "k_hop_2d", "hop2": "k_hop_2d", "mid_combine": "k_mid_combine", "bitmap_add": "k_bitmap_add",
                 "bitmap_range": "k_bits_range",
                 "count_part": "k_rec_part", "count_in": "k_rec_walk",
                 "count_out": "k_rec_walk", "degrees": "k_degrees", "und_count_part": "k_rec_part",
                 "und_count": "k_und_deg", "und_distinct": "k_und_hop1+k_und_hop2", "und_hop1": "k_und_2d",
                 "und_hop2": "k_und_2d"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--scale", type=int, default=26)
    p.add_argument("--edge-factor", type=int, default=16)
    p.add_argument("--modes", default="cold,warm,direct,count",
                   help="comma list of cold, warm (the planner route, N=1), direct, direct_warm (explicit kernel "
                        "calls), stream, count / count_atomic (count(*) of the same match through the route, "
                        "partitioned / per-relationship atomic degrees), und_count / und_distinct (the undirected "
                        "2-hop count(*) / count(DISTINCT c) through the route) (first = value)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-scale", type=int, default=None, help="oracle sample scale (default per workload)")
    p.add_argument("--shard-of", type=int, default=0,
                   help="diagnostic (C3): time every rank's shard of an N-way partition (--rels-by) on one GPU, "
                        "no exchange; the line is not the metric")
    p.add_argument("--rels-by", default="target", choices=("source", "target"),
                   help="C3 at N > 1 / --dist1 / --shard-of: relationships partitioned by the owner of their target "
                        "(default: 15 %% faster per rank at 8 shards, DESIGN.md §7.8) or of their source (north_star; "
                        "the one distribution every route takes)")
    p.add_argument("--c2-route", default="direct", choices=("direct", "planner", "joins"),
                   help="C2: explicit expand kernels (direct), Planner(sg).run routed to the fused expand "
                        "(planner), or the same plan operator by operator through the generic radix joins (joins)")
    p.add_argument("--direct-multi", action="store_true",
                   help="C4/C5 at N > 1: the explicit-kernel calls of rounds 1-3 (replicated trigraph build; "
                        "hand-wired varlen shards) instead of the routed query")
    p.add_argument("--dist1", action="store_true",
                   help="diagnostic (C3, C4, C5): the distributed route at world size 1 over RCCL (launch with "
                        "torch.distributed.run --nproc-per-node 1): the route's fixed per-rank cost, exchanges included")
    p.add_argument("--plan-in-step", action="store_true",
                   help="planned modes (C3; the routed C2 / C4 / C5): build each step's plan inside the timed region (before round 5's "
                        "SURVEY.md 8d timing, the planning was part of every step)")
    p.add_argument("--tri-parts", type=int, default=0,
                   help="diagnostic (C4, one GPU): the interleaved center shares of N ranks of one "
                        "trigraph, each share's count timed alone -- the per-rank triangle phase without contention")
    p.add_argument("--workload", default="c3", choices=("c2", "c3", "c4", "c5"),
                   help="c3 (default, the BASELINE metric) or the single-GPU C2/C4/C5 lines (SURVEY.md 8d)")
    p.add_argument("--c5-upper", type=int, default=3, choices=(3, 4),
                   help="C5's upper bound: 3 (the BASELINE config) or 4 (the four-hop fused count, one GPU; a "
                        "diagnostic line without a fixture: its parity is the tests' against enumeration)")
    return p.parse_args()


def cpu_baseline(scale, ef):
    """The oracle on the host cores: (1) the SAME algorithm as the device path -- the closed form /
    frontier bitmaps of oracle/closed.c orc_two_hop_closed_form_mt -- on the SAME full workload
    (R-MAT `scale`, seed 42), OpenMP over `cores` threads; (2) a second, clearly labelled line: the
    join semantics CAPS runs (every (a, r1, b, r2, c) binding enumerated, oracle/rmat.c) on R-MAT
    scale 20.  Both are CPU restatements, not CAPS-on-Spark (no JVM on the box).  Edge generation is
    ingest and untimed."""
    from oracle import cpu
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, ef << scale)
    t0 = time.perf_counter()
    rows, dist = cpu.two_hop_closed_form_mt(n, src, dst, threads=threads)
    dt = time.perf_counter() - t0
    del src, dst
    es = 20
    s2, d2 = cpu.rmat_edges(es, 0, ef << es)
    t1 = time.perf_counter()
    erows, edist = cpu.two_hop_enumerate(1 << es, s2, d2, threads=threads)
    edt = time.perf_counter() - t1
    return {"value": rows / dt, "unit": "matched rows/s", "cores": threads, "kind": "port",
            "sample": f"CPU restatement, not CAPS: the device algorithm (closed form + frontier bitmaps, "
                      f"oracle/closed.c orc_two_hop_closed_form_mt) on the same workload, R-MAT scale {scale} "
                      f"({ef << scale} rels, seed 42), {threads} OpenMP threads: count(*)={rows}, "
                      f"count(DISTINCT c)={dist}, {dt:.2f} s",
            "enumeration": {"value": erows / edt, "unit": "matched rows/s", "cores": threads,
                            "sample": f"CAPS join semantics (every binding enumerated, oracle/rmat.c "
                                      f"orc_two_hop_enumerate) on R-MAT scale {es}: {erows} bindings, "
                                      f"count(DISTINCT c)={edist}, {edt:.2f} s"}}


def fixture(key):
    """Exact full-size answer from tests/golden/rmat_full.json (oracle closed forms, committed with
    the script that made them: tests/golden/make_rmat_full.py), or None."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "rmat_full.json")) as f:
            return json.load(f)["cases"].get(key)
    except (OSError, ValueError, KeyError):
        return None


def init_dist(dist, local):
    """RCCL (backend "nccl") one rank per GPU; CAPSMI_DIST_BACKEND=gloo rehearses the same ranks and
    collectives on fewer GPUs (RCCL refuses two ranks on one device)."""
    import torch
    backend = os.environ.get("CAPSMI_DIST_BACKEND", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)


# the C4 walk kernels: over the direction-split lists (the library's default whenever the targets are coded,
# i.e. <= 2^24 ids -- C4's config), or the combined lists (config CAPSMI_TRI_SPLIT=0)
TRI_SYMBOL = ("k_tri_big_items+k_tri_small" if os.environ.get("CAPSMI_TRI_SPLIT") == "0"
              else "k_tri_items_sp+k_tri_small_sp")


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of this workload
    (profiles/*_<workload>_pmc.json, newest round first), FETCH_SIZE doubled per MI355X_MICROARCH.md
    (gfx950 tallies 128-B reads at 64 B), or None."""
    if "+" in kernel:  # a timer spanning several kernels: their traffic per timed call, summed
        parts = [_pmc_entry(k, workload) for k in kernel.split("+")]
        if any(p is None for p in parts):
            return None
        calls = min(p["launches"] for p in parts)  # a kernel launched k times per call (C4: the item
        return sum(p["hbm_bytes_per_launch"] * p["launches"] / calls for p in parts)  # kernel, u- and v-mode)
    p = _pmc_entry(kernel, workload)
    return None if p is None else p["hbm_bytes_per_launch"]


def _pmc_entry(kernel, workload):
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{workload}_pmc.json")))
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
            k = d.get("kernels", {}).get(kernel)
            if k and "hbm_bytes_per_launch" in k and k.get("launches"):
                return k
        except (OSError, ValueError):
            continue
    return None


def shard_diagnostic(args):
    """--shard-of N on one GPU: every rank's owner(source) (or --rels-by target) shard of the C3 cold step,
    timed one after the other (kernels only: the frontier exchange and the count all-reduce are not run,
    the node scan is the whole table).  Reports per-rank times and the max -- the projected N-GPU step
    before the collectives.  Not the metric."""
    import torch
    from capsmi import Session, graph
    N = args.shard_of
    torch.cuda.set_device(0)
    sess = Session(0)
    sess.set_stream(torch.cuda.current_stream().cuda_stream)
    scale, ef = args.scale, args.edge_factor
    n, m_total = 1 << scale, ef << scale
    nw = (n + 31) // 32
    persons = graph.rmat_nodes(sess, scale, graph.NODES_ALL)
    mid = torch.zeros(2 * nw, dtype=torch.int32, device="cuda")
    scratch = torch.zeros(nw, dtype=torch.int32, device="cuda")
    dstw = torch.zeros(nw, dtype=torch.int32, device="cuda")
    own_in = torch.zeros(n, dtype=torch.int32, device="cuda")
    in_all = torch.zeros(n, dtype=torch.int32, device="cuda")  # stands in for the gathered in-degrees (timing)
    cnt_dev = torch.zeros(1, dtype=torch.int64, device="cuda")
    per_rank, per_rank_count, rows = [], [], []
    kernel_ms = {}  # rank 0's shard, per launch
    for r in range(N):
        by_src = args.rels_by == "source"
        rels = graph.rmat_rels(sess, scale, 0, m_total, graph.RMAT_GRAPH500, 42,
                               part_col=graph.PART_SOURCE if by_src else graph.PART_TARGET, part=r, nparts=N)
        wb, we = graph.owner_words(n, r, N)
        cs, cd = ("target", "source") if by_src else ("source", "target")  # count(*): reversed over BY_SOURCE

        def step():
            p = graph.NodeBitmap(sess, 0, n).add_scan(persons, "id")
            rp = graph.RelPartition.build_mark_mid(sess, [rels], p, p, mid.data_ptr(), scratch.data_ptr())
            rp.mark_dst(p, p, mid.data_ptr(), dstw.data_ptr())
            rp.release()
            return graph.words_popcount(sess, dstw.data_ptr(), wb, we)

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        per_rank.append((time.perf_counter() - t0) / args.steps * 1e3)
        if r == 0:  # per-kernel times of one shard (separate, profiled steps: the timed ones stay unprofiled)
            import ctypes
            from capsmi import _lib
            _lib.call("capsmi_session_set_profiling", sess.handle, 1)
            for _ in range(args.steps):
                step()
            for k in KERNELS:
                c, ms = ctypes.c_int64(), ctypes.c_double()
                _lib.call("capsmi_session_kernel_time", sess.handle, k.encode(), ctypes.byref(c), ctypes.byref(ms))
                if c.value:
                    kernel_ms[k] = ms.value / c.value
            _lib.call("capsmi_session_set_profiling", sess.handle, 0)

        def step_count():  # count(*) shard: partition + IN walk + owned fold, OUT walk (no gather / all-reduce)
            p = graph.NodeBitmap(sess, 0, n).add_scan(persons, "id")
            sh = graph.CountShard(sess, [rels], p, p, p, 32 * wb, min(32 * we, n), own_in.data_ptr(), cs, cd)
            sh.finish(in_all.data_ptr(), cnt_dev.data_ptr())
            sh.close()

        for _ in range(args.warmup):
            step_count()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_count()
        torch.cuda.synchronize()
        per_rank_count.append((time.perf_counter() - t0) / args.steps * 1e3)
        rows.append(rels.size)
        del rels
    mean = sum(per_rank) / N
    print(json.dumps({"diagnostic": f"C3 cold step, every rank's owner({args.rels_by}) shard of {N} on one GPU, "
                                    "no exchange",
                      "scale": scale, "per_rank_ms": per_rank, "max_ms": max(per_rank), "mean_ms": mean,
                      "imbalance_max_over_mean": max(per_rank) / mean, "rels_per_rank": rows,
                      "count_star_per_rank_ms": per_rank_count, "count_star_max_ms": max(per_rank_count),
                      "rank0_kernel_ms": kernel_ms}),
          flush=True)
    sess.close()


def main():
    args = parse()
    if args.workload != "c3":
        return run_single(args)
    if args.shard_of and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        return shard_diagnostic(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1:
        sys.exit("run with torch.distributed.run for --gpus > 1")
    distributed = world > 1 or args.dist1
    local = local % max(1, torch.cuda.device_count())  # rehearsal: several ranks may share one GPU (gloo)
    torch.cuda.set_device(local)
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        init_dist(dist, local)

    from capsmi import Session, _lib, graph

    sess = Session(local)
    sess.set_stream(torch.cuda.current_stream().cuda_stream)  # library kernels + RCCL on one stream

    scale, ef = args.scale, args.edge_factor
    n = 1 << scale
    m_total = ef << scale
    nw = (n + 31) // 32
    shards = args.shard_of if (args.shard_of and not distributed) else 1
    assert nw % shards == 0, "owner slices must be equal for the all-gather"
    part = rank if shards > 1 else 0  # --shard-of diagnostic only; N > 1 ranks shard by hash below
    wb, we = graph.owner_words(n, part, shards)
    modes = [m.strip() for m in args.modes.split(",") if m.strip()]
    if args.shard_of:  # count(*) of one shard alone is not a share of the count: skip it
        modes = [m for m in modes if not m.startswith("count")] or ["cold"]
    elif distributed:  # the drop-in route on every rank (no explicit-kernel or atomic A/B forms)
        modes = [m for m in modes if m in ("cold", "warm", "count")] or ["cold"]

    # ---- ingest (untimed): relationship table + Person node table ---------------------------------
    # N > 1: every rank generates the graph and keeps its shard -- the relationships whose target it
    # owns and the :Person rows of the ids it owns, ownership by a hash of the id (capsmi_owned_rows) --
    # then registers the shard (capsmi_graph_distribute); ingest is untimed
    t0 = time.perf_counter()
    ingest_gate = None
    if distributed:
        from capsmi.dist import distribute, join_ranks, serial_gate
        join_ranks(sess)  # the rank view first: capsmi_owned_rows owns by (rank, world)
        ingest_gate = serial_gate()  # a serialised rehearsal also serialises the ranks' ingest peaks
        if ingest_gate:
            ingest_gate.acquire()
        rels = owned_rmat_rels(sess, graph, scale, m_total, graph.RMAT_GRAPH500, args.rels_by, n)
    else:
        rels = graph.rmat_rels(sess, scale, 0, m_total, graph.RMAT_GRAPH500, 42,
                               part_col=graph.PART_TARGET if shards > 1 else graph.PART_NONE, part=part, nparts=shards)
    persons = graph.rmat_nodes(sess, scale, graph.NODES_ALL)
    if distributed:
        persons = persons.owned_rows("id", 0, n).as_node_table("id")
        distribute(sess, 0, n, [persons], [rels], nodes_owned=True, rels_by=args.rels_by)
    m_local = rels.size
    sess.sync()
    if ingest_gate:
        ingest_gate.release()
        ingest_gate.busy = 0.0
    ingest_s = time.perf_counter() - t0
    if distributed:  # the shards' sizes (balance of the hash ownership), on every rank
        sizes = torch.zeros(world, dtype=torch.int64, device="cuda")
        sizes[rank] = m_local
        dist.all_reduce(sizes)
        rels_per_rank = sizes.tolist()

    mid = torch.zeros(2 * nw, dtype=torch.int32, device="cuda")
    scratch = torch.zeros(nw, dtype=torch.int32, device="cuda")
    dstw = torch.zeros(nw, dtype=torch.int32, device="cuda")
    cached = {}

    k_own = we - wb
    send = torch.empty(2, k_own, dtype=torch.int32, device="cuda")
    recv = torch.empty(world * 2, k_own, dtype=torch.int32, device="cuda")  # rank-major (rank, X1|X2) rows
    nsend = torch.empty(k_own, dtype=torch.int32, device="cuda")
    nrecv = torch.empty(world * k_own, dtype=torch.int32, device="cuda")
    scan_stats = torch.zeros(2, dtype=torch.int64, device="cuda")  # (owned set bits, duplicate flag), summed
    cnt_dev = torch.zeros(1, dtype=torch.int64, device="cuda")

    def node_scan():
        """The :Person scan (a, b, c).  N > 1: every rank scans its owned rows into its slice of the
        bitmap, then one all-gather of the owned word slices (2^26 ids: 8 MiB in all) completes it."""
        p = graph.NodeBitmap(sess, 0, n).add_scan(persons, "id")
        if not distributed:
            return p
        bits, uniq = p.stats()  # this rank's owned rows (known on the host after the scan)
        p.copy_words(wb, we, nsend.data_ptr(), to_bitmap=False)
        dist.all_gather_into_tensor(nrecv, nsend)
        p.copy_words(0, nw, nrecv.data_ptr(), to_bitmap=True)
        scan_stats[0].fill_(bits)
        scan_stats[1].fill_(0 if uniq else 1)
        dist.all_reduce(scan_stats)  # the gathered bitmap's set bits and any duplicate, in one collective
        total_bits, dups = scan_stats.tolist()  # the step's one host round trip before the partition
        return p.assume(total_bits, dups == 0)

    def exchange_and_finish(p, mark_dst):
        if distributed:  # hop-1 frontier: every rank needs X1/X2 of every middle node; one all-gather
            send.copy_(mid.view(2, nw)[:, wb:we])
            dist.all_gather_into_tensor(recv, send)
            mid.view(2, world, k_own).copy_(recv.view(world, 2, k_own).transpose(0, 1))
        mark_dst(p)
        if distributed:  # owned popcount on the device, summed by the all-reduce: one host read
            graph.words_popcount_device(sess, dstw.data_ptr(), wb, we, cnt_dev.data_ptr())
            dist.all_reduce(cnt_dev)
            return int(cnt_dev.item())
        return graph.words_popcount(sess, dstw.data_ptr(), wb, we)

    own_in = torch.zeros(32 * k_own, dtype=torch.int32, device="cuda")
    in_all = torch.zeros(32 * k_own * world, dtype=torch.int32, device="cuda") if distributed else own_in

    def step_count_shards():
        """count(*) over ranks: each rank partitions its owner(target) relationships and
        writes its owned ids' in-degrees; one all-gather of those slices (2^26 ids: 256 MiB in all)
        gives every rank inA of every source; each rank sums inA(source) over its relationships into
        a device int64 and one all-reduce adds the ranks' parts."""
        p = node_scan()
        sh = graph.CountShard(sess, [rels], p, p, p, 32 * wb, min(32 * we, n), own_in.data_ptr())
        dist.all_gather_into_tensor(in_all, own_in)
        sh.finish(in_all.data_ptr(), cnt_dev.data_ptr())
        dist.all_reduce(cnt_dev)
        r = int(cnt_dev.item())
        sh.close()
        return r

    def step_cold():
        p = node_scan()  # node scan of :Person (a, b, c)
        rp = graph.RelPartition.build_mark_mid(sess, [rels], p, p, mid.data_ptr(), scratch.data_ptr())
        r = exchange_and_finish(p, lambda q: rp.mark_dst(q, q, mid.data_ptr(), dstw.data_ptr()))
        rp.release()
        return r

    def step_warm():
        if "rp" not in cached:
            cached["rp"] = graph.RelPartition(sess, [rels], 0, n)
        rp = cached["rp"]
        p = node_scan()
        rp.mark_mid(p, p, mid.data_ptr(), scratch.data_ptr())
        return exchange_and_finish(p, lambda q: rp.mark_dst(q, q, mid.data_ptr(), dstw.data_ptr()))

    def step_stream():
        p = node_scan()
        graph.two_hop_mark_mid(sess, [rels], p, p, mid.data_ptr(), scratch.data_ptr())
        return exchange_and_finish(p, lambda q: graph.two_hop_mark_dst(sess, [rels], q, q, mid.data_ptr(),
                                                                          dstw.data_ptr()))

    # ---- the drop-in route: the relational plan of the query, as the planner emits it ----------------
    # Planner(sg).run issues the Table[T] calls RelationalPlanner would (node / relationship scans, two
    # Expand joins per hop, the r1 <> r2 filter, the count(DISTINCT c) aggregate); libcapsmi's
    # recogniser maps the lazy plan onto the same fused kernels at materialisation.  The timed region is
    # SURVEY.md §8d's: from handing the plan to the backend (the lazy table's first action: recognition,
    # routing, every kernel) to the answer on the host.  Each timed step executes its own plan, built
    # before the timed region (a lazy plan holds no rows and runs nothing until that action); the
    # planning itself is timed apart (query.plan_ms).  --plan-in-step times planning inside each step.
    from capsmi.planner import EntityTable, Planner, ScanGraph
    person_et = EntityTable("node", frozenset({"Person"}), {}, persons, id_col="id")

    def scan_graph(r):
        return ScanGraph(sess, [person_et], [EntityTable("rel", frozenset({"FRIEND_OF"}), {}, r, id_col="id",
                                                         src_col="source", dst_col="target")])

    sg_cold = scan_graph(rels)
    # Cache analogue: a second handle on the same columns, marked cache() so the route keeps its layout
    rels_cached = rels.select("id", "source", "target").as_rel_table("id", "source", "target").cache()
    if distributed:
        distribute(sess, 0, n, [], [rels_cached], nodes_owned=True, rels_by=args.rels_by)
    sg_warm = scan_graph(rels_cached)

    def run_planner(sg):
        t, outs = Planner(sg).run(C3_QUERY)
        return int(t.column(outs[0][2]).values[0])

    def run_count(atomic=False):  # count(*) of the same match through the route
        # (the session's configuration: a caller's CAPSMI_COUNT in the environment stays in force otherwise)
        with sess.configured(**({"CAPSMI_COUNT": "atomic"} if atomic else {})):
            t, outs = Planner(sg_cold).run(C3_COUNT_QUERY)
            return int(t.column(outs[0][2]).values[0])

    def run_und(q):  # the undirected queries through the route (fused_undirected)
        t, outs = Planner(sg_cold).run(q)
        return int(t.column(outs[0][2]).values[0])

    steps = {"und_count": lambda: run_und(C3U_COUNT_QUERY), "und_distinct": lambda: run_und(C3U_QUERY),
             "cold": lambda: run_planner(sg_cold), "warm": lambda: run_planner(sg_warm),
             "direct": step_cold, "direct_warm": step_warm, "stream": step_stream,
             "count": run_count, "count_atomic": lambda: run_count(True)}
    # the planned modes: (build the lazy plan, execute it)
    plans_of = {"cold": lambda: Planner(sg_cold).run(C3_QUERY), "warm": lambda: Planner(sg_warm).run(C3_QUERY),
                "count": lambda: Planner(sg_cold).run(C3_COUNT_QUERY),
                "und_count": lambda: Planner(sg_cold).run(C3U_COUNT_QUERY),
                "und_distinct": lambda: Planner(sg_cold).run(C3U_QUERY)}

    def execute(plan):
        t, outs = plan
        return int(t.column(outs[0][2]).values[0])
    plan_ms = {}
    if shards != 1:  # --shard-of diagnostic: one shard's kernels, no exchange
        steps["cold"], steps["warm"], steps["count"] = step_cold, step_warm, step_count_shards

    kbytes = {}  # per-launch algorithmic bytes the library declares for a timer (count(*) walks)

    def kernel_times():
        out = {}
        for k in KERNELS:
            cnt, ms, b = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
            _lib.call("capsmi_session_kernel_time", sess.handle, k.encode(), ctypes.byref(cnt), ctypes.byref(ms))
            _lib.call("capsmi_session_kernel_bytes", sess.handle, k.encode(), ctypes.byref(b))
            out[k] = (cnt.value, ms.value)
            if cnt.value and b.value:
                kbytes[k] = b.value / cnt.value
        return out

    results = {}
    medians = {}  # this rank's median step (ms): SURVEY.md 8d asks for the median beside the mean
    gate = None
    if distributed:
        from capsmi.dist import serial_gate
        gate = serial_gate()  # CAPSMI_SERIAL_LOCK: the serialised rehearsal of N ranks on one GPU
    busy = {}
    for mode in modes:
        step = steps[mode]
        if gate is not None:
            def step(inner=steps[mode]):
                gate.acquire()
                try:
                    return inner()
                finally:
                    gate.release()
        for _ in range(args.warmup):
            res = step()
        # every timer over a few untimed steps: the per-kernel breakdown and the dominant kernel.  The timed
        # steps then bracket only the dominant launch (its events are the roofline's live measurement): each
        # timer's two event records leave the device idle for a few microseconds
        _lib.call("capsmi_session_set_profiling", sess.handle, 1)
        kernel_times()  # reset
        for _ in range(PROFILED_STEPS):
            step()
        kt_all = {k: v for k, v in kernel_times().items() if v[0] > 0}
        dom_name = max(kt_all, key=lambda k: kt_all[k][1]) if kt_all else None
        _lib.call("capsmi_session_set_profiling_names", sess.handle, dom_name.encode() if dom_name else None)
        pre = mode in plans_of and shards == 1 and not args.plan_in_step
        if pre:  # this mode's plans, one per timed step, built before the timed region (timed apart)
            tp = time.perf_counter()
            queue = [plans_of[mode]() for _ in range(args.steps)]
            plan_ms[mode] = (time.perf_counter() - tp) / args.steps * 1e3
            step = lambda: execute(queue.pop(0))  # noqa: E731 (each plan executed once, then dropped)
            if gate is not None:
                def step(inner=step):
                    gate.acquire()
                    try:
                        return inner()
                    finally:
                        gate.release()
        if gate is not None:
            gate.busy = 0.0
        kernel_times()  # reset
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        marks = []  # each step ends with its answer on the host (a device sync): per-step times for the median
        for _ in range(args.steps):
            res = step()
            marks.append(time.perf_counter())
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        per_step = [b - a for a, b in zip([t0] + marks[:-1], marks)]
        medians[mode] = sorted(per_step)[len(per_step) // 2] * 1e3 if per_step else None
        kt = dict(kt_all)
        kt.update({k: v for k, v in kernel_times().items() if v[0] > 0})  # the dominant launch, timed steps
        _lib.call("capsmi_session_set_profiling", sess.handle, 0)
        _lib.call("capsmi_session_set_profiling_names", sess.handle, None)
        if distributed:
            tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = float(tt.item())
        if gate is not None:
            bt = torch.zeros(world, dtype=torch.float64, device="cuda")
            bt[rank] = gate.busy / args.steps * 1e3
            dist.all_reduce(bt)
            busy[mode] = [round(x, 3) for x in bt.tolist()]
        results[mode] = (elapsed / args.steps, res, kt, dom_name)
    if "rp" in cached:
        cached["rp"].release()
    routed = sess.route_count("two_hop")

    # ---- untimed checks: matched rows (closed form) and every mode's answer vs the committed fixture -
    matched = check = None
    fx = fixture(f"c3_s{scale}") if ef == 16 else None
    if rank == 0:
        full = graph.rmat_rels(sess, scale, 0, m_total, graph.RMAT_GRAPH500, 42) if distributed else rels
        all_persons = graph.rmat_nodes(sess, scale, graph.NODES_ALL) if distributed else persons
        p = graph.NodeBitmap(sess, 0, n).add_scan(all_persons, "id")
        matched = graph.two_hop_count(sess, [full], p, p, p)
        # the undirected modes' bindings: the undirected count(*) (its own run's answer when und_count ran, else
        # the oracle fixture), so their value is undirected bindings / s, not the directed match's
        fxu0 = fixture(f"c3u_s{scale}") or {}
        und_matched = results["und_count"][1] if "und_count" in results else fxu0.get("count_star")
        answers = {m: r[1] for m, r in results.items()}
        if shards != 1:
            check = f"not applicable (--shard-of {shards}: rank 0's shard alone)"
        elif fx is None:
            check = "no fixture for this scale"
        else:
            fxu = fixture(f"c3u_s{scale}") or {}
            want = {m: (fxu.get("count_star") if m == "und_count" else fxu.get("count_distinct_c") if m == "und_distinct"
                        else fx["count_star"] if m.startswith("count") else fx["count_distinct_c"]) for m in answers}
            bad = {m: v for m, v in answers.items() if v != want[m]}
            if matched != fx["count_star"]:
                bad["count_star"] = matched
            check = "ok" if not bad else f"MISMATCH {bad} vs fixture {fx['count_distinct_c']} / {fx['count_star']}"
        del full

    if rank == 0:
        head = modes[0]
        sec, res, kt, dom = results[head]

        def rows_of(mode):  # matched rows of a mode's query
            return und_matched if mode.startswith("und_") else matched
        # per-kernel algorithmic bytes (this rank's rels): what each kernel must touch by its function
        alg = {"part_scatter1": m_local * 24,        # read 2 x int64, write packed uint2
               "part_scatter2_hop1": m_local * 16 + n // 8,  # read + write uint2, write M
               "part_scatter2": m_local * 16,        # read + write uint2
               "hop1": m_local * 8 + n // 8,         # read uint2 pairs, write M
               "hop2": m_local * 8 + n // 8 * 3,     # read uint2 pairs + X1 + X2, write C
               "mid_combine": n // 8 * 5, "bitmap_add": n * 8,
               "count_part": m_local * 20,  # read 2 x int64, write two 2-byte records
               "und_count_part": m_local * 24,  # read 2 x int64, write up to four 2-byte records
               "und_distinct": m_local * 32 + n * 4,  # two streams of 2 x int64; the per-id state word
               "degrees": m_local * 16 + n * 8}                  # read int64 pairs, inA + outC
        alg.update(kbytes)
        timed = {k: (c, ms) for k, (c, ms) in kt.items() if c > 0}
        avg_ms = timed[dom][1] / timed[dom][0]  # the dominant launch over the timed steps
        achieved = alg[dom] / (avg_ms * 1e-3) / 1e9
        # committed PMC summaries are 1-GPU profiles of the whole table: they say nothing about a shard
        traffic = pmc_traffic(KERNEL_SYMBOL[dom], "c3") if world == 1 and shards == 1 else None
        query_alg = 2 * 24 * m_total + 3 * 8 * n  # SURVEY.md §8d C3 B_alg (whole query, all ranks)
        line = {
            "metric": METRIC,
            "value": rows_of(head) / sec if rows_of(head) is not None else None,
            "unit": "matched rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": sec * 1e3,
            "ms_per_step_median_rank0": medians.get(head),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic R-MAT (on-device counter-based generator, oracle/rmat.c definition)",
            "config": {"workload": MODE_QUERY.get(head, (C3_WORKLOAD,))[0],
                       "mode": head, "scale": scale, "nodes": n, "relationships": m_total,
                       "rmat": [0.57, 0.19, 0.19, 0.05], "seed": 42,
                       "parallelism": (PAR_SOURCE if args.rels_by == "source" else PAR_TARGET).format(w=world)
                       if world > 1 else "single GPU (no exchange)",
                       "route": ("Planner(sg).run(query): lazy Table[T] plan -> fused two-hop kernels "
                                 f"({routed} plans routed on this rank)") if shards == 1 and
                       head in ("cold", "warm", "count") else "explicit phased kernel calls"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": KERNEL_SYMBOL[dom],
                         "kernel_ms": avg_ms, "alg_bytes_per_launch": alg[dom]},
            "query": {MODE_QUERY.get(head, (None, "count_distinct_c"))[1]: res, "matched_rows": rows_of(head),
                      "check_vs_fixture": check,  # tests/golden/rmat_full.json (oracle closed form)
                      "alg_bytes_query": query_alg,
                      "query_alg_GBs": query_alg / sec / 1e9,
                      "query_frac_of_peak": query_alg / sec / 1e9 / (HBM_PEAK_GBS * world),
                      "kernel_ms": {k: v[1] / v[0] for k, v in timed.items()},
                      "kernel_ms_from": (f"{dom}: the timed steps (its timer alone); the others: "
                                         f"{PROFILED_STEPS} untimed steps with every timer"),
                      "rels_local_rank0": m_local, "ingest_s": ingest_s},
        }
        if head in plan_ms:  # planning outside the timed region, reported beside it
            line["query"]["plan_ms"] = plan_ms[head]
            line["query"]["ms_per_step_with_planning"] = sec * 1e3 + plan_ms[head]
            line["query"]["timed_region"] = ("SURVEY.md 8d: from handing each step's lazy plan to the backend to "
                                             "the answer on the host; planning timed apart (plan_ms)")
        if distributed:
            line["query"]["rels_per_rank"] = rels_per_rank
            line["query"]["rels_max_over_mean"] = max(rels_per_rank) / (sum(rels_per_rank) / world)
        if shards != 1:
            line["config"]["diagnostic"] = f"rank 0's shard of {shards} on one GPU, no exchange (not the metric)"
        # warm (layout cached): the query reads the cached layout -- 5-B packed pairs --
        # once per hop, plus the hop bitmaps' slices (the node scans of exact-id tables set a range and
        # read nothing): its PHYSICAL bytes, not SURVEY's B_alg (which is the cold plan's scans)
        warm_phys = 2 * 5 * m_total + 3 * n // 8
        for mode in modes[1:]:
            s2, r2, kt2, _ = results[mode]
            entry = {"ms_per_step": s2 * 1e3, "ms_per_step_median_rank0": medians.get(mode),
                     "value": rows_of(mode) / s2 if rows_of(mode) is not None else None,
                     MODE_QUERY.get(mode, (None, "count_distinct_c"))[1]: r2,
                     "kernel_ms": {k: v[1] / v[0] for k, v in kt2.items() if v[0] > 0}}
            if mode.startswith("und_"):
                entry["workload"] = MODE_QUERY[mode][0]
                entry["matched_rows"] = und_matched
            if mode in ("warm", "direct_warm"):
                entry.update({"phys_bytes_query": warm_phys,
                              "phys_basis": "cached 5-B packed layout read once per hop + hop bitmaps",
                              "phys_frac_of_peak": warm_phys / s2 / 1e9 / (HBM_PEAK_GBS * world)})
            elif mode.startswith("und_"):
                # SURVEY.md 8d's B_alg over the undirected plan: 2^2 branches (outgoing / incoming per hop), each
                # 2 relationship scans (24 B/rel: the ids feed r1 <> r2) and 3 node scans
                und_alg = 8 * 24 * m_total + 12 * 8 * n
                entry.update({"alg_bytes_query": und_alg, "alg_basis": "SURVEY 8d B_alg of the 4-branch undirected plan",
                              "query_frac_of_peak": und_alg / s2 / 1e9 / (HBM_PEAK_GBS * world)})
            else:
                entry.update({"alg_bytes_query": query_alg,
                              "query_frac_of_peak": query_alg / s2 / 1e9 / (HBM_PEAK_GBS * world)})
            line["query"][mode] = entry
        if busy:
            line["rehearsal"] = {"kind": f"{world} gloo ranks sharing one GPU, GPU work serialised by a lock "
                                         f"(CAPSMI_SERIAL_LOCK): a rank's busy ms per step is its share on a device of "
                                         f"its own, collectives excluded; ms_per_step is NOT a multi-GPU time",
                                 "busy_ms_per_rank": busy}
        line["cpu_baseline"] = cpu_baseline(scale, ef) if (not args.no_cpu_baseline and world == 1) else None
        print(json.dumps(line), flush=True)
        if check is not None and check.startswith("MISMATCH"):
            sys.exit(f"bench: result differs from the oracle fixture: {check}")
    sess.close()
    if distributed:
        dist.destroy_process_group()



# ---- single-GPU lines for the other SURVEY.md 8d configs ------------------------------------------
SINGLE = {
    # workload: (scale, edge factor, rmat probs, description, oracle sample scale)
    "c2": (24, 16, (57, 19, 19), "C2: MATCH (a:Person)-[r:FRIEND_OF]->(b:Person) WHERE a.age >= 18 AND a.age < 65 "
                                 "RETURN id(a), id(b)", 22),
    "c4": (24, 16, (57, 19, 19), "C4: MATCH (a)-[r1:FRIEND_OF]->(b)-[r2:FRIEND_OF]->(c)-[r3:FRIEND_OF]->(a) "
                                 "RETURN count(*)", 14),
    "c5": (20, 32, (45, 15, 15), "C5: MATCH (a:Person)-[:KNOWS*1..3]->(b:Person) RETURN id(a), count(*)", 16),
}


# timer name -> kernel symbol (rocprofv3 / PMC summary name) where they differ
SINGLE_SYMBOL = {"direct_join_probe": "k_direct_probe", "radix_join_count": "k_join", "radix_join_write": "k_join",
                 "expand_filter": "k_expand_pairs", "part_scatter1": "k_scatter_l", "varlen_deg": "k_vl_deg",
                 "varlen_w": "k_vl_w", "varlen_t": "k_vl_t", "varlen_rev": "k_vl_bset", "varlen_recip": "k_vl_recip", "varlen_cand": "k_vl_cins", "triangles": TRI_SYMBOL}


def owned_rmat_rels(sess, graph, scale, m, probs, col, n, chunks=8):
    """This rank's shard of the R-MAT relationships (the rows whose `col` id it owns), generated in `chunks`
    edge ranges so that no rank ever holds the whole table (ingest, untimed)."""
    out = None
    step = -(-m // chunks)
    for b in range(0, m, step):
        part = graph.rmat_rels(sess, scale, b, min(m, b + step), probs, 42).owned_rows(col, 0, n)
        out = part if out is None else out.unionAll(part)
        out.size  # materialise: the chunk's full table is released
    return out.as_rel_table("id", "source", "target")


def route_counts(sess):
    names = ("expand", "expand_count", "two_hop", "triangle", "var_length", "miss")
    return ", ".join(f"{k} {sess.route_count(k)}" for k in names if sess.route_count(k))


def run_single(args):
    """C2 / C4 / C5 on one GPU: cold = the whole query from resident entity tables.
    value = matched rows / s; matched rows = the query's bindings (C2: result rows; C4: count(*);
    C5: sum of the per-a counts).  Roofline: the dominant timed kernel's algorithmic bytes."""
    import numpy as np
    import torch
    from capsmi import Session, _lib, graph
    from capsmi.expr import Ands, BinOp, Col, Lit, Ors

    wl = args.workload
    scale, ef, probs, desc, cpu_scale = SINGLE[wl]
    up = args.c5_upper if wl == "c5" else 3
    if up != 3:
        desc = desc.replace("*1..3", f"*1..{up}")
    if args.scale != 26:  # --scale given explicitly
        scale = args.scale
    cpu_scale = args.cpu_scale or cpu_scale
    n, m = 1 << scale, ef << scale
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dw = world > 1 or (args.dist1 and wl in ("c4", "c5"))  # --dist1: the distributed route at world size 1
    if dw and up != 3:
        sys.exit("bench: --c5-upper 4 is the one-GPU four-hop count (the sharded form stops at 3)")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if dw:  # C2: rels by owner(source), local expand; C4: replicated oriented graph, vertex shares;
        # C5: owner(source) shards
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        init_dist(dist, local)
    sess = Session(local)
    sess.set_stream(torch.cuda.current_stream().cuda_stream)
    # N > 1, C4 / C5: the drop-in route over a distributed graph -- every rank runs
    # Planner(sg).run over its shard; libcapsmi's distributed routes exchange through RCCL (C4: the pairs
    # to their lower end's owner and the oriented ranges, all-gathered; C5: owner(source) shards whose
    # in-relationships were exchanged at registration, od / Y all-reduced).  Ingest is untimed.
    dist_route = dw and wl in ("c4", "c5") and not args.direct_multi
    shard_c5 = wl == "c5" and world > 1 and not dist_route
    ingest_gate = None
    if dist_route:
        from capsmi.dist import distribute, join_ranks, serial_gate
        join_ranks(sess)
        ingest_gate = serial_gate()  # a serialised rehearsal also serialises the ranks' ingest peaks
        if ingest_gate:
            ingest_gate.acquire()
        by = "source" if wl == "c5" else "target"
        rels = owned_rmat_rels(sess, graph, scale, m, probs, by, n)
    elif shard_c5:  # ingest (untimed): out-relationships of owned sources + in-relationships from other ranks
        wb, we = graph.owner_words(n, rank, world)
        own_lo, own_hi = min(32 * wb, n), min(32 * we, n)
        rels = graph.rmat_rels(sess, scale, 0, m, probs, 42, part_col=graph.PART_SOURCE, part=rank, nparts=world)
        into = graph.rmat_rels(sess, scale, 0, m, probs, 42, part_col=graph.PART_TARGET, part=rank, nparts=world)
        rels_in = into.filter(Ors((BinOp("<", Col("source"), Lit(own_lo)), BinOp(">=", Col("source"), Lit(own_hi)))))
        del into
        od_buf = torch.zeros(n, dtype=torch.int64, device="cuda")
        y_buf = torch.zeros(n, dtype=torch.int64, device="cuda")
    elif wl == "c2" and world > 1:  # each rank expands its own sources; output stays partitioned
        rels = graph.rmat_rels(sess, scale, 0, m, probs, 42, part_col=graph.PART_SOURCE, part=rank, nparts=world)
    else:
        rels = graph.rmat_rels(sess, scale, 0, m, probs, 42)
    kind = graph.NODES_PERSON if wl == "c2" else graph.NODES_ALL
    nodes = graph.rmat_nodes(sess, scale, kind, 42)
    if dist_route:
        nodes = nodes.owned_rows("id", 0, n).as_node_table("id")
        distribute(sess, 0, n, [nodes], [rels], nodes_owned=True, rels_by=by)
    sess.sync()
    if ingest_gate:
        ingest_gate.release()
        ingest_gate.busy = 0.0
    pred = Ands((BinOp(">=", Col("age"), Lit(18)), BinOp("<", Col("age"), Lit(65))))
    cache = {}
    route = args.c2_route if wl == "c2" and world == 1 else ("planner" if dist_route else "direct")
    if route != "direct":
        from capsmi.planner import EntityTable, Planner, ScanGraph
        props = {"age": 0} if wl == "c2" else {}
        sg = ScanGraph(sess, [EntityTable("node", frozenset({"Person"}), props, nodes, id_col="id")],
                       [EntityTable("rel", frozenset({"KNOWS" if wl == "c5" else "FRIEND_OF"}), {}, rels, id_col="id",
                                    src_col="source", dst_col="target")])
        sess.set_fused(route == "planner")

    def plan_of():  # the routed query's lazy plan (holds no rows, runs nothing until its first action)
        c5q = C5_QUERY if up == 3 else {**C5_QUERY, "clauses": [{"match": f"(a:Person)-[:KNOWS*1..{up}]->(b:Person)"}]}
        return Planner(sg).run({"c4": C4_QUERY, "c5": c5q}.get(wl, C2_QUERY))

    def run_plan(plan):  # from handing the plan to the backend to the answer on the host
        t, outs = plan
        if wl == "c4":  # the routed query on every rank; the count is whole on each
            return int(t.column(outs[0][2]).values[0]), None
        if wl == "c5":  # rows of this rank's owned start nodes (partitioned)
            t.size  # materialise inside the timed region
            cache["c5_cols"] = [outs[0][2], outs[1][2]]
            return None, t
        cache["outs"] = [outs[0][2], outs[1][2]]  # C2 through the planner mirror
        return t.size, t

    def step():
        if route != "direct":
            return run_plan(plan_of())
        if wl == "c2":
            a_ok = graph.NodeBitmap(sess, 0, n).add_scan(nodes, "id", pred)
            b_ok = graph.NodeBitmap(sess, 0, n).add_scan(nodes, "id")
            out = graph.expand_filter(sess, rels, a_ok, b_ok, ["source", "target"], ["a", "b"])
            if world > 1:
                t = torch.tensor([out.size], dtype=torch.int64, device="cuda")
                dist.all_reduce(t)
                return int(t.item()), out
            return out.size, out
        ok = graph.NodeBitmap(sess, 0, n).add_scan(nodes, "id")
        if wl == "c4":  # = graph.triangle_count: build the trigraph, count, release
            g = graph.TriGraph(sess, [rels], ok)
            cache["oriented_edges"] = g.stats()[1]
            if world == 1:
                c = g.count()
                g.release()
                return c, None
            t = torch.tensor([g.count(rank, world)], dtype=torch.int64, device="cuda")
            g.release()
            dist.all_reduce(t)
            return int(t.item()), None
        if shard_c5:  # begin -> all-reduce od -> mid -> all-reduce Y -> finish (rows of owned a)
            sh = graph.VarlenShard(sess, [rels], [rels_in], ok, ok, 1, 3, own_lo, own_hi, od_buf.data_ptr())
            dist.all_reduce(od_buf)
            sh.mid(y_buf.data_ptr())
            dist.all_reduce(y_buf)
            out = sh.finish()
            sh.release()
            return None, out
        out = graph.var_length_count(sess, [rels], ok, ok, 1, up)
        return None, out

    kernels = ("direct_join_probe", "radix_join_count", "radix_join_write", "bitmap_add", "expand_filter", "tri_pack",
               "tri_deg", "tri_sort_und", "tri_order", "tri_sort_or", "tri_post", "tri_work", "triangles", "part_scatter1",
               "varlen_part", "varlen_deg", "varlen_w", "varlen_rev",
               "varlen_cand", "varlen_recip", "varlen_t", "varlen_4", "vls_rev_part", "vls_rev_bloom", "vls_rev_cand",
               "vls_rev_recip")
    gate = None
    if world > 1:
        from capsmi.dist import serial_gate
        gate = serial_gate()  # CAPSMI_SERIAL_LOCK: the serialised rehearsal of N ranks on one GPU
    inner_step = step

    def step():
        if gate is None:
            return inner_step()
        gate.acquire()
        try:
            return inner_step()
        finally:
            gate.release()

    for _ in range(args.warmup):
        step()

    def read_timers():
        t, b_ = {}, {}
        for k in kernels:
            c, ms, b = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
            _lib.call("capsmi_session_kernel_time", sess.handle, k.encode(), ctypes.byref(c), ctypes.byref(ms))
            _lib.call("capsmi_session_kernel_bytes", sess.handle, k.encode(), ctypes.byref(b))
            if c.value:
                t[k] = (c.value, ms.value)
                if b.value:
                    b_[k] = b.value / c.value  # per launch
        return t, b_
    # every timer over a few untimed steps: the per-kernel breakdown and the dominant kernel; the timed steps
    # then bracket only the dominant launch (each timer's two event records leave the device idle a few us)
    _lib.call("capsmi_session_set_profiling", sess.handle, 1)
    read_timers()  # reset
    for _ in range(PROFILED_STEPS):
        step()
    kt, kbytes = read_timers()
    ranked = [k for k in kt if k != "varlen_4"]  # (the four-hop phase: several kernels, no single roofline)
    dom = max(ranked, key=lambda k: kt[k][1]) if ranked else None
    _lib.call("capsmi_session_set_profiling_names", sess.handle, dom.encode() if dom else None)
    plan_ms = None
    if route != "direct" and not args.plan_in_step:  # as the C3 modes: each timed step executes its own
        tp = time.perf_counter()                     # plan, built before the timed region (timed apart)
        queue = [plan_of() for _ in range(args.steps)]
        plan_ms = (time.perf_counter() - tp) / args.steps * 1e3
        inner_step = lambda: run_plan(queue.pop(0))  # noqa: E731 (each plan executed once, then dropped)
    if gate is not None:
        gate.busy = 0.0
    read_timers()  # reset
    if dw:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, out = step()
    torch.cuda.synchronize()
    if dw:
        dist.barrier()
    sec = (time.perf_counter() - t0) / args.steps
    if dw:
        tt = torch.tensor([sec], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        sec = float(tt.item())
    kt_dom, kb_dom = read_timers()  # the dominant launch over the timed steps
    kt.update(kt_dom)
    kbytes.update(kb_dom)
    steps_of = {k: (args.steps if k in kt_dom else PROFILED_STEPS) for k in kt}
    _lib.call("capsmi_session_set_profiling", sess.handle, 0)
    _lib.call("capsmi_session_set_profiling_names", sess.handle, None)
    check = None
    if wl == "c5":
        cnt_col = cache.get("c5_cols", ["id", "count"])[1]
        res = int(out.column(cnt_col).values.sum())  # untimed export
        if shard_c5 or dist_route:  # the ranks' rows are disjoint: total = sum; rank 0 checks the unsharded answer
            t = torch.tensor([res], dtype=torch.int64, device="cuda")
            dist.all_reduce(t)
            res = int(t.item())
            if rank == 0:
                full = graph.rmat_rels(sess, scale, 0, m, probs, 42)
                ok = graph.NodeBitmap(sess, 0, n).add_scan(graph.rmat_nodes(sess, scale, graph.NODES_ALL, 42), "id")
                ref = int(graph.var_length_count(sess, [full], ok, ok, 1, 3).column("count").values.sum())
                check = "ok" if ref == res else f"MISMATCH {res} vs unsharded {ref}"
                del full
    if wl == "c2" and world > 1 and rank == 0:  # the whole table on one device gives the same row count
        full = graph.rmat_rels(sess, scale, 0, m, probs, 42)
        a_ok = graph.NodeBitmap(sess, 0, n).add_scan(nodes, "id", pred)
        b_ok = graph.NodeBitmap(sess, 0, n).add_scan(nodes, "id")
        ref = graph.expand_filter(sess, full, a_ok, b_ok, ["source", "target"], ["a", "b"]).size
        check = "ok" if ref == res else f"MISMATCH {res} vs unsharded {ref}"
        del full
    # every line checks its answer against the committed oracle fixture (tests/golden/rmat_full.json)
    fx = fixture(f"{wl}_s{scale}" if up == 3 else f"{wl}u{up}_s{scale}")  # c5u4_*: the *1..4 answers
    if fx is None or (world > 1 and wl == "c2"):
        fcheck = "no fixture for this scale" if fx is None else "rows only (output stays partitioned)"
        if fx is not None and wl == "c2":
            fcheck = "ok" if res == fx["rows"] else f"MISMATCH rows {res} vs fixture {fx['rows']}"
    elif wl == "c2":
        fp = list(out.fingerprint(cache.get("outs", ["a", "b"])))
        want = [fx["fingerprint"][0], int(fx["fingerprint"][1]), int(fx["fingerprint"][2])]
        fcheck = "ok" if fp == want else f"MISMATCH fingerprint {fp} vs fixture {want}"
    elif wl == "c4":
        fcheck = "ok" if res == fx["count_star"] else f"MISMATCH {res} vs fixture {fx['count_star']}"
    else:
        fcheck = "ok" if res == fx["sum_count"] else f"MISMATCH sum {res} vs fixture {fx['sum_count']}"
        if world == 1 and fcheck == "ok":
            fp = list(out.fingerprint(cache.get("c5_cols", ["id", "count"])))
            want = [fx["fingerprint"][0], int(fx["fingerprint"][1]), int(fx["fingerprint"][2])]
            fcheck = "ok" if fp == want else f"MISMATCH fingerprint {fp} vs fixture {want}"
    matched = res
    m_kern = rels.size if world > 1 and wl in ("c2", "c5") else m  # relationships behind one launch here
    # algorithmic bytes per launch of the kernels whose traffic is a plain function of the input
    alg = {"bitmap_add": n * 8, "expand_filter": m_kern * 16 + (2 * out.size * 8 if wl == "c2" else 0),
           "tri_pack": m * 24, "part_scatter1": m_kern * 24, "varlen_deg": m_kern * 8, "varlen_w": m_kern * 8,
           "varlen_t": m_kern * 8, "varlen_rev": m * 24 + m * 8,  # target partition + filter walk
           # both triangle kernels together: the oriented adjacency read once (8-B offsets, 4-B
           # targets, 8-B multiplicity payload per oriented edge)
           "triangles": n * 8 + 12 * cache.get("oriented_edges", 0)}
    alg.update(kbytes)  # kernels that declare their bytes (generic joins)
    avg_ms = kt[dom][1] / kt[dom][0] if kt else None
    b_alg = {"c2": 16 * m + int(0.75 * n) * 24 + 16 * (res or 0), "c4": 3 * 24 * m + 3 * 8 * n,
             "c5": 3 * 24 * m + 2 * 8 * n + 16 * n}[wl]  # SURVEY.md 8d worked values
    line = {
        "metric": f"matched rows/sec ({wl.upper()})", "value": matched / sec, "unit": "matched rows/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": sec * 1e3, "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic R-MAT (on-device counter-based generator, oracle/rmat.c definition)",
        "config": {"workload": desc, "scale": scale, "nodes": n, "relationships": m,
                   "rmat": [p / 100 for p in probs] + [round(1 - sum(probs) / 100, 2)], "seed": 42},
        "roofline": ({"bound": "hbm", "achieved": alg[dom] / (avg_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": alg[dom] / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                      "traffic": pmc_traffic(SINGLE_SYMBOL.get(dom, "k_" + dom), wl),
                      "kernel": SINGLE_SYMBOL.get(dom, "k_" + dom), "kernel_ms": avg_ms,
                      "alg_bytes_per_launch": alg[dom]} if dom in alg else None),
        "query": {"result": res, "matched_rows": matched, "alg_bytes_query": b_alg,
                  "query_frac_of_peak": b_alg / sec / 1e9 / HBM_PEAK_GBS,
                  "kernel_ms": {k: v[1] / v[0] for k, v in kt.items()},
                  "kernel_ms_from": (f"{dom}: the timed steps (its timer alone); the others: {PROFILED_STEPS} "
                                     "untimed steps with every timer")},
    }
    if world > 1:  # every rank's timed phases (ms per step): the balance of the shares
        kr = torch.zeros(world, len(kernels), dtype=torch.float64, device="cuda")
        for i, k in enumerate(kernels):
            if k in kt:
                kr[rank, i] = kt[k][1] / steps_of[k]
        dist.all_reduce(kr)
        line["query"]["kernel_ms_per_rank"] = {k: [round(x, 3) for x in kr[:, i].tolist()]
                                               for i, k in enumerate(kernels) if kr[:, i].sum() > 0}
    if gate is not None:  # per-rank busy time of the serialised rehearsal (collectives excluded)
        bt = torch.zeros(world, dtype=torch.float64, device="cuda")
        bt[rank] = gate.busy / args.steps * 1e3
        dist.all_reduce(bt)
        line["rehearsal"] = {"kind": f"{world} gloo ranks sharing one GPU, GPU work serialised by a lock "
                                     f"(CAPSMI_SERIAL_LOCK): each rank's busy ms per step is its share on a device of "
                                     f"its own, collectives excluded; ms_per_step above is NOT a multi-GPU time",
                             "busy_ms_per_rank": [round(x, 3) for x in bt.tolist()],
                             "busy_ms_max": round(max(bt.tolist()), 3)}
    if route != "direct":
        if plan_ms is not None:  # planning outside the timed region, reported beside it
            line["query"]["plan_ms"] = plan_ms
            line["query"]["ms_per_step_with_planning"] = sec * 1e3 + plan_ms
        line["query"]["timed_region"] = ("SURVEY.md 8d: from handing each step's lazy plan to the backend to the "
                                         "answer on the host; planning timed apart (plan_ms)" if plan_ms is not None
                                         else "planning inside each step (--plan-in-step)")
    if dist_route:
        line["config"]["route"] = f"Planner(sg).run over a distributed graph ({route_counts(sess)})"
        line["config"]["parallelism"] = (
            f"C4 over {world} GPU(s): relationships by owner(target); sampled degrees all-reduced, every relationship "
            f"packed into its oriented key and exchanged (all-to-all) to the rank of its source's degree-order range, "
            f"sorted and deduplicated there, the ranges all-gathered into a replicated oriented graph, interleaved "
            f"center shares, one all-reduce" if wl == "c4" else
            f"C5 over {world} GPU(s): owner(source) shards, in-relationships exchanged (all-to-all) at registration; "
            f"od and Y all-reduced between phases; each rank the rows of its owned start nodes")
    elif shard_c5:
        line["config"]["parallelism"] = (f"owner(source) shards over {world} GPU(s); od and Y all-reduced between "
                                         f"phases; in-relationships exchanged at ingest")
    elif wl == "c2" and world > 1:
        line["config"]["parallelism"] = f"relationships by owner(source) over {world} GPU(s); row count all-reduced"
    if wl == "c2":
        line["config"]["route"] = {"direct": "explicit bitmap + expand_filter calls",
                                   "planner": "Planner(sg).run, recognised and routed to the fused expand",
                                   "joins": "Planner(sg).run operator by operator: node scans, two generic "
                                            "radix joins, filter, select (fused routing off)"}[route]
    if wl == "c4" and args.tri_parts > 1 and world == 1:
        ok = graph.NodeBitmap(sess, 0, n).add_scan(nodes, "id")
        g = graph.TriGraph(sess, [rels], ok)
        per, tot = [], 0
        for r in range(args.tri_parts):
            g.count(r, args.tri_parts)  # warm
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            c = g.count(r, args.tri_parts)
            torch.cuda.synchronize()
            per.append(round((time.perf_counter() - t1) * 1e3, 3))
            tot += c  # the pair / self terms come with part 0 only: the parts add up to the count
        g.release()
        line["query"]["tri_parts"] = {"parts": args.tri_parts, "ms_per_part": per, "max_ms": max(per),
                                      "mean_ms": sum(per) / len(per), "max_over_mean": max(per) / (sum(per) / len(per)),
                                      "sum_of_parts_ok": tot == res,
                                      "note": "interleaved center shares of one single-GPU trigraph, each part counted "
                                              "alone (wall time incl. the pair/self terms of part 0)"}
    line["query"]["check_vs_fixture"] = fcheck
    if check is not None or (world > 1 and wl in ("c2", "c5")):
        line["query"]["check_vs_unsharded"] = check
    line["cpu_baseline"] = None if (args.no_cpu_baseline or world > 1) else cpu_baseline_single(
        wl, cpu_scale, ef, probs, scale, up)
    if rank == 0:
        print(json.dumps(line), flush=True)
    sess.close()
    if dw:
        dist.destroy_process_group()
    if fcheck.startswith("MISMATCH"):
        sys.exit(f"bench: result differs from the oracle fixture: {fcheck}")


def cpu_baseline_single(wl, scale, ef, probs, full_scale, up=3):
    """The oracle on the host cores, OpenMP over `cores` threads (CPU restatements, not CAPS-on-Spark:
    no JVM on the box).  First line: the SAME algorithm as the device path (oracle/closed.c / rmat.c)
    -- C2 and C5 on the full workload, C4 (triangle listing, ~20 s at scale 20) on a bounded sample;
    second, labelled line: the join semantics CAPS runs (every binding enumerated) on a small sample.
    Edge generation is ingest and untimed."""
    import numpy as np
    from oracle import cpu
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    same_scale = {"c2": full_scale, "c4": min(full_scale, 20), "c5": full_scale}[wl]
    n = 1 << same_scale
    src, dst = cpu.rmat_edges(same_scale, 0, ef << same_scale, probs, 42)
    t0 = time.perf_counter()
    if wl == "c2":
        person, adult = cpu.c2_masks(n)
        rows = cpu.expand_filter(src, dst, adult, person)[0]
        what = "expand with node-filter bitmaps (oracle/rmat.c orc_expand_filter)"
    elif wl == "c4":
        rows = cpu.triangle_closed_form(n, src, dst, threads=threads)
        what = "degree-oriented triangle listing with multiplicities (oracle/closed.c orc_triangle_closed_form)"
    elif up == 3:
        rows, _ = cpu.var_length_closed_form(n, src, dst, 1, 3, threads=threads)
        what = "closed form with reverse multiplicities (oracle/closed.c orc_var_length_closed_form)"
    else:  # *1..4: lengths 1..3 as above plus the four-hop inclusion-exclusion (scipy sparse + closed.c orc_vl4_t14)
        rows, _ = cpu.var_length_closed_form(n, src, dst, 1, 3, threads=threads)
        rows += cpu.var_length4_closed_form(n, src, dst)[0]
        what = ("closed forms, lengths 1..3 (oracle/closed.c) and 4 (inclusion-exclusion, oracle/cpu.py "
                "var_length4_closed_form; its sparse products single-threaded)")
    dt = time.perf_counter() - t0
    del src, dst
    line = {"value": rows / dt, "unit": "matched rows/s", "cores": threads, "kind": "port",
            "sample": f"CPU restatement, not CAPS: the device algorithm -- {what} -- on R-MAT scale {same_scale} "
                      f"({'the full workload' if same_scale == full_scale else 'a bounded sample'}), edge factor "
                      f"{ef}: {rows} rows, {dt:.2f} s"}
    if wl == "c4" and same_scale != full_scale:
        # the same algorithm on the FULL workload is ~20 min of CPU: carried from the fixture run that made the
        # committed answer (tests/golden/make_rmat_full.py, build container, times recorded in rmat_full.json)
        fx = fixture(f"c4_s{full_scale}")
        if fx and fx.get("cpu_seconds"):
            line["full_size"] = {"value": fx["count_star"] / fx["cpu_seconds"], "unit": "matched rows/s",
                                 "seconds": fx["cpu_seconds"], "rows": fx["count_star"],
                                 "sample": f"the same triangle listing on the full R-MAT scale {full_scale} input, "
                                           f"timed when tests/golden/make_rmat_full.py made the fixture (build "
                                           f"container, OpenMP), not re-run on this host"}
    if wl == "c2":
        return line
    if up == 4:
        scale = min(scale, 11)  # 4-hop enumeration: ~10^10 paths at scale 11, seconds on 8 cores
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, ef << scale, probs, 42)
    t0 = time.perf_counter()
    if wl == "c4":
        rows = cpu.triangle_enumerate(n, src, dst, threads=threads)
        what = "triangle binding enumeration (oracle/rmat.c)"
    else:
        rows, _per_a = cpu.var_length_count(n, src, dst, 1, up, threads=threads)
        what = "edge-distinct path enumeration (oracle/rmat.c)"
    dt = time.perf_counter() - t0
    line["enumeration"] = {"value": rows / dt, "unit": "matched rows/s", "cores": threads,
                           "sample": f"CAPS join semantics: {what} on R-MAT scale {scale}, {rows} rows, {dt:.2f} s"}
    return line


if __name__ == "__main__":
    main()
