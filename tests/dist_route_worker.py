"""One rank of the routed multi-GPU rehearsal (tests/test_gpu_dist_route.py), started by
torch.distributed.run.  Every rank reads the same graph, keeps its shard (relationships by owner(target)
or owner(source), node rows by owner(id): capsmi_owned_rows), registers it (capsmi_graph_distribute) and
runs the queries through the planner mirror -- the same Table[T] calls on every rank, routed by libcapsmi
to the distributed kernels, whose exchanges go through torch.distributed (gloo ranks sharing the GPU, or
RCCL at world size 1 with CAPSMI_DIST_BACKEND=nccl).  Writes one JSON file per rank
(<out>.rank<r>.json).  Test infrastructure: the answers are checked by the test, not here.

Graph: an edge list file (`edges lo hi`), or `rmat:<scale>` (the on-device R-MAT generator, ids [0, 2^s))."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cypher-for-apache-spark_amd")]

C3 = "(a:V)-[:E]->(b:V)-[:E]->(c:V)"
TRI = "(a:V)-[:E]->(b:V)-[:E]->(c:V)-[:E]->(a)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("edges")
    ap.add_argument("lo", type=int)
    ap.add_argument("hi", type=int)
    ap.add_argument("nodes", choices=("owned", "replicated"))
    ap.add_argument("--rels-by", default="target", choices=("target", "source"))
    ap.add_argument("--queries", default="c3,tri")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    queries = set(args.queries.split(","))
    out_path = args.out or args.edges
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    backend = os.environ.get("CAPSMI_DIST_BACKEND", "gloo")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    else:
        dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    from capsmi import Session, _lib, graph
    from capsmi.dist import distribute, join_ranks
    from capsmi.expr import I64
    from capsmi.planner import EntityTable, Planner, ScanGraph, result_rows
    s = Session(0)
    s.set_stream(torch.cuda.current_stream().cuda_stream)
    join_ranks(s)
    s.set_unrouted_limit(4 << 30)  # an unrouted plan that would explode is refused, not run out of memory
    col = "target" if args.rels_by == "target" else "source"
    if args.edges.startswith("rmat:"):
        scale = int(args.edges.split(":")[1])
        rels_all = graph.rmat_rels(s, scale, 0, 16 << scale)
        ends = graph.rmat_nodes(s, scale, graph.NODES_ALL)
    else:
        rels_all = s.read_csv([args.edges], ["source", "target"], [I64, I64], delimiter=" ", row_id_col="id")
        ends = rels_all.select("source").withColumnRenamed("source", "id").unionAll(
            rels_all.select("target").withColumnRenamed("target", "id")).distinct()
    rels = rels_all.owned_rows(col, args.lo, args.hi).as_rel_table("id", "source", "target")
    if args.nodes == "owned":
        ends = ends.owned_rows("id", args.lo, args.hi)
    nodes = ends.as_node_table("id")
    distribute(s, args.lo, args.hi, [nodes], [rels], nodes_owned=args.nodes == "owned", rels_by=args.rels_by)
    sg = ScanGraph(s, [EntityTable("node", frozenset({"V"}), {}, nodes, id_col="id")],
                   [EntityTable("rel", frozenset({"E"}), {}, rels, id_col="id", src_col="source", dst_col="target")])
    out = {"rank": rank, "world": world, "rels_local": rels.size, "nodes_local": nodes.size, "backend": backend}

    def run(items, match=C3):
        t, outs = Planner(sg).run({"clauses": [{"match": match}], "return": {"items": items}})
        return result_rows(t, outs, s.dictionary)

    def refused(fn):
        try:
            fn()
            return "ran"
        except _lib.UnsupportedOperationException as e:
            return "refused: " + str(e)[:120]

    if "c3" in queries:  # either mode: all-gather (end's owner holds the walk) or OR-reduce (start's owner) forms
        out["count_star"] = run([["n", ["count*"]]])[0]["n"]
        out["count_distinct_c"] = run([["n", ["count_distinct", ["id", "c"]]]])[0]["n"]
        out["count_distinct_a"] = run([["n", ["count_distinct", ["id", "a"]]]])[0]["n"]
    if "und" in queries:  # undirected 1 / 2 hops: BY_SOURCE shards + their in-relationships
        if args.rels_by == "source":
            u1 = run([["n", ["count*"]], ["d", ["count_distinct", ["id", "b"]]]], "(a:V)-[:E]-(b:V)")[0]
            u2 = run([["n", ["count*"]], ["dc", ["count_distinct", ["id", "c"]]], ["da", ["count_distinct", ["id", "a"]]]],
                     "(a:V)-[:E]-(b:V)-[:E]-(c:V)")[0]
            out["und1"] = [u1["n"], u1["d"]]
            out["und2"] = [u2["n"], u2["dc"], u2["da"]]
        else:
            out["und"] = refused(lambda: run([["n", ["count*"]]], "(a:V)-[:E]-(b:V)-[:E]-(c:V)"))
    if "grouped" in queries:  # RETURN id(a), count(*) / count(DISTINCT c): the rows of this rank's owned starts
        if args.rels_by == "source":
            t, outs = Planner(sg).run({"clauses": [{"match": C3}],
                                       "return": {"items": [["a", ["id", "a"]], ["dc", ["count_distinct", ["id", "c"]]],
                                                            ["n", ["count*"]]]}})
            rows = result_rows(t, outs, s.dictionary)
            out["grouped_rows"] = [[r["a"], r["dc"], r["n"]] for r in rows]
            out["grouped_partitioned"] = t.partitioned
        else:
            out["grouped"] = refused(lambda: run([["a", ["id", "a"]], ["n", ["count*"]]]))
    if "expand" in queries:
        out["expand_count"] = run([["n", ["count*"]]], "(a:V)-[:E]->(b:V)")[0]["n"]
        # rows of this rank's relationships (partitioned result)
        t, outs = Planner(sg).run({"clauses": [{"match": "(a:V)-[r:E]->(b:V)"}],
                                   "return": {"items": [["a", ["id", "a"]], ["b", ["id", "b"]]]}})
        out["expand_rows_local"] = t.size
        out["expand_partitioned"] = t.partitioned
    if "warm" in queries:  # a cached relationship table keeps its layout: the warm route
        cached = rels.cache()
        sgw = ScanGraph(s, sg.nodes, [EntityTable("rel", frozenset({"E"}), {}, cached, id_col="id", src_col="source",
                                                  dst_col="target")])
        tw, ow = Planner(sgw).run({"clauses": [{"match": C3}],
                                   "return": {"items": [["n", ["count_distinct", ["id", "c"]]]]}})
        out["warm_distinct"] = result_rows(tw, ow, s.dictionary)[0]["n"]
    if "tri" in queries:  # the closing ExpandInto: the distributed trigraph build, work shares, one all-reduce
        out["triangle"] = run([["n", ["count*"]]], TRI)[0]["n"]
    if "varlen" in queries:
        if args.rels_by == "source":  # *1..3 grouped by the start: the rows of this rank's owned starts
            t, outs = Planner(sg).run({"clauses": [{"match": "(a:V)-[:E*1..3]->(b:V)"}],
                                       "return": {"items": [["a", ["id", "a"]], ["n", ["count*"]]]}})
            rows = result_rows(t, outs, s.dictionary)
            out["varlen_rows"] = [[r["a"], r["n"]] for r in rows]
            out["varlen_partitioned"] = t.partitioned
        else:
            out["varlen"] = refused(lambda: run([["a", ["id", "a"]], ["n", ["count*"]]], "(a:V)-[:E*1..3]->(b:V)"))
    out["routes"] = {k: s.route_count(k) for k in ("two_hop", "expand_count", "expand", "triangle", "var_length",
                                                   "undirected", "two_hop_grouped", "miss")}
    with open(f"{out_path}.rank{rank}.json", "w") as f:  # one file per rank: stdout lines interleave
        json.dump(out, f)
    s.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
