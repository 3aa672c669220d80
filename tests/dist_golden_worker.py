"""One rank of the distributed golden-vector rehearsal (tests/test_gpu_dist_golden.py), started by
torch.distributed.run: every golden case's graph (the reference's own test graphs, tests/golden/*.json) is
built on every rank, each rank keeps its shard (node rows by owner(id), relationship rows by owner(target):
capsmi_owned_rows), registers it (capsmi_graph_distribute) and runs the case's query through the planner
mirror -- fused routes where they match, otherwise operator by operator with the Exchanges of the generic
executor (csrc/plan.hip dist_join_inputs; hash-partitioned joins / groupings, gathers for global aggregates
and ordering).  Writes <out>.rank<r>.json: per case the rows, whether they are this rank's partition, or the
error.  Test infrastructure: the answers are checked by the test."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cypher-for-apache-spark_amd"), os.path.join(ROOT, "tests")]


def main():
    out_path = sys.argv[1]
    fused = sys.argv[2] == "fused"
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    dist.init_process_group(os.environ.get("CAPSMI_DIST_BACKEND", "gloo"))
    rank = dist.get_rank()
    from capsmi import Session, _lib
    from capsmi.dist import distribute, join_ranks
    from capsmi.planner import EntityTable, Planner, ScanGraph, result_rows, ID, SRC, DST
    from capsmi.table import StringDictionary
    from golden_util import all_cases, property_graph
    s = Session(0)
    s.set_stream(torch.cuda.current_stream().cuda_stream)
    join_ranks(s)
    s.set_fused(fused)
    res = {}
    for _, case in all_cases():
        s.dictionary = StringDictionary()
        try:
            pg, g = property_graph(case)
            sg = ScanGraph.from_property_graph(s, pg)
            ids = [n["id"] for n in g["nodes"]] + [r["src"] for r in g["rels"]] + [r["dst"] for r in g["rels"]]
            lo, hi = (min(ids), max(ids) + 1) if ids else (0, 1)
            nodes = [EntityTable("node", e.labels, e.props, e.table.owned_rows(ID, lo, hi).as_node_table(ID))
                     for e in sg.nodes]
            rels = [EntityTable("rel", e.labels, e.props,
                                e.table.owned_rows(DST, lo, hi).as_rel_table(ID, SRC, DST)) for e in sg.rels]
            distribute(s, lo, hi, [e.table for e in nodes], [e.table for e in rels], nodes_owned=True, rels_by="target")
            t, outs = Planner(ScanGraph(s, nodes, rels)).run(case["query"])
            res[case["name"]] = {"rows": result_rows(t, outs, s.dictionary), "partitioned": t.partitioned}
        except (_lib.UnsupportedOperationException, _lib.NotImplementedException) as e:
            res[case["name"]] = {"error": f"{type(e).__name__}: {str(e)[:200]}"}
    with open(f"{out_path}.rank{rank}.json", "w") as f:
        json.dump(res, f, default=str)
    s.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
