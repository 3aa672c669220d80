import os, sys, time, cProfile, pstats
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cypher-for-apache-spark_amd")]
import torch
from capsmi import Session, graph
from capsmi.planner import EntityTable, Planner, ScanGraph
import bench
s = Session(0)
s.set_stream(torch.cuda.current_stream().cuda_stream)
scale = 14
rels = graph.rmat_rels(s, scale, 0, 16 << scale)
nodes = graph.rmat_nodes(s, scale, graph.NODES_ALL)
sg = ScanGraph(s, [EntityTable("node", frozenset({"Person"}), {}, nodes, id_col="id")],
               [EntityTable("rel", frozenset({"FRIEND_OF"}), {}, rels, id_col="id", src_col="source", dst_col="target")])
for _ in range(20):
    t, outs = Planner(sg).run(bench.C3_QUERY); t.column(outs[0][2])
N = 200
t0 = time.perf_counter()
for _ in range(N):
    t, outs = Planner(sg).run(bench.C3_QUERY)
t1 = time.perf_counter()
print(f"plan build {1e3*(t1-t0)/N:.3f} ms")
pr = cProfile.Profile(); pr.enable()
for _ in range(N):
    t, outs = Planner(sg).run(bench.C3_QUERY)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
