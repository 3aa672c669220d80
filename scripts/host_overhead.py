"""Host-side cost of the planner route for the C3 query (diagnostic): lazy plan construction
(Planner(sg).run without forcing) vs a full forced query, at a small scale so device time is small."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cypher-for-apache-spark_amd")]
import torch  # noqa: E402
from capsmi import Session, graph  # noqa: E402
from capsmi.planner import EntityTable, Planner, ScanGraph  # noqa: E402

import bench  # noqa: E402

s = Session(0)
s.set_stream(torch.cuda.current_stream().cuda_stream)
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 16
rels = graph.rmat_rels(s, scale, 0, 16 << scale)
nodes = graph.rmat_nodes(s, scale, graph.NODES_ALL)
sg = ScanGraph(s, [EntityTable("node", frozenset({"Person"}), {}, nodes, id_col="id")],
               [EntityTable("rel", frozenset({"FRIEND_OF"}), {}, rels, id_col="id", src_col="source", dst_col="target")])
for _ in range(5):
    t, outs = Planner(sg).run(bench.C3_QUERY)
    t.column(outs[0][2])
N = 50
t0 = time.perf_counter()
for _ in range(N):
    t, outs = Planner(sg).run(bench.C3_QUERY)
t1 = time.perf_counter()
for _ in range(N):
    t, outs = Planner(sg).run(bench.C3_QUERY)
    t.column(outs[0][2])
torch.cuda.synchronize()
t2 = time.perf_counter()
p = graph.NodeBitmap(s, 0, 1 << scale).add_scan(nodes, "id")
for _ in range(N):
    p = graph.NodeBitmap(s, 0, 1 << scale).add_scan(nodes, "id")
    graph.two_hop_count_distinct(s, [rels], p, p, p)
torch.cuda.synchronize()
t3 = time.perf_counter()
print(f"scale {scale}: plan build {1e3 * (t1 - t0) / N:.3f} ms, planned+forced {1e3 * (t2 - t1) / N:.3f} ms, "
      f"direct calls {1e3 * (t3 - t2) / N:.3f} ms")
import cProfile, pstats  # noqa: E402,E401
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    t, outs = Planner(sg).run(bench.C3_QUERY)
    t.column(outs[0][2])
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(12)
pr = cProfile.Profile()  # plan construction alone: where the Python time goes
pr.enable()
for _ in range(200):
    t, outs = Planner(sg).run(bench.C3_QUERY)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
s.close()
