"""Host-side profile of the C3 planner route at full size (cProfile over cold steps): where the
≈0.3–0.45 ms between the route and the direct calls goes.  Usage: python3 scripts/route_profile.py [scale]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cypher-for-apache-spark_amd")]
import torch  # noqa: E402
from capsmi import Session, graph  # noqa: E402
from capsmi.planner import EntityTable, Planner, ScanGraph  # noqa: E402
import bench  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 26
s = Session(0)
s.set_stream(torch.cuda.current_stream().cuda_stream)
rels = graph.rmat_rels(s, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
nodes = graph.rmat_nodes(s, scale, graph.NODES_ALL)
sg = ScanGraph(s, [EntityTable("node", frozenset({"Person"}), {}, nodes, id_col="id")],
               [EntityTable("rel", frozenset({"FRIEND_OF"}), {}, rels, id_col="id", src_col="source", dst_col="target")])


def step():
    t, outs = Planner(sg).run(bench.C3_QUERY)
    return int(t.column(outs[0][2]).values[0])


for _ in range(2):
    step()
torch.cuda.synchronize()
N = 10
t0 = time.perf_counter()
for _ in range(N):
    step()
torch.cuda.synchronize()
print(f"route step {1e3 * (time.perf_counter() - t0) / N:.3f} ms")
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    step()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
