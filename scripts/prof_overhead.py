"""Diagnostic (not product): C3 cold route step time with the library's per-kernel HIP-event timers on
and off (capsmi_session_set_profiling), to size the instrumentation's share of the bench's step.
Usage: python3 scripts/prof_overhead.py [scale] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cypher-for-apache-spark_amd")]
import torch  # noqa: E402
from capsmi import Session, _lib, graph  # noqa: E402
from capsmi.planner import EntityTable, Planner, ScanGraph  # noqa: E402

import bench  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 26
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
s = Session(0)
s.set_stream(torch.cuda.current_stream().cuda_stream)
rels = graph.rmat_rels(s, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
nodes = graph.rmat_nodes(s, scale, graph.NODES_ALL)
sg = ScanGraph(s, [EntityTable("node", frozenset({"Person"}), {}, nodes, id_col="id")],
               [EntityTable("rel", frozenset({"FRIEND_OF"}), {}, rels, id_col="id", src_col="source", dst_col="target")])


def step():
    t, outs = Planner(sg).run(bench.C3_QUERY)
    return int(t.column(outs[0][2]).values[0])


for _ in range(3):
    step()
for rep in range(3):
    for prof in (1, 0):
        _lib.call("capsmi_session_set_profiling", s.handle, prof)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        print(f"profiling={prof}: {1e3 * (time.perf_counter() - t0) / steps:.3f} ms/step", flush=True)
