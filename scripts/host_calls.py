"""Host timeline of the C3 cold route (diagnostic): every libcapsmi call one step makes, with its
start offset and duration, so the device-idle window between two steps (result read -> next
query's first launch) can be attributed to Python planning, library calls or syncs.
Usage: python3 scripts/host_calls.py [scale] [plan: pre|in]  (pre: the plan built before the step, as bench.py
times it per SURVEY 8d; in: planning inside the step)"""
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
s = Session(0)
s.set_stream(torch.cuda.current_stream().cuda_stream)
rels = graph.rmat_rels(s, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
nodes = graph.rmat_nodes(s, scale, graph.NODES_ALL)
sg = ScanGraph(s, [EntityTable("node", frozenset({"Person"}), {}, nodes, id_col="id")],
               [EntityTable("rel", frozenset({"FRIEND_OF"}), {}, rels, id_col="id", src_col="source", dst_col="target")])

LOG = []
_orig = _lib.call


def traced(name, *args):
    t0 = time.perf_counter()
    try:
        return _orig(name, *args)
    finally:
        LOG.append((name, t0, time.perf_counter()))


pre = (sys.argv[2] if len(sys.argv) > 2 else "pre") == "pre"


def step(plan=None):
    t, outs = plan if plan is not None else Planner(sg).run(bench.C3_QUERY)
    return int(t.column(outs[0][2]).values[0])


for _ in range(3):
    step()
torch.cuda.synchronize()
_lib.call = traced  # the modules call _lib.call through the module attribute
steps = []
for _ in range(5):
    plan = Planner(sg).run(bench.C3_QUERY) if pre else None
    torch.cuda.synchronize()
    LOG.clear()
    t0 = time.perf_counter()
    r = step(plan)
    t1 = time.perf_counter()
    steps.append((t0, t1, list(LOG)))
for t0, t1, log in steps[-2:]:
    print(f"step {1e3 * (t1 - t0):.3f} ms, {len(log)} calls")
    prev = t0
    for name, a, b in log:
        gap = (a - prev) * 1e6
        print(f"  +{(a - t0) * 1e6:9.1f} us  py-gap {gap:7.1f}  {name:40s} {1e6 * (b - a):9.1f} us")
        prev = b
    print(f"  tail py {(t1 - prev) * 1e6:.1f} us")
