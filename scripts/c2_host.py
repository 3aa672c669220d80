"""Diagnostic (not product): host-side timeline of the C2 direct step (node scans, expand, size) on
resident tables, to attribute the step's time above its kernels.  Usage: python3 scripts/c2_host.py [scale]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cypher-for-apache-spark_amd")]
import torch  # noqa: E402
from capsmi import Session, graph  # noqa: E402
from capsmi.expr import Ands, BinOp, Col, Lit  # noqa: E402


scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
s = Session(0)
s.set_stream(torch.cuda.current_stream().cuda_stream)
n, m = 1 << scale, 16 << scale
rels = graph.rmat_rels(s, scale, 0, m, graph.RMAT_GRAPH500, 42)
nodes = graph.rmat_nodes(s, scale, graph.NODES_PERSON, 42)
pred = Ands((BinOp(">=", Col("age"), Lit(18)), BinOp("<", Col("age"), Lit(65))))  # as bench.py's C2


def step(log):
    t = [time.perf_counter()]
    a_ok = graph.NodeBitmap(s, 0, n).add_scan(nodes, "id", pred)
    t.append(time.perf_counter())
    b_ok = graph.NodeBitmap(s, 0, n).add_scan(nodes, "id")
    t.append(time.perf_counter())
    out = graph.expand_filter(s, rels, a_ok, b_ok, ["source", "target"], ["a", "b"])
    t.append(time.perf_counter())
    rows = out.size
    torch.cuda.synchronize()
    t.append(time.perf_counter())
    if log:
        print("scan a %.1f us, scan b %.1f us, expand call %.1f us, size+sync %.1f us, total %.3f ms, rows %d" % (
            1e6 * (t[1] - t[0]), 1e6 * (t[2] - t[1]), 1e6 * (t[3] - t[2]), 1e6 * (t[4] - t[3]), 1e3 * (t[4] - t[0]), rows),
            flush=True)
    return out


keep = None
for i in range(8):
    keep = step(i >= 3)
