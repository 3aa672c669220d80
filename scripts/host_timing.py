"""Host-side time of each library call in the C3 cold step (rank 0's shard of N on one GPU).
usage: python scripts/host_timing.py [N] -- medians in microseconds, GPU synced only where the API syncs."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cypher-for-apache-spark_amd")]
import torch  # noqa: E402
from capsmi import Session, graph  # noqa: E402

shards = int(sys.argv[1]) if len(sys.argv) > 1 else 8
scale, n = 26, 1 << 26
s = Session(0)
s.set_stream(torch.cuda.current_stream().cuda_stream)
rels = graph.rmat_rels(s, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42, part_col=graph.PART_TARGET if shards > 1
                       else graph.PART_NONE, part=0, nparts=shards)
persons = graph.rmat_nodes(s, scale, graph.NODES_ALL)
nw = n // 32
wb, we = graph.owner_words(n, 0, shards)
mid = torch.zeros(2 * nw, dtype=torch.int32, device="cuda")
scratch = torch.zeros(nw, dtype=torch.int32, device="cuda")
dstw = torch.zeros(nw, dtype=torch.int32, device="cuda")
T = {}


def tick(name, t0):
    t = time.perf_counter()
    T.setdefault(name, []).append((t - t0) * 1e6)
    return t


for it in range(30):
    t = time.perf_counter()
    t0 = t
    p = graph.NodeBitmap(s, 0, n)
    t = tick("bitmap_create", t)
    p.add_scan(persons, "id")
    t = tick("add_scan (syncs)", t)
    rp = graph.RelPartition.build_mark_mid(s, [rels], p, p, mid.data_ptr(), scratch.data_ptr())
    t = tick("build_mark_mid", t)
    rp.mark_dst(p, p, mid.data_ptr(), dstw.data_ptr())
    t = tick("mark_dst", t)
    c = graph.words_popcount(s, dstw.data_ptr(), wb, we)
    t = tick("popcount (syncs)", t)
    rp.release()
    t = tick("relpart_release", t)
    p.release()
    t = tick("bitmap_release", t)
    tick("step", t0)
for k, v in T.items():
    v = sorted(v[5:])
    print(f"{k:20s} {v[len(v) // 2]:9.1f} us")
s.close()
