#!/usr/bin/env python3
"""Emulate the N-rank C3 cold step sequentially on one GPU (no collectives): per rank the
owner(target) relationship share, build + hop 1, then the frontier's owned slices stitched together
(the all-gather), hop 2 per rank, owned popcounts summed (the all-reduce).  Prints per-N answers
against the unpartitioned count.  usage: dist_emulate.py [scale] [N...]"""
import sys

import torch

sys.path.insert(0, "cypher-for-apache-spark_amd")
from capsmi import Session, graph  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
Ns = [int(x) for x in sys.argv[2:]] or [1, 2, 4]
n, m = 1 << scale, 16 << scale
nw = (n + 31) // 32
sess = Session(0)
sess.set_stream(torch.cuda.current_stream().cuda_stream)
persons = graph.rmat_nodes(sess, scale, graph.NODES_ALL)
full = graph.rmat_rels(sess, scale, 0, m, graph.RMAT_GRAPH500, 42)
p = graph.NodeBitmap(sess, 0, n).add_scan(persons, "id")
ref = graph.two_hop_count_distinct(sess, [full], p, p, p)
print("unpartitioned", ref, flush=True)
for N in Ns:
    rels = [graph.rmat_rels(sess, scale, 0, m, graph.RMAT_GRAPH500, 42, part_col=graph.PART_TARGET, part=r, nparts=N)
            for r in range(N)]
    mids = [torch.zeros(2 * nw, dtype=torch.int32, device="cuda") for _ in range(N)]
    scratch = torch.zeros(nw, dtype=torch.int32, device="cuda")
    rps = []
    for r in range(N):
        rps.append(graph.RelPartition.build_mark_mid(sess, [rels[r]], p, p, mids[r].data_ptr(), scratch.data_ptr()))
    mid = torch.zeros(2 * nw, dtype=torch.int32, device="cuda")
    leak = 0
    for r in range(N):
        wb, we = graph.owner_words(n, r, N)
        mid[wb:we] = mids[r][wb:we]
        mid[nw + wb:nw + we] = mids[r][nw + wb:nw + we]
        own = torch.zeros(2 * nw, dtype=torch.bool, device="cuda")
        own[wb:we] = True
        own[nw + wb:nw + we] = True
        leak += int((mids[r][~own] != 0).sum().item())  # marks outside the owned slice (should be 0)
    total = 0
    for r in range(N):
        wb, we = graph.owner_words(n, r, N)
        dst = torch.zeros(nw, dtype=torch.int32, device="cuda")
        rps[r].mark_dst(p, p, mid.data_ptr(), dst.data_ptr())
        total += graph.words_popcount(sess, dst.data_ptr(), wb, we)
        rps[r].release()
    print(f"N={N} count={total} {'ok' if total == ref else 'MISMATCH'} marks outside owned slices: {leak}",
          [r.size for r in rels], flush=True)
