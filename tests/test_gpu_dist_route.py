"""The drop-in path on several ranks: 2 ranks sharing the GPU (gloo collectives -- RCCL
refuses two ranks per device) run Planner(sg).run over their shards of an edge-list graph whose hubs
sit at ids 0..999.  Ownership is a hash of the id (include/capsmi.h capsmi_graph_distribute), so the
shards balance even though contiguous id ranges would not; every rank routes the C3 queries to the
distributed two-hop kernels and gets the whole answer, which must equal the oracle closed form."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _hub_edges(path, seed=7, n=1 << 16, m=400_000, hubs=1000):
    rng = np.random.default_rng(seed)
    src = np.where(rng.random(m) < 0.5, rng.integers(0, hubs, m), rng.integers(0, n, m))
    dst = np.where(rng.random(m) < 0.5, rng.integers(0, hubs, m), rng.integers(0, n, m))
    src[:500] = dst[:500]  # self-loops
    np.savetxt(path, np.stack([src, dst], axis=1), fmt="%d", delimiter=" ")
    return n, src.astype(np.int64), dst.astype(np.int64)


def _ranks(edges, lo, hi, world=2, nodes="owned"):
    env = dict(os.environ, CAPSMI_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tests", "dist_route_worker.py"),
           str(edges), str(lo), str(hi), nodes]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-4000:]
    out = []
    for r in range(world):
        with open(f"{edges}.rank{r}.json") as f:
            out.append(json.load(f))
    assert sorted(o["rank"] for o in out) == list(range(world))
    return out


@pytest.mark.parametrize("nodes", ["owned", "replicated"])
def test_routed_c3_on_two_ranks_with_hubs(tmp_path, nodes):
    from oracle import cpu
    edges = tmp_path / "hubs.txt"
    n, src, dst = _hub_edges(edges)
    lo, hi = int(min(src.min(), dst.min())), int(max(src.max(), dst.max())) + 1
    rows, distinct = cpu.two_hop_closed_form(n, src, dst)
    out = _ranks(edges, lo, hi, nodes=nodes)
    m = len(src)
    for o in out:  # every rank holds the whole answer
        assert o["count_star"] == rows, o
        assert o["count_distinct_c"] == distinct, o
        assert o["warm_distinct"] == distinct, o
        assert o["expand_count"] == m, o
        assert o["expand_partitioned"] is True
        assert o["routes"]["two_hop"] >= 3 and o["routes"]["expand_count"] >= 1 and o["routes"]["expand"] >= 1, o
        assert o["triangle"].startswith("refused"), o
    assert sum(o["expand_rows_local"] for o in out) == m
    assert sum(o["rels_local"] for o in out) == m
    mean = m / len(out)
    assert all(abs(o["rels_local"] - mean) / mean < 0.05 for o in out), [o["rels_local"] for o in out]
    # contiguous owner ranges of the raw ids would put the hubs on rank 0
    assert (dst < n // 2).mean() > 0.7
