"""The drop-in path on several ranks: ranks run Planner(sg).run over their shards of a
distributed graph and libcapsmi routes the plans to the distributed kernels.

- 2 ranks sharing the GPU over gloo (RCCL refuses two ranks per device) on an edge list whose hubs sit
  at ids 0..999.  Ownership is a hash of the id (include/capsmi.h capsmi_graph_distribute), so the
  shards balance even though contiguous id ranges would not.  BY_TARGET shards: the C3 queries, the
  expand, the cached layout, and the cyclic triangle (C4: the distributed trigraph build with its two
  exchanges); BY_SOURCE shards (north_star's owner(source)), registered once: every hot-path shape -- C3
  count(*) / count(DISTINCT c) / count(DISTINCT a), undirected 1- and 2-hop, the grouped 2-hop, the
  triangle and the var-length grouped count (C5: in-relationships exchanged at registration, od / Y
  all-reduced, each rank the rows of its owned starts).  Every answer equals the oracle (oracle/closed.c
  closed forms and enumeration, pinned by tests/test_oracle_pins.py).
- 1 rank over RCCL (backend nccl, world size 1): the same routes with every exchange through
  torch.distributed's NCCL(=RCCL) branch of capsmi.dist.TorchCollective -- all-gathers, all-reduces and
  the ALL_TO_ALL_V, cut into rounds by libcapsmi under a small CAPSMI_COLL_CHUNK -- against the R-MAT
  fixtures (tests/golden/rmat_full.json: C3 s = 20 in both modes, C4 s = 14) and the oracle (the six
  shapes at s = 14 over BY_SOURCE shards)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _err(text):
    """the first Python traceback of a failed rank (torch.distributed.run prints its own summary last)"""
    i = text.find("Traceback (most recent call last)")
    return text[i:i + 5000] if i >= 0 else text[-4000:]


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
    src[500:3000], dst[500:3000] = dst[3000:5500], src[3000:5500]  # reciprocal pairs (C5's reverse terms)
    np.savetxt(path, np.stack([src, dst], axis=1), fmt="%d", delimiter=" ")
    return n, src.astype(np.int64), dst.astype(np.int64)


def _ranks(graph, lo, hi, world=2, nodes="owned", rels_by="target", queries="c3,tri", backend="gloo", out=None,
           env_extra=None):
    env = dict(os.environ, CAPSMI_DIST_BACKEND=backend, MASTER_ADDR="127.0.0.1", **(env_extra or {}))
    out = out or str(graph)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tests", "dist_route_worker.py"),
           str(graph), str(lo), str(hi), nodes, "--rels-by", rels_by, "--queries", queries, "--out", out]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, _err(p.stderr)
    res = []
    for r in range(world):
        with open(f"{out}.rank{r}.json") as f:
            res.append(json.load(f))
    assert sorted(o["rank"] for o in res) == list(range(world))
    return res


@pytest.mark.parametrize("nodes", ["owned", "replicated"])
def test_routed_c3_c4_on_two_ranks_with_hubs(tmp_path, nodes):
    from oracle import cpu
    edges = tmp_path / "hubs.txt"
    n, src, dst = _hub_edges(edges)
    lo, hi = int(min(src.min(), dst.min())), int(max(src.max(), dst.max())) + 1
    rows, distinct = cpu.two_hop_closed_form(n, src, dst)
    _, distinct_a = cpu.two_hop_closed_form(n, dst, src)
    tri = cpu.triangle_closed_form(n, src, dst)
    out = _ranks(edges, lo, hi, nodes=nodes, queries="c3,expand,warm,tri")
    m = len(src)
    for o in out:  # every rank holds the whole answer
        assert o["count_star"] == rows, o
        assert o["count_distinct_c"] == distinct, o
        assert o["count_distinct_a"] == distinct_a, o
        assert o["warm_distinct"] == distinct, o
        assert o["expand_count"] == m, o
        assert o["triangle"] == tri, o
        assert o["expand_partitioned"] is True
        assert o["routes"]["two_hop"] >= 4 and o["routes"]["expand_count"] >= 1 and o["routes"]["expand"] >= 1, o
        assert o["routes"]["triangle"] >= 1, o
    assert sum(o["expand_rows_local"] for o in out) == m
    assert sum(o["rels_local"] for o in out) == m
    mean = m / len(out)
    assert all(abs(o["rels_local"] - mean) / mean < 0.05 for o in out), [o["rels_local"] for o in out]
    # contiguous owner ranges of the raw ids would put the hubs on rank 0
    assert (dst < n // 2).mean() > 0.7


def _six_shapes(n, src, dst):
    """the oracle's answers for the six hot-path shapes over one graph (every node V)"""
    from oracle import cpu
    rows, dc = cpu.two_hop_closed_form(n, src, dst)
    _, da = cpu.two_hop_closed_form(n, dst, src)  # distinct starts = distinct ends of the reversed graph
    u_rows, u_dc = cpu.two_hop_undirected_closed_form(n, src, dst)
    loops = int((src == dst).sum())
    ends = int(np.unique(np.concatenate([src, dst])).size)  # every endpoint is an arc's end
    _, _, grows, gdist = cpu.two_hop_enumerate(n, src, dst, grouped=True)
    grouped = {int(a): (int(gdist[a]), int(grows[a])) for a in np.nonzero(grows)[0]}
    _, per_a = cpu.var_length_closed_form(n, src, dst, 1, 3)
    return {"count_star": rows, "count_distinct_c": dc, "count_distinct_a": da,
            "und1": [2 * len(src) - loops, ends], "und2": [u_rows, u_dc, u_dc],  # (a)-(b)-(c) is symmetric
            "grouped": grouped, "triangle": cpu.triangle_closed_form(n, src, dst),
            "varlen": {int(i): int(per_a[i]) for i in np.nonzero(per_a)[0]}}


def _check_six(out, want, m):
    got_g, got_v = {}, {}
    for o in out:  # the count shapes whole on every rank, the grouped rows partitioned by owned start
        for k in ("count_star", "count_distinct_c", "count_distinct_a", "und1", "und2", "triangle"):
            assert o[k] == want[k], (k, o[k], want[k])
        assert o["expand_count"] == m, o
        r = o["routes"]
        assert r["two_hop"] >= 3 and r["undirected"] >= 2 and r["two_hop_grouped"] >= 1, r
        assert r["triangle"] >= 1 and r["var_length"] >= 1 and r["expand_count"] >= 1, r
        assert r["miss"] == 0, r
        for a, dc, c in o["grouped_rows"]:
            assert a not in got_g, a  # each start id on exactly one rank
            got_g[a] = (dc, c)
        for a, c in o["varlen_rows"]:
            assert a not in got_v, a
            got_v[a] = c
    assert got_g == want["grouped"]
    assert got_v == want["varlen"]


def test_one_by_source_distribution_routes_every_shape(tmp_path):
    """north_star's partitioning (relationships by owner(source)) registered once: C3 count(*) / count(DISTINCT
    c) / count(DISTINCT a), the undirected 1- and 2-hop counts, the grouped 2-hop, the triangle (C4) and the
    var-length grouped count (C5) all routed on 2 ranks, none refused or run operator by operator (miss 0)."""
    edges = tmp_path / "hubs_src.txt"
    n, src, dst = _hub_edges(edges, seed=11, m=200_000)
    want = _six_shapes(n, src, dst)
    # CAPSMI_COLL_CHUNK=4096: at W = 2 every exchange above 2048 words per peer runs in rounds (k_dist.hip
    # collective / collective_a2av); the hub edge list gives the two ranks unequal per-pair counts, so later
    # rounds carry zero words for some peers
    out = _ranks(edges, 0, n, rels_by="source", queries="c3,und,grouped,tri,varlen,expand",
                 env_extra={"CAPSMI_COLL_CHUNK": "4096"})
    _check_six(out, want, len(src))
    for o in out:
        assert o["varlen_partitioned"] is True and o["grouped_partitioned"] is True
    assert sum(o["rels_local"] for o in out) == len(src)


def _fixture(key):
    with open(os.path.join(ROOT, "tests", "golden", "rmat_full.json")) as f:
        return json.load(f)["cases"][key]


def test_routes_over_rccl_world1(tmp_path):
    """The NCCL(=RCCL) branch of TorchCollective (zero-copy device views, no stream drain) under the
    drop-in route before the driver's multi-GPU run: C3 at s = 20 (BY_TARGET: all-gathers of the node
    scan, the frontier and the in-degrees, all-reduces) and C4 at s = 14 (BY_SOURCE: the in-relationship
    ALL_TO_ALL_V at registration, the trigraph build's two exchanges and its all-gathers)."""
    c3 = _fixture("c3_s20")
    o = _ranks("rmat:20", 0, 1 << 20, world=1, rels_by="target", queries="c3", backend="nccl",
               out=str(tmp_path / "r20"))[0]
    assert o["backend"] == "nccl" and o["world"] == 1
    assert o["count_distinct_c"] == c3["count_distinct_c"], o
    assert o["count_star"] == c3["count_star"], o
    assert o["routes"]["two_hop"] >= 2, o
    o = _ranks("rmat:20", 0, 1 << 20, world=1, rels_by="source", queries="c3", backend="nccl",
               out=str(tmp_path / "r20s"))[0]
    assert o["count_distinct_c"] == c3["count_distinct_c"], o
    assert o["count_star"] == c3["count_star"], o
    c4 = _fixture("c4_s14")
    # CAPSMI_COLL_CHUNK: every collective above 2^12 words cut by libcapsmi into rounds (k_dist.hip collective,
    # collective_a2av) -- the path that keeps a full-size C4 build's 2^28-word exchanges in bounded RCCL calls
    o = _ranks("rmat:14", 0, 1 << 14, world=1, rels_by="source", queries="c3,und,grouped,tri,varlen,expand",
               backend="nccl", out=str(tmp_path / "r14"), env_extra={"CAPSMI_COLL_CHUNK": str(1 << 12)})[0]
    assert o["triangle"] == c4["count_star"], o
    from oracle import cpu
    src, dst = cpu.rmat_edges(14, 0, 16 << 14)
    _check_six([o], _six_shapes(1 << 14, src, dst), len(src))
