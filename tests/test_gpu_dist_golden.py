"""Every golden vector of the reference's acceptance tests (tests/golden/acceptance.json, predicates.json)
over a graph distributed on 2 ranks (gloo ranks sharing the GPU; tests/dist_golden_worker.py), and on one rank
over RCCL: routed plans
and operator-by-operator plans whose joins, groupings, distincts, global aggregates and orderings take the
generic executor's Exchanges (csrc/plan.hip; Spark's Exchange before joins and aggregates, SparkTable.scala:
133, 226).  A partitioned result's rows, summed over the ranks, and a whole result on every rank must equal
the case's expected rows (order too for ORDER BY cases); list columns (collect results) travel with their
values.""" 
import json
import os
import socket
import subprocess
import sys

import pytest

from golden_util import all_cases, same_rows

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


# (ranks, backend, mode): 2 gloo ranks sharing the GPU, routed and unrouted; and 1 rank over RCCL (backend
# nccl), unrouted, so every Exchange of the generic executor -- the ALL_TO_ALL_V of hash-partitioned joins
# and groupings, the all-gathers of global aggregates and ordering -- runs through RCCL, in chunked calls
# (CAPSMI_COLL_CHUNK=64 on every backend: the golden graphs are small, so at two gloo ranks the all-gathers
# stage rank-major rounds and the ALL_TO_ALL_V rounds carry unequal, partly empty per-peer counts)
@pytest.mark.parametrize("world,backend,mode", [(2, "gloo", "fused"), (2, "gloo", "unfused"), (1, "nccl", "unfused")])
def test_golden_vectors_on_two_ranks(tmp_path, world, backend, mode):
    out = str(tmp_path / "golden")
    env = dict(os.environ, CAPSMI_DIST_BACKEND=backend, MASTER_ADDR="127.0.0.1")
    env["CAPSMI_COLL_CHUNK"] = "64"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}", "--master-addr",
           "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tests", "dist_golden_worker.py"), out, mode]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, _err(p.stderr)
    ranks = []
    for r in range(world):
        with open(f"{out}.rank{r}.json") as f:
            ranks.append(json.load(f))
    refused, checked = [], 0
    for _, case in all_cases():
        name = case["name"]
        res = [x[name] for x in ranks]
        if any("error" in x for x in res):
            refused.append((name, [x.get("error") for x in res]))
            continue
        assert len({x["partitioned"] for x in res}) == 1, name
        if res[0]["partitioned"]:
            got = [row for x in res for row in x["rows"]]
            assert same_rows(got, case["expected"]), (name, got, case["expected"])
        else:
            for x in res:
                assert same_rows(x["rows"], case["expected"], case.get("ordered", False)), (name, x["rows"],
                                                                                               case["expected"])
        checked += 1
    assert not refused, refused
    print(f"{mode}: {checked} golden vectors equal on {world} rank(s) over {backend}")


def test_nulls_on_one_rank_only(tmp_path):
    """A nullable column whose validity buffer exists on one rank only (tests/dist_nulls_worker.py): the ranks
    agree on which columns carry validity before an Exchange (csrc/k_dist.hip agreed_validity), so they issue
    the same collectives; grouping on it, projecting it through the expand's joins and counting it give the
    expected rows (nulls grouped together and not counted, SparkTable.scala:121-188)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from dist_nulls_worker import N, age, edges
    out = str(tmp_path / "nulls")
    env = dict(os.environ, CAPSMI_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tests", "dist_nulls_worker.py"), out]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    assert p.returncode == 0, _err(p.stderr)
    ranks = []
    for r in range(2):
        with open(f"{out}.rank{r}.json") as f:
            ranks.append(json.load(f))
    assert [x["has_valid"] for x in ranks] == [True, False]  # the case the agreement is for
    ages = {x: age(x, 2) for x in range(N)}
    groups = {}
    for a in ages.values():
        groups[a] = groups.get(a, 0) + 1
    want = {"group": [{"k": k, "n": n} for k, n in groups.items()],
            "expand": [{"x": ages[s], "y": ages[t]} for _, s, t in edges()],
            "count": [{"c": sum(a is not None for a in ages.values())}]}
    for name, rows in want.items():
        res = [x[name] for x in ranks]
        if res[0]["partitioned"]:
            got = [row for x in res for row in x["rows"]]
            assert same_rows(got, rows), (name, got, rows)
        else:
            for x in res:
                assert same_rows(x["rows"], rows), (name, x["rows"], rows)
