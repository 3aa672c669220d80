"""The multi-GPU bench lines rehearsed with 2 ranks on one GPU (gloo collectives; RCCL refuses two
ranks per device): each rank holds its owner shard, the exchanges run as in an N-GPU job, and the
answers must equal the committed oracle fixture (C3, C5) / the unsharded table (C2, C5)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(wl, scale, n=2):
    env = dict(os.environ, CAPSMI_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"), "--gpus", str(n),
           "--workload", wl, "--scale", str(scale), "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_c3_two_ranks():
    """bench.py's N-rank C3: every mode (cold, warm, count(*)) is Planner(sg).run through the route on
    every rank of the distributed graph; shards balanced by the hash ownership."""
    d = _run("c3", 16)
    assert d["n_gpus"] == 2
    assert d["query"]["check_vs_fixture"] == "ok"
    assert d["query"]["rels_local_rank0"] < 16 << 16  # rank 0 holds only its owner(target) share
    assert d["query"]["rels_max_over_mean"] < 1.05
    assert d["config"]["route"].startswith("Planner(sg).run") and "plans routed" in d["config"]["route"]
    assert d["roofline"]["traffic"] is None  # the committed PMC profiles are 1-GPU runs


def test_c5_two_ranks():
    d = _run("c5", 14)
    assert d["query"]["check_vs_fixture"] == "ok" and d["query"]["check_vs_unsharded"] == "ok"


def test_c2_two_ranks():
    d = _run("c2", 16)
    assert d["query"]["check_vs_fixture"] == "ok" and d["query"]["check_vs_unsharded"] == "ok"
