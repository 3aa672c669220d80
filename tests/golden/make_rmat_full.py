#!/usr/bin/env python3
"""Generate tests/golden/rmat_full.json: exact answers of the BASELINE configs C2-C5 at their full
sizes, computed by the CPU checker's closed forms (oracle/closed.c, pinned against enumeration and
the reference's golden graphs by tests/test_oracle_pins.py).  TEST INFRASTRUCTURE: bench.py and the
-m gpu tests compare the device results with these numbers.

Run from the repo root (needs ~20 GB of host memory for C3; several minutes on 8 cores):
    python tests/golden/make_rmat_full.py [--only c3,c2,...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden", "rmat_full.json")

G500, LDBC = (57, 19, 19), (45, 15, 15)


def c3(scale):
    from oracle import cpu
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale, G500, 42)
    rows, dist = cpu.two_hop_closed_form_mt(1 << scale, src, dst)
    return {"query": "MATCH (a:Person)-[:FRIEND_OF]->(b:Person)-[:FRIEND_OF]->(c:Person) RETURN count(DISTINCT c)",
            "scale": scale, "edge_factor": 16, "rmat": list(G500), "seed": 42, "nodes": "all ids Person",
            "count_star": rows, "count_distinct_c": dist, "oracle": "closed.c orc_two_hop_closed_form_mt"}


def c3u(scale):
    from oracle import cpu
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale, G500, 42)
    rows, dist = cpu.two_hop_undirected_closed_form(1 << scale, src, dst)
    return {"query": "MATCH (a:Person)-[:FRIEND_OF]-(b:Person)-[:FRIEND_OF]-(c:Person) RETURN count(*), count(DISTINCT c)",
            "scale": scale, "edge_factor": 16, "rmat": list(G500), "seed": 42, "nodes": "all ids Person",
            "count_star": rows, "count_distinct_c": dist, "oracle": "closed.c orc_two_hop_undirected_closed_form"}


def c2(scale):
    from oracle import cpu
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale, G500, 42)
    person, adult = cpu.c2_masks(n, 42)
    rows, s, x = cpu.expand_filter(src, dst, adult, person)
    return {"query": "MATCH (a:Person)-[r:FRIEND_OF]->(b:Person) WHERE a.age >= 18 AND a.age < 65 RETURN id(a), id(b)",
            "scale": scale, "edge_factor": 16, "rmat": list(G500), "seed": 42, "age_seed": 42,
            "rows": rows, "fingerprint": [rows, str(s), str(x)],
            "oracle": "rmat.c orc_expand_filter (row hash fingerprint over (id(a), id(b)))"}


def c4(scale):
    from oracle import cpu
    src, dst = cpu.rmat_edges(scale, 0, 16 << scale, G500, 42)
    rows = cpu.triangle_closed_form(1 << scale, src, dst)
    return {"query": "MATCH (a)-[r1:FRIEND_OF]->(b)-[r2:FRIEND_OF]->(c)-[r3:FRIEND_OF]->(a) RETURN count(*)",
            "scale": scale, "edge_factor": 16, "rmat": list(G500), "seed": 42, "count_star": rows,
            "oracle": "closed.c orc_triangle_closed_form"}


def c5(scale):
    from oracle import cpu
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, 32 << scale, LDBC, 42)
    tot, per_a = cpu.var_length_closed_form(n, src, dst, 1, 3)
    ids = np.nonzero(per_a)[0].astype(np.int64)
    cnt, s, x = cpu.fingerprint([ids, per_a[ids]])
    return {"query": "MATCH (a:Person)-[:KNOWS*1..3]->(b:Person) RETURN id(a), count(*)", "scale": scale,
            "edge_factor": 32, "rmat": list(LDBC), "seed": 42, "rows": int(len(ids)), "sum_count": tot,
            "fingerprint": [cnt, str(s), str(x)], "oracle": "closed.c orc_var_length_closed_form"}


def c5u4(scale):
    from oracle import cpu
    n = 1 << scale
    src, dst = cpu.rmat_edges(scale, 0, 32 << scale, LDBC, 42)
    _, per3 = cpu.var_length_closed_form(n, src, dst, 1, 3)
    _, per4 = cpu.var_length4_closed_form(n, src, dst)
    per_a = per3 + per4
    ids = np.nonzero(per_a)[0].astype(np.int64)
    cnt, s, x = cpu.fingerprint([ids, per_a[ids]])
    return {"query": "MATCH (a:Person)-[:KNOWS*1..4]->(b:Person) RETURN id(a), count(*)", "scale": scale,
            "edge_factor": 32, "rmat": list(LDBC), "seed": 42, "rows": int(len(ids)), "sum_count": int(per_a.sum()),
            "fingerprint": [cnt, str(s), str(x)],
            "oracle": "closed.c orc_var_length_closed_form (1..3) + cpu.py var_length4_closed_form (4)"}


JOBS = {"c3_s26": (c3, 26), "c3_s20": (c3, 20), "c3_s16": (c3, 16), "c3u_s26": (c3u, 26),
        "c3u_s20": (c3u, 20), "c3u_s16": (c3u, 16), "c2_s24": (c2, 24), "c2_s16": (c2, 16),
        "c4_s24": (c4, 24), "c4_s14": (c4, 14), "c5_s20": (c5, 20), "c5_s14": (c5, 14),
        "c5u4_s20": (c5u4, 20), "c5u4_s14": (c5u4, 14)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    want = [j for j in JOBS if not args.only or any(j.startswith(o) for o in args.only.split(","))]
    out = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            out = json.load(f)
    out.setdefault("about", "Exact answers of BASELINE configs C2-C5 (SURVEY.md 8d) from the CPU checker's closed "
                            "forms (oracle/closed.c, pinned by tests/test_oracle_pins.py); generated by "
                            "tests/golden/make_rmat_full.py.  Fingerprint = (rows, sum, xor) of the row hashes "
                            "(oracle/rmat.c orc_row_hash), sums and xors as decimal strings.")
    cases = out.setdefault("cases", {})
    for j in want:
        fn, scale = JOBS[j]
        t0 = time.perf_counter()
        cases[j] = fn(scale)
        cases[j]["cpu_seconds"] = round(time.perf_counter() - t0, 1)
        print(j, cases[j], flush=True)
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
