#!/usr/bin/env python3
"""Print the key numbers of a bench JSON line (last JSON line of the given log)."""
import json
import sys

import os

for f in sys.argv[1:]:
    if not os.path.exists(f):
        print(f"{f}: missing")
        continue
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f"{f}: no JSON line")
        continue
    line = lines[-1]
    d = json.loads(line)
    q = d.get("query", {})
    print(f"{f}: {d['ms_per_step']:.3f} ms/step  value={d['value']:.4g}  kernel={d['roofline'] and d['roofline']['kernel']} "
          f"frac={d['roofline'] and round(d['roofline']['frac'], 3)}  query_frac={q.get('query_frac_of_peak', 0):.3f}")
    for k, v in q.get("kernel_ms", {}).items():
        print(f"    {k:22s} {v:8.3f} ms")
    print("    check:", q.get("check_vs_fixture"), q.get("check_vs_unsharded", ""))
    for k, v in q.items():  # secondary modes of the C3 line
        if isinstance(v, dict) and "ms_per_step" in v:
            print(f"    mode {k}: {v['ms_per_step']:.3f} ms  " + " ".join(f"{a}={b:.3f}" for a, b in v.get("kernel_ms", {}).items()))
    if d.get("rehearsal"):
        print("    rehearsal busy ms per rank:", d["rehearsal"].get("busy_ms_per_rank"))
    for k, v in q.get("kernel_ms_per_rank", {}).items():
        print(f"    per rank {k:16s}", v)
