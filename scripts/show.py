import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
q = d["query"]
print("cold ms", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 3), d["roofline"]["kernel"], q["check_vs_unpartitioned"])
print(" ", {k: round(v, 3) for k, v in q["kernel_ms"].items()})
for m in ("warm", "stream"):
    if m in q:
        print(m, round(q[m]["ms_per_step"], 3), {k: round(v, 3) for k, v in q[m]["kernel_ms"].items()})
