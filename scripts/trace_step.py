"""One step's device timeline from a rocprofv3 csv trace directory (kernels + copies, gaps between them).

usage: python3 scripts/trace_step.py DIR FIRST_KERNEL [occurrence]
  DIR: the -d directory of `rocprofv3 --kernel-trace [--memory-copy-trace] -f csv -o run`
  FIRST_KERNEL: a substring of the step's first kernel name; the step runs to its next occurrence
  occurrence: which step (default -2: the last complete one)
"""
import csv
import os
import sys


def main():
    d, first = sys.argv[1], sys.argv[2]
    occ = int(sys.argv[3]) if len(sys.argv) > 3 else -2
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:48]))
    mc = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(mc):
        for r in csv.DictReader(open(mc)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M " + r.get("Direction", "?")))
    ev.sort()
    idx = [i for i, e in enumerate(ev) if first in e[2]]
    st, en = idx[occ], idx[occ + 1] if occ + 1 < 0 or occ + 1 < len(idx) else len(ev)
    t0, prev, busy, gaps = ev[st][0], None, 0, 0
    for s, e, n in ev[st:en]:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        busy += e - s
        gaps += max(gap, 0.0)
        print("%8.3f %7.3f gap=%6.1fus %s" % ((s - t0) / 1e6, (e - s) / 1e6, gap, n))
        prev = e
    print("device busy %.3f ms, gaps %.3f ms, span %.3f ms" % (busy / 1e6, gaps / 1e3, (ev[en - 1][1] - t0) / 1e6))


if __name__ == "__main__":
    main()
