"""Generic-join strategy sweep (session configuration CAPSMI_JOIN=hash|radix): inner joins of random 64-bit keys
(no dense range, so the direct-address table is out) with 2 payload columns a side, build sizes
2^22..2^26, probe = 4 x build, ~1 match per probe row.  Prints one JSON line per (size, strategy)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cypher-for-apache-spark_amd"))


def main():
    from capsmi import ColumnData, Session
    from capsmi.expr import I64
    s = Session(0)
    rng = np.random.default_rng(0)
    for lg in [int(x) for x in os.environ.get("SIZES", "22 24 26").split()]:
        nb = 1 << lg
        bkeys = rng.integers(-(1 << 62), 1 << 62, nb)
        pkeys = bkeys[rng.integers(0, nb, 4 * nb)]
        B = s.table([ColumnData("bk", I64, bkeys), ColumnData("b1", I64, np.arange(nb)),
                     ColumnData("b2", I64, np.arange(nb) * 3)])
        Pt = s.table([ColumnData("pk", I64, pkeys), ColumnData("p1", I64, np.arange(4 * nb)),
                      ColumnData("p2", I64, np.arange(4 * nb) * 5)])
        B.size, Pt.size
        for mode in ("hash", "radix"):
            s.set_config("CAPSMI_JOIN", mode)
            times = []
            for it in range(4):
                s.sync()
                t0 = time.perf_counter()
                j = Pt.join(B, "inner", ("pk", "bk"))
                n = j.size
                s.sync()
                times.append(time.perf_counter() - t0)
                del j
            ms = min(times[1:]) * 1e3
            print(json.dumps({"build_rows": nb, "probe_rows": 4 * nb, "out_rows": n, "strategy": mode,
                              "ms": round(ms, 3), "probe_rows_per_s": 4 * nb / ms * 1e3}), flush=True)
        del B, Pt
    s.close()


if __name__ == "__main__":
    main()
