#!/usr/bin/env python3
"""Fold rocprofv3 --pmc counter CSVs (one pass per counter) into profiles/<name>_pmc.json.

hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 per dispatch, averaged per kernel
(FETCH_SIZE doubled: gfx950 tallies 128-B reads at 64 B, MI355X_MICROARCH.md §HBM).
Usage: scripts/pmc_summary.py OUT.json FETCH_DIR WRITE_DIR [label]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def load(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = re.sub(r"\(.*$", "", r["Kernel_Name"]).split("<")[0].split("::")[-1].strip()
            vals[(name, r.get("Dispatch_Id", r.get("Correlation_Id")))].append(float(r["Counter_Value"]))
    per = defaultdict(list)
    for (name, _), v in vals.items():
        per[name].append(sum(v))
    return per


def main():
    out, fdir, wdir = sys.argv[1:4]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [])))
        w = sum(write.get(k, [0])) / max(1, len(write.get(k, [])))
        kernels[k] = {"launches": max(len(fetch.get(k, [])), len(write.get(k, []))),
                      "fetch_kb": f, "write_kb": w, "hbm_bytes_per_launch": int((2 * f + w) * 1024)}
    json.dump({"label": label, "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving)",
               "kernels": kernels}, open(out, "w"), indent=1)
    for k, v in kernels.items():
        print(f"{k:30s} {v['launches']:4d} {v['hbm_bytes_per_launch'] / 1e9:10.3f} GB/launch")


if __name__ == "__main__":
    main()
