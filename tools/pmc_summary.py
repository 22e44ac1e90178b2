#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs for one kernel: per-dispatch counter sums (median over dispatches).

    python tools/pmc_summary.py gpurun_out/pmc2 k_eval_pdf_v4
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def summarise(root, pattern):
    out = {}
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        per = collections.defaultdict(float)
        dur = {}
        for r in csv.DictReader(open(f)):
            if pattern not in r["Kernel_Name"]:
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        byc = collections.defaultdict(list)
        for (d, c), v in per.items():
            byc[c].append(v)
        for c, v in byc.items():
            out[c] = statistics.median(v)
        if dur:
            out.setdefault("dispatch_ns", statistics.median(dur.values()))
    return out


if __name__ == "__main__":
    print(json.dumps(summarise(sys.argv[1], sys.argv[2]), indent=1))
