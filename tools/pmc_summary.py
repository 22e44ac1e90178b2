#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs for one kernel: per-dispatch counter sums (median over dispatches); when the
pattern matches several kernels, the one with the longest median dispatch.

    python tools/pmc_summary.py gpurun_out/pmc2 k_eval_pdf_v4            # {counter: median, dispatch_ns: ...}
    python tools/pmc_summary.py --by-kernel gpurun_out/pmc2 k_check      # {kernel name: {counter: median, ...}}

`root` holds one sub-directory per counter pass (rocprofv3 -d <root>/<pass>); every *counter_collection.csv
below a pass directory is read.
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def _rows(root):
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        yield f, csv.DictReader(open(f))


def summarise(root, pattern, by_kernel=False):
    per = collections.defaultdict(float)            # (kernel, file, dispatch, counter) -> sum over dimensions
    dur = collections.defaultdict(dict)              # kernel -> {(file, dispatch): ns}
    for f, rows in _rows(root):
        for r in rows:
            k = r["Kernel_Name"]
            if pattern not in k:
                continue
            kk = k
            per[(kk, f, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            dur[kk][(f, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    byc = collections.defaultdict(lambda: collections.defaultdict(list))
    for (kk, _, _, c), v in per.items():
        byc[kk][c].append(v)
    out = {}
    for kk, cs in byc.items():
        out[kk] = {c: statistics.median(v) for c, v in cs.items()}
        out[kk]["dispatch_ns"] = statistics.median(dur[kk].values())
        out[kk]["dispatches"] = len(dur[kk])
    if by_kernel:
        return out
    # one kernel per summary: the pattern can also match a short companion kernel (k_check -> k_check_final), whose
    # dispatches must not enter the medians -- the matching kernel with the longest median dispatch is the one
    return max(out.values(), key=lambda c: c["dispatch_ns"]) if out else {}


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--by-kernel"]
    print(json.dumps(summarise(args[0], args[1], by_kernel="--by-kernel" in sys.argv), indent=1))
