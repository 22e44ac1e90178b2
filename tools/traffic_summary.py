#!/usr/bin/env python3
"""Per-launch HBM bytes of one kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python tools/traffic_summary.py gpurun_out/pmc_traffic k_eval_pdf_v4 CookTorrance 100000000

FETCH_SIZE and WRITE_SIZE are reported in KiB.  On gfx950 FETCH_SIZE counts exactly half of the
bytes of a 16-B-per-lane streaming read (MI355X_MICROARCH.md, HBM section), so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Median over the profiled launches.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarise  # noqa: E402


def main():
    root, kernel, model, pairs = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    c = summarise(root, kernel)
    fetch = 2.0 * c["FETCH_SIZE"] * 1024.0
    write = c["WRITE_SIZE"] * 1024.0
    print(json.dumps({"model": model, "pairs": pairs, "kernel": kernel,
                      "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                      "hbm_bytes_per_launch": fetch + write,
                      "algorithmic_bytes_per_launch": 40 * pairs,
                      "raw": {"FETCH_SIZE_KiB": c["FETCH_SIZE"], "WRITE_SIZE_KiB": c["WRITE_SIZE"]},
                      "correction": "FETCH_SIZE x2 (gfx950 16B/lane streaming reads), KiB -> bytes"}, indent=1))


if __name__ == "__main__":
    main()
