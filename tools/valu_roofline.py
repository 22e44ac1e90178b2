#!/usr/bin/env python3
"""Build profiles/pmc_valu.json (the VALU counter summaries bench.py's config-4/5 rooflines read) from
tools/gpu_step.sh pmc:... output:

    python tools/valu_roofline.py gpurun_out/pmc_sample:sample:125000000 gpurun_out/pmc_fit:fit:52488000 \
        gpurun_out/pmc_he_after:evalpdf:10000000 > profiles/pmc_valu.json
    python tools/valu_roofline.py --merge profiles/pmc_valu.json profiles/r04_pmc_models:models:10000000 > new.json

Each argument is <dir>:<workload>:<units per dispatch>; every <dir>/<model>.json (tools/pmc_summary.py output for
the workload's kernel) becomes workloads["<workload>:<model>"] with
  valu_lane_instr_per_unit = SQ_INSTS_VALU x 64 / units   (wave instructions x lanes: issue slots per unit)
  issue_frac = SQ_INSTS_VALU / (dispatch_ns x 1.2288e12)   (the chip's VALU issue rate: 256 CUs x 4 SIMDs x 0.5 x 2.4 GHz)
  valu_busy_per_active = SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES
"""
import glob
import json
import os
import sys

ISSUE_PEAK = 256 * 4 * 0.5 * 2.4e9


def main(specs):
    out = {"peak_tflops": 157.3, "issue_peak_wave_instr_per_s": ISSUE_PEAK,
           "definition": __doc__.strip().split("\n\n")[-1], "workloads": {}}
    if specs and specs[0] == "--merge":       # keep an existing summary's workloads, replace / add the given ones
        with open(specs[1]) as f:
            out["workloads"] = json.load(f).get("workloads", {})
        specs = specs[2:]
    for spec in specs:
        d, workload, units = spec.rsplit(":", 2)
        units = float(units)
        for f in sorted(glob.glob(os.path.join(d, "*.json"))):
            if f.endswith(".bench.json"):
                continue
            model = os.path.basename(f)[:-5]
            c = json.load(open(f))
            if "SQ_INSTS_VALU" not in c:
                continue
            e = {"source": f"{os.path.basename(d)}/{model}.json", "units_per_dispatch": units,
                 "dispatch_ns": c.get("dispatch_ns"),
                 "valu_lane_instr_per_unit": c["SQ_INSTS_VALU"] * 64 / units,
                 "issue_frac": c["SQ_INSTS_VALU"] / (c["dispatch_ns"] * 1e-9 * ISSUE_PEAK),
                 "counters": {k: v for k, v in c.items() if k.startswith("SQ_") or k.startswith("GRBM_")}}
            if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c and c["SQ_ACTIVE_INST_VALU"]:
                e["valu_active_lane_frac"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
            out["workloads"][f"{workload}:{model}"] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
