#!/bin/bash
# VALU counters for BASELINE configs 4 (importance-sample MC loop, k_check) and 5 (fitting loss, k_loss), then
# gpurun_out/pmc_valu.json (copy to profiles/pmc_valu.json: bench.py's config-4/5 rooflines read it).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
WORKLOAD=sample MODELS="CookTorrance GGX" KERNEL="k_check<" bash tools/gpu_pmc_workload.sh || exit 1
WORKLOAD=fit MODELS="Aggregate" KERNEL="k_loss<" bash tools/gpu_pmc_workload.sh || exit 1
python3 tools/valu_roofline.py gpurun_out/pmc_sample:sample:125000000 gpurun_out/pmc_fit:fit:52488000 \
  ${HE_DIR:+$HE_DIR:evalpdf:10000000} > gpurun_out/pmc_valu.json && python3 -c "
import json; d=json.load(open('gpurun_out/pmc_valu.json'))
for k,v in d['workloads'].items(): print(k, '%.0f VALU/unit'%v['valu_lane_instr_per_unit'], 'issue %.3f'%v['issue_frac'], '%.3f ms'%(v['dispatch_ns']/1e6))"
