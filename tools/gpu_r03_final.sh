#!/bin/bash
# Round-3 evidence in one call: all GPU tests; VALU counters (headline, He family, configs 4 / 5, lane utilisation)
# -> gpurun_out/pmc_valu.json (copied over profiles/pmc_valu.json in the box's tree, so the config-4/5 rooflines pair
# this build's counters with this build's times); the headline bench + rocprof + PMC traffic + configs 3-5 + f64
# (tools/gpu_final.sh); the 12.5 M-pair shard (one rank of the 8-GPU strong-scaled config) graph-timed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
bash tools/gpu_r03_pmc.sh > gpurun_out/pmc_r03.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_r03.log; exit 1; }
WORKLOAD=fit MODELS="Aggregate" KERNEL="k_loss<" EXTRA_PASS="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES" bash tools/gpu_pmc_workload.sh > gpurun_out/pmc_fit.log 2>&1 || { echo "pmc fit failed"; tail -20 gpurun_out/pmc_fit.log; exit 1; }
python3 tools/valu_roofline.py gpurun_out/pmc_headline:evalpdf:100000000 gpurun_out/pmc_sample:sample:125000000 \
  gpurun_out/pmc_fit:fit:52488000 gpurun_out/pmc_he_r03:evalpdf:10000000 > gpurun_out/pmc_valu.json || exit 1
cp gpurun_out/pmc_valu.json profiles/pmc_valu.json || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_valu.json'))
for k,v in d['workloads'].items(): print(k, '%.0f VALU/unit'%v['valu_lane_instr_per_unit'], 'issue %.3f'%v['issue_frac'], 'lanes %s'%v.get('valu_active_lane_frac'))"
bash tools/gpu_final.sh || exit 1
timeout -k 10 300 python bench.py --pairs 12500000 --graph on --steps 40 --warmup 5 > gpurun_out/final/bench_12m5.json 2> gpurun_out/final/bench_12m5.err || { echo "12.5M failed"; tail gpurun_out/final/bench_12m5.err; exit 1; }
cut -c1-400 gpurun_out/final/bench_12m5.json
