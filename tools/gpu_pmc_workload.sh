#!/bin/bash
# VALU / wave-occupancy counters for one bench workload (one counter group per rocprofv3 run), summarised
# per kernel into gpurun_out/pmc_<workload>/summary.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
W=${WORKLOAD:-sample}
mkdir -p gpurun_out/pmc_$W
cd /tmp && export TMPDIR=/tmp
for P in "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_CVT"; do
  tag=$(echo $P | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_$W/$tag" -o run -- python3 "$R/bench.py" --workload $W --steps 2 --warmup 1 > "$R/gpurun_out/pmc_$W/$tag.log" 2>&1 || { echo "pmc $tag failed"; tail -5 "$R/gpurun_out/pmc_$W/$tag.log"; exit 1; }
done
cd "$R"
python3 tools/pmc_summary.py "gpurun_out/pmc_$W" "${KERNEL:-k_check}" | tee "gpurun_out/pmc_$W/summary.txt"
