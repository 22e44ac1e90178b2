#!/bin/bash
# PMC HBM-traffic passes for the bench kernel (one counter group per rocprofv3 run, as
# MI355X_MICROARCH.md prescribes), summarised into gpurun_out/traffic.json (copy to profiles/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
M=${MODEL:-CookTorrance}
mkdir -p gpurun_out/pmc_traffic
cd /tmp && export TMPDIR=/tmp
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_traffic/$P" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --settle-s 0 --no-cpu --no-exact --model $M > "$R/gpurun_out/pmc_traffic/$P.log" 2>&1 || { echo "pmc $P failed"; tail -5 "$R/gpurun_out/pmc_traffic/$P.log"; exit 1; }
done
cd "$R"
python3 tools/traffic_summary.py gpurun_out/pmc_traffic k_eval_pdf_v4 $M 100000000 > gpurun_out/traffic.json && cat gpurun_out/traffic.json
