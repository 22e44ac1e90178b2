#!/bin/bash
# rocprofv3 kernel-trace summary of the config-3 bench on the final tree -> gpurun_out/final/prof_models
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/final/prof_models" -o run -- python3 "$R/bench.py" --workload models --steps 5 --warmup 2 > "$R/gpurun_out/final/prof_models.log" 2>&1 || { echo "rocprof models failed"; tail -20 "$R/gpurun_out/final/prof_models.log"; exit 1; }
cd "$R"
find gpurun_out/final/prof_models -name "*kernel_stats.csv"
