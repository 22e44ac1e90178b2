#!/bin/bash
# Round-end evidence on one MI355X: headline bench (with the CPU leg), its rocprofv3 kernel-trace summary,
# the PMC HBM-traffic passes, and the config 3-5 benches.  Every GPU step under its own limit, chained.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 300 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { echo "bench failed"; tail -20 gpurun_out/final/bench.err; exit 1; }
cut -c1-300 gpurun_out/final/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/final/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu --no-exact > "$R/gpurun_out/final/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/final/prof.log"; exit 1; }
cd "$R"
bash tools/gpu_traffic.sh || exit 1
for W in models sample fit f64; do
  timeout -k 10 300 python bench.py --workload $W --steps 10 --warmup 3 > gpurun_out/final/bench_$W.json 2> gpurun_out/final/bench_$W.err || { echo "bench $W failed"; tail -20 gpurun_out/final/bench_$W.err; exit 1; }
  cut -c1-200 gpurun_out/final/bench_$W.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/final/prof_models" -o run -- python3 "$R/bench.py" --workload models --steps 5 --warmup 2 > "$R/gpurun_out/final/prof_models.log" 2>&1 || { echo "rocprof models failed"; tail -20 "$R/gpurun_out/final/prof_models.log"; exit 1; }
cd "$R"
find gpurun_out/final/prof gpurun_out/final/prof_models -name "*kernel_stats.csv" | head -3
