#!/bin/bash
# Final tree: every GPU test, then config 3 (all models, graph-timed over four operand sets) and the headline line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/y
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/y/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/y/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/y/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --workload models --steps 10 --warmup 3 > gpurun_out/y/bench_models.json 2> gpurun_out/y/bench_models.err || { echo "models failed"; tail gpurun_out/y/bench_models.err; exit 1; }
cut -c1-300 gpurun_out/y/bench_models.json
timeout -k 10 300 python bench.py > gpurun_out/y/bench.json 2> gpurun_out/y/bench.err || { echo "bench failed"; tail gpurun_out/y/bench.err; exit 1; }
cut -c1-300 gpurun_out/y/bench.json
rm -rf gpurun_out/gpu_outputs
