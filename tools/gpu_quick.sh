#!/bin/bash
# Quick GPU iteration: parity tests + short bench (no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "passed|failed|golden|large" gpurun_out/pytest_gpu.log | tail -30
for M in ${BENCH_MODELS:-CookTorrance}; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --model $M > gpurun_out/bench_$M.json 2> gpurun_out/bench_$M.err || { echo bench failed; tail -20 gpurun_out/bench_$M.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$M.json'));print('$M', '%.4e pairs/s'%d['value'], '%.1f GB/s'%d['roofline']['achieved'], 'frac %.3f'%d['roofline']['frac'], '%.3f ms'%d['roofline']['kernel_ms'])"
done
