#!/bin/bash
# A/B of library builds / env variants on the bench kernel (interleaved rounds in one call).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
grep -E "^(golden|large|sample) (CookTorrance|GGX)" gpurun_out/pytest_gpu.log | cut -c1-150 | head -20
cat gpurun_out/adapter_check.jsonl 2>/dev/null
for round in 1 2; do
for V in ${AB_VARIANTS:-"BBM_HIP_NT=1"}; do
  for M in ${BENCH_MODELS:-CookTorrance}; do
  env $(echo $V | tr "," " ") timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --model $M > gpurun_out/v.json 2>gpurun_out/v.err || { echo "variant $V failed"; tail gpurun_out/v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v.json'));print('r$round $M $V', '%.4e'%d['value'], '%.1f GB/s'%d['roofline']['achieved'], 'frac %.3f'%d['roofline']['frac'], '%.3f ms'%d['roofline']['kernel_ms'])"
  done
done
done
