#!/bin/bash
# All GPU tests, then the config 4 / 5 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
for W in ${WORKLOADS:-sample fit}; do
  timeout -k 10 300 python bench.py --workload $W --steps 10 --warmup 3 > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err || { tail -20 gpurun_out/bench_$W.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/bench_$W.json'))
print('$W', '%.4e'%d['value'], d['unit'], ' '.join('%s %.3f ms'%(k,v['kernel_ms']) for k,v in d.get('per_model',{}).items()), 'roofline frac', d['roofline'].get('frac'))"
done
