#!/bin/bash
# After the doubleRGB quotient work: every GPU test on the default build, then the doubleRGB bench line (CookTorrance
# 100 M pairs + every f64 model over 10 M pairs, graph-timed) -> gpurun_out/v/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/v
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/v/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/v/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/v/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py --workload f64 --steps 10 --warmup 3 > gpurun_out/v/bench_f64.json 2> gpurun_out/v/bench_f64.err || { echo "f64 bench failed"; tail gpurun_out/v/bench_f64.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/v/bench_f64.json'))
print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])
for k,v in sorted(d['per_model_10M'].items(), key=lambda kv: kv[1]['roofline_frac']): print('%-45s %.4f %.3f'%(k, v['kernel_ms'], v['roofline_frac']))"
rm -rf gpurun_out/gpu_outputs
