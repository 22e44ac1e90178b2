#!/bin/bash
# exact-subnormal mode: its parity test, the whole GPU suite, and the headline with the mode off / on (interleaved)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r
timeout -k 10 600 python -u -m pytest -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_parity.py -k exact > gpurun_out/r/exact_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r/exact_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r/exact_tests.log | head -20; exit $rc; }
python3 -c "
import json
for f in ['exact_01','exact_00']:
    d=json.load(open('gpurun_out/parity_%s.json'%f))
    for k,v in d.items(): print(f, k, '%.2e'%v['max_rel_normal'], v['lanes_outside_bar'], '%.6f'%v['frac_bit_exact'], 'default %.6f'%v['frac_bit_exact_default_mode'])
"
for round in 1 2 3; do
  for V in off on; do
    e=0; [ $V = on ] && e=1
    BBM_HIP_EXACT_SUBNORMALS=$e timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu > gpurun_out/v.json 2>gpurun_out/v.err || { echo "bench $V failed"; tail gpurun_out/v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('r$round exact=$V', '%.4e'%d['value'], 'frac %.4f'%d['roofline']['frac'], '%.4f ms'%d['roofline']['kernel_ms'])"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/r/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r/pytest_gpu.log; [ $rc -eq 0 ] || grep -E "^E |FAILED" gpurun_out/r/pytest_gpu.log | head -30
rm -rf gpurun_out/gpu_outputs
exit $rc
