#!/bin/bash
# doubleRGB after the reciprocal hoists: every f64 model (10 M pairs) + the f64 headline, exp A/B (device library
# exp, Estrin polynomials), f64 parity
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 tools/bin/f64math_probe_estrin > gpurun_out/f64math_estrin.log 2>&1; head -4 gpurun_out/f64math_estrin.log
for V in default expocml estrin; do
  lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
  env $lib timeout -k 10 400 python bench.py --workload f64 --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_f64_$V.json 2>gpurun_out/bench_f64.err || { echo "f64 failed"; tail gpurun_out/bench_f64.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/bench_f64_$V.json'))
print('$V headline %.4e pairs/s %.3f ms frac %.3f'%(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']))
print('$V', ' '.join('%s %.4f %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model_10M'].items()))"
done
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f64.py tests/test_gpu_nested.py > gpurun_out/f64_tests.log 2>&1; rc=$?
tail -3 gpurun_out/f64_tests.log
exit $rc
