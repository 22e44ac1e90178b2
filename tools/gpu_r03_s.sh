#!/bin/bash
# doubleRGB Bagher P22 on exp_dd (default) vs exp_d (bexpd); f64 tests; config 5 to convergence; the headline line
# with its exact-subnormal figure
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
for round in 1 2 3; do
  for V in default bexpd; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    env $lib timeout -k 10 300 python bench.py --workload f64 --models 'Bagher,Aggregate<Lambertian,Bagher>,CookTorrance' --steps 5 --warmup 2 --no-cpu > gpurun_out/f.json 2>gpurun_out/f.err || { echo "f64 $V failed"; tail gpurun_out/f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/f.json'))
print('f64 r$round $V', ' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model_10M'].items()))"
  done
done
timeout -k 10 600 python -u -m pytest -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_f64.py tests/test_gpu_fits.py > gpurun_out/s/f64_tests.log 2>&1; rc=$?
tail -3 gpurun_out/s/f64_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/s/f64_tests.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --workload fit --steps 10 --warmup 3 > gpurun_out/s/bench_fit.json 2> gpurun_out/s/bench_fit.err || { echo "fit failed"; tail gpurun_out/s/bench_fit.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/s/bench_fit.json'));print(d['value'], d['fit'])"
timeout -k 10 300 python bench.py > gpurun_out/s/bench.json 2> gpurun_out/s/bench.err || { echo "bench failed"; tail gpurun_out/s/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/s/bench.json'));print(d['value'], d['roofline']['kernel_ms'], d['exact_subnormals_mode'])"
rm -rf gpurun_out/gpu_outputs
