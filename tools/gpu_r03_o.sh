#!/bin/bash
# Westin sort key (m* vs g) on the f32 He family; f64 Bagher after the squared-chord compare
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
for V in default gkey; do
  lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
  env $lib timeout -k 10 200 python bench.py --workload models --models He,HeWestin,NganHe,Bagher --steps 5 --warmup 2 > gpurun_out/m.json 2>gpurun_out/m.err || { echo "models $V failed"; tail gpurun_out/m.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/m.json'))
print('r$r $V', ' '.join('%s %.3f ms'%(k,v['kernel_ms']) for k,v in d['per_model'].items()))"
done
done
timeout -k 10 300 python bench.py --workload f64 --models 'Bagher,Aggregate<Lambertian,Bagher>' --steps 5 --warmup 2 --no-cpu > gpurun_out/f.json 2>gpurun_out/f.err || { echo "f64 failed"; tail gpurun_out/f.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/f.json'))
print('f64', ' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model_10M'].items()))"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f64.py tests/test_gpu_parity.py tests/test_gpu_fits.py -k "Bagher or He or large or fits" > gpurun_out/o_tests.log 2>&1; rc=$?
tail -3 gpurun_out/o_tests.log
exit $rc
