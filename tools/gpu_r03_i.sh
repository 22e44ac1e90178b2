#!/bin/bash
# f64 He prelude / series split (heprobe: no series), Bagher f64 after the half-chord branch; f64 tests
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for V in default heprobe; do
  lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
  env $lib timeout -k 10 300 python bench.py --workload f64 --models He,HeWestin,HeHolzschuch,NganHe,Bagher,Aggregate\<Lambertian,Bagher\> --steps 5 --warmup 2 --no-cpu > gpurun_out/f.json 2>gpurun_out/f.err || { echo "f64 $V failed"; tail gpurun_out/f.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/f.json'))
print('f64 $V', ' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model_10M'].items()))"
  env $lib timeout -k 10 200 python bench.py --workload models --models He,HeWestin,HeHolzschuch,NganHe --steps 5 --warmup 2 > gpurun_out/m.json 2>gpurun_out/m.err || { echo "models $V failed"; tail gpurun_out/m.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/m.json'))
print('f32 $V', ' '.join('%s %.3f ms'%(k,v['kernel_ms']) for k,v in d['per_model'].items()))"
done
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f64.py tests/test_gpu_nested.py > gpurun_out/f64_tests.log 2>&1; rc=$?
tail -3 gpurun_out/f64_tests.log
exit $rc
