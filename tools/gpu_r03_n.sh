#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
for V in default bagf4; do
  lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
  env $lib timeout -k 10 300 python bench.py --workload f64 --models 'Bagher,Aggregate<Lambertian,Bagher>,EPD,Ribardiere,He,HeWestin,HeHolzschuch,NganHe,CookTorrance' --steps 5 --warmup 2 --no-cpu > gpurun_out/f.json 2>gpurun_out/f.err || { echo "f64 $V failed"; tail gpurun_out/f.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/f.json'))
print('r$r f64 $V', ' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model_10M'].items()))"
done
done
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_f64.py -k "large or golden or sample" > gpurun_out/f64he.log 2>&1; rc=$?
tail -2 gpurun_out/f64he.log
exit $rc
