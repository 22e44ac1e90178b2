#!/bin/bash
# f64 heavy models one pair per thread at 1-4 waves/SIMD; last-bit diagnostics of the Beckmann models
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for V in default f64hw1 f64hw3 f64hw4; do
  lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
  env $lib timeout -k 10 300 python bench.py --workload f64 --models He,HeWestin,HeHolzschuch,NganHe --steps 5 --warmup 2 --no-cpu > gpurun_out/f.json 2>gpurun_out/f.err || { echo "f64 $V failed"; tail gpurun_out/f.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/f.json'))
print('f64 $V', ' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model_10M'].items()))"
done
for ms in "CookTorrance 0" "CookTorrance 3" "Ward 0" "GGX 0"; do
  timeout -k 10 200 python tools/bitexact_diag.py $ms 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_f64.py -k "large or golden" > gpurun_out/f64he.log 2>&1; rc=$?
tail -2 gpurun_out/f64he.log
exit $rc
