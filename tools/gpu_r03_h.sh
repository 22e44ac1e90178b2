#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BBM_HIP_LIB=bbm_amd/lib_ab/hegeb/libbbm_hip.so timeout -k 10 200 python tools/he_geb.py HeWestin He > gpurun_out/he_geb.log 2>&1 || { echo "he_geb failed"; tail gpurun_out/he_geb.log; exit 1; }
cat gpurun_out/he_geb.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --workload f64 --models He,HeWestin,HeHolzschuch,NganHe,Bagher --steps 5 --warmup 2 --no-cpu > gpurun_out/f.json 2>gpurun_out/f.err || { echo "f64 failed"; tail gpurun_out/f.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/f.json'))
print(' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model_10M'].items()))"
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_f64.py -k "large" > gpurun_out/f64he.log 2>&1; rc=$?
tail -2 gpurun_out/f64he.log
exit $rc
