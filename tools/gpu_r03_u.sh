#!/bin/bash
# doubleRGB: Student-T fast divisions / rsqrt (fdiv), Bagher parameters kept in VGPRs (vparam) = both; + microfacet fast
# halfway / Fresnel / scale divisions = all; then the f64 parity tests on all
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/u
for round in 1 2 3; do
  for V in default all; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    env $lib timeout -k 10 300 python bench.py --workload f64 --models 'Bagher,Aggregate<Lambertian,Bagher>,Ribardiere,RibardiereAnisotropic,CookTorrance,GGX,CookTorranceHeitz,PhongWalter' --steps 5 --warmup 2 --no-cpu > gpurun_out/f.json 2>gpurun_out/f.err || { echo "f64 $V failed"; tail gpurun_out/f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/f.json'))
print('f64 r$round $V', ' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model_10M'].items()))"
  done
done
BBM_HIP_LIB=bbm_amd/lib_ab/all/libbbm_hip.so timeout -k 10 600 python -u -m pytest -q --timeout 500 --timeout-method thread -m gpu tests -k "f64" > gpurun_out/u/f64_tests.log 2>&1; rc=$?
tail -3 gpurun_out/u/f64_tests.log; [ $rc -eq 0 ] || grep -E "^E |FAILED" gpurun_out/u/f64_tests.log | head -20
rm -rf gpurun_out/gpu_outputs
exit $rc
