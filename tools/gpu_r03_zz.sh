#!/bin/bash
# floatRGB PhongWalter: the Phong G1 quotient by f_div_d (default) vs the IEEE double division (phieee); parity

set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/z
for round in 1 2 3; do
  for V in default phieee; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    env $lib timeout -k 10 200 python bench.py --workload models --models PhongWalter,CookTorranceHeitz --steps 5 --warmup 2 > gpurun_out/m.json 2>gpurun_out/m.err || { echo "models $V failed"; tail gpurun_out/m.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/m.json'))
print('r$round $V', ' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model'].items()))"
  done
done
timeout -k 10 600 python -u -m pytest -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "large_batch or golden or sample or reflectance" > gpurun_out/z/tests.log 2>&1; rc=$?
tail -3 gpurun_out/z/tests.log; [ $rc -eq 0 ] || grep -E "^E |FAILED" gpurun_out/z/tests.log | head -20
python3 -c "
import json
for f in ['parity_large_00.json','parity_large_01.json','parity_golden.json']:
    d=json.load(open('gpurun_out/'+f))
    for k,v in d.items():
        if k.startswith('PhongWalter'): print(f[:-5], k, '%.2e'%v['max_rel_normal'], v['lanes_outside_bar'], v.get('proven_by'), '%.5f'%v['frac_bit_exact'])
"
rm -rf gpurun_out/gpu_outputs
exit $rc
