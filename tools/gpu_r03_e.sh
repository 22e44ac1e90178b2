#!/bin/bash
# Round 3: headline occupancy A/B; He two-phase (sorted series) vs one-phase; He parity.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AB_LIBS="default ctw6 ctw8 expdn" ROUNDS=3 bash tools/gpu_r03_ab.sh || exit 1
for round in 1 2; do
  for V in default he1p; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    env $lib timeout -k 10 200 python bench.py --workload models --models He,HeWestin,HeHolzschuch,NganHe --steps 5 --warmup 2 > gpurun_out/m.json 2>gpurun_out/m.err || { echo "models $V failed"; tail gpurun_out/m.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/m.json'))
print('r$round $V', ' '.join('%s %.3f ms'%(k,v['kernel_ms']) for k,v in d['per_model'].items()))"
  done
done
for round in 1 2; do
  for V in default lobedn; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    env $lib timeout -k 10 200 python bench.py --workload models --models Ward,WardDuer,NganWard,Bagher,EPD --steps 5 --warmup 2 > gpurun_out/m.json 2>gpurun_out/m.err || { echo "models $V failed"; tail gpurun_out/m.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/m.json'))
print('r$round $V', ' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model'].items()))"
  done
done
AB_LIBS="default" WORKLOADS=sample ROUNDS=1 bash tools/gpu_ab_work.sh
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fits.py tests/test_gpu_aggregate.py -k "large or golden or fits or He or composed" > gpurun_out/he_tests.log 2>&1; rc=$?
tail -3 gpurun_out/he_tests.log
python3 -c "
import json
for f in ['gpurun_out/parity_large_00.json','gpurun_out/parity_large_01.json']:
    d=json.load(open(f))
    for k,v in d.items():
        if 'He' in k: print(f[-7:-5], k, '%.2e'%v['max_rel_normal'], v['lanes_outside_bar'], v['proven_by'], '%.5f'%v['frac_bit_exact'])
"
exit $rc
