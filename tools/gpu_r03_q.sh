#!/bin/bash
# exp_tab in the He series (f32 and f64) + the concave Westin exit in f64 (default) against exp_dd (hedd);
# exact subnormal-safe quotients at the three CookTorrance sites (divcr) against div_nr: time and bit-exactness.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/q
AB_LIBS="default divcr" ROUNDS=3 bash tools/gpu_r03_ab.sh || exit 1
for round in 1 2; do
  for V in default hedd f64poly; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    if [ "$V" != f64poly ]; then
    env $lib timeout -k 10 200 python bench.py --workload models --models He,HeWestin,HeHolzschuch,NganHe --steps 5 --warmup 2 > gpurun_out/m.json 2>gpurun_out/m.err || { echo "models $V failed"; tail gpurun_out/m.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/m.json'))
print('f32 r$round $V', ' '.join('%s %.4f ms'%(k,v['kernel_ms']) for k,v in d['per_model'].items()))"
    fi
    env $lib timeout -k 10 300 python bench.py --workload f64 --models 'He,HeWestin,HeHolzschuch,NganHe,Bagher,Aggregate<Lambertian,Bagher>,CookTorrance,Ribardiere,EPD' --steps 5 --warmup 2 --no-cpu > gpurun_out/f.json 2>gpurun_out/f.err || { echo "f64 $V failed"; tail gpurun_out/f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/f.json'))
print('f64 r$round $V', ' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model_10M'].items()))"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/q/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/q/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/q/pytest_gpu.log | head -30; }
cp gpurun_out/parity_large_0*.json gpurun_out/q/ ; for f in gpurun_out/parity_f64_large_0*.json; do cp $f gpurun_out/q/; done
BBM_HIP_LIB=bbm_amd/lib_ab/divcr/libbbm_hip.so timeout -k 10 600 python -u -m pytest -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "large_batch or golden" > gpurun_out/q/divcr_tests.log 2>&1; rc2=$?
tail -3 gpurun_out/q/divcr_tests.log
for f in gpurun_out/parity_large_0*.json; do cp $f gpurun_out/q/divcr_$(basename $f); done
python3 -c "
import json
for tag in ['', 'divcr_']:
  for f in ['parity_large_00.json','parity_large_01.json']:
    d=json.load(open('gpurun_out/q/'+tag+f))
    for k,v in d.items():
        if k.startswith(('CookTorrance[','He','NganHe','Aggregate<Lambertian,CookTorrance>')): print(tag or 'default', f[-7:-5], k, '%.2e'%v['max_rel_normal'], v['lanes_outside_bar'], '%.5f'%v['frac_bit_exact'])
"
rm -rf gpurun_out/gpu_outputs
exit $((rc + rc2))
