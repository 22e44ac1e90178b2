#!/bin/bash
# Round 3: full GPU suite after sqrt_nr / div_nr_n / f64 He series; headline A/B vs the round-2 exponential; the
# f64 He A/B; Beckmann parity statistics.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "pytest rc $rc: stopping"; exit 1; }
AB_LIBS="default expdn" ROUNDS=3 bash tools/gpu_r03_ab.sh || exit 1
for round in 1 2; do
  for V in default hev1; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    env $lib timeout -k 10 200 python bench.py --workload f64 --models He,HeWestin,HeHolzschuch,NganHe --pairs 10000000 --steps 5 --warmup 2 > gpurun_out/f.json 2>gpurun_out/f.err || { echo "f64 $V failed"; tail gpurun_out/f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/f.json'))
print('r$round $V', ' '.join('%s %.3f ms'%(k,v['kernel_ms']) for k,v in d['per_model_10M'].items()))"
  done
done
M=CookTorrance,NganCookTorrance,CookTorranceHeitz,GGX,Ward,Bagher
timeout -k 10 400 python -u tools/parity_diag.py --models "$M" --out gpurun_out/r03_parity_d.npz > gpurun_out/r03_parity_d.log 2>&1 || { echo parity failed; tail -20 gpurun_out/r03_parity_d.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03_parity_d.json'))
for k,v in d.items():
  if 'backscatter' not in k: print(k, v['bad_lanes'], v['explained_by_2ulp_inputs'], '%.2e'%v['max_rel_normal'], '%.6f'%v['frac_bit_exact'])"
exit $rc
