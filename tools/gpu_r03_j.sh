#!/bin/bash
# exact subnormal division fallback (divsub) vs default: headline time, config 4, bit-exact fractions
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AB_LIBS="default divsub" ROUNDS=3 bash tools/gpu_r03_ab.sh || exit 1
AB_LIBS="default divsub" WORKLOADS=sample ROUNDS=1 bash tools/gpu_ab_work.sh || exit 1
M=CookTorrance,NganCookTorrance,CookTorranceHeitz,GGX,Ward,LowCookTorrance
for V in default divsub; do
  lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
  env $lib timeout -k 10 400 python -u tools/parity_diag.py --models "$M" --out gpurun_out/r03_parity_$V.npz > gpurun_out/r03_parity_$V.log 2>&1 || { echo parity failed; tail -20 gpurun_out/r03_parity_$V.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_parity_$V.json'))
for k,v in d.items():
  if 'backscatter' not in k and 'golden' not in k: print('$V', k, v['bad_lanes'], '%.2e'%v['max_rel_normal'], '%.6f'%v['frac_bit_exact'], v['max_ulp'])"
done
