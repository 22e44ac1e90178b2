#!/bin/bash
# Round 3: full GPU suite on the ABI-8 tree (nested / f64 composed aggregates, glibc-exact expf in Beckmann), the
# Beckmann models' per-lane parity statistics, and the interleaved bench A/B of the three exponentials.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "pytest rc $rc: stopping"; exit 1; }
M=${PARITY_MODELS:-CookTorrance,NganCookTorrance,CookTorranceHeitz,LowCookTorrance}
timeout -k 10 400 python -u tools/parity_diag.py --models "$M" --out gpurun_out/r03_parity_exp.npz > gpurun_out/r03_parity_exp.log 2>&1 || { echo parity failed; tail -20 gpurun_out/r03_parity_exp.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03_parity_exp.json'))
for k,v in d.items(): print(k, v['bad_lanes'], v['explained_by_2ulp_inputs'], '%.2e'%v['max_rel_normal'], '%.6f'%v['frac_bit_exact'])"
for round in 1 2 3; do
  for V in BBM_HIP_NT=1 BBM_HIP_LIB=bbm_amd/lib_ab/exprn/libbbm_hip.so BBM_HIP_LIB=bbm_amd/lib_ab/expdn/libbbm_hip.so; do
    env $V timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu --model CookTorrance > gpurun_out/v.json 2>gpurun_out/v.err || { echo "variant $V failed"; tail gpurun_out/v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('r$round $V', '%.4e'%d['value'], 'frac %.4f'%d['roofline']['frac'], '%.4f ms'%d['roofline']['kernel_ms'])"
  done
done
exit $rc
