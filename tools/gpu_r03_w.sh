#!/bin/bash
# Default-mode quotients on the subnormal grid in f32 (BBM_HIP_SUB_SCALED=1: scaled numerator; =2: + round to odd)
# against the current default: headline kernel time (interleaved), and the default mode's bit-exact fraction from
# the exact-subnormal test (frac_bit_exact_default_mode per Beckmann model and parameter set)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/w
AB_LIBS="default sc1 sc2" ROUNDS=3 BENCH_ARGS="--no-exact" bash tools/gpu_r03_ab.sh || exit 1
for V in default sc1 sc2; do
  lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
  env $lib timeout -k 10 600 python -u -m pytest -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "exact_subnormal or large_batch" > gpurun_out/w/tests_$V.log 2>&1; rc=$?
  tail -1 gpurun_out/w/tests_$V.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/w/tests_$V.log | head -10; }
  mkdir -p gpurun_out/w/$V; cp gpurun_out/parity_exact_*.json gpurun_out/parity_large_*.json gpurun_out/w/$V/ 2>/dev/null
  python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/w/$V/parity_exact_*.json')):
    d=json.load(open(f)); print('$V', f[-7:-5], ' '.join('%s %.6f'%(k, v['frac_bit_exact_default_mode']) for k,v in d.items()))
for f in sorted(glob.glob('gpurun_out/w/$V/parity_large_*.json')):
    d=json.load(open(f)); print('$V large', f[-7:-5], ' '.join('%s %s/%.5f'%(k, v['lanes_outside_bar'], v['frac_bit_exact']) for k,v in d.items() if 'CookTorrance' in k))"
done
rm -rf gpurun_out/gpu_outputs
