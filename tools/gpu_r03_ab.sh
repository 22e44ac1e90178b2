#!/bin/bash
# Interleaved bench A/B of library variants on --model (default CookTorrance): AB_LIBS = names under bbm_amd/lib_ab
# ("default" = bbm_amd/lib), ROUNDS rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for round in $(seq 1 ${ROUNDS:-3}); do
  for V in ${AB_LIBS:-default}; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    env $lib timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu --model ${MODEL:-CookTorrance} ${BENCH_ARGS} > gpurun_out/v.json 2>gpurun_out/v.err || { echo "variant $V failed"; tail gpurun_out/v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('r$round $V', '%.4e'%d['value'], 'frac %.4f'%d['roofline']['frac'], '%.4f ms'%d['roofline']['kernel_ms'])"
  done
done
