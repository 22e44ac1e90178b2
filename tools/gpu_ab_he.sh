#!/bin/bash
# A/B of library variants on the He-family eval+pdf kernels (10M pairs), interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for round in 1 2; do
  for V in ${AB_LIBS:-default w4}; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    for M in ${BENCH_MODELS:-HeWestin He HeHolzschuch}; do
      env $lib timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --pairs 10000000 --model $M > gpurun_out/v.json 2>gpurun_out/v.err || { echo "variant $V $M failed"; tail gpurun_out/v.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('r$round $V $M', '%.3f ms'%d['roofline']['kernel_ms'])"
    done
  done
done
