#!/bin/bash
# A/B of library variants on the config-4 / config-5 workloads (sample MC loop, fitting loss), interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for round in 1 2; do
  for V in ${AB_LIBS:-default}; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    for W in ${WORKLOADS:-sample fit}; do
      env $lib timeout -k 10 200 python bench.py --workload $W --steps 5 --warmup 2 > gpurun_out/w.json 2>gpurun_out/w.err || { echo "variant $V $W failed"; tail gpurun_out/w.err; exit 1; }
      python3 -c "
import json;d=json.load(open('gpurun_out/w.json'))
pm=d.get('per_model',{})
print('r$round $V $W', '%.4e %s'%(d['value'],d['unit']), ' '.join('%s %.3f ms'%(k,v['kernel_ms']) for k,v in pm.items()) or '%.3f ms'%d.get('kernel_ms',0))"
    done
  done
done
