#!/bin/bash
# GPU round: all parity tests, then the bench workloads (configs 2-5).  Each step under its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -40
[ $rc -eq 0 ] || [ -n "$CONTINUE_ON_FAIL" ] || exit $rc
for W in ${WORKLOADS:-models sample fit}; do
  timeout -k 10 300 python bench.py --workload $W --steps ${STEPS:-10} --warmup 3 > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err || { echo "bench $W failed"; tail -20 gpurun_out/bench_$W.err; exit 1; }
  cut -c1-600 gpurun_out/bench_$W.json
done
