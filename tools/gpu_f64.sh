#!/bin/bash
# doubleRGB evidence: the f64 parity tests, the C++ adapter check (doubleRGB model objects included), the f64
# bench and the config-3 bench (floatRGB grid caps).  Every GPU step under its own limit, chained.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_parity.py -k "f64 or adapter" -m gpu -x -v \
  --timeout 400 --timeout-method thread > gpurun_out/pytest_f64.log 2>&1
rc=$?; tail -22 gpurun_out/pytest_f64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload f64 --steps 20 --warmup 5 > gpurun_out/bench_f64.json 2> gpurun_out/bench_f64.err || { tail -5 gpurun_out/bench_f64.err; exit 1; }
cut -c1-300 gpurun_out/bench_f64.json
timeout -k 10 300 python bench.py --workload models --steps 10 --warmup 3 > gpurun_out/bench_models.json 2> gpurun_out/bench_models.err || { tail -5 gpurun_out/bench_models.err; exit 1; }
cut -c1-300 gpurun_out/bench_models.json
