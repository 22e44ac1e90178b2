#!/bin/bash
# erfinv in f32 (Beckmann VNDF sampling): sample / check parity tests, then the config-4 A/B against the f64 variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_check.py tests/test_gpu_parity.py -k "sample or check or Check or reflectance" > gpurun_out/erf_tests.log 2>&1 || { tail -30 gpurun_out/erf_tests.log; exit 1; }
tail -3 gpurun_out/erf_tests.log
AB_LIBS="default erfd" WORKLOADS=sample bash tools/gpu_ab_work.sh
