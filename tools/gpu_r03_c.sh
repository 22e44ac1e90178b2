#!/bin/bash
# Round 3: exp gather A/B on the headline, then the config-4 sample workload with the new erfinv vs erfv1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AB_LIBS="default nogather expdn" ROUNDS=3 bash tools/gpu_r03_ab.sh || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_check.py -k "sample or check or Check" > gpurun_out/erf_tests.log 2>&1 || { tail -30 gpurun_out/erf_tests.log; exit 1; }
tail -2 gpurun_out/erf_tests.log
grep -h '"CookTorrance' gpurun_out/parity_sample_large.json | head -3
AB_LIBS="default erfv1" WORKLOADS=sample bash tools/gpu_ab_work.sh
