#!/bin/bash
# Round-end evidence in one call: all GPU tests, the headline bench + rocprof + PMC traffic + configs 3-5
# (tools/gpu_final.sh), then the VALU counters of configs 4/5 and the He family (tools/gpu_valu.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
bash tools/gpu_final.sh || exit 1
TAG=final bash tools/gpu_he_pmc.sh > /dev/null || exit 1
HE_DIR=gpurun_out/pmc_he_final bash tools/gpu_valu.sh || exit 1
