#!/bin/bash
# Round-end evidence in one call: all GPU tests, the VALU counters of configs 4/5 and the He family
# (tools/gpu_valu.sh; copied over profiles/pmc_valu.json in the box's tree first, so the config-4/5 rooflines
# below pair this build's counters with this build's times), then the headline bench + rocprof + PMC traffic +
# configs 3-5 (tools/gpu_final.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
TAG=final bash tools/gpu_he_pmc.sh > /dev/null || exit 1
HE_DIR=gpurun_out/pmc_he_final bash tools/gpu_valu.sh || exit 1
cp gpurun_out/pmc_valu.json profiles/pmc_valu.json || exit 1
bash tools/gpu_final.sh || exit 1
