#!/bin/bash
# All GPU tests, adapter_check, then VALU counters for configs 4/5 and the He family (TAG).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; [ $rc -eq 1 ] || exit $rc; }
grep -h '"ok": false' gpurun_out/adapter_check.jsonl | cut -c1-300
HE_DIR=gpurun_out/pmc_he_${TAG:-w4} bash -c 'TAG='${TAG:-w4}' bash tools/gpu_he_pmc.sh > /dev/null && bash tools/gpu_valu.sh' || exit 1
