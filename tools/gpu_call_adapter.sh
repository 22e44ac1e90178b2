#!/bin/bash
# GPU parity (test_gpu_parity.py), adapter_check (BBM_BACKBONE=hip drop-in: all exported models + Merl +
# aggregates + bsdf_ptr), then He-family VALU counters without (before) and with (after) live-pair compaction.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_parity.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_parity.log | head -20; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 500 ./tests/cpp/_build/adapter_check > gpurun_out/adapter_check.jsonl 2> gpurun_out/adapter_check.err
rc=$?
echo "adapter_check rc=$rc"; python3 -c "import sys,json
for l in open('gpurun_out/adapter_check.jsonl'):
    d=json.loads(l); print(('OK ' if d['ok'] else 'BAD'), d.get('model','')[:60], {k:v for k,v in d.items() if k not in ('model','ok')})"
[ $rc -le 1 ] || exit $rc
BBM_HIP_COMPACT=0 TAG=before bash tools/gpu_he_pmc.sh || exit 1
TAG=after bash tools/gpu_he_pmc.sh || exit 1
