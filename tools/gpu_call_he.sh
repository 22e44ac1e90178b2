#!/bin/bash
# He-family iteration: GPU parity (all models, aggregates), adapter_check, He VALU counters (TAG), counter list.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_aggregate.py -m gpu -q --timeout 600 --timeout-method thread -k "not cpp_adapter" > gpurun_out/pytest_parity.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_parity.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_parity.log | head -30; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 500 ./tests/cpp/_build/adapter_check > gpurun_out/adapter_check.jsonl 2> gpurun_out/adapter_check.err
rc=$?
echo "adapter_check rc=$rc"; grep '"ok": false' gpurun_out/adapter_check.jsonl | cut -c1-400; head -40 gpurun_out/adapter_check.err
[ $rc -le 1 ] || exit $rc
TAG=${TAG:-iter} bash tools/gpu_he_pmc.sh || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/counters_avail.txt" 2>&1; echo "list rc=$?"
