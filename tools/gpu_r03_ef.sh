#!/bin/bash
# call5 + call6 in one box: stop at the first GPU fault / abort / timeout (rc > 1)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_r03_e.sh > gpurun_out/call5.log 2>&1; rc=$?
echo "call5 rc=$rc"; tail -40 gpurun_out/call5.log
[ $rc -le 1 ] || exit $rc
bash tools/gpu_r03_f.sh > gpurun_out/call6.log 2>&1; rc=$?
echo "call6 rc=$rc"; cat gpurun_out/call6.log | tail -30
exit $rc
