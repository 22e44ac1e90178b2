#!/bin/bash
# tools/gpu_r03_final.sh, then the layout probe (tools/roofprobe.py: SoA streams vs the pair-array layout), then
# the bulky per-lane dumps and raw counter CSVs are dropped so gpurun_out/ stays under the 64 MiB copy-back cap
# (the summaries they fed are kept).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r03_final.sh; rc=$?
if [ $rc -eq 0 ]; then
  PROBE_VARIANTS=1,5,6,12,13,14 timeout -k 10 300 python tools/roofprobe.py > gpurun_out/roofprobe.txt 2>&1 || { echo "roofprobe failed"; tail gpurun_out/roofprobe.txt; rc=1; }
  grep -v amdgpu.ids gpurun_out/roofprobe.txt
fi
rm -rf gpurun_out/gpu_outputs
find gpurun_out -type f -size +3M ! -name "*kernel_stats.csv" -delete
du -sh gpurun_out
exit $rc
