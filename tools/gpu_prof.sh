#!/bin/bash
# Profiling pass on the GPU box: roofline probe, grid sweep, PMC counters for the bench kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
R="$GRAFT_REPO_ROOT"
echo "== roofprobe"
timeout -k 10 300 python tools/roofprobe.py > gpurun_out/roofprobe.txt 2>&1 || { echo roofprobe failed; tail -20 gpurun_out/roofprobe.txt; exit 1; }
cat gpurun_out/roofprobe.txt
echo "== grid sweep"
for B in 1024 2048 4096 8192 16384 100000; do
  BBM_HIP_MAX_BLOCKS=$B timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/sweep_$B.json 2>/dev/null || { echo "sweep $B failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sweep_$B.json'));print('blocks=$B', '%.3e'%d['value'], '%.1f GB/s'%d['roofline']['achieved'], '%.3f ms'%d['roofline']['kernel_ms'])"
done
cd /tmp && export TMPDIR=/tmp
echo "== counters"
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1 || echo "listing failed (non-fatal)"
grep -oE "(SQ|TCC|TCP|GRBM|TA|TD)_[A-Z0-9_]+" "$R/gpurun_out/pmc/counters.txt" | sort -u > "$R/gpurun_out/pmc/counter_names.txt" || true
wc -l "$R/gpurun_out/pmc/counter_names.txt"
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  tag=$(echo $P | cut -d' ' -f1)
  echo "-- pmc $P"
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/$tag" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc/$tag.log" 2>&1 || { echo "pmc $tag failed"; tail -5 "$R/gpurun_out/pmc/$tag.log"; exit 1; }
done
echo done
