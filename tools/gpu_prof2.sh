#!/bin/bash
# Variant sweep + categorised PMC counters for the bench kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc2
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
grep -E "^(golden|large|sample)" gpurun_out/pytest_gpu.log | awk '{print $1, $2, $3, $4, $5, $6, $7, $8, $9}' | head -60
for V in "BBM_HIP_NT=1" "BBM_HIP_NT=0" "BBM_HIP_NT=1 BBM_HIP_MAX_BLOCKS=2048" "BBM_HIP_NT=1 BBM_HIP_MAX_BLOCKS=8192"; do
  env $V timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/v.json 2>/dev/null || { echo "variant $V failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v.json'));print('$V', '%.4e'%d['value'], '%.1f GB/s'%d['roofline']['achieved'], 'frac %.3f'%d['roofline']['frac'], '%.3f ms'%d['roofline']['kernel_ms'])"
done
cd /tmp && export TMPDIR=/tmp
for P in "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $P | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$R/gpurun_out/pmc2/$tag" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc2/$tag.log" 2>&1 || { echo "pmc $tag failed"; tail -5 "$R/gpurun_out/pmc2/$tag.log"; exit 1; }
done
echo done
