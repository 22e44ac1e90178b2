#!/bin/bash
# One iteration: parity tests, bench (2 rounds), categorised VALU counters for the bench kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc3
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
grep -E "^(golden|large|sample) (CookTorrance|GGX)" gpurun_out/pytest_gpu.log | cut -c1-120 | head -20
for round in 1 2; do for M in ${BENCH_MODELS:-CookTorrance}; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --model $M > gpurun_out/v.json 2>gpurun_out/v.err || { echo "bench failed"; tail gpurun_out/v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v.json'));print('r$round $M', '%.4e'%d['value'], '%.1f GB/s'%d['roofline']['achieved'], 'frac %.3f'%d['roofline']['frac'], '%.3f ms'%d['roofline']['kernel_ms'])"
done; done
if [ -n "$PMC" ]; then
cd /tmp && export TMPDIR=/tmp
for P in "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT"; do
  tag=$(echo $P | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$R/gpurun_out/pmc3/$tag" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc3/$tag.log" 2>&1 || { echo "pmc $tag failed"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc3" k_eval_pdf_v4
fi
