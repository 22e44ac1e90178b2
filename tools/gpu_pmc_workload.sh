#!/bin/bash
# VALU counters for the VALU-bound workloads (BASELINE configs 4 and 5; He-family eval+pdf), one counter group per
# rocprofv3 pass and one model per run, summarised per kernel into gpurun_out/pmc_<workload>/<model>.json;
# tools/valu_roofline.py turns them into profiles/pmc_valu.json.
#   WORKLOAD=sample MODELS="CookTorrance GGX" KERNEL=k_check bash tools/gpu_pmc_workload.sh
#   WORKLOAD=fit MODELS=Aggregate KERNEL=k_loss bash tools/gpu_pmc_workload.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
W=${WORKLOAD:-sample}
OUT="$R/gpurun_out/pmc_$W"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for M in ${MODELS:-CookTorrance GGX}; do
  mkdir -p "$OUT/$M"
  for P in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64" ${EXTRA_PASS:+"$EXTRA_PASS"}; do
    tag=$(echo $P | cut -d' ' -f1)
    sel=""; [ "$W" = "fit" ] || sel="--models $M"
    timeout -k 10 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/$M/$tag" -o run -- python3 "$R/bench.py" --workload $W $sel --steps 2 --warmup 1 --settle-s 0 > "$OUT/$M/$tag.log" 2>&1 || { echo "pmc $W $M $tag failed"; tail -5 "$OUT/$M/$tag.log"; exit 1; }
  done
  (cd "$R" && python3 tools/pmc_summary.py "$OUT/$M" "${KERNEL:-k_check}" > "$OUT/$M.json") || exit 1
  grep -h '^{' "$OUT/$M/SQ_INSTS_VALU.log" | tail -1 > "$OUT/$M.bench.json"
  echo "== $W $M"; cat "$OUT/$M.json"
done
