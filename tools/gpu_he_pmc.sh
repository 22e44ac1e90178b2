#!/bin/bash
# He-family VALU counters: one counter group per rocprofv3 pass over a short bench of
# one model (10M pairs), summarised per kernel into gpurun_out/pmc_he_<TAG>/<model>.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG=${TAG:-before}
OUT="$R/gpurun_out/pmc_he_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for M in ${MODELS:-HeWestin NganHe He HeHolzschuch}; do
  for P in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64" ${EXTRA_PASS:+"$EXTRA_PASS"}; do
    tag=$(echo $P | cut -d' ' -f1); mkdir -p "$OUT/$M"
    timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/$M/$tag" -o run -- python3 "$R/bench.py" --model $M --pairs 10000000 --steps 3 --warmup 1 --settle-s 0 --no-cpu > "$OUT/$M/$tag.log" 2>&1 || { echo "pmc $M $tag failed"; tail -5 "$OUT/$M/$tag.log"; exit 1; }
  done
  (cd "$R" && python3 tools/pmc_summary.py "$OUT/$M" k_eval_pdf > "$OUT/$M.json") || exit 1
  echo "== $M"; cat "$OUT/$M.json"
done
