#!/bin/bash
# Round 3 counters: the headline kernel's VALU counters (k_eval_pdf_v4<CookTorrance>) and VALU lane utilisation
# (SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64), the VALUUtilization metric of rocprofiler's counter_defs)
# for the He family (eval+pdf, 10 M pairs) and config 4.  One counter group per rocprofv3 pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
LANE="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES"
OUT="$R/gpurun_out/pmc_headline"; mkdir -p "$OUT/CookTorrance"
cd /tmp && export TMPDIR=/tmp
for P in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64" "$LANE"; do
  tag=$(echo $P | cut -d' ' -f1)-$(echo $P | wc -w)
  timeout -k 10 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/CookTorrance/$tag" -o run -- python3 "$R/bench.py" --model CookTorrance --steps 3 --warmup 1 --settle-s 0 --no-cpu --no-exact > "$OUT/CookTorrance/$tag.log" 2>&1 || { echo "pmc headline $tag failed"; tail -5 "$OUT/CookTorrance/$tag.log"; exit 1; }
done
(cd "$R" && python3 tools/pmc_summary.py "$OUT/CookTorrance" k_eval_pdf_v4 > "$OUT/CookTorrance.json") || exit 1
echo "== headline"; cat "$OUT/CookTorrance.json"
cd "$R"
MODELS="${HE_MODELS:-HeWestin He NganHe HeHolzschuch}" TAG=r03 EXTRA_PASS="$LANE" bash tools/gpu_he_pmc.sh || exit 1
cd "$R"
WORKLOAD=sample MODELS="CookTorrance GGX" KERNEL="k_check<" EXTRA_PASS="$LANE" bash tools/gpu_pmc_workload.sh || exit 1
