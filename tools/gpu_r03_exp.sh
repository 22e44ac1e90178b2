#!/bin/bash
# Round 3, item 1: Beckmann eval with the correctly rounded branch-free expf (default build) against the 1.4-ulp
# expf_dn (bbm_amd/lib_ab/expdn): per-lane parity of the Beckmann models, then interleaved bench A/B, then the
# VALU counters of the headline kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
M=${PARITY_MODELS:-CookTorrance,NganCookTorrance,CookTorranceHeitz}
timeout -k 10 400 python -u tools/parity_diag.py --models "$M" --out gpurun_out/r03_parity_exp.npz > gpurun_out/r03_parity_exp.log 2>&1 || { echo parity failed; tail -20 gpurun_out/r03_parity_exp.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03_parity_exp.json'))
for k,v in d.items(): print(k, v['bad_lanes'], v['explained_by_2ulp_inputs'], '%.2e'%v['max_rel_normal'], '%.6f'%v['frac_bit_exact'])"
AB_VARIANTS=${AB_VARIANTS:-"BBM_HIP_NT=1 BBM_HIP_LIB=bbm_amd/lib_ab/expdn/libbbm_hip.so"}
for round in 1 2 3; do
  for V in $AB_VARIANTS; do
    env $V timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu --model CookTorrance > gpurun_out/v.json 2>gpurun_out/v.err || { echo "variant $V failed"; tail gpurun_out/v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('r$round $V', '%.4e'%d['value'], 'frac %.4f'%d['roofline']['frac'], '%.4f ms'%d['roofline']['kernel_ms'])"
  done
done
[ -n "$SKIP_PMC" ] && exit 0
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_ct"
R="$GRAFT_REPO_ROOT"
mkdir -p "$OUT/CookTorrance"
cd /tmp && export TMPDIR=/tmp
P="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64"
timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/CookTorrance/SQ_INSTS_VALU" -o run -- python3 "$R/bench.py" --model CookTorrance --steps 3 --warmup 1 --settle-s 0 --no-cpu > "$OUT/CookTorrance/SQ_INSTS_VALU.log" 2>&1 || { echo "pmc failed"; tail -5 "$OUT/CookTorrance/SQ_INSTS_VALU.log"; exit 1; }
cd "$R" && python3 tools/pmc_summary.py "$OUT/CookTorrance" k_eval_pdf_v4 > "$OUT/CookTorrance.json" && cat "$OUT/CookTorrance.json"
