#!/bin/bash
# One parameterised runner for every GPU step (replaces the per-call lease scripts of rounds 1-3).
# Each step runs under its own time limit; the first failing step ends the call (no retries).
#
#   bash tools/gpu_step.sh STEP [STEP ...]
#
# STEP (arguments after ':' separated by ','):
#   tests[:PYTEST_K]             pytest -m gpu (optionally -k PYTEST_K) -> gpurun_out/pytest_gpu.log
#   bench:TAG[,ARGS...]          python bench.py ARGS -> gpurun_out/bench_TAG.json (e.g. bench:ggx,--model,GGX)
#   stats:TAG[,ARGS...]          rocprofv3 --kernel-trace --stats around bench.py ARGS -> gpurun_out/stats_TAG/
#   traffic:MODEL[,PAIRS]        FETCH_SIZE / WRITE_SIZE passes of the eval+pdf kernel -> gpurun_out/traffic_MODEL.json
#   pmc:WORKLOAD,KERNEL,UNITS,M1[,M2...]  VALU counter passes, one model per run -> gpurun_out/pmc_WORKLOAD/M.json
#   ab:TAG,ROUNDS,LIBS...        interleaved A/B of library builds (bbm_amd/lib_ab/<LIB>) with bench.py $AB_ARGS
#   py:TAG,SCRIPT[,ARGS...]      python SCRIPT ARGS -> gpurun_out/py_TAG.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SQ8="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64"
LANE="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES"
# PMC_WAIT=1: a third pass -- where the wave cycles go (parked on s_waitcnt, issue-stalled, issuing) and the
# GPU-busy cycles (GRBM_GUI_ACTIVE summed over the 8 XCDs: / 8 / dispatch time = the clock the kernel ran at)
WAIT="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"

step_tests() {
  local k=()
  [ -n "$1" ] && k=(-k "$1")
  timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s -x --timeout 300 --timeout-method thread "${k[@]}" \
      > gpurun_out/pytest_gpu.log 2>&1
  local rc=$?
  grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -20
  return $rc
}

step_bench() {
  local tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > "gpurun_out/bench_$tag.json" 2> "gpurun_out/bench_$tag.err" \
      || { echo "bench $tag failed"; tail -20 "gpurun_out/bench_$tag.err"; return 1; }
  cut -c1-900 "gpurun_out/bench_$tag.json"
}

step_stats() {
  local tag=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/stats_$tag" -o run -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/stats_$tag.log" 2>&1) \
      || { echo "stats $tag failed"; tail -20 "gpurun_out/stats_$tag.log"; return 1; }
  find "gpurun_out/stats_$tag" -name "*kernel_stats.csv" -exec cut -c1-200 {} \; | head -8
}

step_traffic() {
  local m=$1 pairs=${2:-100000000}
  mkdir -p "gpurun_out/pmc_traffic_$m"
  for P in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --pmc $P --kernel-trace --output-format csv \
        -d "$R/gpurun_out/pmc_traffic_$m/$P" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --settle-s 0 \
        --no-cpu --no-exact --graph off --model "$m" --pairs "$pairs" > "$R/gpurun_out/pmc_traffic_$m/$P.log" 2>&1) \
        || { echo "pmc $P failed"; tail -5 "gpurun_out/pmc_traffic_$m/$P.log"; return 1; }
  done
  python3 tools/traffic_summary.py "gpurun_out/pmc_traffic_$m" k_eval_pdf "$m" "$pairs" > "gpurun_out/traffic_$m.json" \
      && cat "gpurun_out/traffic_$m.json"
}

step_pmc() {
  local w=$1 kern=$2 units=$3; shift 3
  local out="$R/gpurun_out/pmc_$w"
  mkdir -p "$out"
  for M in "$@"; do
    mkdir -p "$out/$M"
    local sel=(--models "$M")
    case $w in
      evalpdf) sel=(--model "$M" --pairs "$units" --no-exact --graph off);;
      fit) sel=(--fit-max-steps 0);;
      models) sel=(--models "$M" --graph off);;
      sample) sel=(--models "$M" --no-exact);;    # the default sampler, not the exact-mode twin timed after it
    esac
    local passes=("$SQ8" "$LANE")
    [ -n "$PMC_WAIT" ] && passes+=("$WAIT")
    for P in "${passes[@]}"; do
      local tag
      tag=$(echo $P | cut -d' ' -f1)-$(echo $P | wc -w)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc $P --kernel-trace --output-format csv \
          -d "$out/$M/$tag" -o run -- python3 "$R/bench.py" --workload "$w" "${sel[@]}" --steps 2 --warmup 1 \
          --settle-s 0 --no-cpu > "$out/$M/$tag.log" 2>&1) \
          || { echo "pmc $w $M $tag failed"; tail -5 "$out/$M/$tag.log"; return 1; }
    done
    python3 tools/pmc_summary.py "$out/$M" "$kern" > "$out/$M.json" || return 1
    python3 - "$out/$M.json" "$units" "$M" <<'EOF'
import json, sys
c = json.load(open(sys.argv[1])); u = float(sys.argv[2])
v = c.get("SQ_INSTS_VALU", 0)
print(sys.argv[3], "valu/unit %.0f" % (v * 64 / u), "issue %.3f" % (v / (c["dispatch_ns"] * 1e-9 * 1.2288e12)),
      "lane %.3f" % (c.get("SQ_THREAD_CYCLES_VALU", 0) / max(64 * c.get("SQ_ACTIVE_INST_VALU", 1), 1)),
      "f64fma %.0f" % (c.get("SQ_INSTS_VALU_FMA_F64", 0) * 64 / u), "ms %.4f" % (c["dispatch_ns"] / 1e6))
if "SQ_WAIT_ANY" in c:
    w = max(c.get("SQ_WAVE_CYCLES", 1), 1)
    print("   wait %.3f inst-stall %.3f active %.3f  clock %.2f GHz" % (c["SQ_WAIT_ANY"] / w, c["SQ_WAIT_INST_ANY"] / w,
          c["SQ_ACTIVE_INST_ANY"] / w, c.get("GRBM_GUI_ACTIVE", 0) / 8 / c["dispatch_ns"]))
EOF
    rm -rf "${out:?}/$M"/*/   # raw CSVs: the summary above is what is kept
  done
}

step_ab() {
  local tag=$1 rounds=$2; shift 2
  for r in $(seq 1 "$rounds"); do
    for L in "$@"; do
      BBM_HIP_LIB="$R/bbm_amd/lib_ab/$L/libbbm_hip.so" timeout -k 10 300 python bench.py ${AB_ARGS:---steps 20 --warmup 3 --no-cpu --no-exact} \
          > gpurun_out/ab_v.json 2> gpurun_out/ab_v.err || { echo "ab $L failed"; tail gpurun_out/ab_v.err; return 1; }
      python3 - "$r" "$L" >> "gpurun_out/ab_$tag.txt" <<'EOF'
import json, sys
d = json.load(open("gpurun_out/ab_v.json"))
if "per_model" in d:
    for m, e in d["per_model"].items():
        print("r%s %s %s %.4f ms" % (sys.argv[1], sys.argv[2], m, e.get("kernel_ms", float("nan"))))
else:
    print("r%s %s %s %.4f ms %.4e" % (sys.argv[1], sys.argv[2], d["config"].get("model", ""), d["roofline"]["kernel_ms"], d["value"]))
EOF
    done
  done
  cat "gpurun_out/ab_$tag.txt"
}

step_py() {
  local tag=$1 script=$2; shift 2
  timeout -k 10 600 python -u "$script" "$@" > "gpurun_out/py_$tag.log" 2>&1 \
      || { echo "py $tag failed"; tail -30 "gpurun_out/py_$tag.log"; return 1; }
  tail -30 "gpurun_out/py_$tag.log"
}

for S in "$@"; do
  name=${S%%:*}
  args=""
  [ "$name" != "$S" ] && args=${S#*:}
  IFS=, read -r -a A <<< "$args"
  echo "=== $S"
  "step_$name" "${A[@]}" || { echo "step $S failed"; exit 1; }
done
