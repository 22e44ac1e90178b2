#!/bin/bash
# Submit one gpurun call, resubmitting only while the pool reports that nothing ran (exit 3: no box / slot free,
# or status "transient" with run_s 0: the box failed before the command started).  A call whose command ran --
# pass or fail -- is never repeated.  Waits as long as the pool's own back-off hint ("retry in Ns"), at least 120 s.
#   tools/gpurun_retry.sh TIMEOUT_S 'COMMAND'
t=$1; shift
log=$(mktemp)
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1 | tee "$log"
  rc=${PIPESTATUS[0]}
  nothing_ran=$(python3 -c "
import json
try:
    d = json.load(open('gpurun_out/.last_call.json'))
    print(int(d.get('status') == 'transient' and not d.get('run_s')))
except Exception:
    print(0)")
  if [ "$rc" -ne 3 ] && [ "$nothing_ran" != 1 ]; then rm -f "$log"; exit "$rc"; fi
  hint=$(grep -o 'retry in [0-9]*s' "$log" | tail -1 | grep -o '[0-9]*')
  wait_s=$(( ${hint:-0} + 20 ))
  [ "$wait_s" -lt 120 ] && wait_s=120
  echo "[retry] nothing ran (rc=$rc), attempt $i; waiting $wait_s s"
  sleep "$wait_s"
done
rm -f "$log"
exit 3
