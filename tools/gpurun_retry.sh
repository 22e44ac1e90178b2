#!/bin/bash
# Submit one gpurun call, resubmitting only while the pool reports that nothing ran (exit 3: no box / slot free,
# or status "transient" with run_s 0: the box failed before the command started).  A call whose command ran --
# pass or fail -- is never repeated.
#   tools/gpurun_retry.sh TIMEOUT_S 'COMMAND'
t=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  nothing_ran=$(python3 -c "
import json
try:
    d = json.load(open('gpurun_out/.last_call.json'))
    print(int(d.get('status') == 'transient' and not d.get('run_s')))
except Exception:
    print(0)")
  if [ $rc -ne 3 ] && [ "$nothing_ran" != 1 ]; then exit $rc; fi
  # honour the pool's own back-off hint ("retry in Ns"), at least 90 s
  wait_s=$(python3 -c "
import json, re
try:
    m = re.search(r'retry in (\\d+)s', json.load(open('gpurun_out/.last_call.json')).get('msg', '') or '')
    print(max(90, int(m.group(1)) + 15) if m else 90)
except Exception:
    print(90)")
  echo "[retry] nothing ran (rc=$rc), attempt $i; waiting $wait_s s"
  sleep "$wait_s"
done
exit 3
