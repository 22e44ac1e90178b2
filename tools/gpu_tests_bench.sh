#!/bin/bash
# All GPU tests, then the headline bench line (with the CPU leg) and the He-family eval+pdf times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-200 gpurun_out/bench.json; python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['cpu_baseline'])"
for M in HeWestin NganHe He HeHolzschuch Bagher EPD; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --pairs 10000000 --model $M > gpurun_out/v.json 2>gpurun_out/v.err || { tail gpurun_out/v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('$M', '%.3f ms'%d['roofline']['kernel_ms'])"
done
