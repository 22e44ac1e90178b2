set -o pipefail
timeout -k 10 300 tests/cpp/_build/adapter_check > gpurun_out/adapter_n.jsonl 2> gpurun_out/adapter_n.err; echo adapter rc=$?
grep -c '"ok": false' gpurun_out/adapter_n.jsonl
timeout -k 10 1100 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_n.log 2>&1; echo pytest rc=$?; tail -6 gpurun_out/pytest_n.log
mkdir -p gpurun_out/parity_n && cp gpurun_out/parity_*.json gpurun_out/parity_n/
