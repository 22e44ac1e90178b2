# Full GPU verification: the C++ adapter check against the reference, then every -m gpu test (records under gpurun_out/).
set -o pipefail
timeout -k 10 300 tests/cpp/_build/adapter_check > gpurun_out/adapter_m.jsonl 2> gpurun_out/adapter_m.err; echo adapter rc=$?
grep -c '"ok": false' gpurun_out/adapter_m.jsonl
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_m.log 2>&1; echo pytest rc=$?; tail -8 gpurun_out/pytest_m.log
mkdir -p gpurun_out/parity_m && cp gpurun_out/parity_*.json gpurun_out/parity_m/ 2>/dev/null; true
