set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_merl.py -m gpu > gpurun_out/pytest_merl.log 2>&1; rc=$?; grep -E "bin-edge|passed|failed|Error" gpurun_out/pytest_merl.log | head; [ $rc -eq 0 ] || exit 1
export AB_ARGS="--workload models --models Merl,CookTorrance --steps 20 --warmup 3 --no-cpu"
bash tools/gpu_step.sh ab:merl1,3,exact,new || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_aggregate.py -m gpu -k "scratch or graph" > gpurun_out/pytest_agg.log 2>&1; echo agg rc=$?; tail -3 gpurun_out/pytest_agg.log
