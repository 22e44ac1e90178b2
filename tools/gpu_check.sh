set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== smoke" 
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo "== pytest gpu"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/pytest_gpu.log
echo "== bench"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== rocprof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo rocprof failed; tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*"
