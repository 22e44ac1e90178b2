set -o pipefail
timeout -k 10 200 python -u tools/dbg_he_cdf.py > gpurun_out/dbg_he_cdf.log 2>&1 || { tail -5 gpurun_out/dbg_he_cdf.log; exit 1; }
cut -c1-150 gpurun_out/dbg_he_cdf.log
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/pytest_par.log 2>&1; echo pytest rc=$?; tail -4 gpurun_out/pytest_par.log
mkdir -p gpurun_out/parity_n && cp gpurun_out/parity_*.json gpurun_out/parity_n/
export AB_ARGS="--workload models --models He,HeWestin,HeHolzschuch,NganHe --steps 10 --warmup 2 --no-cpu"
bash tools/gpu_step.sh ab:he2,2,base,hetab || exit 1
export AB_ARGS="--workload models --models EPD --steps 20 --warmup 3 --no-cpu"
bash tools/gpu_step.sh ab:epd1,2,base,epdtab || exit 1
