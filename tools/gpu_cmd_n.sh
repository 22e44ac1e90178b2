set -o pipefail
BBM_HIP_LIB=$GRAFT_REPO_ROOT/bbm_amd/lib_ab/poison/libbbm_hip.so timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_aggregate.py -m gpu > gpurun_out/pytest_poison.log 2>&1; echo poison pytest rc=$?; tail -4 gpurun_out/pytest_poison.log
export AB_ARGS="--workload models --models GGX,GGXHeitz,Lambertian,CookTorrance --steps 20 --warmup 3 --no-cpu"
bash tools/gpu_step.sh ab:nt1,3,base,new || exit 1
export AB_ARGS="--model GGX --steps 20 --warmup 3 --no-cpu --no-exact"
bash tools/gpu_step.sh ab:nt2,3,base,new || exit 1
