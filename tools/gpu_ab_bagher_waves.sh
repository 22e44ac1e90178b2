set -o pipefail
export AB_ARGS="--workload models --models Bagher --steps 20 --warmup 3 --no-cpu"
bash tools/gpu_step.sh ab:bw,3,base,w2,w4 || exit 1
