set -o pipefail
export AB_ARGS="--workload models --models CookTorranceWalter,CookTorranceHeitz,PhongWalter,CookTorrance --steps 20 --warmup 3 --no-cpu"
bash tools/gpu_step.sh ab:mid1,3,base,w5,w6,nopf,w5nopf || exit 1
