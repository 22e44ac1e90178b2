set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
M=Ribardiere,RibardiereAnisotropic,PhongWalter,Bagher,EPD,CookTorrance,GGX,LowMicrofacet,OrenNayar,HeHolzschuch,Merl
for B in 0 1024 2048 4096 8192; do
  if [ $B -eq 0 ]; then unset BBM_HIP_MAX_BLOCKS; else export BBM_HIP_MAX_BLOCKS=$B; fi
  timeout -k 10 200 python bench.py --workload models --models $M --steps 10 --warmup 3 > gpurun_out/ab/models_$B.json 2> gpurun_out/ab/models_$B.err || exit 1
  echo "blocks=$B done"
done
