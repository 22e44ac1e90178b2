#!/bin/bash
# Headline gap on one box: the 6in/4out pattern ceiling (roofprobe) against the CookTorrance kernel and variants:
# expdn (no table gather), nogather (timing only), bperm (table via ds_bpermute), ctw8 (8 waves/SIMD)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PROBE_VARIANTS=1,6 timeout -k 10 200 python tools/roofprobe.py > gpurun_out/roofprobe_p.txt 2>&1 || { echo "roofprobe failed"; tail gpurun_out/roofprobe_p.txt; exit 1; }
grep blocks= gpurun_out/roofprobe_p.txt | grep 97657
AB_LIBS="default expdn nogather bperm ctw8" ROUNDS=3 bash tools/gpu_r03_ab.sh || exit 1
for M in GGX Ward Lambertian; do MODEL=$M AB_LIBS=default ROUNDS=1 bash tools/gpu_r03_ab.sh | sed "s/^/$M /" || exit 1; done
PROBE_VARIANTS=1 timeout -k 10 200 python tools/roofprobe.py > gpurun_out/roofprobe_p2.txt 2>&1 || exit 1
grep blocks= gpurun_out/roofprobe_p2.txt | grep 97657
