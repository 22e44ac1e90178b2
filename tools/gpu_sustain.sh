#!/bin/bash
# Sustained-load experiment (tools/sustain.py) + a PMC traffic pass for the bench kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/sustain.py --launches ${LAUNCHES:-200} --models ${MODELS:-CookTorrance,GGX,Lambertian} > gpurun_out/sustain.txt 2>&1 || { echo sustain failed; tail -20 gpurun_out/sustain.txt; exit 1; }
cat gpurun_out/sustain.txt
