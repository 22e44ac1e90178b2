#!/bin/bash
# Round 3: doubleRGB exp / log / pow restatements -- the math probe against glibc, f64 parity, and the per-model A/B
# against the device library (bbm_amd/lib_ab/f64ocml: -DBBM_HIP_F64_OCML).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 tools/bin/f64math_probe > gpurun_out/f64math.log 2>&1; rc=$?
cat gpurun_out/f64math.log
[ $rc -le 1 ] || exit $rc
M=${F64_MODELS:-Bagher,AshikhminShirleyFull,AshikhminShirley,Ribardiere,RibardiereAnisotropic,EPD,Phong,Lafortune,NganLafortune,PhongWalter,CookTorrance,LowSmooth,NganAshikhminShirley}
for round in $(seq 1 ${F64_ROUNDS:-2}); do
  for V in ${F64_LIBS:-default f64ocml}; do
    lib=""; [ "$V" = default ] || lib="BBM_HIP_LIB=bbm_amd/lib_ab/$V/libbbm_hip.so"
    env $lib timeout -k 10 200 python bench.py --workload f64 --models $M --steps 5 --warmup 2 --no-cpu > gpurun_out/f.json 2>gpurun_out/f.err || { echo "f64 $V failed"; tail gpurun_out/f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/f.json'))
print('r$round $V', ' '.join('%s %.4f ms %.3f'%(k,v['kernel_ms'],v['roofline_frac']) for k,v in d['per_model_10M'].items()))"
  done
done
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f64.py tests/test_gpu_nested.py -k "f64 or composed" > gpurun_out/f64_tests.log 2>&1; rc=$?
tail -5 gpurun_out/f64_tests.log
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/parity_f64_large_*.json')):
    d = json.load(open(f))
    worst = sorted(((v.get('max_rel_normal', 0), k) for k, v in d.items()), reverse=True)[:8]
    print(f[-7:-5], ' '.join('%s %.2e' % (k, e) for e, k in worst))
PY
exit $rc
