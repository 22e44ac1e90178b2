#!/bin/bash
# f64 restatement check, He series lengths (diagnostics build), round-3 counters
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
F64_LIBS=default F64_ROUNDS=1 bash tools/gpu_r03_f.sh > gpurun_out/call7.log 2>&1; rc=$?
echo "f64 rc=$rc"; tail -12 gpurun_out/call7.log
[ $rc -le 1 ] || exit $rc
BBM_HIP_LIB=bbm_amd/lib_ab/heterms/libbbm_hip.so timeout -k 10 300 python tools/he_terms.py He HeWestin NganHe > gpurun_out/he_terms.log 2>&1 || { echo "he_terms failed"; tail gpurun_out/he_terms.log; exit 1; }
head -3 gpurun_out/he_terms.log
bash tools/gpu_r03_pmc.sh > gpurun_out/pmc_r03.log 2>&1; rc2=$?
echo "pmc rc=$rc2"; grep -A3 "^==" gpurun_out/pmc_r03.log | head -60
exit $(( rc > rc2 ? rc : rc2 ))
