set -o pipefail
for v in hediag1 hediag2 hediag3; do
  BBM_HIP_LIB=bbm_amd/lib_ab/$v/libbbm_hip.so timeout -k 10 300 python tools/dbg_he_parts.py $v pairs || exit 1
done
timeout -k 10 300 python tools/dbg_he_parts.py main pairs
