#!/bin/bash
# Build an A/B variant of libbbm_hip.so with extra compile flags into bbm_amd/lib_ab/<name>/ (select it at run
# time with BBM_HIP_LIB=bbm_amd/lib_ab/<name>/libbbm_hip.so).   tools/build_variant.sh w4 -DBBM_HIP_COMPACT_WAVES=4
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=bbm_amd/lib_ab/$name
mkdir -p $out/obj
python3 - "$out" "$@" <<'PY'
import os, subprocess, sys
sys.path.insert(0, ".")
import __graft_entry__ as g
out, extra = sys.argv[1], sys.argv[2:]
procs, objs = [], []
for src in g.HIP_SOURCES:
    obj = os.path.join(out, "obj", os.path.basename(src).replace(".hip", ".o"))
    objs.append(obj)
    procs.append(subprocess.Popen([g.HIPCC] + g.HIP_FLAGS + extra + ["-c", "-o", obj, src]))
assert all(p.wait() == 0 for p in procs)
subprocess.run([g.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out, "libbbm_hip.so")] + objs, check=True)
PY
echo built $out/libbbm_hip.so
