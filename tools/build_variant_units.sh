#!/bin/bash
# Like tools/build_variant.sh, but recompiles only the named units with the extra flags and links them with the
# default build's objects for the rest (bbm_amd/lib/obj): a variant that only touches one model family builds in
# the time of that unit.   tools/build_variant_units.sh bperm "inst_microfacet" -DBBM_HIP_EXPF_BPERM
set -e
cd "$(dirname "$0")/.."
name=$1; units=$2; shift 2
out=bbm_amd/lib_ab/$name
mkdir -p $out/obj
python3 - "$out" "$units" "$@" <<'PY'
import os, shutil, subprocess, sys
sys.path.insert(0, ".")
import __graft_entry__ as g
out, units, extra = sys.argv[1], sys.argv[2].split(), sys.argv[3:]
procs, objs = [], []
for src in g.HIP_SOURCES:
    base = os.path.basename(src).replace(".hip", "")
    obj = os.path.join(out, "obj", base + ".o")
    objs.append(obj)
    if base in units:
        procs.append(subprocess.Popen([g.HIPCC] + g.HIP_FLAGS + extra + ["-c", "-o", obj, src]))
    else:
        shutil.copy(os.path.join(g.OBJ_DIR, base + ".o"), obj)
assert all(p.wait() == 0 for p in procs)
subprocess.run([g.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out, "libbbm_hip.so")] + objs, check=True)
PY
echo built $out/libbbm_hip.so
