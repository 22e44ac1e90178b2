#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for mode in normal serial; do
  if [ $mode = serial ]; then export AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3; fi
  timeout -k 10 300 ./tests/cpp/_build/adapter_check > gpurun_out/adapter_$mode.jsonl 2> gpurun_out/adapter_$mode.err
  rc=$?; echo "== $mode rc=$rc"; grep '"ok": false' gpurun_out/adapter_$mode.jsonl | cut -c1-200; head -6 gpurun_out/adapter_$mode.err | cut -c1-250
  [ $rc -le 1 ] || exit $rc
done
