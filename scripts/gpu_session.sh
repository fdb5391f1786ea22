#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; stop at the first fatal exit
# (timeout/kill/abort/segfault) so nothing runs on a GPU in a bad state.
# usage: scripts/gpu_session.sh "name:timeout:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for step in "$@"; do
  name="${step%%:*}"; rest="${step#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout ${to}s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  case $rc in 124|137|134|139|143) echo "fatal exit $rc: stopping"; exit $rc;; esac
done
exit 0
