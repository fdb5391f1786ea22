#!/bin/bash
# The one GPU-session runner (round 5 folded the per-session gpu_r*.sh
# scripts into it; they remain in git history).  Runs a sequence of steps on
# the gpurun box, each under its own time limit, and stops at the first fatal
# exit (timeout / kill / abort / segfault) so nothing more runs on a GPU in a
# bad state.  Logs go to $OUT (default gpurun_out/session)/<name>.log.
# usage: OUT=gpurun_out/r5s1 scripts/gpu_session.sh "name:timeout:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="${OUT:-gpurun_out/session}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
for step in "$@"; do
  name="${step%%:*}"; rest="${step#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout ${to}s): $cmd" | tee -a "$OUT/CMDS.txt"
  timeout -k 10 "$to" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"; tail -n 6 "$OUT/$name.log" | cut -c1-400
  case $rc in 124|137|134|139|143|-6|-11) echo "fatal exit $rc: stopping"; exit $rc;; esac
done
exit 0
