#!/bin/bash
# how much of a short timed window is the closing synchronize (in-flight batches behind the last completion)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ax
for i in 1 2 3 4; do
  for s in 20 300; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps $s --warmup 5 > gpurun_out/r3ax/s${s}_$i.log 2>&1 || exit 1
    echo "run=$i steps=$s $(grep -h '^{' gpurun_out/r3ax/s${s}_$i.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); c = d["cpu_cores_by_thread"]
print(d["value"], "ms/step", d["ms_per_step"], "window_ms", round(d["ms_per_step"] * d["steps"], 2),
      "start_sync_ms", c.get("start_sync_ms"), "end_sync_ms", c.get("end_sync_ms"))')"
  done
done
