#!/bin/bash
# the driver's exact command with the new default placement (2 L3 groups), plus the 2-rank self-launch
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3aw
for i in 1 2 3 4 5 6; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3aw/driver_$i.log 2>&1 || exit 1
  echo "run=$i $(grep -h '^{' gpurun_out/r3aw/driver_$i.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); c = d["cpu_cores_by_thread"]; h = c.get("host", {})
print(d["value"], d["p50_latency_ms"], "recv", c.get("io_us_per_req_recv"), "node", h.get("node_busy"),
      "llcs", h.get("threads_on", {}).get("llcs"), "cpus", d["diagnostics"][0]["placement"]["cpus"])')"
done
