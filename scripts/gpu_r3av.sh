#!/bin/bash
# last-level-cache placement: the rank's whole NUMA-node share (default) vs its 1 or 2 least-busy
# L3 groups (--llc-groups), interleaved; threads_on says how many L3s the hot threads ended on
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/${OUT:-r3av}
python -c "
import os
from rust_tensorflow_serving2_amd.parallel import topology as t
pl = t.plan(1)[0]
g = t.llc_groups(pl.cpus)
print('node', pl.numa_node, 'cpus', t.compress(pl.cpus), 'llc groups', len(g), [t.compress(x) for x in g[:4]])
" > gpurun_out/${OUT:-r3av}/llc_probe.log 2>&1 || exit 1
cat gpurun_out/${OUT:-r3av}/llc_probe.log
summ() {
  grep -h '^{' "$1" | python -c '
import sys, json
d = json.loads(sys.stdin.read()); c = d["cpu_cores_by_thread"]; h = c.get("host", {})
print(d["value"], d["p50_latency_ms"], "recv", c.get("io_us_per_req_recv"), "h2", c.get("io_us_per_req_h2"),
      "node", h.get("node_busy"), "llcs", h.get("threads_on", {}).get("llcs"), "cpus", d["diagnostics"][0]["placement"]["cpus"])'
}
for i in ${RUNS:-1 2 3 4 5}; do
  for m in ${ARMS:-0 1 2}; do
    timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --llc-groups $m > gpurun_out/${OUT:-r3av}/llc${m}_$i.log 2>&1 || exit 1
    echo "run=$i llc=$m $(summ gpurun_out/${OUT:-r3av}/llc${m}_$i.log)"
  done
done
