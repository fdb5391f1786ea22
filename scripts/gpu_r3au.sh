#!/bin/bash
# per-thread core pinning (--pin-threads) vs the default rank pinning, interleaved, with the
# host-contention diagnostics (node / host busy share, run-queue wait, quota throttling)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3au
summ() {
  grep -h '^{' "$1" | python -c '
import sys, json
d = json.loads(sys.stdin.read()); c = d["cpu_cores_by_thread"]; h = c.get("host", {})
print(d["value"], d["p50_latency_ms"], "recv", c.get("io_us_per_req_recv"), "node", h.get("node_busy"),
      "host", h.get("host_busy"), "rq", json.dumps(h.get("runq_wait")), "thr", h.get("throttled_ms"))'
}
for i in 1 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/r3au/base_$i.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --pin-threads > gpurun_out/r3au/pin_$i.log 2>&1 || exit 1
  echo "run=$i base $(summ gpurun_out/r3au/base_$i.log)"
  echo "run=$i pin  $(summ gpurun_out/r3au/pin_$i.log)"
done
