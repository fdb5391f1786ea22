#!/bin/bash
# double-buffered native lanes (TFSERVE_LANE_SIDES=2) vs the default, same box, interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3z
run() { # name, bench args..., (env via prefix)
  local name=$1; shift
  env $ENVV timeout -k 10 240 python -u bench.py --steps 300 --warmup 30 "$@" > gpurun_out/r3z/$name.log 2>&1 || exit 1
  python - "$name" <<'PY'
import json, sys
name = sys.argv[1]
l = [x for x in open(f"gpurun_out/r3z/{name}.log") if x.startswith("{")][-1]
d = json.loads(l)
c = d.get("cpu_cores_by_thread") or {}
print(name, d["value"], "p50", d["p50_latency_ms"], "p99", d["p99_latency_ms"], "c1", d.get("p50_c1_ms"),
      "err", d["errors"], "busy", (d.get("gpu_busy_pct") or [{}])[0].get("mean"), "fast", d.get("fast_path_share"),
      "avg_batch", c.get("avg_batch"), flush=True)
PY
}
ENVV="TFSERVE_LANE_SIDES=1" run base1 --lanes 4
ENVV="TFSERVE_LANE_SIDES=2" run s2_l2_c128 --lanes 2 --concurrency 128
ENVV="TFSERVE_LANE_SIDES=2" run s2_l3_c192 --lanes 3 --concurrency 192
ENVV="TFSERVE_LANE_SIDES=2" run s2_l3_c128 --lanes 3 --concurrency 128
ENVV="TFSERVE_LANE_SIDES=1" run base_c192 --lanes 4 --concurrency 192
ENVV="TFSERVE_LANE_SIDES=1" run base2 --lanes 4
