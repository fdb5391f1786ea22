#!/bin/bash
# re-tune the tile-pick table with 8 hardware queues (the concurrent graph-tune of the largest bucket
# measures 4 replays in flight), then A/B it against the committed table in the serving regime
set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
mkdir -p gpurun_out/r3an
TFSERVE_TUNED_CACHE=0 timeout -k 10 600 python -u scripts/probe_concurrency.py --buckets 1 2 4 8 16 --save-tuned gpurun_out/r3an/tuned_r50.json > gpurun_out/r3an/tune_r50.log 2>&1 &&
TFSERVE_TUNED_CACHE=0 timeout -k 10 600 python -u scripts/probe_concurrency.py --model bert-base --buckets 1 2 4 8 16 --save-tuned gpurun_out/r3an/tuned_bert.json > gpurun_out/r3an/tune_bert.log 2>&1 &&
TFSERVE_TUNED_CACHE=gpurun_out/r3an/tuned_r50.json timeout -k 10 300 python -u scripts/probe_concurrency.py > gpurun_out/r3an/probe_new.log 2>&1 &&
timeout -k 10 300 python -u scripts/probe_concurrency.py > gpurun_out/r3an/probe_old.log 2>&1 &&
TFSERVE_TUNED_CACHE=gpurun_out/r3an/tuned_r50.json timeout -k 10 300 python -u scripts/probe_concurrency.py > gpurun_out/r3an/probe_new2.log 2>&1 &&
timeout -k 10 300 python -u scripts/probe_concurrency.py > gpurun_out/r3an/probe_old2.log 2>&1
for f in probe_new probe_old probe_new2 probe_old2; do echo "$f $(grep -h ms_per_batch gpurun_out/r3an/$f.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print({k[13:]: v for k, v in d.items() if k.startswith("ms_per_batch")})')"; done
# double-buffered lanes again, now with 8 hardware queues (the first test ran with 4: 8 streams on 4 queues)
for cfg in base s2 base s2; do
  if [ $cfg = s2 ]; then sides=2; c=192; l=3; else sides=1; c=128; l=4; fi
  TFSERVE_LANE_SIDES=$sides timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --lanes $l --concurrency $c > gpurun_out/r3an/bench_$cfg.log 2>&1 || exit 1
  echo "$cfg $(grep -h '^{' gpurun_out/r3an/bench_$cfg.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d["p50_c1_ms"], d["gpu_busy_pct"][0]["mean"])')"
done
