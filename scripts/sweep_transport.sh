#!/bin/bash
# Transport sweep: "io client conns concurrency" configs on a model (default tiny:
# same 602 KB payload as ResNet-50, negligible compute).  Prints RPC/s, p50 and
# the CPU cores used by the server IO threads and the whole process.
MODEL=${MODEL:-tiny}
CFGS=${CFGS:-"6 4 16 128|8 8 32 128|8 8 32 256|12 8 32 256|8 12 48 256"}
IFS='|' read -ra LIST <<< "$CFGS"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  out=$(timeout -k 5 150 python bench.py --model $MODEL --steps ${STEPS:-800} --warmup 30 --io-threads $1 --client-threads $2 \
        --connections $3 --concurrency $4 --lanes ${5:-4} --cpu-report 2>/dev/null | tail -1)
  rc=$?
  echo "model=$MODEL io=$1 client=$2 conns=$3 conc=$4 lanes=${5:-4} rc=$rc $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d["cpu_cores_by_thread"])' 2>/dev/null)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
