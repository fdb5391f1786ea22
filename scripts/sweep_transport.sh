#!/bin/bash
# Transport ceiling sweep on the tiny probe model (same 602 KB payload as ResNet-50).
for cfg in "4 4 16" "6 4 16" "8 4 16" "4 8 32" "8 8 32" "12 4 16" "6 6 24"; do
  set -- $cfg
  for rep in 1 2; do
    out=$(timeout -k 5 120 python bench.py --model tiny --steps 400 --warmup 20 --io-threads $1 --client-threads $2 --connections $3 2>/dev/null | tail -1)
    rc=$?
    echo "io=$1 client=$2 conns=$3 rep=$rep rc=$rc $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])' 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
