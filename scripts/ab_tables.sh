#!/bin/bash
# A/B of two tile-pick tables on one box: engine replays of ResNet-50 (b1, b32)
# and BERT-base (b32), alternating A B A B.  usage: ab_tables.sh OUTDIR TABLE_A TABLE_B
set -o pipefail
OUT=$1; A=$2; B=$3
for round in 1 2; do
  for t in A B; do
    tab=$A; [ $t = B ] && tab=$B
    TFSERVE_TUNED_CACHE=$tab timeout -k 10 150 python scripts/bench_engine.py --model resnet50 --batch 1 32 --iters 50 2>/dev/null | grep graph_ms | sed "s/^/$t r$round /" >> $OUT/ab.log || exit 1
    TFSERVE_TUNED_CACHE=$tab timeout -k 10 150 python scripts/bench_engine.py --model bert-base --batch 32 --iters 30 2>/dev/null | grep graph_ms | sed "s/^/$t r$round /" >> $OUT/ab.log || exit 1
  done
done
