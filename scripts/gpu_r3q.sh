set -o pipefail
mkdir -p gpurun_out/r3q
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r3q/bench1.log 2>&1 &&
timeout -k 10 400 python bench.py --model resnet50-v2 > gpurun_out/r3q/bench1_v2.log 2>&1 &&
timeout -k 10 400 python bench.py --model bert-base > gpurun_out/r3q/bench1_bert.log 2>&1
