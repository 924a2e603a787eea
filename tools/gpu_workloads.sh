#!/bin/bash
# One gpurun call: the bench line of every BASELINE config on one GPU (c3 = headline default).
# usage: bash tools/gpu_workloads.sh TAG
set -e -o pipefail
OUT=gpurun_out/${1:-wl}
mkdir -p $OUT
for w in c2 c4 c5 c3; do
  steps=5; [ $w = c5 ] && steps=2
  timeout -k 10 400 python -u bench.py --workload $w --steps $steps --warmup 1 --cpu-samples 20000 \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err
done
echo done > $OUT/DONE
