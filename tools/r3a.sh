#!/bin/bash
# round 3 first GPU call: body-check tests, then C3 (with the all-core CPU baseline) and C5 lines
set -e -o pipefail
O=gpurun_out/r3a; mkdir -p $O
bash tools/gpu_tests.sh r3a "body or capi or shared or fixture"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
echo done > $O/DONE2
