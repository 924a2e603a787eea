#!/bin/bash
# One gpurun call: the whole GPU suite, then the C3 and C5 bench lines.  usage: bash tools/full_ab.sh TAG
set -e -o pipefail
O=gpurun_out/${1:-full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-alt > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
echo done > $O/DONE
