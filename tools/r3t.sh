#!/bin/bash
# HEAD measured: full GPU suite, smoke, the four bench lines, C3 kernel-trace stats
set -e -o pipefail
T=${1:-r3t}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
for W in c2 c4 c5; do
  timeout -k 10 400 python -u bench.py --workload $W --steps 3 --warmup 1 > $O/bench_$W.json 2> $O/bench_$W.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt > $O/prof_bench.json 2> $O/prof.err
echo done > $O/DONE
