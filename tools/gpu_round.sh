#!/bin/bash
# One gpurun call: GPU tests, smoke(), the default bench line and a rocprofv3 kernel-trace
# summary of the same bench command.  usage: bash tools/gpu_round.sh TAG [SKIP_TESTS]
set -e -o pipefail
TAG=${1:-r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
fi
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt > $OUT/prof_bench.json 2> $OUT/prof.err
echo done > $OUT/DONE
