#!/bin/bash
# One gpurun call: GPU parity tests, the bench line, a kernel-trace profile and two PMC passes.
# usage (from the repo root on the GPU box): bash tools/gpu_check.sh TAG [tests|notests]
set -e -o pipefail
TAG=${1:-run}
MODE=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$MODE" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --verbose > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt > $OUT/trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run \
  --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-alt > $OUT/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run \
  --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-alt > $OUT/pmc_write.log 2>&1
echo done > $OUT/DONE
