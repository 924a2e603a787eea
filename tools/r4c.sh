#!/bin/bash
# round-3 final (part 1): full GPU suite, smoke, the default bench line
set -e -o pipefail
T=${1:-r4c}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
echo done > $O/DONE
