#!/bin/bash
# One gpurun call: the GPU test suite (optionally a -k filter), then smoke().
# usage: bash tools/gpu_tests.sh TAG [PYTEST_K_EXPR]
set -e -o pipefail
OUT=gpurun_out/${1:-tests}
mkdir -p $OUT
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $OUT/gpu_tests.log 2>&1
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo done > $OUT/DONE
