#!/bin/bash
# A/B of the nearest-scan variants (TCMP_NN_MODE): parity subset, then the C3 bench line each.
# usage: bash tools/nn_ab.sh TAG "MODES"
set -e -o pipefail
O=gpurun_out/${1:-nnab}; mkdir -p $O
MODES=${2:-"0 1"}
for M in $MODES; do
  [ "$M" = 0 ] && continue
  TCMP_NN_MODE=$M timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "nearest or c2_full or batched_frontier" > $O/t$M.log 2>&1
done
for M in $MODES; do
  TCMP_NN_MODE=$M timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-alt > $O/b$M.json 2> $O/b$M.err
done
