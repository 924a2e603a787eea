#!/bin/bash
# A/B of an engine environment switch: parity subset per value, then the C3 bench line each.
# usage: bash tools/env_ab.sh TAG VAR "VALUES" [PYTEST_K]
set -e -o pipefail
O=gpurun_out/${1:-envab}; VAR=$2; VALUES=$3; K=${4:-"nearest or c2_full or batched_frontier"}
mkdir -p $O
for V in $VALUES; do
  env $VAR=$V timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/t$V.log 2>&1
done
for V in $VALUES; do
  env $VAR=$V timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-alt > $O/b$V.json 2> $O/b$V.err
done
