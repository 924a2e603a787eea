#!/bin/bash
# A/B of the nearest scan's candidate grouping (TCMP_NN_GROUP, 0 = one candidate per wave):
# parity subset per setting, then bench lines.  usage: bash tools/nng_ab.sh TAG "G..." [CBITS]
set -e -o pipefail
O=gpurun_out/${1:-nng}; mkdir -p $O
GS=${2:-"0 4"}
export TCMP_NN_CBITS=${3:-16}
for G in $GS; do
  [ $G = 0 ] && continue
  TCMP_NN_GROUP=$G timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "nearest or c2_full or batched_frontier" > $O/t$G.log 2>&1
done
for G in $GS; do
  TCMP_NN_GROUP=$G timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-alt > $O/b$G.json 2> $O/b$G.err
done
echo done > $O/DONE
