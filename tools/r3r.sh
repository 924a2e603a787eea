#!/bin/bash
# two lanes per edge in small rounds: parity subset (split on), then same-box C2 / C4 / C3 lines
# with TCMP_EDGE_SPLIT=1 / 2 / 4, two passes
set -e -o pipefail
T=${1:-r3r}; O=gpurun_out/$T; mkdir -p $O
K=${2:-"edges or batched_frontier or golden or c2_full or fixture or shared or group or mesh_batched or self or retrace"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
for r in 1 2; do
  for V in 1 2 4; do
    for W in c2 c4; do
      TCMP_EDGE_SPLIT=$V timeout -k 10 300 python -u bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline --no-alt > $O/${W}_s${V}_$r.json 2> $O/${W}_s${V}_$r.err
    done
  done
done
echo done > $O/DONE
