#!/bin/bash
# Round graphs on/off: GPU tests (graphs on), then the C3 bench line with TCMP_GRAPHS=0 and 1.
# usage: bash tools/graph_ab.sh TAG
set -e -o pipefail
O=gpurun_out/${1:-graph}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
for G in 0 1; do
  TCMP_GRAPHS=$G timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/b$G.json 2> $O/b$G.err
done
