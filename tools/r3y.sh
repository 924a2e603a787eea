#!/bin/bash
# LDS-staged certificate data, with / without the facet trial axes: mesh GPU tests, then a
# same-box C5 A/B against the first sphere build (s1)
set -e -o pipefail
T=${1:-r3y}; O=gpurun_out/$T; mkdir -p $O
K=${2:-"mesh or self or fixture or c5 or body"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
for r in 1 2; do
  for L in s1 nof new; do
    [ $L = new ] && P=torque_constrained_motion_planning_amd/libtcmp.so || P=torque_constrained_motion_planning_amd/libtcmp_$L.so
    TCMP_LIB_PATH=$P timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_${L}_$r.json 2> $O/c5_${L}_$r.err
  done
done
echo done > $O/DONE
