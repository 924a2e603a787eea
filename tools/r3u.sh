#!/bin/bash
# sphere certificates: mesh / self / fixture GPU tests, then same-box C5 and C3 A/B
# (HEAD library, new library with TCMP_SPHERES=0, new library)
set -e -o pipefail
T=${1:-r3u}; O=gpurun_out/$T; mkdir -p $O
K=${2:-"mesh or self or fixture or c5 or body"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
B=torque_constrained_motion_planning_amd/libtcmp_base.so
N=torque_constrained_motion_planning_amd/libtcmp.so
for r in 1 2; do
  TCMP_LIB_PATH=$B timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_base_$r.json 2> $O/c5_base_$r.err
  TCMP_SPHERES=0 TCMP_LIB_PATH=$N timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_off_$r.json 2> $O/c5_off_$r.err
  TCMP_LIB_PATH=$N timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_new_$r.json 2> $O/c5_new_$r.err
done
for L in base new; do
  [ $L = base ] && P=$B || P=$N
  TCMP_LIB_PATH=$P timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-alt > $O/c3_$L.json 2> $O/c3_$L.err
done
echo done > $O/DONE
