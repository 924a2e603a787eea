#!/bin/bash
# wave-cooperative facet trial axes at the head of the mesh chain: mesh GPU tests, C5 stage
# profile, same-box C5 A/B against the LDS-staged certificate build without them (nof)
set -e -o pipefail
T=${1:-r4b}; O=gpurun_out/$T; mkdir -p $O
K=${2:-"mesh or self or fixture or c5 or body"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
TCMP_LIB_PATH=torque_constrained_motion_planning_amd/libtcmp_prof.so timeout -k 10 300 python -u tools/mesh_profile.py 1000000 > $O/prof_c5.json 2> $O/prof_c5.err
for r in 1 2; do
  for L in if new; do
    [ $L = new ] && P=torque_constrained_motion_planning_amd/libtcmp.so || P=torque_constrained_motion_planning_amd/libtcmp_$L.so
    TCMP_LIB_PATH=$P timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_${L}_$r.json 2> $O/c5_${L}_$r.err
  done
done
echo done > $O/DONE
