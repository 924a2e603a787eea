#!/bin/bash
# facet trial axes in the mesh certificate: mesh GPU tests, C5 stage profile, same-box C5 / C3
# A/B of the first sphere build (s1) against this one
set -e -o pipefail
T=${1:-r3x}; O=gpurun_out/$T; mkdir -p $O
K=${2:-"mesh or self or fixture or c5 or body"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
P=torque_constrained_motion_planning_amd/libtcmp_prof.so
TCMP_LIB_PATH=$P timeout -k 10 300 python -u tools/mesh_profile.py 1000000 > $O/prof_c5.json 2> $O/prof_c5.err
A=torque_constrained_motion_planning_amd/libtcmp_s1.so
N=torque_constrained_motion_planning_amd/libtcmp.so
for r in 1 2; do
  TCMP_LIB_PATH=$A timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_s1_$r.json 2> $O/c5_s1_$r.err
  TCMP_LIB_PATH=$N timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_new_$r.json 2> $O/c5_new_$r.err
  TCMP_LIB_PATH=$A timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-alt > $O/c3_s1_$r.json 2> $O/c3_s1_$r.err
  TCMP_LIB_PATH=$N timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-alt > $O/c3_new_$r.json 2> $O/c3_new_$r.err
done
echo done > $O/DONE
