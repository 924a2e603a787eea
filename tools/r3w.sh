#!/bin/bash
# ball / box certificates: edge / mesh GPU tests, C5 and C3 stage profiles (TCMP_PROF build),
# same-box A/B of the first sphere build (s1) against this one (certificates on / off)
set -e -o pipefail
T=${1:-r3w}; O=gpurun_out/$T; mkdir -p $O
K=${2:-"mesh or self or fixture or c5 or body or edges or batched_frontier or golden or c2_full"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
P=torque_constrained_motion_planning_amd/libtcmp_prof.so
TCMP_LIB_PATH=$P timeout -k 10 300 python -u tools/mesh_profile.py 1000000 > $O/prof_c5.json 2> $O/prof_c5.err
TCMP_LIB_PATH=$P timeout -k 10 300 python -u tools/edge_profile.py 2 > $O/prof_c3.json 2> $O/prof_c3.err
TCMP_SPHERES=0 TCMP_LIB_PATH=$P timeout -k 10 300 python -u tools/edge_profile.py 2 > $O/prof_c3_off.json 2> $O/prof_c3_off.err
A=torque_constrained_motion_planning_amd/libtcmp_s1.so
N=torque_constrained_motion_planning_amd/libtcmp.so
for r in 1 2; do
  TCMP_LIB_PATH=$A timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-alt > $O/c3_s1_$r.json 2> $O/c3_s1_$r.err
  TCMP_SPHERES=0 TCMP_LIB_PATH=$N timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-alt > $O/c3_off_$r.json 2> $O/c3_off_$r.err
  TCMP_LIB_PATH=$N timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-alt > $O/c3_new_$r.json 2> $O/c3_new_$r.err
  TCMP_LIB_PATH=$A timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_s1_$r.json 2> $O/c5_s1_$r.err
  TCMP_LIB_PATH=$N timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_new_$r.json 2> $O/c5_new_$r.err
done
echo done > $O/DONE
