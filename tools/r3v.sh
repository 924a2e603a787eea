#!/bin/bash
# mesh-stage profile (TCMP_PROF build) of the C5 edges, spheres off / on
set -e -o pipefail
T=${1:-r3v}; O=gpurun_out/$T; mkdir -p $O
P=torque_constrained_motion_planning_amd/libtcmp_prof.so
TCMP_SPHERES=0 TCMP_LIB_PATH=$P timeout -k 10 300 python -u tools/mesh_profile.py 1000000 > $O/prof_off.json 2> $O/prof_off.err
TCMP_LIB_PATH=$P timeout -k 10 300 python -u tools/mesh_profile.py 1000000 > $O/prof_on.json 2> $O/prof_on.err
echo done > $O/DONE
