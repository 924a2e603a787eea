#!/bin/bash
# same-box A/B of the base and new libraries (C3, C5); the gfx950 counter list
set -e -o pipefail
T=${1:-r3i}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
bash tools/ab_lib.sh $T/c3 "torque_constrained_motion_planning_amd/libtcmp_base.so torque_constrained_motion_planning_amd/libtcmp.so"
bash tools/ab_lib.sh $T/c5 "torque_constrained_motion_planning_amd/libtcmp_base.so torque_constrained_motion_planning_amd/libtcmp.so" --workload c5 --steps 2 --warmup 1
echo done > $O/DONE
