#!/bin/bash
# node counting sort: nearest / tree parity subset, then same-box A/B against the radix build (C3, C5)
set -e -o pipefail
T=${1:-r3n}; O=gpurun_out/$T; mkdir -p $O
K=${2:-"nearest or fixture or batched_frontier or golden or c2_full or shared or group or mesh_batched"}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
bash tools/ab_lib.sh $T/c3 "torque_constrained_motion_planning_amd/libtcmp_base.so torque_constrained_motion_planning_amd/libtcmp.so"
bash tools/ab_lib.sh $T/c5 "torque_constrained_motion_planning_amd/libtcmp_base.so torque_constrained_motion_planning_amd/libtcmp.so" --workload c5 --steps 2 --warmup 1
echo done > $O/DONE
