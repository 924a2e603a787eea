#!/bin/bash
# nearest-scan rework: parity subset, then same-box A/B of the base and new libraries (C3, C5)
set -e -o pipefail
T=${1:-r3h}; O=gpurun_out/$T; mkdir -p $O
K=${2:-"nearest or fullsize or fixture or batched_frontier or golden or retrace or shared or group or c2_full"}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
bash tools/ab_lib.sh $T/c3 "torque_constrained_motion_planning_amd/libtcmp_base.so torque_constrained_motion_planning_amd/libtcmp.so"
bash tools/ab_lib.sh $T/c5 "torque_constrained_motion_planning_amd/libtcmp_base.so torque_constrained_motion_planning_amd/libtcmp.so" --workload c5 --steps 2 --warmup 1
echo done > $O/DONE
