#!/bin/bash
# parity subset on the default library, then same-box A/B of base vs default (C3)
set -e -o pipefail
T=${1:-r3l}; O=gpurun_out/$T; mkdir -p $O
K=${2:-"nearest or fixture or batched_frontier or golden or retrace or c2_full"}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
bash tools/ab_lib.sh $T/c3 "torque_constrained_motion_planning_amd/libtcmp_base.so torque_constrained_motion_planning_amd/libtcmp.so"
echo done > $O/DONE
