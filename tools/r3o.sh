#!/bin/bash
# node counting sort + four-pairs-per-wave mesh certificates: parity subset, then same-box A/B
# (base = radix sort + wave certificates, cs = counting sort only, new = both)
set -e -o pipefail
T=${1:-r3o}; O=gpurun_out/$T; mkdir -p $O
L=torque_constrained_motion_planning_amd
K=${2:-"nearest or fixture or batched_frontier or golden or c2_full or shared or group or mesh or self or c5"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
bash tools/ab_lib.sh $T/c5 "$L/libtcmp_base.so $L/libtcmp_cs.so $L/libtcmp.so" --workload c5 --steps 2 --warmup 1
bash tools/ab_lib.sh $T/c3 "$L/libtcmp_base.so $L/libtcmp.so"
echo done > $O/DONE
