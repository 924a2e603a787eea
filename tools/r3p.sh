#!/bin/bash
# same-box A/B: base (radix + wave certificates), cs (counting sort), lod (cs + four-per-wave
# LOD certificates), new (cs + four-per-wave LOD and full-hull stages)
set -e -o pipefail
T=${1:-r3p}; O=gpurun_out/$T; mkdir -p $O
L=torque_constrained_motion_planning_amd
bash tools/ab_lib.sh $T/c3 "$L/libtcmp_base.so $L/libtcmp_cs.so"
bash tools/ab_lib.sh $T/c5 "$L/libtcmp_base.so $L/libtcmp_cs.so $L/libtcmp_lod.so" --workload c5 --steps 2 --warmup 1
echo done > $O/DONE
