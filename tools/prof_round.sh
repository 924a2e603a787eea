#!/bin/bash
# One gpurun call: profiling-build clock breakdowns of the scan and the edge kernel (C3), then
# SQ counter passes over one bench step.  usage: bash tools/prof_round.sh TAG
set -e -o pipefail
O=gpurun_out/${1:-prof}; mkdir -p $O
export TMPDIR=/tmp
TCMP_LIB_PATH=torque_constrained_motion_planning_amd/libtcmp_prof.so timeout -k 10 200 python -u tools/nn_profile.py 2 > $O/nn_profile.json 2> $O/nn_profile.err
TCMP_LIB_PATH=torque_constrained_motion_planning_amd/libtcmp_prof.so timeout -k 10 200 python -u tools/edge_profile.py 2 > $O/edge_profile.json 2> $O/edge_profile.err
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $O/p$i -o run --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-alt > $O/p$i.log 2>&1
done
echo done > $O/DONE
