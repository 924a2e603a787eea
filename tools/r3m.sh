#!/bin/bash
# kernel-trace (+stats) of the C3 and C5 bench lines; PMC FETCH/WRITE and SQ passes over one C3 step
set -e -o pipefail
T=${1:-r3m}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3 -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt > $O/c3.json 2> $O/c3.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c5 -o run --output-format csv \
  -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5.json 2> $O/c5.err
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-trace -d $O/p$i -o run --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-alt > $O/p$i.log 2>&1
done
echo done > $O/DONE
