#!/bin/bash
# PMC counter passes over one bench step (C3), one rocprofv3 run per counter group.
# usage: bash tools/pmc_passes.sh OUTDIR
set -e -o pipefail
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-alt > $OUT/p$i.log 2>&1
done
echo done > $OUT/DONE
