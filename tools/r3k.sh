#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over one C3 bench step for each library given
# usage: bash tools/r3k.sh TAG "LIB_A LIB_B"
set -e -o pipefail
T=$1; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
i=0
for L in $2; do
  i=$((i+1))
  j=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    j=$((j+1))
    TCMP_LIB_PATH=$L timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-trace -d $O/l${i}_p$j -o run --output-format csv \
      -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-alt > $O/l${i}_p$j.log 2>&1
  done
done
echo done > $O/DONE
