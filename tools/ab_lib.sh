#!/bin/bash
# Same-box A/B of builds of libtcmp.so (device clocks differ from box to box, so kernel timings
# are only comparable inside one call): bench lines for each library, two passes.
# usage: bash tools/ab_lib.sh TAG "LIB_A LIB_B ..." [bench args...]
set -e -o pipefail
O=gpurun_out/${1:-ablib}; LIBS=$2; shift 2
mkdir -p $O
for r in 1 2; do
  i=0
  for L in $LIBS; do
    i=$((i+1))
    TCMP_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-alt --no-sublines "$@" > $O/bench_${i}_$r.json 2> $O/bench_${i}_$r.err
  done
done
echo done > $O/DONE
