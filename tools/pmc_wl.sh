#!/bin/bash
# One gpurun call: PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters; one rocprofv3 run each)
# over one bench step of each named workload, plus each workload's bench line and kernel-trace
# summary when BENCH is set.  usage: [BENCH=1] bash tools/pmc_wl.sh TAG "c3 c5"
set -e -o pipefail
TAG=$1; WLS=${2:-c3}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for W in $WLS; do
  mkdir -p $O/pmc_$W
  if [ -n "$BENCH" ]; then
    S=5; [ $W = c5 ] && S=2
    timeout -k 10 600 python -u bench.py --workload $W --steps $S --warmup 1 > $O/bench_$W.json 2> $O/bench_$W.err
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/stats_$W -o run --output-format csv \
      -- python3 bench.py --workload $W --steps $S --warmup 1 --no-cpu-baseline --no-alt > $O/stats_$W.json 2> $O/stats_$W.err
  fi
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $grp --kernel-trace -d $O/pmc_$W/p$i -o run --output-format csv \
      -- python3 bench.py --workload $W --steps 1 --warmup 0 --no-cpu-baseline --no-alt > $O/pmc_$W/p$i.log 2>&1
  done
done
echo done > $O/DONE
