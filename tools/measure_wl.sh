#!/bin/bash
# One gpurun call for one workload: its bench line, the rocprofv3 kernel-trace summary of the
# same bench command, and the PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters), each in a
# run of its own.  usage: bash tools/measure_wl.sh TAG WORKLOAD STEPS [TESTS]
set -e -o pipefail
TAG=$1; W=$2; S=${3:-5}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$4" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
timeout -k 10 600 python -u bench.py --workload $W --steps $S --warmup 1 > $O/bench_$W.json 2> $O/bench_$W.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/stats_$W -o run --output-format csv \
  -- python3 bench.py --workload $W --steps $S --warmup 1 --no-cpu-baseline --no-alt > $O/stats_$W.json 2> $O/stats_$W.err
i=0
mkdir -p $O/pmc_$W
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace -d $O/pmc_$W/p$i -o run --output-format csv \
    -- python3 bench.py --workload $W --steps 1 --warmup 0 --no-cpu-baseline --no-alt > $O/pmc_$W/p$i.log 2>&1
done
echo done > $O/DONE
