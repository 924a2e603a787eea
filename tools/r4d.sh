#!/bin/bash
# round-3 final (part 2): C2 / C4 / C5 bench lines, kernel-trace stats of C3 and C5, PMC HBM
# passes (FETCH_SIZE, WRITE_SIZE) over one C5 step
set -e -o pipefail
T=${1:-r4d}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for W in c2 c4; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 5 --warmup 1 > $O/bench_$W.json 2> $O/bench_$W.err
done
timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3 -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt > $O/c3_rocprof.json 2> $O/c3_rocprof.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5 -o run --output-format csv \
  -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_rocprof.json 2> $O/c5_rocprof.err
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace -d $O/pmc_c5/p$i -o run --output-format csv \
    -- python3 bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline --no-alt > $O/pmc_c5_p$i.log 2>&1
done
echo done > $O/DONE
