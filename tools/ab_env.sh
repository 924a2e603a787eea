#!/bin/bash
# Same-box A/B of environment settings for one library: bench lines per setting, two passes.
# usage: bash tools/ab_env.sh TAG "VAR=a VAR=b ..." [bench args...]   (use NONE for no setting)
set -e -o pipefail
O=gpurun_out/${1:-abenv}; SETS=$2; shift 2
mkdir -p $O
for r in 1 2; do
  i=0
  for S in $SETS; do
    i=$((i+1))
    if [ "$S" = NONE ]; then
      timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-alt --no-sublines "$@" > $O/bench_${i}_$r.json 2> $O/bench_${i}_$r.err
    else
      env $S timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-alt --no-sublines "$@" > $O/bench_${i}_$r.json 2> $O/bench_${i}_$r.err
    fi
  done
done
echo done > $O/DONE
