set -e
O=gpurun_out/$1; mkdir -p $O
for cfg in "3 1" "4 1" "6 1" "3 2" "0 3"; do
  set -- $cfg
  timeout -k 10 900 python -u bench.py --workload c5 --steps 12 --warmup 1 --fleet $1 --pipeline $2 --no-cpu-baseline --no-alt > $O/c5_f$1_p$2.json 2> $O/c5_f$1_p$2.err
done
