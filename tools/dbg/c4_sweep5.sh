set -e
O=gpurun_out/r7j; mkdir -p $O
for cfg in "16 2" "16 3" "16 4" "8 4" "21 3"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 2 --fleet $1 --pipeline $2 --no-cpu-baseline --no-alt > $O/c4_f$1_p$2.json 2> $O/c4_f$1_p$2.err
done
