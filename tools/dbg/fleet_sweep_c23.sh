set -e
O=gpurun_out/r7k; mkdir -p $O
for cfg in "c3 4 1" "c3 4 2" "c3 2 2" "c2 8 2" "c2 16 1" "c2 8 1"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload $1 --steps 16 --warmup 1 --fleet $2 --pipeline $3 --no-cpu-baseline --no-alt > $O/$1_f$2_p$3.json 2> $O/$1_f$2_p$3.err
done
