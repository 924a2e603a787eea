set -e
O=gpurun_out/r7l; mkdir -p $O
for cfg in "c3 4 3" "c3 8 2" "c3 3 3" "c3 6 2" "c2 16 2" "c2 8 3" "c2 12 2"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload $1 --steps 24 --warmup 1 --fleet $2 --pipeline $3 --no-cpu-baseline --no-alt > $O/$1_f$2_p$3.json 2> $O/$1_f$2_p$3.err
done
