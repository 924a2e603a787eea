set -e
O=gpurun_out/$1; mkdir -p $O
for p in 2 3; do
  timeout -k 10 400 python -u bench.py --workload c5 --steps 3 --warmup 1 --pipeline $p --no-cpu-baseline --no-alt > $O/c5_p$p.json 2> $O/c5_p$p.err
done
