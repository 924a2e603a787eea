set -e
O=gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  for cb in 16 13 10; do
    TCMP_NN_CBITS=$cb timeout -k 10 200 python -u bench.py --steps 16 --warmup 1 --no-cpu-baseline --no-alt > $O/c3_cb${cb}_$r.json 2> $O/c3_cb${cb}_$r.err
  done
done
