set -e -o pipefail
O=gpurun_out/r2d; mkdir -p $O
for G in 4 8; do
TCMP_NN_GROUP=$G timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "nearest or c2_full or batched_frontier" > $O/t$G.log 2>&1
done
for G in 0 4 8 16; do
TCMP_NN_GROUP=$G timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-alt > $O/b$G.json 2> $O/b$G.err
done
