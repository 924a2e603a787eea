set -e
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fleet.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for cfg in "0 3" "3 1" "2 2" "3 2"; do
  set -- $cfg
  timeout -k 10 600 python -u bench.py --workload c5 --steps 6 --warmup 1 --fleet $1 --pipeline $2 --no-cpu-baseline --no-alt > $O/c5_f$1_p$2.json 2> $O/c5_f$1_p$2.err
done
