set -e
O=gpurun_out/r7i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fleet.py tests/test_gpu_parity.py tests/test_gpu_trajectory.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for cfg in "16 2" "16 4"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 1 --fleet $1 --pipeline $2 --no-cpu-baseline --no-alt > $O/c4_f$1_p$2.json 2> $O/c4_f$1_p$2.err
done
