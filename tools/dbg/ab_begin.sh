set -e
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  for L in libtcmp_base libtcmp; do
    TCMP_LIB_PATH=torque_constrained_motion_planning_amd/$L.so timeout -k 10 200 python -u bench.py --workload c4 --steps 6 --warmup 1 --no-cpu-baseline --no-alt > $O/c4_${L}_$r.json 2> $O/c4_${L}_$r.err
  done
done
