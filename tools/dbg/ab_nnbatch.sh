set -e
O=gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  for L in libtcmp libtcmp_nb8 libtcmp_nb2; do
    TCMP_LIB_PATH=torque_constrained_motion_planning_amd/$L.so timeout -k 10 200 python -u bench.py --steps 16 --warmup 1 --no-cpu-baseline --no-alt > $O/c3_${L}_$r.json 2> $O/c3_${L}_$r.err
  done
done
