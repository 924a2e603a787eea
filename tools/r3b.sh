#!/bin/bash
# C3 / C5 bench lines and the C5 mesh-stage profile (profiling build)
set -e -o pipefail
O=gpurun_out/${1:-r3b}; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
TCMP_LIB_PATH=torque_constrained_motion_planning_amd/libtcmp_prof.so timeout -k 10 200 python -u tools/mesh_profile.py 1000000 > $O/mesh_profile.json 2> $O/mesh_profile.err
echo done > $O/DONE
