#!/bin/bash
# One gpurun call after a kernel change: the parity subset that exercises the nearest scan and
# the edge kernel, the C3 bench line, the profiling-build clock breakdowns.
# usage: bash tools/quick_ab.sh TAG [pytest -k expr]
set -e -o pipefail
O=gpurun_out/${1:-ab}; mkdir -p $O
K=${2:-"nearest or c2_full or batched_frontier or golden or edges"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-alt > $O/bench.json 2> $O/bench.err
TCMP_LIB_PATH=torque_constrained_motion_planning_amd/libtcmp_prof.so timeout -k 10 200 python -u tools/nn_profile.py 1 > $O/nn_profile.json 2> $O/nn_profile.err
echo done > $O/DONE
