#!/bin/bash
# One gpurun call: the whole GPU suite + smoke(), then every workload's bench line.
# usage: bash tools/r3g.sh TAG
set -e -o pipefail
T=${1:-r3g}; O=gpurun_out/$T; mkdir -p $O
bash tools/gpu_tests.sh $T
bash tools/gpu_workloads.sh $T
echo done > $O/DONE
