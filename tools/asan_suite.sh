#!/bin/bash
# The CPU test suite against AddressSanitizer + UBSan builds of the oracle and of libtcmp.so's
# host code (CPU only, no GPU).  usage: bash tools/asan_suite.sh [LOG]
set -e -o pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r3_asan_suite.log}
make -C oracle asan
make -C torque_constrained_motion_planning_amd/csrc asan
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
# leaks: CPython and numpy keep allocations until exit by design; odr: two libraries
# carry the same generated geometry tables
export ASAN_OPTIONS=detect_leaks=0:detect_odr_violation=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export ORC_LIB_PATH=$PWD/oracle/build/liboracle_asan.so
export TCMP_LIB_PATH=$PWD/torque_constrained_motion_planning_amd/libtcmp_asan.so
{
  echo "# $(date -u) asan+ubsan: $ORC_LIB_PATH $TCMP_LIB_PATH runtime $RT"
  LD_PRELOAD=$RT python -m pytest tests -m "not gpu" -q -p no:cacheprovider \
    --deselect tests/test_dist_gloo.py::test_gather_two_ranks_gloo 2>&1
} | tee "$LOG"
# the instrumented library is large and not used by any GPU run
rm -f torque_constrained_motion_planning_amd/libtcmp_asan.so
