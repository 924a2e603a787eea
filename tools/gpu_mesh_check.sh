set -o pipefail
mkdir -p gpurun_out/mesh1
timeout -k 10 600 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/mesh1/tests.log 2>&1
rc=$?
tail -30 gpurun_out/mesh1/tests.log
[ $rc -eq 0 ] && timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/mesh1/bench.json 2> gpurun_out/mesh1/bench.err
exit $rc
