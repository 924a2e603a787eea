set -e
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_default_1.json 2> $O/bench_default_1.err
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench_default_2.json 2> $O/bench_default_2.err
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --no-alt > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python -u bench.py --workload c2 --steps 24 --no-cpu-baseline --no-alt > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 600 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > $O/bench_c5.json 2> $O/bench_c5.err
