set -e
O=gpurun_out/r7e; mkdir -p $O
for cfg in "8 3" "16 2" "16 1" "4 4" "32 1"; do
  set -- $cfg
  f=$1; p=$2; [ $f -gt 31 ] && f=31
  timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 1 --fleet $f --pipeline $p --no-cpu-baseline --no-alt > $O/c4_f${f}_p${p}.json 2> $O/c4_f${f}_p${p}.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > $O/trace_c4.json 2> $O/trace_c4.err
