set -e
O=gpurun_out/$1; mkdir -p $O
for cfg in "4 2" "4 3" "5 2" "6 2" "8 2" "3 3" "4 2"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 24 --warmup 1 --fleet $1 --pipeline $2 --no-cpu-baseline --no-alt > $O/c3_f$1_p$2_$RANDOM.json 2> /dev/null
done
