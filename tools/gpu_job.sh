#!/bin/bash
# One gpurun call made of named stages, run in order; the first failing stage ends the call.
#   bash tools/gpu_job.sh TAG STAGE [STAGE ...]
# stages:
#   tests[=K]        pytest -m gpu (optionally -k K), then smoke()
#   bench[=W]        bench.py line for workload W (c3 default), 5 steps (c5: 2)
#   default          the driver's own default command, `python bench.py` (C3, CPU baseline too)
#   trace[=W]        rocprofv3 --kernel-trace --stats of the same bench command
#   pmc[=W]          PMC passes FETCH_SIZE / WRITE_SIZE (one run each) over one bench step
#   sq[=W]           PMC pass of SQ wave / busy counters over one bench step
#   sq2[=W]          PMC pass of the issue-side SQ counters (WAIT_INST_ANY, ACTIVE_INST_ANY /
#                    VALU / SCA / VMEM / LDS / MISC) over one bench step
#   tcc[=W]          PMC pass of the L2 hit / miss and TCP request counters
#   list             rocprofv3 -L (the box's counter names)
#   res              kernel resource usage (tools/resource.py, a CPU-side compile) into the stage dir
#   valu[=W]         PMC pass of the SQ_INSTS_VALU_* / FLOPS counters over one bench step
#   mix[=W]          PMC pass of the instruction mix (SQ_INSTS total / VALU / SALU / branch /
#                    LDS / VMEM / SMEM, SQ_THREAD_CYCLES_VALU) over one bench step
#   meshprof[=N]     profiling build (make prof): tools/mesh_profile.py on C5 (N samples, 1e6)
#   prof             profiling-build (make prof) clock breakdowns: tools/nn_profile.py and
#                    tools/edge_profile.py on C3
#   ab=LIBS          same-box A/B of libtcmp builds (space-separated .so paths): C3 bench lines,
#                    two passes (tools/ab_lib.sh; bench arguments via env:AB_ARGS=...)
#   c5seeds=B,S,N    tools/c5_fixture_search.py B S N (goal-reaching seeds of the C5 fixture)
#   sweep=W:F/P,...  bench lines of workload W at each fleet size F / fleets in flight P
#                    (steps via env:SWEEP_STEPS=N, default 16; c5 3)
#   line=W:ARGS      one bench line of workload W with extra bench arguments (commas for spaces),
#                    e.g. line=c5:--steps,6,--fleet,3 ; output line_W_<n>.json
#   abw=W            ab (the TCMP_LIB_PATH builds listed in env:AB_LIBS) on workload W
#   abenv=W          same-box A/B of environment settings (env:AB_SETS="VAR=a VAR=b", NONE for
#                    none) on workload W, two passes (tools/ab_env.sh)
#   env:VAR=V        export VAR=V for the following stages (A/B knobs, TCMP_LIB_PATH=...)
# Outputs under gpurun_out/TAG/.
set -e -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
agg() {  # PASS_DIR -> PASS_DIR.json (per-kernel totals), raw CSVs removed (gpurun_out <= 64 MiB)
  python3 tools/pmc_agg.py "$1" > "$1.json" && rm -rf "$1"
}
pmc_args() {  # workload -> bench.py arguments of a counter pass: whole fleets, one in flight
  case "$1" in
    c3|"") echo "--steps 4 --warmup 0 --pipeline 1 --no-sublines" ;;   # one fleet of 4 (+ the timing pass's)
    c2) echo "--workload c2 --steps 8 --warmup 0 --pipeline 1" ;;
    c5) echo "--workload c5 --steps 3 --warmup 0 --pipeline 1 --no-single" ;;   # one fleet of 3
    *) echo "--workload $1 --steps 1 --warmup 0 --pipeline 1" ;;
  esac
}
bench_args() {  # workload -> bench.py arguments of one measured line
  case "$1" in
    c5) echo "--workload c5 --steps 2 --warmup 1" ;;
    c3|"") echo "--steps 5 --warmup 1 --no-sublines" ;;
    *) echo "--workload $1 --steps 5 --warmup 1" ;;
  esac
}
for st in "$@"; do
  name=${st%%=*}; arg=""; [ "$name" != "$st" ] && arg=${st#*=}
  case "$name" in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$arg" > $O/gpu_tests.log 2>&1
      else
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
      fi
      timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    bench)
      w=${arg:-c3}
      timeout -k 10 300 python -u bench.py $(bench_args $w) > $O/bench_$w.json 2> $O/bench_$w.err ;;
    default)
      timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err ;;
    trace)
      w=${arg:-c3}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$w -o run --output-format csv \
        -- python3 bench.py $(bench_args $w) --no-cpu-baseline --no-alt > $O/trace_$w.json 2> $O/trace_$w.err
      python3 tools/trace_split.py $O/trace_$w/run_kernel_trace.csv > $O/trace_split_$w.json
      cp $O/trace_$w/run_kernel_stats.csv $O/kernel_stats_$w.csv && rm -rf $O/trace_$w ;;
    pmc)
      w=${arg:-c3}; i=0
      for grp in FETCH_SIZE WRITE_SIZE; do
        i=$((i+1))
        timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace -d $O/pmc_$w/p$i -o run --output-format csv \
          -- python3 bench.py $(pmc_args $w) --no-cpu-baseline --no-alt > $O/pmc_${w}_p$i.log 2>&1
      done
      python3 tools/pmc_summary.py $O/pmc_hbm_$w.json "FETCH_SIZE / WRITE_SIZE passes: bench.py $(pmc_args $w)" $O/pmc_$w/p1 $O/pmc_$w/p2
      rm -rf $O/pmc_$w ;;
    sq)
      w=${arg:-c3}
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
        --kernel-trace -d $O/sq_$w -o run --output-format csv \
        -- python3 bench.py $(pmc_args $w) --no-cpu-baseline --no-alt > $O/sq_$w.log 2>&1
      agg $O/sq_$w ;;
    sq2)
      w=${arg:-c3}
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
        --kernel-trace -d $O/sq2_$w -o run --output-format csv \
        -- python3 bench.py $(pmc_args $w) --no-cpu-baseline --no-alt > $O/sq2_$w.log 2>&1
      agg $O/sq2_$w ;;
    tcc)
      w=${arg:-c3}
      timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
        --kernel-trace -d $O/tcc_$w -o run --output-format csv \
        -- python3 bench.py $(pmc_args $w) --no-cpu-baseline --no-alt > $O/tcc_$w.log 2>&1
      agg $O/tcc_$w ;;
    list)
      timeout -s KILL 120 rocprofv3 -L > $O/counters.txt 2>&1 ;;
    valu)
      w=${arg:-c3}
      timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 \
        --kernel-trace -d $O/valu_$w -o run --output-format csv \
        -- python3 bench.py $(pmc_args $w) --no-cpu-baseline --no-alt > $O/valu_$w.log 2>&1
      python3 tools/pmc_summary.py $O/pmc_valu_$w.json "SQ_INSTS_VALU_* pass: bench.py $(pmc_args $w)" $O/valu_$w
      agg $O/valu_$w ;;
    mix)
      w=${arg:-c3}
      timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_THREAD_CYCLES_VALU \
        --kernel-trace -d $O/mix_$w -o run --output-format csv \
        -- python3 bench.py $(pmc_args $w) --no-cpu-baseline --no-alt > $O/mix_$w.log 2>&1
      agg $O/mix_$w ;;
    prof)
      P=torque_constrained_motion_planning_amd/libtcmp_prof.so
      TCMP_LIB_PATH=$P timeout -k 10 200 python -u tools/nn_profile.py 2 > $O/nn_profile.json 2> $O/nn_profile.err
      TCMP_LIB_PATH=$P timeout -k 10 200 python -u tools/edge_profile.py 2 > $O/edge_profile.json 2> $O/edge_profile.err ;;
    meshprof)
      TCMP_LIB_PATH=torque_constrained_motion_planning_amd/libtcmp_prof.so timeout -k 10 300 \
        python -u tools/mesh_profile.py ${arg:-1000000} > $O/mesh_profile.json 2> $O/mesh_profile.err ;;
    ab)
      bash tools/ab_lib.sh $TAG/ab "$arg" ${AB_ARGS:-} ;;
    sweep)
      w=${arg%%:*}; n=${SWEEP_STEPS:-16}; [ "$w" = c5 ] && n=${SWEEP_STEPS:-3}
      IFS=',' read -ra cfgs <<< "${arg#*:}"
      for fp in "${cfgs[@]}"; do
        f=${fp%/*}; p=${fp#*/}
        timeout -k 10 600 python -u bench.py --workload $w --steps $n --warmup 1 --fleet $f --pipeline $p \
          --no-cpu-baseline --no-alt --no-sublines > $O/sweep_${w}_f${f}_p${p}.json 2> $O/sweep_${w}_f${f}_p${p}.err
      done ;;
    line)
      w=${arg%%:*}; extra=${arg#*:}; [ "$extra" = "$arg" ] && extra=""
      nl=$(ls $O 2>/dev/null | grep -c "^line_${w}_" || true)
      timeout -k 10 600 python -u bench.py --workload $w ${extra//,/ } > $O/line_${w}_$nl.json 2> $O/line_${w}_$nl.err ;;
    abw)
      bash tools/ab_lib.sh $TAG/ab_$arg "${AB_LIBS:?env:AB_LIBS=...}" --workload $arg --no-sublines ${AB_ARGS:-} ;;
    abenv)
      bash tools/ab_env.sh $TAG/abenv_$arg "${AB_SETS:?env:AB_SETS=...}" --workload $arg ${AB_ARGS:-} ;;
    c5seeds)
      timeout -k 10 300 python -u tools/c5_fixture_search.py ${arg//,/ } > $O/c5seeds.jsonl 2> $O/c5seeds.err ;;
    env:*)
      export "${st#env:}" ;;
    *) echo "unknown stage $st" >&2; exit 2 ;;
  esac
  echo "$st ok" >> $O/STAGES
done
echo done > $O/DONE
