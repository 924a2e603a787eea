#!/bin/bash
# Multi-GPU preflight: the exact 8-GPU commands of the scaling runs and the fields
# their JSON lines must carry for the run to prove itself.  This pipeline's own GPU box has one
# GPU, so the script only prints the commands unless --run is given (on a node with N GPUs).
#
#   bash tools/scale_preflight.sh            # print the commands and the checks
#   bash tools/scale_preflight.sh --run [N]  # run them on N GPUs (default 8), check every line
#   bash tools/scale_preflight.sh --check FILE...  # check JSON lines written elsewhere
#
# What each line must show (bench.py adds these fields whenever WORLD_SIZE > 1):
#   rccl_ranks       == N   RCCL's own count of the communicator the job ran on
#   samples_per_rank        N entries, every one > 0 (each rank planned its share)
#   gather_ok        true   (query-sharded runs) every query id arrived at rank 0 exactly once
#                           with the all-gathered row counts (tcmp_gather_paths + unpack checks)
#   tree_consistent  true   (--shared-tree runs) every rank's device digest and node count of
#                           the last step's tree are equal: the ranks grew ONE tree
#   n_gpus           == N, value > 0
set -e -o pipefail
cd "$(dirname "$0")/.."
MODE=${1:-print}
N=${2:-8}
PORT=${TCMP_PREFLIGHT_PORT:-29611}
launch() {  # workload args -> the driver's own launcher line
  echo "python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $PORT bench.py --gpus $N $*"
}
CMDS=(
  "$(launch --workload c3 --steps 5 --warmup 1)"
  "$(launch --workload c4 --steps 2 --warmup 1)"
  "$(launch --workload c5 --steps 2 --warmup 1)"
  "$(launch --workload c5 --shared-tree --steps 2 --warmup 1)"
  "$(launch --workload c3 --shared-tree --steps 5 --warmup 1)"
)
check() {  # JSON line file -> pass/fail on the fields above
  python3 - "$N" "$@" <<'EOF'
import json, sys
n = int(sys.argv[1]); bad = 0
for path in sys.argv[2:]:
    lines = [l for l in open(path).read().splitlines() if l.strip().startswith("{")]
    if not lines:
        print("%s: no JSON line" % path); bad += 1; continue
    d = json.loads(lines[-1])
    shared = "shared-tree" in d["config"].get("parallelism", "")
    errs = []
    if d.get("n_gpus") != n: errs.append("n_gpus %r" % d.get("n_gpus"))
    if not d.get("value", 0) > 0: errs.append("value %r" % d.get("value"))
    if d.get("rccl_ranks") != n: errs.append("rccl_ranks %r" % d.get("rccl_ranks"))
    spr = d.get("samples_per_rank") or []
    if len(spr) != n or min(spr or [0]) <= 0: errs.append("samples_per_rank %r" % spr)
    if shared and d.get("tree_consistent") is not True: errs.append("tree_consistent %r" % d.get("tree_consistent"))
    if not shared and d.get("gather_ok") is not True: errs.append("gather_ok %r" % d.get("gather_ok"))
    print("%s: %s (%s, %.3g %s)" % (path, "ok" if not errs else "FAIL " + "; ".join(errs),
                                   d["config"].get("parallelism"), d.get("value", 0), d.get("unit")))
    bad += bool(errs)
sys.exit(1 if bad else 0)
EOF
}
case "$MODE" in
  print)
    printf '%s\n' "${CMDS[@]}"
    echo "# each JSON line: rccl_ranks == $N, samples_per_rank ($N entries > 0), gather_ok (sharded)"
    echo "# or tree_consistent (--shared-tree) true; check with: bash tools/scale_preflight.sh --check FILE..." ;;
  --run)
    mkdir -p gpurun_out/preflight
    i=0
    for c in "${CMDS[@]}"; do
      i=$((i+1))
      echo "[$i] $c" >&2
      timeout -k 10 900 $c > gpurun_out/preflight/line_$i.json 2> gpurun_out/preflight/line_$i.err
    done
    check gpurun_out/preflight/line_*.json ;;
  --check)
    shift; N=${N_GPUS:-8}; check "$@" ;;
  *) echo "usage: $0 [--run [N] | --check FILE...]" >&2; exit 2 ;;
esac
