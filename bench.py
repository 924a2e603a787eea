#!/usr/bin/env python3
"""Benchmark: torque-feasible, collision-checked RRT* samples/s (BASELINE.json metric).

Workload (BASELINE.json configs[2], "C3"): Panda 7-DOF, 16 axis-aligned box obstacles,
5 kg payload, torque_test=rne (static RNE per extend step during search; min-jerk v/a +
dynamic RNE in the final validation), 1e6 RRT* samples per query on one MI355X.  A step is
one full planning query: 1e6 Philox-drawn candidates in batched frontier rounds (nearest,
extend, collision, torque, insert, rewire on the device), then retrace + min-jerk +
final validation.  Synthetic scene, seed = 1234 + query id.

N > 1 (torchrun, one process per GPU): every rank plans its own queries (independent
queries shard with no data-path collective, scaling "weak"); solved trajectories are
gathered to rank 0 over RCCL at the end of each step, as in configs[3].  The collectives
(barrier, max-over-ranks time, the trajectory gather) are libtcmp.so's own RCCL
communicator (tcmp_dist_*, tcmp_gather_paths): no PyTorch in this process.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from torque_constrained_motion_planning_amd import _lib, shard  # noqa: E402
from torque_constrained_motion_planning_amd.scene import (mesh_pack, obstacle_array,  # noqa: E402
                                                           random_box_scene, random_mesh_scene)

START = np.array([0, -np.pi / 4, 0.0, -6 * np.pi / 8, 0, np.pi / 2, np.pi / 4])  # utils.py:45
PEAK_FP32_TFLOPS = 157.3    # MI355X fp32 vector peak (spec, MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0       # MI355X HBM3E peak (MI355X_MICROARCH.md)
PEAK_FP64_TFLOPS = 78.6     # MI355X fp64 vector peak (spec)
NN_FLOP_PER_PAIR = 21       # 7 sub + 7 fma per (candidate, node) pair, fp32 first pass (SURVEY 8d F_nn)
# SURVEY 8d per-edge-step work: FK, link-vs-box cull per (link, obstacle), static RNE (rne and
# nov during search), SAT per pair surviving the cull
F_FK, F_BP, F_RNE_STATIC, F_SAT, N_LINKS = 720, 48, 3000, 260, 10


def _plan_dispatches(rows):
    """The planner's own launches of a kernel among a PMC summary's dispatches: the bench's scene
    setup runs the same kernels on a few configurations (grids of a few hundred threads), which
    would otherwise dilute the per-launch averages."""
    big = max((x.get("grid") or 0 for x in rows), default=0)
    return [x for x in rows if (x.get("grid") or 0) * 8 >= big]


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of THIS
    workload (profiles/<tag>_pmc_hbm_<workload>.json): 2 x FETCH_SIZE (gfx950 correction) +
    WRITE_SIZE.  None when the workload was never profiled."""
    prof = os.path.join(REPO, "profiles")
    suffix = "_pmc_hbm_%s.json" % workload
    pmc = sorted(f for f in os.listdir(prof) if f.endswith(suffix)) if os.path.isdir(prof) else []
    if not pmc:
        return None
    d = _plan_dispatches(json.load(open(os.path.join(prof, pmc[-1])))["dispatches"].get(kernel, []))
    fetch = [x["value_KiB"] for x in d if x["counter"] == "FETCH_SIZE"]
    write = [x["value_KiB"] for x in d if x["counter"] == "WRITE_SIZE"]
    if not fetch or len(fetch) != len(write):
        return None
    return (2 * sum(fetch) + sum(write)) * 1024 / len(fetch)


def pmc_valu(kernel, workload, peak, counters=("SQ_INSTS_VALU_FLOPS_FP64",)):
    """Measured VALU flop of `kernel` from the newest committed PMC summary of THIS workload
    (profiles/<tag>_pmc_valu_<workload>.json: a rocprofv3 --pmc pass of the SQ_INSTS_VALU_*
    counters over one bench step): flop per launch (summed over `counters`, averaged over the
    step's launches) and the rate over the same dispatches' traced durations.  None when the
    workload was never profiled that way."""
    prof = os.path.join(REPO, "profiles")
    suffix = "_pmc_valu_%s.json" % workload
    pmc = sorted(f for f in os.listdir(prof) if f.endswith(suffix)) if os.path.isdir(prof) else []
    if not pmc:
        return None
    d = _plan_dispatches(json.load(open(os.path.join(prof, pmc[-1])))["dispatches"].get(kernel, []))
    rows = [x for x in d if x["counter"] == counters[0]]
    if not rows:
        return None
    # SQ_INSTS_VALU_FLOPS_* count flop per wave instruction (they equal 2 FMA + ADD + MUL of
    # the SQ_INSTS_VALU_*_F64 instruction counts): x 64 lanes, exec-masked lanes included, so
    # an upper bound of the lanes' own flop
    flop = 64.0 * sum(x["value_KiB"] for x in d if x["counter"] in counters)
    us = sum(x["dur_us"] or 0.0 for x in rows)
    tf = flop / (us * 1e-6) / 1e12 if us > 0 else None
    return {"flop_per_launch": flop / len(rows), "tflops_traced": tf,
            "frac_traced": tf / peak if tf else None, "counters": list(counters),
            "source": "profiles/" + pmc[-1]}


# BASELINE.json configs (SURVEY 8 sizes): boxes, meshes, torque test, payload, samples per
# query, queries per step (all ranks together), scaling.  Batch per round: SURVEY 8d's
# 65,536 for the 1e5-sample queries (C2 17.4M -> 28.0M, C4 26.7M -> 39.7M samples/s over
# 32,768), 262,144 for the 1e6 / 1e7-sample ones.
WORKLOADS = {
    "c2": dict(boxes=4, meshes=0, mode=_lib.TORQUE_NOV, mass=2.0, samples=100_000, batch=65536,
               queries=1, scaling="weak", pipeline=3, fleet=8,
               text="C2: Panda 7-DOF, 4 axis-aligned boxes, 2 kg payload, torque_test=nov, 1e5 "
                    "batched samples per query, one query per GPU per step (queries_in_flight "
                    "of them planned concurrently, fused_queries per fused round)"),
    "c3": dict(boxes=16, meshes=0, mode=_lib.TORQUE_RNE, mass=5.0, samples=1_000_000,
               batch=262144, alt_batch=65536, queries=1, scaling="weak", pipeline=2, fleet=4,
               text="C3: Panda 7-DOF, 16 axis-aligned boxes, 5 kg payload, torque_test=rne + "
                    "min-jerk v/a validation, 1e6 samples per query, one query per GPU per step "
                    "(queries_in_flight of them planned concurrently, fused_queries per fused "
                    "round; config_single_query = one at a time)"),
    "c4": dict(boxes=16, meshes=0, mode=_lib.TORQUE_RNE, mass=5.0, samples=100_000, batch=65536,
               queries=64, scaling="strong", pipeline=3, fleet=16,
               text="C4: 64 independent start/goal queries (16 boxes each, 5 kg, rne, 1e5 "
                    "samples each) per step, sharded round-robin over the GPUs, solved paths "
                    "gathered to rank 0 over RCCL; a GPU's queries grow their trees in fused "
                    "rounds, `fleet` queries per set of kernel launches"),
    "c5": dict(boxes=0, meshes=256, mode=_lib.TORQUE_RNE, mass=5.0, samples=10_000_000,
               batch=262144, queries=1, scaling="strong", pipeline=1, fleet=3,
               text="C5: dense clutter, 256 convex meshes (Panda link hulls scaled 0.5-1.5, "
                    "random poses), 5 kg, rne, 1e7 samples per step split over the GPUs -- "
                    "throughput mode: N independent replica trees of 1e7/N samples on the same "
                    "scene (smaller trees than the 1-GPU 1e7-sample tree: not the same problem "
                    "as N grows)"),
}


def make_query(seed, n_obs=16, mode=_lib.TORQUE_RNE, mass=5.0, engine=None, n_mesh=0):
    """Scene + goal: obstacles rejected while start/goal collide; goal collision-free and
    torque-feasible, straight start->goal edge blocked.  Returns (boxes (n, 15),
    MeshPack or None, goal)."""
    rng = np.random.default_rng(seed)
    eng = engine
    lo = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
    hi = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])
    empty = np.zeros((0, 15))
    while True:
        goal = lo + (hi - lo) * rng.random(7)
        eng.set_scene(empty)
        if eng.collides(np.stack([START, goal])).any():
            continue
        boxes = []
        for _ in range(200 if n_obs else 0):
            cand = random_box_scene(rng, 1)
            eng.set_scene(obstacle_array(cand))
            if not eng.collides(np.stack([START, goal])).any():
                boxes += cand
            if len(boxes) == n_obs:
                break
        if len(boxes) < n_obs:
            continue
        meshes = []
        for _ in range(40 * n_mesh):
            cand = random_mesh_scene(rng, 1)
            eng.set_scene(empty, cand)
            if not eng.collides(np.stack([START, goal])).any():
                meshes += cand
            if len(meshes) == n_mesh:
                break
        if len(meshes) < n_mesh:
            continue
        obs = obstacle_array(boxes)
        pack = mesh_pack(meshes)
        eng.set_scene(obs, pack)
        if not (eng.torque_ok([goal], mode, mass)[0] and eng.torque_ok([START], mode, mass)[0]):
            continue
        # the straight start->goal edge must be blocked, so the tree has to grow to the goal
        ns, nt, _ = eng.check_edges([START], [goal], mode, mass)
        if ns[0] < nt[0]:
            return obs, pack, goal


HOST_MS = {"begin": 0.0, "run": 0.0, "finish": 0.0, "fetch": 0.0}  # host wall time per call
HOST_MS_LOCK = threading.Lock()  # run_query runs on several pool threads at once
GATHER = {"ok": True, "queries": 0, "rows": 0}  # rank 0's checks of the timed steps' gathers


def run_query(eng, obs, goal, n_samples, batch, seed, mode=_lib.TORQUE_RNE, mass=5.0,
              exec_time=5.0, meshes=None, shared=None):
    """One planning query.  shared: a communicator -- the ranks then grow ONE tree together
    (tcmp_plan_run_shared: each rank takes its share of every round's lanes)."""
    eng.set_scene(obs, meshes)
    world = shared.world if shared is not None else 1
    t0 = time.perf_counter()
    st = eng.plan_begin(START, goal, mode, mass, exec_time, max_nodes=n_samples + 1,
                        max_batch=-(-batch // world), seed=seed)
    if st != _lib.PLAN_OK:
        raise RuntimeError("start/goal in collision")
    t1 = time.perf_counter()
    if shared is not None:
        eng.plan_run_shared(shared, n_samples, batch)
    else:
        eng.plan_run(n_samples, batch)
    t2 = time.perf_counter()
    r = eng.plan_finish()
    t3 = time.perf_counter()
    out = eng.plan_fetch(r) if r.goal_found else None
    t4 = time.perf_counter()
    with HOST_MS_LOCK:
        for k, a, b in (("begin", t0, t1), ("run", t1, t2), ("finish", t2, t3), ("fetch", t3, t4)):
            HOST_MS[k] += (b - a) * 1e3
    return r, out


def run_fleet(engs, qs, n_samples, batch, seeds, mode=_lib.TORQUE_RNE, mass=5.0, exec_time=5.0):
    """len(qs) independent queries (each its own scene, goal and seed) as one fleet: begin each
    plan on its own engine, grow every tree in fused rounds (tcmp_plan_run_fused: one set of
    kernel launches per round for all of them), then finish and fetch each plan."""
    t0 = time.perf_counter()
    engs = engs[:len(qs)]
    for e, (obs, pack, goal) in zip(engs, qs):
        e.set_scene(obs, pack)
    cfgs = [_lib.plan_cfg(START, goal, mode, mass, exec_time, n_samples + 1, batch, seed)
            for (obs, pack, goal), seed in zip(qs, seeds)]
    if any(st != _lib.PLAN_OK for st in _lib.plan_begin_many(engs, cfgs)):
        raise RuntimeError("start/goal in collision")
    t1 = time.perf_counter()
    _lib.plan_run_fused(engs, n_samples, batch)
    t2 = time.perf_counter()
    rs = _lib.plan_finish_many(engs)
    t3 = time.perf_counter()
    outs = [e.plan_fetch(r) if r.goal_found else None for e, r in zip(engs, rs)]
    t4 = time.perf_counter()
    with HOST_MS_LOCK:
        for k, a, b in (("begin", t0, t1), ("run", t1, t2), ("finish", t2, t3), ("fetch", t3, t4)):
            HOST_MS[k] += (b - a) * 1e3
    return list(zip(rs, outs))


def usable_cores():
    """CPUs this process may actually run on: the affinity mask, capped by a cgroup v2 CPU
    quota (a GPU box shares its host: nproc counts the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def log(msg):
    print("[bench %.0fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


T_START = time.perf_counter()


def cpu_baseline(obs, goal, n_samples, seed, workers, mode=2, mass=5.0, meshes=None,
                 what="C3 scene (16 boxes, 5 kg, rne)"):
    """Oracle (C restatement of the reference loop, B = 1 = rrt_star.py semantics) on the
    same scene and Philox sample stream: single core in-process, then one independent query
    per host core (separate worker processes that never touch the GPU).  The all-core rate
    is the reported value (SURVEY 8d / BASELINE.md CPU-baseline plan)."""
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    O.set_meshes(meshes)
    t0 = time.perf_counter()
    ref = O.rrt_run(START, goal, n_samples, obs, mode, mass, 5.0, batch=1, seed=seed, cull=2,
                    tree=True)
    dt1 = time.perf_counter() - t0
    g = int(ref["goal_node"])
    depth = 0
    if g >= 0:
        n = g
        while n > 0:
            n = int(ref["tree_parent"][n])
            depth += 1
    q1 = quality([{"goal_node": g, "goal_cost": float(ref["tree_cost"][g]) if g >= 0 else 0.0,
                   "goal_depth": depth, "launches_nearest": n_samples,
                   "status": int(ref["status"])}])
    single = n_samples / dt1
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "scene.npz")
        extra = {}
        if meshes is not None:
            extra = dict(m_verts=meshes.verts, m_vert_off=meshes.vert_off, m_planes=meshes.planes,
                         m_plane_off=meshes.plane_off, m_edges=meshes.edges,
                         m_edge_off=meshes.edge_off, m_boxes=meshes.boxes)
        np.savez(path, start=START, goal=goal, obs=obs, mode=mode, mass=mass, **extra)
        worker = os.path.join(REPO, "oracle", "bench_worker.py")
        t0 = time.perf_counter()
        procs = [subprocess.Popen([sys.executable, worker, path, str(n_samples), str(seed + 1 + i)],
                                  stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
                 for i in range(workers)]
        outs = [p.communicate()[0] for p in procs]
        dtw = time.perf_counter() - t0
        done = [json.loads(o) for o, p in zip(outs, procs) if p.returncode == 0 and o.strip()]
    multi = sum(d["samples"] for d in done) / dtw if done else None
    nproc = os.cpu_count() or 1
    per_core = multi / len(done) if multi else single
    log("cpu baseline: %d workers, %.0f samples/s" % (len(done), multi or single))
    return {"value": multi if multi else single, "unit": "samples/s",
            "cores": len(done) if multi else 1, "host_nproc": nproc,
            "usable_cores": usable_cores(), "kind": "port",
            "single_core": single,
            # the single-core query's tree: B = 1, one sample per round
            "quality": q1,
            # SURVEY 8d asks for all host cores: the measured per-core rate scaled to nproc
            # (a shared GPU box lets this process use only its share of them), and one GPU's
            # share of an 8-GPU node's host cores
            "all_cores_scaled": {"cores": nproc, "value": per_core * nproc},
            "per_gpu_share": {"cores": nproc / 8.0, "value": per_core * nproc / 8.0},
            "sample": "oracle/tcmp_oracle.c sequential RRT* (B=1, reference loop semantics) on the "
                      "same %s: %d samples per query; single core "
                      "%.1f s (%d nodes, %d extend steps); %d independent queries, one per core, "
                      "%.1f s wall" % (what, n_samples, dt1, ref["n_nodes"], ref["edge_steps"],
                                       len(done), dtw)}


def quality(res):
    """What the timed queries planned, beside how fast: rounds per query (one nearest / edge
    launch set each), how many reached the goal, the goal node's cost (goal_n.cost,
    rrt_star.py:25-27 -- the returned path's summed distance fn) and depth (edges root -> goal),
    and the final statuses (0 ok, 2 no goal, 3 validation failure)."""
    found = [x for x in res if x.get("goal_node", -1) >= 0]
    costs = sorted(x["goal_cost"] for x in found)
    st = {}
    for x in res:
        st[str(x["status"])] = st.get(str(x["status"]), 0) + 1
    return {"queries": len(res),
            "rounds_per_query": sum(x["launches_nearest"] for x in res) / max(1, len(res)),
            "goal_rate": len(found) / max(1, len(res)),
            "path_cost_mean": sum(costs) / len(costs) if costs else None,
            "path_cost_median": costs[len(costs) // 2] if costs else None,
            "goal_depth_mean": (sum(x["goal_depth"] for x in found) / len(found)) if found else None,
            "status_counts": st}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS),
                    help="BASELINE.json config (default c3, the headline metric's config)")
    ap.add_argument("--samples", type=int, default=None, help="samples per query")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--obstacles", type=int, default=None, help="boxes per scene")
    ap.add_argument("--queries", type=int, default=None,
                    help="queries per step over all ranks (c4: 64; --queries 8 on one GPU is "
                         "one GPU's share of c4 at N = 8)")
    ap.add_argument("--cpu-samples", type=int, default=40000)
    ap.add_argument("--cpu-workers", type=int, default=usable_cores(),
                    help="worker processes of the multi-core CPU baseline (default: every "
                         "core this process may use -- affinity and cgroup quota; the all-core "
                         "and per-GPU (nproc/8) figures are the measured per-core rate scaled "
                         "to the host's nproc, reported beside it)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-alt", action="store_true",
                    help="skip the SURVEY 8d default-batch line (config_alt)")
    ap.add_argument("--no-sublines", action="store_true",
                    help="c3 on one GPU: skip the config_c4 / config_c5 sub-lines (BASELINE "
                         "configs[3] and [4] measured in the same run, after the headline)")
    ap.add_argument("--no-single", action="store_true",
                    help="skip the one-query-at-a-time pass of a single-query workload "
                         "(config_single_query; the sub-lines skip it)")
    ap.add_argument("--c5-steps", type=int, default=3,
                    help="steps of the config_c5 sub-line (one fleet of three 1e7-sample trees)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--self-collisions", action="store_true",
                    help="add the arm's self-collision pairs (off in the reference planner)")
    ap.add_argument("--shared-tree", action="store_true",
                    help="c3/c5: the GPUs grow ONE tree of the workload's samples per step "
                         "(shared-tree rounds, strong scaling) instead of one tree per GPU")
    ap.add_argument("--streams", type=int, default=None,
                    help="engines (one HIP stream each) driven concurrently by host threads "
                         "when a rank plans several queries per step (default 16 for c4, at most one per query)")
    ap.add_argument("--fleet", type=int, default=None,
                    help="queries per fused round (tcmp_plan_run_fused): a step's queries (c4) or "
                         "consecutive steps' queries (c2, c3) grow their trees in one set of "
                         "launches per round (default c2 8, c3 4, c4 16, c5 3, the best of a "
                         "one-box sweep; 0 or 1: one engine per query; a mesh scene fleets only "
                         "one query's replica trees, whose scene is the same)")
    ap.add_argument("--pipeline", type=int, default=None,
                    help="steps in flight at once: P consecutive steps' queries run concurrently "
                         "on separate engines from host threads, so one query's host calls and "
                         "kernel tails overlap another's kernels (not with --shared-tree); "
                         "default per workload (c2 3 fleets of 8, c3 2 fleets of 4, c4 3 fleets "
                         "of 16, c5 1 fleet of 3: the best of a one-box sweep); --pipeline 1 --fleet "
                         "0 runs the steps one after another")
    return ap.parse_args(argv)


SUBLINE_KEYS = ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "scaling", "config",
                "roofline", "roofline_other", "quality", "kernel_ms_per_step", "kernel_timing",
                "host_ms_per_step", "stats_last_step")


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    gpu = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; the collectives are libtcmp.so's RCCL communicator (no torch)
    comm = shard.comm_from_env(device=gpu) if world > 1 else None
    line = measure(args, world, rank, gpu, comm)
    # BASELINE configs[3] (C4, 64 queries) and configs[4] (C5, 256 meshes, 1e7 samples) in the
    # same default run, after the headline and its CPU baseline, so the driver's own run times
    # them too: each a full bench line of its workload (its own engines, warmup, timed steps and
    # rooflines), condensed; one GPU only (at N > 1 run --workload c4 / c5 for the sharded form)
    default_c3 = (args.workload == "c3" and args.samples is None and args.batch is None and
                  args.obstacles is None and not args.shared_tree and not args.self_collisions)
    if world == 1 and default_c3 and not args.no_sublines:
        for wl, steps in (("c4", args.steps), ("c5", args.c5_steps)):
            sub = parse_args(["--workload", wl, "--steps", str(max(1, steps)), "--warmup",
                              str(min(1, args.warmup)), "--no-cpu-baseline", "--no-alt",
                              "--no-single"])
            try:
                sl = measure(sub, world, rank, gpu, comm)
                line["config_%s" % wl] = {k: sl[k] for k in SUBLINE_KEYS if k in sl}
            except Exception as e:  # the headline stands; the sub-line says what failed
                line["config_%s" % wl] = {"error": "%s: %s" % (type(e).__name__, e)}
            log("sub-line %s done" % wl)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()


def measure(args, world, rank, gpu, comm):
    """One workload's bench line (a dict; printed by main on rank 0)."""
    W = dict(WORKLOADS[args.workload])
    if args.samples is not None:
        W["samples"] = args.samples
    if args.batch is not None:
        W["batch"] = args.batch
    if args.obstacles is not None:
        W["boxes"] = args.obstacles
    if args.queries is not None and W["queries"] > 1:
        W["queries"] = args.queries
    shared = args.shared_tree and W["queries"] == 1
    if shared:
        W["scaling"] = "strong"
        W["text"] = W["text"].split(" -- ")[0].split(", one query per GPU")[0] + \
            " -- shared tree: the GPUs grow one tree per step together (each rank takes its " \
            "share of every round's lanes; goal lane, counts and new nodes exchanged over RCCL)"
    elif args.workload == "c5":
        W["samples"] = W["samples"] // world  # 1e7 per step over all GPUs
    mode, mass = W["mode"], W["mass"]
    n_obs_total = W["boxes"] + W["meshes"]

    eng = _lib.Engine(gpu)
    # the spec peaks re-measured on this device, reported beside the spec figures
    try:
        measured = eng.microbench()
    except _lib.TcmpError as e:  # older library builds (A/B runs) lack the entry point
        measured = {"error": str(e)}
    # query ids of this rank: c4 shards 64 queries round-robin (scene and goal fixed per query
    # id); the single-query workloads run the same scene (query id 0) on every rank with
    # rank-dependent sample seeds -- independent trees of identical expected work, so the
    # per-GPU work stays fixed as N grows (weak scaling; c5 splits its samples instead)
    if W["queries"] > 1:
        qids = shard.queries_for_rank(W["queries"], world, rank)
        labels = list(qids)
        all_labels = list(range(W["queries"]))
    else:
        qids = [0]
        labels = [rank]
        all_labels = list(range(world))
    eng.set_self_collision(args.self_collisions)
    queries = [make_query(1234 + q, n_obs=W["boxes"], mode=mode, mass=mass, engine=eng,
                          n_mesh=W["meshes"]) for q in qids]

    def barrier():
        # every engine stream of this rank drained, then the ranks meet (RCCL all-reduce)
        for e in engines:
            e.synchronize()
        if comm is not None:
            comm.barrier()

    # a shared tree needs the same seed on every rank (one Philox stream, split by lanes)
    step_seed = (lambda s: 1234 + s) if shared else (lambda s: 1234 + rank * 100003 + s)  # noqa: E731

    # several queries per rank (c4): independent queries run concurrently on separate engines
    # (handles, one HIP stream each) from host threads -- the C-ABI calls release the GIL and
    # one 1e5-sample query's rounds do not fill the GPU on their own.  Single-query workloads
    # with --pipeline P run P consecutive steps at once the same way (step s on engine s mod P).
    pipe = max(1, args.pipeline if args.pipeline is not None else W.get("pipeline", 1)) \
        if not shared else 1
    # fused rounds (tcmp_plan_run_fused): the (query, step) pairs of the steps in flight, in
    # order, are dealt in fleets of `fleet` -- c4: a step's queries; a single-query workload:
    # consecutive steps' queries (each its own seed) -- with `pipe` fleets in flight, each on
    # its own group of engines
    fleet = args.fleet if args.fleet is not None else W.get("fleet", 0)
    # (convex-mesh scenes fuse only plans of one scene: the single-query workloads' steps)
    fleet = 0 if shared or ((W["meshes"] or args.self_collisions) and len(queries) > 1) else fleet
    fleets = fleet > 1
    if fleets:
        n_streams = max(1, args.streams if args.streams else pipe)
        n_engines = n_streams * fleet
    else:
        fleet = 0
        n_streams = max(1, min(len(queries) * pipe, args.streams if args.streams else 16))
        n_engines = n_streams
    engines = [eng] + [_lib.Engine(gpu) for _ in range(n_engines - 1)]
    for e in engines[1:]:
        e.set_self_collision(args.self_collisions)
    pool = None
    if n_streams > 1:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(n_streams)
    # one fleet at a time (c5): no launch overlaps another's, so the fleet's lead engine keeps
    # its event timing through the timed steps and those give the per-kernel figures (no
    # second pass of 1e7-sample fleets)
    lead_timed = fleets and n_streams == 1
    if n_engines > 1:
        # concurrent queries: no per-family event timing (an overlapped launch's span would
        # include its neighbours' kernels, and the round graphs then hold kernel nodes only; fused
        # rounds record none); the per-kernel figures come from the one-at-a-time pass after
        # the timed region
        for e in engines:
            e.set_timing(False)
        if lead_timed:
            engines[0].set_timing(True)

    def run_jobs(jobs):
        """jobs: (query index, step) pairs, or lists of them (fleets).  Each engine's thread
        takes the next job as soon as its last one is done, so P steps stay in flight the whole
        time (no barrier between groups of steps, no idle GPU while the slowest query of a
        group finishes)."""
        nxt = iter(range(len(jobs)))
        take = threading.Lock()

        def lane(k):
            got = []
            while True:
                with take:
                    idx = next(nxt, None)
                if idx is None:
                    return got
                if fleets:
                    # a fleet of (query, step) pairs on this thread's group of engines
                    pairs = jobs[idx]
                    done = run_fleet(engines[k * fleet:(k + 1) * fleet],
                                     [queries[j] for j, _ in pairs], W["samples"], W["batch"],
                                     [step_seed(s) + 7919 * j for j, s in pairs], mode, mass)
                    got += [(idx * fleet + t, s) + d for t, ((_, s), d) in enumerate(zip(pairs, done))]  # noqa: E501
                    continue
                j, s = jobs[idx]
                obs, pack, goal = queries[j]
                got.append((idx, s) + run_query(engines[k], obs, goal, W["samples"], W["batch"],
                                                step_seed(s) + 7919 * j, mode, mass, meshes=pack,
                                                shared=comm if shared else None))
        return sorted(sum(pool.map(lane, range(n_streams)) if pool else [lane(0)], []),
                      key=lambda x: x[0])

    def step_group(ss):
        pairs = [(j, s) for s in ss for j in range(len(queries))]
        # fleets of at most `fleet`, as equal as the pairs allow and a multiple of the threads
        # in number, so that every thread's group stays busy to the end (10 steps in fleets of
        # 4 on two threads: 3 + 2 + 3 + 2, not 4 + 4 + 2 with one thread idle at the end)
        if fleets:
            nf = n_streams * -(-len(pairs) // (n_streams * fleet))
            cut = [len(pairs) * i // nf for i in range(nf + 1)]
            jobs = [pairs[a:b] for a, b in zip(cut, cut[1:]) if b > a]
        else:
            jobs = pairs
        done = run_jobs(jobs)
        res = []
        for s in ss:
            part = [d for d in done if d[1] == s]
            outs = [d[3] for d in part]
            res += [d[2].as_dict() for d in part]
            if comm is not None and not shared:
                # RCCL gather of the solved trajectories (q, qd, qdd, dt) to rank 0 (configs[3]),
                # checked on rank 0: every rank's query ids arrived, row counts as all-gathered
                trajs = [shard.pack_trajectory(o) for o in outs]
                sizes = comm.allgather_i64([len(labels), sum(len(t) for t in trajs)])
                ids, rows, data = shard.pack_paths(trajs, labels)
                got = comm.gather_paths(ids, rows, data, int(sizes[:, 0].sum()),
                                        int(sizes[:, 1].sum()), sizes=sizes)
                if rank == 0:
                    got = shard.unpack_paths(*got)
                    GATHER["ok"] &= shard.gather_ok(got, all_labels, sizes)
                    GATHER["queries"] += len(got)
                    GATHER["rows"] += int(sizes[:, 1].sum())
        return res

    log("workload %s ready on rank %d of %d" % (args.workload, rank, world))
    if args.warmup:
        step_group([10_000 + i for i in range(
            args.warmup * pipe * (fleet if fleets and len(queries) == 1 else 1))])
    log("warmup done")

    barrier()
    for k in HOST_MS:
        HOST_MS[k] = 0.0
    GATHER.update(ok=True, queries=0, rows=0)
    t0 = time.perf_counter()
    results = []
    results += step_group(list(range(args.steps)))  # gathers (N > 1) follow, in step order
    barrier()
    dt = time.perf_counter() - t0
    log("timed steps done: %.3f s" % dt)
    # samples the devices actually drew (tcmp_plan_result.n_samples), summed over all ranks
    total_samples = float(sum(x["n_samples"] for x in results))
    if comm is not None:
        dt = float(comm.allreduce([dt], _lib.REDUCE_MAX)[0])
        total_samples = float(comm.allreduce([total_samples], _lib.REDUCE_SUM)[0])
    n_queries_total = W["queries"] if W["queries"] > 1 else (1 if shared else world)
    S = args.steps
    host_ms = {k: v / S for k, v in HOST_MS.items()}
    gathered = dict(GATHER)
    # Per-kernel figures (kernel_ms, the rooflines) need each launch's own duration.  With
    # queries in flight the engines ran without event timing (an overlapped launch's span would
    # include its neighbour's share of the GPU), so they come from as many queries again, run
    # one at a time on one engine after the timed region (same workload, fresh seeds, the
    # engine's graph captured first); for a single-query workload that pass is also the
    # one-query-at-a-time throughput (config_single_query), same build, same box.
    kres = results
    single = None
    if fleets and not lead_timed:
        # fused rounds: S fleets one at a time on one group of engines, timed on its first
        # engine (the fleet's kernel times are reported there; every plan counts the rounds);
        # a fleet = the first `fleet` (query, step) pairs' queries, fresh seeds
        grp = engines[:fleet]
        grp[0].set_timing(True)
        ids = [t % len(queries) for t in range(fleet)]
        qs = [queries[j] for j in ids]
        kseeds = lambda s: [step_seed(s) + 7919 * t for t in range(fleet)]  # noqa: E731
        for w in range(max(1, args.warmup)):
            run_fleet(grp, qs, W["samples"], W["batch"], kseeds(40_000 + 100 + w), mode, mass)
        kres = []
        for s in range(S):
            kres += [r.as_dict() for r, _ in run_fleet(grp, qs, W["samples"], W["batch"],
                                                       kseeds(40_000 + s), mode, mass)]
        grp[0].synchronize()
        grp[0].set_timing(False)
        barrier()
    if n_engines > 1 and (not fleets or (len(queries) == 1 and not args.no_single)):
        e0 = engines[0]
        e0.set_timing(True)
        obs, pack, goal = queries[0]
        for w in range(max(1, args.warmup)):  # the first query captures the round graph
            run_query(e0, obs, goal, W["samples"], W["batch"], step_seed(30_000 + 100 + w), mode,
                      mass, meshes=pack)
        e0.synchronize()
        t1 = time.perf_counter()
        kq = [run_query(e0, obs, goal, W["samples"], W["batch"], step_seed(30_000 + s), mode,
                        mass, meshes=pack)[0].as_dict() for s in range(S)]
        e0.synchronize()
        dts = time.perf_counter() - t1
        if not fleets:
            kres = kq
        if len(queries) == 1:
            single = {"value": sum(x["n_samples"] for x in kq) / dts * world,
                      "unit": "samples/s", "ms_per_step": dts / S * 1e3, "steps": S,
                      "queries_in_flight": 1,
                      "note": "the same workload one query at a time on one engine per GPU, "
                              "after the timed region (rank 0's time x ranks); the headline "
                              "value keeps %d queries in flight" % (pipe * max(1, fleet))}
        barrier()
    kernel_ms = {k: sum(x[k] for x in kres) / S for k in
                 ("ms_nearest", "ms_nn_scan", "ms_edge_prep", "ms_edges", "ms_insert", "ms_rewire",
                  "ms_finish")}
    if args.verbose and rank == 0:
        print(json.dumps({"per_step": results, "kernel_ms_per_step": kernel_ms}), file=sys.stderr)
    # one k_edges launch per round; one scan per round, except a one-node first round (nearest =
    # the root, no index).  The plans of a fleet share their rounds' launches.
    launches = int(round(sum(x["launches_nearest"] / max(1, x.get("fused_plans", 0)) for x in kres)))
    scans = int(round(sum(x["launches_nn_scan"] / max(1, x.get("fused_plans", 0)) for x in kres)))
    ek_name = ("k_fl_edges_mesh" if W["meshes"] else "k_fl_edges") if fleets else "k_edges"
    # (the fused-rounds scan's PMC entry: tools/pmc_summary.py)
    nn_key = "k_nearest_wave32@fleet" if fleets else "k_nearest_wave32"

    # k_nearest_wave32: 21 flop (fp32 first pass) per (candidate, node) pair it evaluated.  The
    # brute-force-equivalent rate (SURVEY 8d F_nn = 21 T per sample) counts pairs the pruned
    # search never touches, so it is reported beside it, not as "achieved".
    nn_pairs = sum(x["nn_pairs"] for x in kres)
    nn_full = sum(x["nn_full_pairs"] for x in kres)
    nn_ms = sum(x["ms_nn_scan"] for x in kres)
    nn_tf = NN_FLOP_PER_PAIR * nn_pairs / (nn_ms * 1e-3) / 1e12 if nn_ms > 0 else 0.0
    roof_nn = {
        "kernel": "k_nearest_wave32<FLEET>" if fleets else "k_nearest_wave32",
        "avg_launch_ms": nn_ms / max(1, scans),
        "bound": "valu_fp32", "achieved": nn_tf, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
        "frac": nn_tf / PEAK_FP32_TFLOPS, "traffic": pmc_traffic(nn_key, args.workload),
        "measured_valu": pmc_valu(nn_key, args.workload, PEAK_FP32_TFLOPS,
                                  ("SQ_INSTS_VALU_FLOPS_FP32",)),
        "algorithmic": "%d flop per evaluated (candidate, node) pair; %d pairs over %d launches "
                       "(brute force would be %d pairs: %.1f PFLOP/s equivalent)" % (
                           NN_FLOP_PER_PAIR, nn_pairs, scans, nn_full,
                           NN_FLOP_PER_PAIR * nn_full / (nn_ms * 1e-3) / 1e15 if nn_ms else 0.0)}
    # k_edges: SURVEY 8d per-step work F_fk + F_bp * L * n_obs + F_rne, + F_sat per pair that
    # survives the cull (device counters).  The steps are k_edges' own: edge_steps less the
    # rewire edges' (k_rewire_apply, timed under ms_rewire).  Tier 0's F_bp runs in packed
    # fp32, the rest in fp64, so the bound is the mixed one: the time the fp64 flop need at the
    # fp64 peak plus the time the fp32 flop need at the fp32 peak; "peak" is the flop rate that
    # time implies and frac = that time / the measured time.  frac_fp64_contract is the
    # round-1..4 figure (every flop charged at the fp64 peak).
    steps = sum(x["edge_steps"] - x.get("rewire_steps", 0) for x in kres)
    sat = sum(x["pairs_sat"] for x in kres)
    f_rne = 0 if mode == _lib.TORQUE_BASE else F_RNE_STATIC
    flop64 = steps * (F_FK + f_rne) + F_SAT * sat
    flop32 = steps * F_BP * N_LINKS * n_obs_total
    edge_flop = flop64 + flop32
    t_min = flop64 / (PEAK_FP64_TFLOPS * 1e12) + flop32 / (PEAK_FP32_TFLOPS * 1e12)
    ed_ms = sum(x["ms_edges"] for x in kres)
    ed_tf = edge_flop / (ed_ms * 1e-3) / 1e12 if ed_ms > 0 else 0.0
    peak_mixed = edge_flop / t_min / 1e12 if t_min > 0 else PEAK_FP64_TFLOPS
    roof_ed = {
        "kernel": ek_name, "avg_launch_ms": ed_ms / max(1, launches),
        "bound": "valu_fp64+fp32", "achieved": ed_tf, "peak": peak_mixed, "unit": "TFLOP/s",
        "frac": ed_tf / peak_mixed, "frac_fp64_contract": ed_tf / PEAK_FP64_TFLOPS,
        "traffic": pmc_traffic(ek_name, args.workload),
        # the hardware's own count of the kernel's fp64 VALU flop (PMC), beside the SURVEY 8d
        # contract flop above
        "measured_valu": pmc_valu(ek_name, args.workload, PEAK_FP64_TFLOPS),
        "algorithmic": "per extend step F_fk %d + F_rne %d (fp64) + F_bp %d x %d links x %d "
                       "obstacles (packed fp32), + F_sat %d per pair past the cull (fp64); %d "
                       "edge steps (rewire steps excluded), %d such pairs, %d launches" % (
                           F_FK, f_rne, F_BP, N_LINKS, n_obs_total, F_SAT, steps, sat,
                           launches)}
    for roof, peak in ((roof_nn, PEAK_FP32_TFLOPS), (roof_ed, PEAK_FP64_TFLOPS)):
        mv = roof["measured_valu"]
        if mv and roof["avg_launch_ms"] > 0:
            # the PMC flop per launch over this run's event-timed average launch
            mv["tflops_live"] = mv["flop_per_launch"] / (roof["avg_launch_ms"] * 1e-3) / 1e12
            mv["frac_live"] = mv["tflops_live"] / peak
    mv32 = pmc_valu(ek_name, args.workload, PEAK_FP32_TFLOPS, ("SQ_INSTS_VALU_FLOPS_FP32",))
    mv = roof_ed["measured_valu"]
    if mv and mv32 and roof_ed["avg_launch_ms"] > 0:
        # the hardware's fp64 and fp32 flop against the same mixed bound as "frac"
        t_hw = mv["flop_per_launch"] / (PEAK_FP64_TFLOPS * 1e12) + \
            mv32["flop_per_launch"] / (PEAK_FP32_TFLOPS * 1e12)
        mv["fp32_flop_per_launch"] = mv32["flop_per_launch"]
        mv["frac_live_mixed"] = t_hw / (roof_ed["avg_launch_ms"] * 1e-3)
    for roof, key in ((roof_nn, "fp32_tflops"), (roof_ed, "fp64_tflops")):
        if measured.get(key):
            roof["peak_measured"] = measured[key]
            roof["frac_measured"] = roof["achieved"] / measured[key]
    dominant, other = (roof_nn, roof_ed) if nn_ms >= ed_ms else (roof_ed, roof_nn)
    # north-star HBM figure: compulsory bytes per query = 68 T_r per round (tree read
    # once) + 72 B_r per round (candidates written) + trajectory rows, over the step time
    snap = sum(x["snap_sum"] for x in results)
    hbm_bytes = 68 * snap + 72 * sum(x["n_samples"] for x in results) + \
        22 * 8 * sum(x["n_traj"] for x in results)
    hbm_gbs = hbm_bytes / (dt / 1.0) / 1e9 * world if dt > 0 else 0.0
    hbm_peak_meas = measured.get("hbm_gbs")

    line = {
        "metric": "torque-feasible collision-checked RRT* samples/sec, Panda 7-DOF, 1/2/4/8 GPU",
        "value": total_samples / dt,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": W["scaling"],
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY 8d %s scene, Philox4x32-10 samples)" % (
            "convex-mesh" if W["meshes"] else "box"),
        "config": {"workload": W["text"], "boxes": W["boxes"], "meshes": W["meshes"],
                   "samples_per_query": W["samples"], "queries_per_step": n_queries_total,
                   "batch_per_round": W["batch"], "execution_time_s": 5.0,
                   "parallelism": ("shared-tree x%d" if shared else "query-sharded x%d") % world,
                   "streams_per_gpu": n_engines, "pipelined_steps": pipe,
                   "queries_in_flight": (n_streams * fleet if fleets
                                         else min(n_streams, len(queries) * pipe)),
                   "fused_queries": fleet if fleets else 1,
                   "self_collisions": bool(args.self_collisions)},
        "roofline": dominant,
        "roofline_other": other,
        "hbm_roofline": {"bytes_per_step": hbm_bytes / S, "achieved": hbm_gbs, "unit": "GB/s",
                         "peak": PEAK_HBM_GBS, "frac": hbm_gbs / PEAK_HBM_GBS,
                         "peak_measured": hbm_peak_meas,
                         "definition": "SURVEY 8d compulsory bytes: 68 T_r + 72 B_r per round "
                                       "+ 176 B per trajectory row, whole job"},
        "measured_peaks": measured,
        "kernel_ms_per_step": kernel_ms,
        "kernel_timing": ("the timed steps: one fleet of %d queries at a time, kernel times on "
                          "its lead engine, kernel_ms per step (query)" % fleet if lead_timed else
                          "%d fleets of %d queries run one at a time after the timed steps, "
                          "kernel_ms per fleet (fleets in flight run untimed per kernel)" % (
                              S, fleet) if fleets else
                          "%d queries run one at a time on one engine after the timed steps "
                          "(queries in flight run untimed per kernel)" % S
                          if kres is not results else "the timed steps"),
        # host wall time inside the C-ABI calls (rank 0; the GPU work of a step completes
        # inside plan_finish's first wait, so "finish" holds most of the step)
        "host_ms_per_step": host_ms,
        "host_ms_note": ("per step, summed over the host threads of the queries in flight"
                         if n_engines > 1 else "per step"),
        "stats_last_step": {k: results[-1][k] for k in ("status", "n_nodes", "n_waypoints", "n_traj",
                                                        "edge_steps", "pairs_tested", "pairs_sat",
                                                        "pairs_exact")},
        # rank 0's timed queries: rounds, goal rate, path cost / depth, statuses
        "quality": quality(results),
    }
    if comm is not None:
        # proof of the collective world the run used: RCCL's own rank count, and rank 0's check
        # that every gather delivered every query id with the all-gathered row counts
        line["rccl_ranks"] = comm.rccl_ranks()
        # every rank's drawn samples (replica / sharded mode: each rank's own trees)
        per_rank = comm.allgather_i64([int(sum(x["n_samples"] for x in results))])
        line["samples_per_rank"] = [int(v) for v in per_rank[:, 0]]
        if shared:
            # proof that the ranks grew ONE tree: the device digest of the last step's tree
            # (tcmp_plan_digest), all-gathered; equal digests and node counts on every rank
            d, nn = eng.plan_digest()
            g = comm.allgather_i64([d - (1 << 64) if d >= (1 << 63) else d, nn])
            line["tree_consistent"] = bool((g == g[0]).all())
            line["tree_digest"] = "%016x" % d
            line["tree_nodes"] = int(nn)
        if not shared:
            line["gather_ok"] = bool(gathered["ok"])
            line["gathered"] = {"queries": gathered["queries"], "rows": gathered["rows"],
                                "steps": S}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        obs, pack, goal = queries[0]
        cpu_n = args.cpu_samples if not W["meshes"] else max(1000, args.cpu_samples // 10)
        line["cpu_baseline"] = cpu_baseline(obs, goal, cpu_n, step_seed(0), args.cpu_workers,
                                            mode, mass, meshes=pack,
                                            what=W["text"].split(",")[0] + " scene")
    if rank == 0 and world == 1 and W.get("alt_batch") and not args.no_alt:
        # the same workload at SURVEY 8d's default batch, beside the headline's tuned batch
        # (the batch changes the tree: more, smaller rounds see fresher snapshots)
        alt = dict(W, batch=W["alt_batch"])
        obs, pack, goal = queries[0]
        for w in range(args.warmup):
            run_query(eng, obs, goal, alt["samples"], alt["batch"], step_seed(20_000 + w), mode,
                      mass, meshes=pack)
        eng.synchronize()
        t1 = time.perf_counter()
        alt_res = [run_query(eng, obs, goal, alt["samples"], alt["batch"], step_seed(s), mode,
                             mass, meshes=pack)[0].as_dict() for s in range(args.steps)]
        eng.synchronize()
        dta = time.perf_counter() - t1
        line["config_alt"] = {
            "batch_per_round": alt["batch"], "steps": args.steps,
            "value": sum(x["n_samples"] for x in alt_res) / dta, "unit": "samples/s",
            "ms_per_step": dta / args.steps * 1e3,
            "edge_steps_per_sample": sum(x["edge_steps"] for x in alt_res) /
            max(1, sum(x["n_samples"] for x in alt_res)),
            "quality": quality(alt_res),
            "note": "SURVEY 8d default batch; the headline line runs batch_per_round %d" % W["batch"]}
        line["config"]["edge_steps_per_sample"] = steps / max(1.0, float(
            sum(x["n_samples"] for x in kres)))
    if single is not None:
        line["config_single_query"] = single
    if pool is not None:
        pool.shutdown(wait=True)
    for e in reversed(engines):  # every engine released explicitly, the first one last
        e.close()
    return line


if __name__ == "__main__":
    main()
