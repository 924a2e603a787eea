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
gathered to rank 0 over RCCL at the end of each step, as in configs[3].

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from torque_constrained_motion_planning_amd import _lib, shard  # noqa: E402
from torque_constrained_motion_planning_amd.scene import obstacle_array, random_box_scene  # noqa: E402

START = np.array([0, -np.pi / 4, 0.0, -6 * np.pi / 8, 0, np.pi / 2, np.pi / 4])  # utils.py:45
PEAK_FP32_TFLOPS = 157.3    # MI355X fp32 vector peak (spec, MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0       # MI355X HBM3E peak (MI355X_MICROARCH.md)
NN_FLOP_PER_PAIR = 21       # 7 sub + 7 fma per (candidate, node) pair, fp32 first pass (SURVEY 8d F_nn)
NN_BYTES_PER_NODE = 64      # one tree record (q0..q6, cost) streamed per block


def make_query(seed, n_obs=16, mode=_lib.TORQUE_RNE, mass=5.0, engine=None):
    """Scene + goal: boxes rejected while start/goal collide; goal collision-free and
    torque-feasible."""
    rng = np.random.default_rng(seed)
    eng = engine
    lo = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
    hi = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])
    while True:
        goal = lo + (hi - lo) * rng.random(7)
        boxes = []
        for _ in range(200):
            cand = random_box_scene(rng, 1)
            arr = obstacle_array(boxes + cand)
            eng.set_scene(arr)
            if not eng.collides(np.stack([START, goal])).any():
                boxes += cand
            if len(boxes) == n_obs:
                break
        if len(boxes) < n_obs:
            continue
        obs = obstacle_array(boxes)
        eng.set_scene(obs)
        if not (eng.torque_ok([goal], mode, mass)[0] and eng.torque_ok([START], mode, mass)[0]):
            continue
        # the straight start->goal edge must be blocked, so the tree has to grow to the goal
        ns, nt, _ = eng.check_edges([START], [goal], mode, mass)
        if ns[0] < nt[0]:
            return obs, goal


def run_query(eng, obs, goal, n_samples, batch, seed, mode=_lib.TORQUE_RNE, mass=5.0,
              exec_time=5.0):
    eng.set_scene(obs)
    st = eng.plan_begin(START, goal, mode, mass, exec_time, max_nodes=n_samples + 1,
                        max_batch=batch, seed=seed)
    if st != _lib.PLAN_OK:
        raise RuntimeError("start/goal in collision")
    eng.plan_run(n_samples, batch)
    r = eng.plan_finish()
    out = eng.plan_fetch(r) if r.goal_found else None
    return r, out


def cpu_baseline(obs, goal, n_samples, seed, mode=2, mass=5.0):
    """Oracle (C restatement of the reference loop, B = 1 = rrt_star.py semantics) on the
    same scene and Philox sample stream, single core."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    t0 = time.perf_counter()
    ref = O.rrt_run(START, goal, n_samples, obs, mode, mass, 5.0, batch=1, seed=seed, cull=2)
    dt = time.perf_counter() - t0
    return {"value": n_samples / dt, "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": "oracle/tcmp_oracle.c sequential RRT* (B=1, reference loop semantics), "
                      "first %d samples of the same C3 query (16 boxes, 5 kg, rne), %.1f s, "
                      "%d nodes, %d extend steps" % (n_samples, dt, ref["n_nodes"], ref["edge_steps"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--samples", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--obstacles", type=int, default=16)
    ap.add_argument("--cpu-samples", type=int, default=50000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl")
        dist = tdist

    eng = _lib.Engine(local_rank)
    # one scene per rank (query id = rank); the goal is fixed per rank, seeds vary per step
    obs, goal = make_query(1234 + rank, n_obs=args.obstacles, engine=eng)

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    def gather(out, qid):
        # RCCL gather of the solved trajectories (q, qd, qdd, dt) to rank 0 (configs[3])
        if dist is None:
            return
        shard.gather_trajectories(dist, [shard.pack_trajectory(out)], [qid], world, rank,
                                  device="cuda")

    step_seed = lambda s: 1234 + rank * 100003 + s  # noqa: E731
    for w in range(args.warmup):
        r, out = run_query(eng, obs, goal, args.samples, args.batch, step_seed(10_000 + w))
        gather(out, w)

    barrier()
    t0 = time.perf_counter()
    results = []
    for s in range(args.steps):
        r, out = run_query(eng, obs, goal, args.samples, args.batch, step_seed(s))
        gather(out, s * world + rank)
        results.append(r.as_dict())
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    total_samples = args.samples * args.steps * world
    # dominant kernel: k_nearest_wave32 (pruned Morton-chunk argmin over the snapshot, fp32
    # first pass + exact fp64 refinement); ms_nn_scan = hipEvents around its launches only,
    # on the engine's stream.  Achieved = 21 flop x evaluated pairs / scan time.
    nn_pairs = sum(x["nn_pairs"] for x in results)
    nn_ms = sum(x["ms_nn_scan"] for x in results)
    nn_launches = sum(x["launches_nearest"] for x in results)
    achieved_tflops = NN_FLOP_PER_PAIR * nn_pairs / (nn_ms * 1e-3) / 1e12 if nn_ms > 0 else 0.0
    # HBM traffic per k_nearest_wave32 launch from the committed rocprofv3 PMC passes of this same
    # workload (profiles/*_pmc_hbm.json; FETCH_SIZE doubled per the gfx950 correction)
    traffic = None
    pmc = sorted(f for f in os.listdir(os.path.join(REPO, "profiles")) if f.endswith("_pmc_hbm.json")) \
        if os.path.isdir(os.path.join(REPO, "profiles")) else []
    if pmc:
        d = json.load(open(os.path.join(REPO, "profiles", pmc[-1])))["dispatches"].get(
            "k_nearest_wave32", [])
        fetch = [x["value_KiB"] for x in d if x["counter"] == "FETCH_SIZE"]
        write = [x["value_KiB"] for x in d if x["counter"] == "WRITE_SIZE"]
        if fetch and len(fetch) == len(write):
            traffic = (2 * sum(fetch) + sum(write)) * 1024 / len(fetch)
    kernel_ms = {k: sum(x[k] for x in results) / args.steps for k in
                 ("ms_nearest", "ms_nn_scan", "ms_edges", "ms_insert", "ms_rewire", "ms_finish")}
    if args.verbose and rank == 0:
        print(json.dumps({"per_step": results, "kernel_ms_per_step": kernel_ms}), file=sys.stderr)

    line = {
        "metric": "torque-feasible collision-checked RRT* samples/sec, Panda 7-DOF, 1/2/4/8 GPU",
        "value": total_samples / dt,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY 8d box scene, Philox4x32-10 samples)",
        "config": {"workload": "C3: Panda 7-DOF, %d axis-aligned boxes, 5 kg payload, torque_test=rne "
                               "+ min-jerk v/a validation, %d samples per query, one query per "
                               "GPU per step" % (args.obstacles, args.samples),
                   "batch_per_round": args.batch, "execution_time_s": 5.0,
                   "parallelism": "query-sharded x%d" % world},
        "roofline": {
            "kernel": "k_nearest_wave32",
            "avg_launch_ms": nn_ms / max(1, nn_launches),
            "bound": "valu_fp32",
            "achieved": achieved_tflops,
            "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved_tflops / PEAK_FP32_TFLOPS,
            "traffic": traffic,
            "traffic_unit": "bytes per launch (rocprofv3 PMC, %s)" % (pmc[-1] if pmc else "none"),
            "algorithmic": "%d flop per (candidate, node) pair; %d pairs over %d launches" % (
                NN_FLOP_PER_PAIR, nn_pairs, nn_launches),
        },
        "kernel_ms_per_step": kernel_ms,
        "stats_last_step": {k: results[-1][k] for k in ("status", "n_nodes", "n_waypoints", "n_traj",
                                                        "edge_steps", "pairs_tested", "pairs_sat",
                                                        "pairs_exact")},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(obs, goal, args.cpu_samples, step_seed(0))
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
