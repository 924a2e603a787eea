#!/usr/bin/env python3
"""Planned vs executed extend steps per round on the C3 workload: how many steps a fully
speculative (all steps of every edge at once) edge check would evaluate beyond the sequential
walk's first failing step.  usage: python tools/edge_waste.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from torque_constrained_motion_planning_amd import _lib  # noqa: E402

RES = 0.1


def main():
    eng = _lib.Engine(0)
    obs, _, goal = bench.make_query(1234, engine=eng)
    B = 262144
    eng.set_scene(obs)
    eng.plan_begin(bench.START, goal, _lib.TORQUE_RNE, 5.0, 5.0, max_nodes=1_000_001,
                   max_batch=B, seed=1234)
    prev_steps = 0
    for r in range(4):
        eng.plan_run(B, B)
        cand, nn, score, snap = eng.plan_debug_round(B)
        nb = len(cand)
        cfg = eng.plan_tree(2_000_000)[0]
        d = (cand - cfg[nn]) / RES
        planned = (np.floor(np.sqrt((d * d).sum(1))).astype(np.int64) + 1)
        print(json.dumps({"round": r, "snap": int(snap), "nb": int(nb),
                          "planned_steps": int(planned.sum()),
                          "planned_mean": float(planned.mean()),
                          "planned_p50": float(np.median(planned)),
                          "planned_max": int(planned.max())}), flush=True)
    r = eng.plan_finish()
    print(json.dumps({"executed_steps_all_rounds": int(r.edge_steps), "n_samples": int(r.n_samples)}))


if __name__ == "__main__":
    main()
