#!/usr/bin/env python3
"""GPU helper for tests/golden/gen_fullsize.py: on the bench's C5 scene (bench.make_query(1234,
n_mesh=256)), which (batch, sample seed) plan reaches the goal, so the bit-exact C5 fixture can
cover several rounds, the goal, min-jerk and validation.  Prints one JSON line per plan: batch,
seed, samples, status, nodes, goal node, rewires.

    python tools/c5_fixture_search.py                      # the round-3 search (small batches)
    python tools/c5_fixture_search.py 262144 562816 40     # the bench's batch: two full rounds
                                                           # (k_edges<true,1>) + a 38,528-lane
                                                           # round (k_edges<true,2>), 40 seeds
    python tools/c5_fixture_search.py 262144 562816:824960 16   # several sample counts
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from torque_constrained_motion_planning_amd import _lib  # noqa: E402

eng = _lib.engine(0)
obs, pack, goal = bench.make_query(1234, n_obs=0, mode=2, mass=5.0, engine=eng, n_mesh=256)
if len(sys.argv) > 1:
    batch = int(sys.argv[1])
    n_seeds = int(sys.argv[3]) if len(sys.argv) > 3 else 24
    plans = [(batch, int(s), n_seeds) for s in sys.argv[2].split(":")]  # samples: a:b:c
else:
    plans = [(16384, 16384 * 8, 12), (32768, 32768 * 6, 12), (65536, 65536 * 5, 12)]
for batch, samples, n_seeds in plans:
    for seed in range(1234, 1234 + n_seeds):
        r, out = bench.run_query(eng, obs, goal, samples, batch, seed, meshes=pack)
        print(json.dumps(dict(batch=batch, seed=seed, samples=samples, status=r.status,
                              nodes=r.n_nodes, goal_node=r.goal_node, rewires=r.n_rewires,
                              n_traj=r.n_traj)), flush=True)
