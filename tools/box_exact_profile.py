#!/usr/bin/env python3
"""Exit stages and stage clocks of the hull-vs-box exact test on C3 (profiling build:
make -C torque_constrained_motion_planning_amd/csrc prof; TCMP_LIB_PATH=.../libtcmp_prof.so)."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from torque_constrained_motion_planning_amd import _lib  # noqa: E402

eng = _lib.Engine(0)
obs, _, goal = bench.make_query(1234, engine=eng)
r, _ = bench.run_query(eng, obs, goal, 1_000_000, 262144, 1234)
c = eng.debug_counters(52)
tot = max(1, c[0])
clk = c[28:32]
print(json.dumps({
    "pairs_exact": r.pairs_exact, "box_face_exit": c[12], "facet_exit": c[13],
    "edge_or_full": c[14], "edge_early_free": c[47], "full_collision": c[48],
    "full_free": c[49], "degenerate": c[15],
    "exact_clk_share_of_edges": c[5] / tot, "k_edges_clk": c[0],
    "stage_clk": {"box_faces": clk[0], "facets": clk[2], "edges": clk[3]},
    "stage_clk_share_of_exact": {k: v / max(1, c[5]) for k, v in
                                 zip(("box_faces", "-", "facets", "edges"), clk) if k != "-"}}))
