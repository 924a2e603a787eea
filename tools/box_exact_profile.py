#!/usr/bin/env python3
"""Exit stages of the hull-vs-box exact test on C3 (profiling build with TCMP_PROF_EXACT)."""
import json, sys, os
sys.path.insert(0, os.getcwd())
import bench
from torque_constrained_motion_planning_amd import _lib
eng = _lib.Engine(0)
obs, _, goal = bench.make_query(1234, engine=eng)
r, _ = bench.run_query(eng, obs, goal, 1_000_000, 262144, 1234)
c = eng.debug_counters(16)
tot = max(1, c[0])
print(json.dumps({"pairs_exact": r.pairs_exact, "box_face_exit": c[12], "facet_exit": c[13], "edge_or_full": c[14], "degenerate": c[15], "exact_clk_share": c[5]/tot}))
