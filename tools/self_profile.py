#!/usr/bin/env python3
"""k_edges clock breakdown on C3 with the self-collision pairs on (profiling build).

usage: TCMP_LIB_PATH=torque_constrained_motion_planning_amd/libtcmp_prof.so \
       python tools/self_profile.py
"""
import json, sys, os
sys.path.insert(0, os.getcwd())
import bench
from torque_constrained_motion_planning_amd import _lib
eng = _lib.Engine(0)
eng.set_self_collision(True)
obs, pack, goal = bench.make_query(1234, engine=eng)
r, _ = bench.run_query(eng, obs, goal, 1_000_000, 262144, 1234)
c = eng.debug_counters(36)
tot = max(1, c[0])
print(json.dumps({"ms_edges": r.ms_edges, "fetch": c[1]/tot, "collision": c[2]/tot, "torque": c[3]/tot,
   "exact": c[5]/tot, "t123_flush": c[7]/tot, "sincos": c[6]/tot,
   "mesh_counts": {"outer_box_free": c[16], "outer_lod_free": c[17], "inner_collision": c[18], "fp64": c[19]},
   "mesh_stage_clk_share_of_total": [round(x/tot, 4) for x in c[28:33]],
   "pairs_sat": r.pairs_sat, "pairs_exact": r.pairs_exact}))
