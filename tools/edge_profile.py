#!/usr/bin/env python3
"""k_edges clock breakdown on the C3 workload (profiling build libtcmp_prof.so, -DTCMP_PROF).

usage: TCMP_LIB_PATH=torque_constrained_motion_planning_amd/libtcmp_prof.so \
       python tools/edge_profile.py [n_queries]
Prints, per query, the share of wave clocks k_edges spends fetching work, in the collision
check (and its tier-4 exact part), in the torque check and in bookkeeping.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from torque_constrained_motion_planning_amd import _lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    eng = _lib.Engine(0)
    obs, _, goal = bench.make_query(1234, engine=eng)
    prev = [0] * 4
    pprev = [0] * 8
    for q in range(n):
        r, _ = bench.run_query(eng, obs, goal, 1_000_000, 262144, 1234 + q)
        c = eng.debug_counters(128)
        ex = [a - b for a, b in zip(c[8:12], prev)]
        prev = c[8:12]
        ps = [a - b for a, b in zip(c[120:128], pprev)]
        pprev = c[120:128]
        npass = max(1, ps[0])
        tot = max(1, c[0])
        print(json.dumps({"query": q, "ms_edges": r.ms_edges, "total_clk": c[0],
                          "fetch": c[1] / tot, "collision": c[2] / tot, "torque": c[3] / tot,
                          "tail": c[4] / tot, "exact_in_collision": c[5] / tot,
                          "sincos": c[6] / tot, "tiers123_in_collision": c[7] / tot,
                          "exact32_box_exit": ex[0], "exact32_facets_would_exit": ex[1],
                          "exact32_full": ex[2], "exact32_degenerate": ex[3],
                          "edge_steps": r.edge_steps, "pairs_sat": r.pairs_sat,
                          "pairs_exact": r.pairs_exact, "box_cert_collision": c[33],
                          "box_cert_free": c[34],
                          # phase B's 64-entry passes: entries, distinct source lanes and
                          # (lane, link) per pass, entries of links 7..9, and the share of
                          # wave clocks from a pass's start to its exact loop (pose + tiers 1-3)
                          "phaseB": {"passes": ps[0], "entries_per_pass": ps[1] / npass,
                                     "lanes_per_pass": ps[2] / npass,
                                     "lane_links_per_pass": ps[3] / npass,
                                     "distal_share": ps[4] / max(1, ps[1]),
                                     "pose_tiers_clk": ps[5] / tot}}), flush=True)


if __name__ == "__main__":
    main()
