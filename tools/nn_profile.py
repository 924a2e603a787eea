#!/usr/bin/env python3
"""k_nearest_wave32 clock breakdown on the C3 workload (profiling build, -DTCMP_PROF).

usage: TCMP_LIB_PATH=torque_constrained_motion_planning_amd/libtcmp_prof.so \\
       python tools/nn_profile.py [n_queries]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from torque_constrained_motion_planning_amd import _lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    eng = _lib.Engine(0)
    obs, _, goal = bench.make_query(1234, engine=eng)
    for q in range(n):
        r, _ = bench.run_query(eng, obs, goal, 1_000_000, 262144, 1234 + q)
        cc = eng.debug_counters(44)
        c, v = cc[36:41], cc[41:44]
        tot = max(1, sum(c))
        print(json.dumps({"query": q, "ms_nn_scan": r.ms_nn_scan, "nn_pairs": r.nn_pairs,
                          "nn_box_tests": r.nn_box_tests,
                          "setup_home": c[0] / tot, "super_bounds": c[1] / tot,
                          "chunk_bounds": c[2] / tot, "chunk_scans": c[3] / tot,
                          "final": c[4] / tot,
                          "super_box_wave_tests": v[0], "cell_box_wave_tests": v[1],
                          "cells_scanned": v[2]}), flush=True)


if __name__ == "__main__":
    main()
