#!/usr/bin/env python3
"""CPU-baseline worker for bench.py (test/benchmark infrastructure, never product code).

Runs the oracle's sequential RRT* (B = 1, reference loop semantics) on one query and prints
one JSON line.  bench.py starts one worker process per host core so the multi-core baseline
is "one independent query per core" (SURVEY 8d); the workers never touch the GPU.

usage: python oracle/bench_worker.py SCENE.npz N_SAMPLES SEED
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle as O  # noqa: E402


def main():
    z = np.load(sys.argv[1])
    n, seed = int(sys.argv[2]), int(sys.argv[3])
    if "m_verts" in z:
        class Pack:  # the MeshPack fields the oracle reads
            def __init__(self):
                for k in ("verts", "vert_off", "planes", "plane_off", "edges", "edge_off", "boxes"):
                    setattr(self, k, z["m_" + k])
                self.n = len(self.boxes)

            def __len__(self):
                return self.n
        O.set_meshes(Pack())
    t0 = time.perf_counter()
    r = O.rrt_run(z["start"], z["goal"], n, z["obs"], int(z["mode"]), float(z["mass"]), 5.0,
                  batch=1, seed=seed, cull=2)
    dt = time.perf_counter() - t0
    print(json.dumps({"samples": n, "seconds": dt, "n_nodes": r["n_nodes"],
                      "edge_steps": r["edge_steps"]}))


if __name__ == "__main__":
    main()
