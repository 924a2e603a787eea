"""Queries in flight together (bench.py --pipeline, C4's engines): several engines on one GPU,
each driven from its own host thread, must build exactly the trees and trajectories they build
one at a time -- nothing of one handle's state may leak into another's while their kernels
overlap.  Box and convex-mesh scenes."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(eng, q, n, batch, seed, mode, mass):
    import bench
    obs, pack, goal = q
    r, out = bench.run_query(eng, obs, goal, n, batch, seed, mode, mass, meshes=pack)
    # (not pairs_exact: which pairs an exact test skips because its lane already collides
    # depends on which edges share a wave, i.e. on the persistent kernel's dynamic deal)
    return (eng.plan_digest(), r.status, r.n_nodes, r.n_waypoints, r.n_traj, r.edge_steps,
            out["q"].tobytes() if out is not None else b"")


@pytest.mark.parametrize("n_obs,n_mesh,n,batch,k", [
    (16, 0, 100_000, 65536, 3),   # C3-like boxes, rne
    (0, 16, 20_000, 4096, 2),     # convex meshes (the C5 kernels)
])
def test_concurrent_queries_equal_one_at_a_time(n_obs, n_mesh, n, batch, k):
    import bench
    from torque_constrained_motion_planning_amd import _lib
    mode, mass = _lib.TORQUE_RNE, 5.0
    engines = [_lib.Engine(0) for _ in range(k)]
    queries = [bench.make_query(4242 + j, n_obs=n_obs, mode=mode, mass=mass, engine=engines[0],
                                n_mesh=n_mesh) for j in range(k)]
    seeds = [9000 + 17 * j for j in range(k)]
    alone = [_run(engines[0], queries[j], n, batch, seeds[j], mode, mass) for j in range(k)]
    assert all(a[2] > 1000 for a in alone)
    got = [None] * k
    go = threading.Barrier(k)

    def lane(j):
        go.wait()
        got[j] = _run(engines[j], queries[j], n, batch, seeds[j], mode, mass)

    for rep in range(2):
        ts = [threading.Thread(target=lane, args=(j,)) for j in range(k)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert got == alone, "rep %d" % rep
        got = [None] * k
    for e in engines:
        e.close()
