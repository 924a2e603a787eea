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


@pytest.mark.parametrize("n_obs,n_mesh,n,batch", [
    (16, 0, 60_000, 16384),   # boxes
    (0, 16, 20_000, 4096),    # convex meshes (the C5 kernels)
])
def test_concurrent_graph_capture_then_replay(n_obs, n_mesh, n, batch):
    """Round-graph capture while other engines' threads dispatch (the round-4 C5 trace abort,
    DESIGN.md section 8): three engines see a shape for the first time together and capture it
    (one at a time under the exclusive dispatch lock, while the others wait or sit in a host
    wait), then replay it together, twice -- with event timing off on one of them (a graph of
    kernel nodes only).  Every pass builds the trees and trajectories of the same
    queries run one at a time on a fourth engine, and the plan results say which passes ran
    as a captured graph."""
    import bench
    from torque_constrained_motion_planning_amd import _lib
    mode, mass, k = _lib.TORQUE_RNE, 5.0, 3
    engines = [_lib.Engine(0) for _ in range(k + 1)]
    ref = engines[k]
    engines[1].set_timing(False)
    queries = [bench.make_query(777 + j, n_obs=n_obs, mode=mode, mass=mass, engine=ref,
                                n_mesh=n_mesh) for j in range(k)]
    seeds = [5100 + 31 * j for j in range(k)]
    alone = [_run(ref, queries[j], n, batch, seeds[j], mode, mass) for j in range(k)]
    go = threading.Barrier(k)
    for rep, want_graph in enumerate((1, 1, 1)):
        got, gl, ms = [None] * k, [None] * k, [None] * k

        def lane(j):
            go.wait()
            eng = engines[j]
            obs, pack, goal = queries[j]
            r, out = bench.run_query(eng, obs, goal, n, batch, seeds[j], mode, mass, meshes=pack)
            gl[j], ms[j] = r.graph_launches, r.ms_edges
            got[j] = (eng.plan_digest(), r.status, r.n_nodes, r.n_waypoints, r.n_traj,
                      r.edge_steps, out["q"].tobytes() if out is not None else b"")

        ts = [threading.Thread(target=lane, args=(j,)) for j in range(k)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert got == alone, "pass %d" % rep
        assert gl == [want_graph] * k, (rep, gl)
        # timing off on engine 1: no event spans, in direct launches and in its graph
        assert ms[1] == 0.0 and ms[0] > 0.0 and ms[2] > 0.0, ms
    for e in engines:
        e.close()


def test_plan_run_shape_change_keeps_event_spans():
    """plan_run(n1, B) then plan_run(n2, B) on one engine: the second call captures a new
    round graph and destroys the first one's event nodes -- their spans must have been read
    first (this sequence aborted in the HIP runtime at plan_finish before the fix), and the
    per-family times keep counting both calls."""
    import bench
    from torque_constrained_motion_planning_amd import _lib
    eng = _lib.Engine(0)
    obs, pack, goal = bench.make_query(4343, n_obs=12, mode=2, mass=5.0, engine=eng)
    eng.set_scene(obs)
    assert eng.plan_begin(bench.START, goal, 2, 5.0, 5.0, max_nodes=17_001, max_batch=4608,
                          seed=3) == _lib.PLAN_OK
    eng.plan_run(10_000, 4608)
    eng.plan_run(7_000, 4608)
    r = eng.plan_finish()
    assert r.n_samples == 17_000 and r.n_nodes > 1000
    assert r.ms_edges > 0 and r.ms_nearest > 0 and r.graph_launches == 2
    eng.close()
