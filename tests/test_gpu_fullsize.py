"""GPU parity at BASELINE.json's full sizes (configs[1] C2 and configs[2] C3).

C2 (4 boxes, 2 kg, nov, 1e5 batched samples) is small enough for the oracle's batched
restatement: node count, extend-step count, goal node and trajectory are compared directly.
C3 (16 boxes, 5 kg, rne, 1e6 samples) is checked through size-independent properties:
determinism, tree invariants (parents precede children, cost = parent cost + distance,
exactly as rrt_star.py:18-63 maintains them), every sampled tree node is a valid
configuration for the oracle (limits, collision, torque), the goal node is within the goal
tolerance and the returned trajectory passes the oracle's dynamic torque test.
"""
import numpy as np
import pytest

import oracle as O  # noqa: E402  (test infrastructure)

pytestmark = pytest.mark.gpu

START = np.array([0, -np.pi / 4, 0.0, -6 * np.pi / 8, 0, np.pi / 2, np.pi / 4])
LO = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
HI = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])


@pytest.fixture(scope="module")
def eng():
    from torque_constrained_motion_planning_amd import _lib
    return _lib.engine(0)


def _query(seed, n_obs, mode, mass):
    """SURVEY 8d query: start/goal collision-free and torque-feasible, straight edge blocked
    (so the tree has to grow)."""
    from torque_constrained_motion_planning_amd.scene import obstacle_array, random_box_scene
    rng = np.random.default_rng(seed)
    while True:
        goal = LO + (HI - LO) * rng.random(7)
        obs = obstacle_array(random_box_scene(rng, n_obs))
        if O.collision(START, obs) or O.collision(goal, obs):
            continue
        if not (O.torque_ok(goal, mode, mass) and O.torque_ok(START, mode, mass)):
            continue
        nsafe, nsteps, _ = O.check_edge(START, goal, obs, mode, mass, cull=2)
        if nsafe == nsteps:
            continue
        return obs, goal


def _dist(a, b):
    d = b - a
    return np.sqrt((10.0 * (d * d)).sum(axis=-1))


def test_c2_full_size_vs_oracle(eng):
    from torque_constrained_motion_planning_amd.rrt_star import rrt_star_batched
    obs, goal = _query(21, 4, 1, 2.0)
    (path, vels, accels, psg), r, raw = rrt_star_batched(
        START, goal, obs, 1, 2.0, 5.0, 100_000, batch=65536, seed=77, engine=eng)
    ref = O.rrt_run(START, goal, 100_000, obs, 1, 2.0, 5.0, batch=65536, seed=77, cull=2)
    assert r.n_nodes == ref["n_nodes"]
    assert r.edge_steps == ref["edge_steps"]
    assert r.goal_node == ref["goal_node"]
    assert r.status == ref["status"]
    if ref["status"] in (0, 3):
        assert np.abs(raw["waypoints"] - ref["waypoints"]).max() < 1e-12
        assert np.abs(raw["q"] - ref["q"]).max() < 1e-9
        assert np.abs(raw["qd"] - ref["qd"]).max() < 1e-9
        assert np.abs(raw["qdd"] - ref["qdd"]).max() < 1e-9


def test_nearest_at_bench_scale_vs_bruteforce(eng):
    """k_nearest_wave32 inside the plan path at the bench's own C3 size (B = 262,144 per
    round, 1e6 samples): for candidates of rounds 3 and 4 (snapshots of ~0.4-0.66M nodes,
    the super-cell block walk fully exercised) the chosen node is the brute-force argmin of
    rrt_star.py:9-14 (first index on ties) and its exact score matches the distance."""
    obs, goal = _query(1234, 16, 2, 5.0)
    eng.set_scene(obs)
    B = 262144
    assert eng.plan_begin(START, goal, 2, 5.0, 5.0, max_nodes=4 * B + 1, max_batch=B,
                          seed=5) == 0
    rng = np.random.default_rng(1)
    for r in range(4):
        eng.plan_round(nb=B, sync=False)
        if r < 2:
            continue
        cand, nn, score, snap = eng.plan_debug_round(B)
        assert len(cand) == B and snap > 200_000
        cfg, _, _, n = eng.plan_tree(snap)
        assert n >= snap
        pick = np.concatenate([np.arange(64), rng.choice(B, 1500, replace=False)])
        idx, dist = O.nearest(cfg[:snap], cand[pick])
        bad = np.nonzero(nn[pick] != idx)[0]
        assert len(bad) == 0, (r, snap, pick[bad[:5]], nn[pick][bad[:5]], idx[bad[:5]])
        assert np.allclose(np.sqrt(10.0 * score[pick]), dist, rtol=1e-12, atol=0)
    eng.plan_finish()


def test_c3_full_size_properties(eng):
    from torque_constrained_motion_planning_amd.rrt_star import rrt_star_batched
    obs, goal = _query(1234, 16, 2, 5.0)
    args = (START, goal, obs, 2, 5.0, 5.0, 1_000_000)
    (path, vels, accels, psg), r, raw = rrt_star_batched(*args, batch=262144, seed=5,
                                                         engine=eng)
    cfg, cost, par, n = eng.plan_tree(r.n_nodes)
    assert n == r.n_nodes and 1 < n <= 1_000_001
    # determinism of the batched frontier
    (_, _, _, _), r2, raw2 = rrt_star_batched(*args, batch=262144, seed=5, engine=eng)
    assert (r2.n_nodes, r2.edge_steps, r2.goal_node) == (r.n_nodes, r.edge_steps, r.goal_node)
    # tree invariants: root first, parents inserted before children, costs consistent
    assert np.allclose(cfg[0], START) and cost[0] == 0.0
    idx = np.arange(1, n)
    assert np.all(par[1:] >= 0) and np.all(par[1:] < idx)
    d = _dist(cfg[par[1:]], cfg[1:])
    assert np.allclose(cost[1:], cost[par[1:]] + d, rtol=1e-12, atol=1e-12)
    # every node is a valid configuration (limits, collision, search-time torque)
    rng = np.random.default_rng(0)
    pick = rng.choice(n, size=min(n, 3000), replace=False)
    for i in pick:
        assert not O.collision(cfg[i], obs)
        assert O.torque_ok(cfg[i], 2, 5.0)
    if r.goal_found:
        g = cfg[r.goal_node]
        assert _dist(g, goal) < 1e-2
        wp = raw["waypoints"]
        assert np.allclose(wp[0], START) and np.array_equal(wp[-1], g)
        if r.status == 0:
            # the returned trajectory passes the reference's dynamic torque test
            q, qd, qdd = raw["q"], raw["qd"], raw["qdd"]
            sel = np.arange(0, len(q), max(1, len(q) // 500))
            for i in sel:
                assert O.torque_ok(q[i], 2, 5.0, qd=qd[i], qdd=qdd[i])


def _digest(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["c3", "c5", "c5b"])
def test_bench_query_vs_oracle_fixture(eng, name):
    """The bench's own query at its own size, bit for bit against the oracle's batched
    restatement (tests/golden/fullsize_<name>.npz, made by tests/golden/gen_fullsize.py):
    C3 = bench.py make_query(1234), 16 boxes, 5 kg, rne, 1e6 samples, B = 262,144, seed 1234
    (step 0 of rank 0); C5 = make_query(1234, n_mesh=256), 131,072 samples in eight rounds of
    16,384 (Philox seed 1243, the goal found in a late round: the nearest scan on a mesh tree,
    insertion across rounds, retrace, min-jerk and validation at C5 scale); C5b = the same
    scene at the bench's B = 262,144, 562,816 samples (two full rounds through
    k_edges<true,1>'s persistent refill and a 38,528-lane round through k_edges<true,2>, the
    bench's own kernels; no goal yet, so the tree is what is pinned).  The scene is
    regenerated on the device by bench.make_query and must be the fixture's; then the final
    tree (configs, costs, parents: sha256), counters, waypoints and trajectory rows match."""
    import os
    import sys
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                        "fullsize_%s.npz" % name)
    if not os.path.exists(path):
        pytest.skip("fixture not generated")
    F = np.load(path)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n_mesh = int(F["n_mesh"])
    obs, pack, goal = bench.make_query(1234, n_obs=16 if not n_mesh else 0, mode=2, mass=5.0,
                                       engine=eng, n_mesh=n_mesh)
    assert np.array_equal(obs, F["obs"]) and np.array_equal(goal, F["goal"])
    if n_mesh:
        import hashlib
        h = hashlib.sha256()
        for f in ("verts", "vert_off", "planes", "plane_off", "edges", "edge_off", "boxes"):
            h.update(np.ascontiguousarray(getattr(pack, f)).tobytes())
        assert h.hexdigest() == str(F["sha_pack"])
    r, out = bench.run_query(eng, obs, goal, int(F["samples"]), int(F["batch"]), int(F["seed"]),
                             meshes=pack)
    assert (r.n_samples, r.n_nodes, r.edge_steps, r.goal_node, r.status) == \
        (int(F["n_samples"]), int(F["n_nodes"]), int(F["edge_steps"]), int(F["goal_node"]),
         int(F["status"]))
    cfg, cost, par, n = eng.plan_tree(r.n_nodes)
    stride = F["tree_stride"]
    assert np.array_equal(cfg[stride], F["tree_cfg_sel"])
    assert np.array_equal(par[stride], F["tree_parent_sel"])
    assert _digest(cfg) == str(F["sha_cfg"])
    assert _digest(cost) == str(F["sha_cost"])
    assert _digest(par.astype(np.int32)) == str(F["sha_parent"])
    if int(F["status"]) in (0, 3):
        assert (r.n_waypoints, r.n_traj) == (int(F["n_waypoints"]), int(F["n_traj"]))
        assert np.array_equal(out["waypoints"], F["waypoints"])
        sel = F["traj_sel"]
        for k in ("q", "qd", "qdd"):
            assert np.abs(out[k][sel] - F[k]).max() < 1e-9, k
        assert np.abs(out["psg"][sel] - F["psg"]).max() < 1e-12


def test_c4_eight_concurrent_queries_vs_oracle_fixture():
    """C4's per-GPU shape at N = 8 (BASELINE configs[3]): eight 16-box rne queries of 1e5 samples
    at B = 65,536 planned at once on eight engines from eight host threads (bench.py's C4 path),
    each bit for bit against the oracle's batched restatement (tests/golden/fullsize_c4.npz:
    bench.make_query(1234 + q), sample seed 5000 + q) -- tree digests, counters, waypoints and
    trajectory rows."""
    import os
    import sys
    import threading
    from torque_constrained_motion_planning_amd import _lib
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize_c4.npz")
    if not os.path.exists(path):
        pytest.skip("fixture not generated")
    F = np.load(path)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n_q = int(F["n_queries"])
    engines = [_lib.Engine(0) for _ in range(n_q)]
    queries = [bench.make_query(1234 + q, n_obs=16, mode=2, mass=5.0, engine=engines[q])
               for q in range(n_q)]
    for q, (obs, pack, goal) in enumerate(queries):
        assert np.array_equal(obs, F["q%d_obs" % q]) and np.array_equal(goal, F["q%d_goal" % q])
    got = [None] * n_q
    go = threading.Barrier(n_q)

    def lane(q):
        go.wait()
        obs, pack, goal = queries[q]
        r, out = bench.run_query(engines[q], obs, goal, int(F["q%d_samples" % q]),
                                 int(F["q%d_batch" % q]), int(F["q%d_seed" % q]))
        cfg, cost, par, n = engines[q].plan_tree(r.n_nodes)
        got[q] = (r, out, cfg, cost, par)

    ts = [threading.Thread(target=lane, args=(q,)) for q in range(n_q)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for q in range(n_q):
        f = lambda k: F["q%d_%s" % (q, k)]  # noqa: E731
        r, out, cfg, cost, par = got[q]
        assert (r.n_samples, r.n_nodes, r.edge_steps, r.goal_node, r.status) == \
            (int(f("n_samples")), int(f("n_nodes")), int(f("edge_steps")), int(f("goal_node")),
             int(f("status"))), q
        assert _digest(cfg) == str(f("sha_cfg")) and _digest(cost) == str(f("sha_cost"))
        assert _digest(par.astype(np.int32)) == str(f("sha_parent"))
        if int(f("status")) in (0, 3):
            assert (r.n_waypoints, r.n_traj) == (int(f("n_waypoints")), int(f("n_traj")))
            assert np.array_equal(out["waypoints"], f("waypoints"))
            sel = f("traj_sel")
            for k in ("q", "qd", "qdd"):
                assert np.abs(out[k][sel] - f(k)).max() < 1e-9, (q, k)
    assert sum(int(F["q%d_status" % q]) == 0 for q in range(n_q)) >= 2  # solved paths among them
    for e in engines:
        e.close()
