"""Shared-tree rounds (SURVEY 8e's alternative to replica trees, tcmp_plan_run_group /
tcmp_plan_run_shared): k engines each take a consecutive range of every round's lanes and
exchange the goal lane, their accepted-edge counts, the lowest goal node and their new node
records.  Every engine must end with exactly the tree one engine builds from the whole round
(node order = lane order), so the trees are compared bit for bit with a lone engine's -- and
the lone engine's with the oracle's batched restatement.  On one GPU the engines share the
device; the RCCL form differs only in how the four exchanges move (one rank per GPU).
"""
import numpy as np
import pytest

import oracle as O  # noqa: E402  (test infrastructure)

pytestmark = pytest.mark.gpu

START = np.array([0, -np.pi / 4, 0.0, -6 * np.pi / 8, 0, np.pi / 2, np.pi / 4])
LO = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
HI = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])


def _query(seed, n_obs, mode, mass):
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
        if nsafe < nsteps:
            return obs, goal


def _begin(eng, obs, goal, mode, mass, n, max_batch, seed):
    from torque_constrained_motion_planning_amd import _lib
    eng.set_scene(obs)
    st = eng.plan_begin(START, goal, mode, mass, 5.0, max_nodes=n + 1, max_batch=max_batch,
                        seed=seed)
    assert st == _lib.PLAN_OK


def _tree(eng, n):
    cfg, cost, par, m = eng.plan_tree(n + 1)
    return cfg, cost, par, m


@pytest.mark.parametrize("k,n,batch,n_obs,mode,mass", [
    (2, 20_000, 4096, 4, 1, 2.0),
    (3, 20_000, 4096, 16, 2, 5.0),      # 4096 lanes do not split evenly over 3 engines
    (4, 30_000, 8192, 16, 2, 5.0),
    (2, 3_000, 64, 8, 3, 5.0),          # dyn torque mode, small rounds
])
def test_group_rounds_equal_one_engine(k, n, batch, n_obs, mode, mass):
    from torque_constrained_motion_planning_amd import _lib
    obs, goal = _query(900 + k + n_obs, n_obs, mode, mass)
    seed = 77 + k
    one = _lib.Engine(0)
    _begin(one, obs, goal, mode, mass, n, batch, seed)
    one.plan_run(n, batch)
    ref = _tree(one, n)
    r1 = one.plan_finish()
    group = [_lib.Engine(0) for _ in range(k)]
    for e in group:
        _begin(e, obs, goal, mode, mass, n, -(-batch // k), seed)
    _lib.plan_run_group(group, n, batch)
    for e in group:
        cfg, cost, par, m = _tree(e, n)
        assert m == ref[3]
        assert np.array_equal(cfg, ref[0])
        assert np.array_equal(cost, ref[1])
        assert np.array_equal(par, ref[2])
    # every engine finishes the same plan; the samples drawn add up to the lone engine's
    drawn = 0
    for e in group:
        r = e.plan_finish()
        assert (r.status, r.n_nodes, r.goal_found, r.n_waypoints, r.n_traj) == \
            (r1.status, r1.n_nodes, r1.goal_found, r1.n_waypoints, r1.n_traj)
        drawn += r.n_samples
    assert drawn == r1.n_samples
    # and the lone engine's tree is the oracle's batched restatement's
    ref_o = O.rrt_run(START, goal, n, obs, mode, mass, 5.0, batch=batch, seed=seed, cull=2)
    assert ref_o["n_nodes"] == r1.n_nodes
    assert ref_o["status"] == r1.status


def test_group_rounds_meshes():
    """The same on a convex-mesh scene (k_edges<true>, the mesh rewire)."""
    from torque_constrained_motion_planning_amd import _lib
    from torque_constrained_motion_planning_amd.scene import mesh_pack, random_mesh_scene
    rng = np.random.default_rng(5)
    empty = np.zeros((0, 15))
    chk = _lib.Engine(0)
    while True:
        goal = LO + (HI - LO) * rng.random(7)
        meshes = random_mesh_scene(rng, 12)
        pack = mesh_pack(meshes)
        chk.set_scene(empty, pack)
        if not chk.collides(np.stack([START, goal])).any():
            break
    n, batch, k = 8_000, 2048, 2
    engines = [_lib.Engine(0) for _ in range(k + 1)]
    for i, e in enumerate(engines):
        e.set_scene(empty, pack)
        e.plan_begin(START, goal, 2, 5.0, 5.0, max_nodes=n + 1,
                     max_batch=batch if i == 0 else -(-batch // k), seed=3)
    engines[0].plan_run(n, batch)
    _lib.plan_run_group(engines[1:], n, batch)
    ref = _tree(engines[0], n)
    for e in engines[1:]:
        got = _tree(e, n)
        assert got[3] == ref[3]
        for a, b in zip(got[:3], ref[:3]):
            assert np.array_equal(a, b)


def test_shared_one_rank_is_plan_run():
    """tcmp_plan_run_shared over a one-rank communicator is tcmp_plan_run."""
    from torque_constrained_motion_planning_amd import _lib
    obs, goal = _query(61, 4, 2, 5.0)
    n, batch = 10_000, 2048
    a, b = _lib.Engine(0), _lib.Engine(0)
    _begin(a, obs, goal, 2, 5.0, n, batch, 9)
    _begin(b, obs, goal, 2, 5.0, n, batch, 9)
    a.plan_run(n, batch)
    comm = _lib.Comm(0, 1, 0)
    b.plan_run_shared(comm, n, batch)
    ta, tb = _tree(a, n), _tree(b, n)
    assert ta[3] == tb[3] and np.array_equal(ta[0], tb[0]) and np.array_equal(ta[2], tb[2])


def test_group_rejects_bad_shapes():
    from torque_constrained_motion_planning_amd import _lib
    obs, goal = _query(62, 4, 2, 5.0)
    es = [_lib.Engine(0) for _ in range(2)]
    for e in es:
        _begin(e, obs, goal, 2, 5.0, 5000, 512, 1)
    with pytest.raises(_lib.TcmpError):
        _lib.plan_run_group(es, 4000, 2048)   # 1024 lanes per engine > max_batch 512
    with pytest.raises(_lib.TcmpError):
        _lib.plan_run_group(es, 4000, 1)      # fewer lanes than engines


def test_tree_digest_proves_one_tree():
    """tcmp_plan_digest (what bench.py --shared-tree all-gathers as tree_consistent): the
    engines of a group round report the lone engine's digest; the host restatement
    (shard.tree_digest) over the fetched tree gives the same value; a different tree
    (another seed) gives another."""
    from torque_constrained_motion_planning_amd import _lib, shard
    obs, goal = _query(71, 16, 2, 5.0)
    n, batch = 20_000, 4096
    one = _lib.Engine(0)
    _begin(one, obs, goal, 2, 5.0, n, batch, 5)
    one.plan_run(n, batch)
    es = [_lib.Engine(0) for _ in range(3)]
    for e in es:
        _begin(e, obs, goal, 2, 5.0, n, -(-batch // 3), 5)
    _lib.plan_run_group(es, n, batch)
    d1, n1 = one.plan_digest()
    cfg, cost, par, m = _tree(one, n)
    assert n1 == m > 1000
    assert shard.tree_digest(cfg, cost, par) == d1
    assert [e.plan_digest() for e in es] == [(d1, n1)] * 3
    other = _lib.Engine(0)
    _begin(other, obs, goal, 2, 5.0, n, batch, 6)
    other.plan_run(n, batch)
    assert other.plan_digest()[0] != d1
