"""GPU parity: libtcmp (HIP, gfx950) against the CPU oracle and the reference's golden vectors.

Tolerances: torques / trajectories within 1e-9 abs (north_star asks 1e-5 on joint angles
and torques); integer results (nearest index, safe-prefix length, collision flags) exact.
"""
import glob
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN

import oracle as O  # noqa: E402  (test infrastructure)

pytestmark = pytest.mark.gpu

LO = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
HI = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])
TOL = 1e-9


@pytest.fixture(scope="module")
def eng():
    from torque_constrained_motion_planning_amd import _lib
    e = _lib.engine(0)
    return e


def rand_q(rng, n):
    return LO + (HI - LO) * rng.random((n, 7))


def boxes(rng, n, aligned=True):
    from torque_constrained_motion_planning_amd.scene import random_box_scene, obstacle_array
    return obstacle_array(random_box_scene(rng, n, aligned=aligned))


def test_rne_golden(eng):
    z = np.load(os.path.join(GOLDEN, "rne_golden.npz"))
    for m in (0, 2, 5):
        t = "m%d" % m
        q, qd, qdd = z["q_" + t], z["qd_" + t], z["qdd_" + t]
        ts = eng.rne(q, np.zeros_like(q), np.zeros_like(q), float(m))
        td = eng.rne(q, qd, qdd, float(m))
        assert np.abs(ts - z["tau_static_" + t]).max() < TOL
        assert np.abs(td - z["tau_dyn_" + t]).max() < TOL


def test_torque_tests_vs_oracle(eng):
    rng = np.random.default_rng(11)
    q = rand_q(rng, 3000)
    qd = rng.uniform(-2, 2, q.shape)
    qdd = rng.uniform(-6, 6, q.shape)
    for mode in (0, 1, 2, 3):
        for mass in (0.0, 0.005, 2.0, 5.0, 9.0):
            ok_s = eng.torque_ok(q, mode, mass)
            ok_d = eng.torque_ok(q, mode, mass, qd=qd, qdd=qdd)
            ref_s = np.array([O.torque_ok(x, mode, mass) for x in q])
            ref_d = np.array([O.torque_ok(x, mode, mass, a, b) for x, a, b in zip(q, qd, qdd)])
            assert (ok_s == ref_s).all(), (mode, mass)
            assert (ok_d == ref_d).all(), (mode, mass)


def test_minjerk_golden(eng):
    z = np.load(os.path.join(GOLDEN, "minjerk_golden.npz"))
    for c in range(int(z["ncases"])):
        P, ni = z["P%d" % c], int(z["ni%d" % c])
        q, qd, qdd = eng.minjerk(P, ni)
        assert np.abs(q - z["x%d" % c]).max() < 1e-12
        assert np.abs(qd - z["v%d" % c]).max() < 1e-12
        assert np.abs(qdd - z["a%d" % c]).max() < 1e-12


def test_collision_vs_oracle(eng):
    rng = np.random.default_rng(5)
    for n_obs, aligned in ((0, True), (4, True), (16, True), (16, False), (64, True)):
        obs = boxes(rng, n_obs, aligned) if n_obs else np.zeros((0, 15))
        eng.set_scene(obs)
        q = rand_q(rng, 2000)
        q[:50] = LO - 1e-3 + (HI - LO + 2e-3) * rng.random((50, 7))  # some out of limits
        got = eng.collides(q)
        # oracle: bounds + Gauss-map exact test; brute-force exact test on a subset
        ref = np.array([O.collision(x, obs, cull=2) for x in q])
        assert (got == ref).all(), (n_obs, aligned, np.nonzero(got != ref))
        sub = q[:60]
        ref0 = np.array([O.collision(x, obs[:8], cull=0) for x in sub])
        eng.set_scene(obs[:8])
        assert (eng.collides(sub) == ref0).all()


def test_check_edges_vs_oracle(eng):
    rng = np.random.default_rng(7)
    for n_obs, mode, mass in ((0, 2, 5.0), (4, 1, 2.0), (16, 2, 5.0), (16, 0, 0.0),
                              (8, 3, 5.0)):
        obs = boxes(rng, n_obs) if n_obs else np.zeros((0, 15))
        eng.set_scene(obs)
        a = rand_q(rng, 400)
        b = rand_q(rng, 400)
        b[:200] = np.clip(a[:200] + rng.normal(0, 0.3, (200, 7)), LO, HI)
        ns, nt, last = eng.check_edges(a, b, mode, mass)
        for i in range(len(a)):
            s, n, l = O.check_edge(a[i], b[i], obs, mode, mass, cull=2)
            assert ns[i] == s and nt[i] == n, (i, ns[i], s, nt[i], n)
            if s:
                assert np.array_equal(last[i], l), i


def test_nearest_exact(eng):
    """tcmp_nearest runs the planner's own index + k_nearest_wave32 (rrt_star.py:9-14)."""
    rng = np.random.default_rng(3)
    tree = rand_q(rng, 5000)
    tree[100] = tree[7]  # duplicate: first index must win
    s = rand_q(rng, 1000)
    s[0] = tree[7]
    idx = eng.nearest(tree, s)
    ref, _ = O.nearest(tree, s)
    assert (idx == ref).all()
    assert idx[0] == 7
    # many exact duplicates (cells of identical keys), a single-node tree
    dup = np.repeat(rand_q(rng, 50), 40, axis=0)
    s2 = np.concatenate([dup[::97], rand_q(rng, 300)])
    assert (eng.nearest(dup, s2) == O.nearest(dup, s2)[0]).all()
    assert (eng.nearest(tree[:1], s) == 0).all()


def test_nearest_weights_and_range(eng):
    """Non-uniform weights (the weighted scan) and coordinates outside the joint-limit box
    (the fp32 error terms scale with the data's bound)."""
    rng = np.random.default_rng(4)
    tree = rand_q(rng, 40000)
    s = rand_q(rng, 3000)
    w = np.array([10.0, 3.0, 7.5, 1.0, 20.0, 0.5, 10.0])
    assert (eng.nearest(tree, s, w) == O.nearest(tree, s, w)[0]).all()
    big = rng.uniform(-40, 40, (20000, 7))
    sb = rng.uniform(-40, 40, (2000, 7))
    assert (eng.nearest(big, sb) == O.nearest(big, sb)[0]).all()
    # clustered nodes (a grown tree is dense near its edges): near-ties within fp32 resolution
    base = rand_q(rng, 1)
    clus = base + rng.normal(0, 1e-5, (30000, 7))
    sc = base + rng.normal(0, 2e-5, (2000, 7))
    assert (eng.nearest(clus, sc) == O.nearest(clus, sc)[0]).all()


def test_validate_traj_vs_oracle(eng):
    rng = np.random.default_rng(9)
    wp = rand_q(rng, 6)
    for ni in (40, 200):
        q, qd, qdd = eng.minjerk(wp, ni)
        for mode, mass in ((1, 5.0), (2, 5.0), (2, 0.0), (0, 0.0), (3, 5.0), (3, 9.0)):
            ff, tau = eng.validate(q, qd, qdd, mode, mass)
            ref_ff = -1
            for i in range(len(q)):
                if not O.torque_ok(q[i], mode, mass, qd[i], qdd[i]):
                    ref_ff = i
                    break
            assert ff == ref_ff
            assert np.abs(tau - O.rne(q, qd, qdd, 0.0)).max() < TOL


RRT_GOLDEN = sorted(glob.glob(os.path.join(GOLDEN, "rrt_*.npz")))


def _numpy_dynam(exec_time):
    """A foreign dynam_fn (plain function): the package's numpy min-jerk utilities."""
    from torque_constrained_motion_planning_amd import min_jerk_v2 as MJ

    def dynam_fn(path, dur=None):
        traj = MJ.minjerk_trajectory(MJ.minjerk_coefficients(np.array(path)),
                                     int(exec_time * 1000 / len(path)))
        q = [list(t[0]) for t in traj]
        return (q, [exec_time * n / len(traj) for n in range(len(traj))],
                [list(t[1]) for t in traj], [list(t[2]) for t in traj])
    return dynam_fn


VARIANTS = ["native", "foreign_distance", "foreign_extend", "foreign_dynam"]


def _golden_radius(z):
    return float(z["radius"]) if "radius" in z else 0.01


def _golden_problem(z):
    from torque_constrained_motion_planning_amd import panda_primitives as PP
    from torque_constrained_motion_planning_amd import utils as U
    mode = int(z["mode"])
    mass = float(z["mass"])
    prob = U.Problem(U.PandaRobot(), list(z["obs"]), U.Payload(mass), mass, float(z["exec_time"]),
                     torque_test={0: "base", 1: "nov", 2: "rne"}[mode])
    resolutions = 0.2 ** np.ones(7)
    radius = resolutions / 2
    joints = U.get_arm_joints(prob.robot)
    return dict(torque_fn=PP.select_torque_test(prob),
                dynam_fn=PP.get_dynamics_fn_v5(prob, resolutions),
                sample=U.get_sample_fn(prob.robot, joints),
                distance=U.get_distance_fn(prob.robot, joints, weights=np.reciprocal(radius)),
                extend=U.get_extend_fn(prob.robot, joints, resolutions=radius),
                collision=U.get_collision_fn(prob.robot, joints, list(z["obs"]),
                                             self_collisions=False))


REWIRE_GOLDEN = [p for p in RRT_GOLDEN if "tree_cfg" in np.load(p)]


@pytest.mark.parametrize("loop", ["engine", "host"])
@pytest.mark.parametrize("path", REWIRE_GOLDEN, ids=[os.path.basename(p) for p in REWIRE_GOLDEN])
def test_rrt_golden_tree_and_rewires(eng, path, loop):
    """The reference runs at rewire radii 4-8 (rrt_star.py:183-192 fires tens to hundreds of
    times): the drop-in's whole tree -- every node's configuration, parent and cost, in node
    order -- and its rewire count equal the reference's OptimalNode graph.  engine: the device
    loop (tcmp_plan_round per iteration, k_rewire_scan / k_rewire_apply; n_rewires from
    tcmp_plan_result); host: the host loop of a foreign distance fn (tree on the host, the
    engine checking edges)."""
    from torque_constrained_motion_planning_amd import rrt_star as R
    z = np.load(path)
    assert int(z["n_rewires"]) > 0
    f = _golden_problem(z)
    seed = int(z["seed"])
    random.seed(seed)
    np.random.seed(seed)
    radius = [_golden_radius(z)]
    if loop == "engine":
        (path_, _, _, _), r, _ = R._rrt_engine(
            tuple(z["start"]), tuple(z["goal"]), f["distance"], f["sample"], f["extend"],
            f["collision"], f["torque_fn"], f["dynam_fn"], radius, int(z["iters"]), 0.2)
        assert r.n_rewires == int(z["n_rewires"])
        # the engine loop plans on the collision fn's own handle (utils.CollisionFn)
        cfg, cost, par, n = f["collision"].engine.plan_tree(r.n_nodes)
    else:
        st = {}
        dist = (lambda fn: (lambda a, b: fn(a, b)))(f["distance"])
        path_, _, _, _ = R._rrt_host(
            tuple(z["start"]), tuple(z["goal"]), dist, f["sample"], f["extend"], f["collision"],
            f["torque_fn"], f["dynam_fn"], radius, max_time=50, max_iterations=int(z["iters"]),
            stats=st)
        assert st["n_rewires"] == int(z["n_rewires"])
        t = st["tree"]
        n = len(t)
        cfg, cost, par = t.q[:n], np.array(t.cost), np.array(t.parent)
    assert n == len(z["tree_cfg"])
    assert np.array_equal(cfg, z["tree_cfg"])
    assert np.array_equal(par, z["tree_parent"])
    assert np.abs(cost - z["tree_cost"]).max() < 1e-12
    assert (path_ is not None) == bool(z["found"])
    if path_ is not None:
        q = np.array(path_)
        assert len(q) == int(z["n_traj"])
        assert np.abs(q[z["traj_idx"]] - z["q"]).max() < 1e-9


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("path", RRT_GOLDEN, ids=[os.path.basename(p) for p in RRT_GOLDEN])
def test_rrt_golden_drop_in(eng, path, variant):
    """The package's rrt_star_force_aware, seeded like the reference run, reproduces the
    reference RRT* output (waypoints, q, qd, qdd, psg) -- with its own closures (the engine
    loop), and with one foreign callback each: a foreign distance or extend fn runs the host
    loop (engine edge checks / batched collision + torque for the package's own tests), a
    foreign dynam_fn runs the engine loop and then the callback on the retraced path."""
    from torque_constrained_motion_planning_amd import panda_primitives as PP
    from torque_constrained_motion_planning_amd import utils as U
    from torque_constrained_motion_planning_amd.rrt_star import rrt_star_force_aware
    z = np.load(path)
    mode = int(z["mode"])
    mass = float(z["mass"])
    prob = U.Problem(U.PandaRobot(), list(z["obs"]), U.Payload(mass), mass, float(z["exec_time"]),
                     torque_test={0: "base", 1: "nov", 2: "rne"}[mode])
    torque_fn = PP.select_torque_test(prob)
    resolutions = 0.2 ** np.ones(7)
    radius = resolutions / 2
    dyn = PP.get_dynamics_fn_v5(prob, resolutions)
    joints = U.get_arm_joints(prob.robot)
    sample = U.get_sample_fn(prob.robot, joints)
    dist = U.get_distance_fn(prob.robot, joints, weights=np.reciprocal(radius))
    ext = U.get_extend_fn(prob.robot, joints, resolutions=radius)
    coll = U.get_collision_fn(prob.robot, joints, list(z["obs"]), self_collisions=False)
    if variant == "foreign_distance":
        dist = (lambda f: (lambda a, b: f(a, b)))(dist)
    elif variant == "foreign_extend":
        ext = (lambda f: (lambda a, b: f(a, b)))(ext)
    elif variant == "foreign_dynam":
        dyn = _numpy_dynam(float(z["exec_time"]))
    seed = int(z["seed"])
    random.seed(seed)
    np.random.seed(seed)
    path_, vels, accels, psg = rrt_star_force_aware(
        tuple(z["start"]), tuple(z["goal"]), dist, sample, ext, coll, torque_fn, dyn,
        radius=[_golden_radius(z)], max_time=50, max_iterations=int(z["iters"]),
        informed=bool(z["informed"]) if "informed" in z else False)
    assert (path_ is not None) == bool(z["found"])
    if path_ is None:
        return
    q = np.array(path_)
    assert len(q) == int(z["n_traj"])
    idx = z["traj_idx"]
    assert np.abs(q[idx] - z["q"]).max() < 1e-9
    assert np.abs(np.array(vels)[idx] - z["qd"]).max() < 1e-9
    assert np.abs(np.array(accels)[idx] - z["qdd"]).max() < 1e-9
    assert np.abs(np.array(psg)[idx] - z["psg"]).max() < 1e-12
    assert np.abs(q.sum(0) - z["sum_q"]).max() < 1e-6


def _tree_digest(cfg, cost, par):
    import hashlib
    h = hashlib.sha256()
    for a in (np.ascontiguousarray(cfg, dtype=np.float64), np.ascontiguousarray(cost, dtype=np.float64),
              np.ascontiguousarray(par, dtype=np.int32)):
        h.update(a.tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("batch,n_obs,mode,mass,radius", [
    (1, 4, 2, 5.0, 0.01), (64, 8, 1, 2.0, 0.01), (256, 16, 2, 5.0, 0.01),
    (4096, 16, 2, 5.0, 0.01), (256, 8, 3, 5.0, 0.01),
    # rewire radii where rrt_star.py:187-192 fires: every rewire of every round is compared
    (256, 16, 2, 5.0, 4.0), (256, 16, 2, 5.0, 8.0), (4096, 16, 2, 5.0, 4.0),
    (4096, 16, 2, 5.0, 8.0), (1, 8, 1, 2.0, 8.0)])
def test_batched_frontier_vs_oracle(eng, batch, n_obs, mode, mass, radius):
    """Device-sampled batched rounds (Philox) == the oracle's batched restatement: the whole
    tree (sha256 of cfg, cost, parent), the rewire count, the goal and the trajectory."""
    from torque_constrained_motion_planning_amd.rrt_star import rrt_star_batched
    rng = np.random.default_rng(100 + batch)
    start = np.array([0, -np.pi / 4, 0.0, -6 * np.pi / 8, 0, np.pi / 2, np.pi / 4])
    while True:
        goal = rand_q(rng, 1)[0]
        obs = boxes(rng, n_obs)
        if not (O.collision(start, obs) or O.collision(goal, obs)) and O.torque_ok(goal, mode, mass):
            break
    n_samples = 3 * batch + 17 if batch > 1 else (60 if radius < 1 else 600)
    (path, vels, accels, psg), r, raw = rrt_star_batched(
        start, goal, obs, mode, mass, 1.0, n_samples, batch=batch, seed=1234 + batch, engine=eng,
        radius=radius)
    ref = O.rrt_run(start, goal, n_samples, obs, mode, mass, 1.0, batch=batch, seed=1234 + batch,
                    cull=2, radius=radius, tree=True, threads=16 if batch >= 4096 else 1)
    assert r.n_nodes == ref["n_nodes"]
    assert r.edge_steps == ref["edge_steps"]
    assert r.goal_node == ref["goal_node"]
    assert r.n_rewires == ref["n_rewires"]
    if radius > 1:
        assert ref["n_rewires"] > 0
    cfg, cost, par, n = eng.plan_tree(r.n_nodes)
    assert n == ref["n_nodes"]
    assert _tree_digest(cfg, cost, par) == _tree_digest(ref["tree_cfg"], ref["tree_cost"],
                                                        ref["tree_parent"])
    if ref["status"] in (0, 3):
        assert r.status == ref["status"]
        assert r.n_waypoints == ref["n_waypoints"]
        assert np.abs(raw["waypoints"] - ref["waypoints"]).max() < 1e-12
        assert np.abs(raw["q"] - ref["q"]).max() < 1e-9
        assert np.abs(raw["qd"] - ref["qd"]).max() < 1e-9
        assert np.abs(raw["qdd"] - ref["qdd"]).max() < 1e-9
    else:
        assert r.status == ref["status"]


@pytest.mark.parametrize("exec_time", [0.0, 1.0])
def test_plan_retrace_only(eng, exec_time):
    """tcmp_plan_retrace (the finish of a foreign dynam_fn): the same waypoints as
    tcmp_plan_finish, no trajectory, status 0 even where the engine's min-jerk would assert
    (execution time 0 -> zero intervals)."""
    from torque_constrained_motion_planning_amd import _lib
    rng = np.random.default_rng(77)
    start = np.array([0, -np.pi / 4, 0.0, -6 * np.pi / 8, 0, np.pi / 2, np.pi / 4])
    while True:
        goal = start + rng.uniform(-0.4, 0.4, 7)
        obs = boxes(rng, 8)
        if not (O.collision(start, obs) or O.collision(goal, obs)) and O.torque_ok(goal, 2, 5.0):
            break
    eng.set_scene(obs)

    def plan():
        assert eng.plan_begin(start, goal, 2, 5.0, exec_time, max_nodes=2049, max_batch=256,
                              seed=99) == 0
        eng.plan_run(2048, 256)

    plan()
    rt = eng.plan_retrace()
    assert rt.goal_found == 1 and rt.status == 0
    assert rt.n_traj == 0 and rt.first_fail == -1 and rt.n_waypoints >= 2
    wp = eng.plan_fetch(rt)["waypoints"]
    plan()
    fin = eng.plan_finish()
    assert fin.goal_node == rt.goal_node and fin.n_waypoints == rt.n_waypoints
    if exec_time == 0:
        assert fin.status == _lib.PLAN_MINJERK_ASSERT and fin.n_traj == 0
    else:
        assert fin.status in (_lib.PLAN_OK, _lib.PLAN_VALIDATION_FAILED) and fin.n_traj > 0
    assert np.array_equal(eng.plan_fetch(fin)["waypoints"], wp)


# ---- goal IK ------------------------------------------------------------
def test_dyn_torque_test_host(eng):
    """get_torque_limits_not_exceded_test_v2 through the host mirror == the oracle."""
    from torque_constrained_motion_planning_amd import panda_primitives as pp
    from torque_constrained_motion_planning_amd.scene import PandaRobot, Payload
    from torque_constrained_motion_planning_amd.utils import Problem
    rng = np.random.default_rng(5)
    prob = Problem(PandaRobot(), [], Payload.coke(6.0), 6.0, 1.0, torque_test="dyn")
    test = pp.select_torque_test(prob)
    q = rand_q(rng, 200)
    qd = rng.uniform(-2, 2, q.shape)
    qdd = rng.uniform(-6, 6, q.shape)
    for x, a, b in zip(q, qd, qdd):
        assert test(list(x)) == O.torque_ok(x, 3, 6.0)
        assert test(list(x), velocities=list(a), accelerations=list(b)) == \
            O.torque_ok(x, 3, 6.0, a, b)


def test_fk_golden(eng):
    """tcmp_fk == the reference DH chain (rne.py:46-63 via fk_golden.npz)."""
    z = np.load(os.path.join(GOLDEN, "fk_golden.npz"))
    P = eng.fk(z["q"])
    T = z["T"]
    assert np.abs(P[:, :9] - T[:, :3, :3].reshape(-1, 9)).max() < 1e-12
    assert np.abs(P[:, 9:] - T[:, :3, 3]).max() < 1e-12


def test_ik_vs_oracle(eng):
    """tcmp_ik == the oracle solver, branch by branch, and every solution maps back through
    the reference FK; the generating configuration is among the solutions."""
    rng = np.random.default_rng(31)
    q = rand_q(rng, 3000)
    T = np.stack([O.fk8(r) for r in q])
    free = q[:, 6].copy()
    free[::3] = rng.uniform(LO[6], HI[6], size=len(free[::3]))  # other free values too
    sols, cnt = eng.ik(T, free)
    back = eng.fk(sols.reshape(-1, 7)).reshape(len(q), 8, 12)
    hit = 0
    for i in range(len(q)):
        ref, _ = O.ik8(T[i], free[i])
        assert cnt[i] == len(ref)
        if cnt[i]:
            assert np.abs(sols[i, :cnt[i]] - ref).max() < 1e-9
            Tb = back[i, :cnt[i]]
            assert np.abs(Tb[:, :9] - T[i, :3, :3].reshape(9)).max() < 1e-9
            assert np.abs(Tb[:, 9:] - T[i, :3, 3]).max() < 1e-9
        if i % 3 and cnt[i]:
            d = (sols[i, :cnt[i]] - q[i] + np.pi) % (2 * np.pi) - np.pi
            hit += np.abs(d).max(1).min() < 1e-8
    assert hit == sum(1 for i in range(len(q)) if i % 3)


def test_planner_fn_force_aware_end_to_end(eng):
    """panda_primitives.planner_fn_force_aware: top grasp -> GPU IK -> RRT* -> Trajectory.
    The goal conf must put the grasp target on the requested gripper pose."""
    import random as pyrandom
    from torque_constrained_motion_planning_amd import ik as IK
    from torque_constrained_motion_planning_amd import panda_primitives as PP
    from torque_constrained_motion_planning_amd.scene import Box, PandaRobot, Payload
    from torque_constrained_motion_planning_amd.utils import Problem
    np.random.seed(3)
    pyrandom.seed(3)
    robot = PandaRobot()
    table = Box(center=(0.5, 0.0, -0.02), size=(0.6, 1.0, 0.04))
    payload = Payload.coke(1.0)
    problem = Problem(robot, [table], payload, 1.0, 1.0, torque_test="rne")
    start = IK.TOP_HOLDING_LEFT_ARM
    pose = ((0.45, 0.1, 0.2), IK.quat_from_euler((0, 0, 0)))
    grasp_conf = IK.grasp_conf_for_pose(problem, start, pose, engine=eng)
    assert grasp_conf is not None
    grasp = IK.get_top_grasp(payload)
    gripper = IK.to_matrix(IK.multiply(pose, IK.invert(grasp.value)))
    P = eng.fk(np.array([grasp_conf]))[0]
    T8 = np.eye(4)
    T8[:3, :3] = P[:9].reshape(3, 3)
    T8[:3, 3] = P[9:]
    assert np.abs(T8 @ IK.EE_TO_TOOL - gripper).max() < 1e-9
    np.random.seed(4)
    pyrandom.seed(4)
    traj = PP.planner_fn_force_aware(start, pose, problem)
    if traj is not None:
        last = np.array(traj.path[-1].values)
        P = eng.fk(last[None])[0]
        T8[:3, :3] = P[:9].reshape(3, 3)
        T8[:3, 3] = P[9:]
        assert np.abs(T8 @ IK.EE_TO_TOOL - gripper).max() < 1e-6
