#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE Python in this container.

Dev-time only (needs /root/reference, which never reaches the GPU box).  It imports the
reference modules that are importable without pybullet:
  rne.py          (with the `np.Inf = np.inf` shim numpy 2 needs, rne.py:203)
  min_jerk_v2.py
  rrt_star.py
and drives rrt_star.rrt_star_force_aware (rrt_star.py:151) with closures restated from
the pybullet-backed utils.py / panda_primitives.py factories (cited below).  Obstacle
collision uses the oracle's hull-vs-box semantics (pybullet is absent: parity of that
piece against Bullet is unpinned).

Outputs (small npz fixtures, no pickles) in tests/golden/:
  rne_golden.npz       reference rne() torques, static and dynamic, payload 0/2/5 kg
  minjerk_golden.npz   reference minjerk_coefficients/minjerk_trajectory outputs
  fk_golden.npz        reference DH forward kinematics panda_link0 -> panda_link8
                       (X = rne.get_parent_to_child_transform(q, 0, 8) = inv(T_0^8),
                       rne.py:46-63, and T = inv(X)): pins the
                       FK the IK round trip is checked with (ikfast itself is unbuildable here)
  rrt_<name>.npz       full reference RRT* runs: RNG streams consumed, waypoints,
                       trajectory q/qd/qdd/psg (strided subsample for long ones)
"""
import os
import random
import sys
import time

import numpy as np

REF_SRC = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REF_SRC)
sys.path.insert(0, os.path.join(REPO, "oracle"))
np.Inf = np.inf  # numpy 2 removed np.Inf; rne.py:203 uses it

import min_jerk_v2 as ref_mj  # noqa: E402
import rne as ref_rne  # noqa: E402
import rrt_star as ref_rrt  # noqa: E402

import oracle  # noqa: E402

# panda_mod.urdf joint limits / efforts
LO = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
HI = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])
EFFORT = [87.0, 87.0, 87.0, 87.0, 12.0, 12.0, 12.0]
TOP_HOLDING_LEFT_ARM = [0, -np.pi / 4, 0.0, -6 * np.pi / 8, 0, np.pi / 2, np.pi / 4]  # utils.py:45
RESOLUTIONS = 0.2 ** np.ones(7)          # panda_primitives.py:248
RADIUS = RESOLUTIONS / 2                 # panda_primitives.py:274 radius=resolutions/2
WEIGHTS = np.reciprocal(RADIUS)          # panda_primitives.py:333-334


# ---- restated utils.py closures (pybullet-free) -------------------------------------------
def difference_fn(q2, q1):               # utils.py:2995-3001 (no circular joints on the Panda)
    return tuple(v2 - v1 for v2, v1 in zip(q2, q1))


def distance_fn(q1, q2):                 # utils.py:3010-3017
    diff = np.array(difference_fn(q2, q1))
    return np.sqrt(np.dot(WEIGHTS, diff * diff))


def refine_fn(q1, q2, num_steps):        # utils.py:3031-3041
    num_steps = num_steps + 1
    q = q1
    for i in range(num_steps):
        positions = (1. / (num_steps - i)) * np.array(difference_fn(q2, q)) + q
        q = tuple(positions)
        yield q


def extend_fn(q1, q2):                   # utils.py:3068-3077
    steps = int(np.linalg.norm(np.divide(difference_fn(q2, q1), RADIUS), ord=2))
    return refine_fn(q1, q2, steps)


def all_between(lo, v, hi):              # utils.py:1150-1154
    return np.less_equal(lo, v).all() and np.less_equal(v, hi).all()


class SampleRecorder:                    # utils.py:2941-2990 uniform_generator/convex_combination
    def __init__(self):
        self.u = []

    def __call__(self):
        w = np.random.uniform(size=7)
        self.u.append(np.array(w))
        return tuple((1 - w) * np.array(LO) + w * np.array(HI))


class RandomRecorder:                    # rrt_star.py:3 `from random import random`
    def __init__(self):
        self.vals = []
        self._r = random.random

    def __call__(self):
        x = self._r()
        self.vals.append(x)
        return x


def make_collision_fn(obs):              # utils.py:3165-3218 (limits first, then obstacles)
    obs = oracle.obstacles_array(obs)

    def collision_fn(q, verbose=False):
        if not all_between(LO, q, HI):
            return True
        if len(obs) == 0:
            return False
        return oracle.collision(np.array(q, dtype=np.float64), obs, cull=1)
    return collision_fn


class Problem:                           # utils.py:86-93
    def __init__(self, payload_mass, execution_time, torque_test):
        self.payload_mass = payload_mass
        self.payload = None if payload_mass is None else object()
        self.execution_time = execution_time
        self.torque_test = torque_test


def torque_test_base(problem):           # panda_primitives.py:13-16
    def test(poses=None, ptotalMass=None, velocities=None, accelerations=None):
        return True
    return test


def torque_test_nov(problem):            # panda_primitives.py:118-153
    def test(poses=None, ptotalMass=None, velocities=None, accelerations=None):
        totalMass = problem.payload_mass
        if problem.payload is None:
            totalMass = 0
        velocities = [0] * len(poses)
        accelerations = [0] * len(poses)
        if totalMass > 0.01:
            ref_rne.add_payload([0, 0, 0.05], totalMass)
        torques = ref_rne.rne(poses, velocities, accelerations)
        for i in range(len(EFFORT) - 1):
            if abs(torques[i]) >= EFFORT[i]:
                ref_rne.remove_payload()
                return False
        ref_rne.remove_payload()
        return True
    return test


def torque_test_rne(problem):            # panda_primitives.py:155-193 (_v4)
    def test(poses=None, ptotalMass=problem.payload_mass, velocities=None, accelerations=None):
        totalMass = ptotalMass
        if velocities is None or accelerations is None:
            velocities = [0] * len(poses)
            accelerations = [0] * len(poses)
        if totalMass > 0.01:
            ref_rne.add_payload([0, 0, 0.03], totalMass)
        torques = ref_rne.rne(poses, velocities, accelerations)
        for i in range(len(EFFORT) - 1):
            if abs(torques[i]) >= EFFORT[i]:
                ref_rne.remove_payload()
                return False
        ref_rne.remove_payload()
        return True
    return test


TESTS = {"base": torque_test_base, "nov": torque_test_nov, "rne": torque_test_rne}
MODE_ID = {"base": 0, "nov": 1, "rne": 2}


def make_dynam_fn(problem, record):      # panda_primitives.py:295-318 (get_dynamics_fn_v5)
    def dynam_fn(path, dur=None):
        record.append(np.array(path, dtype=np.float64))
        m_coeff = ref_mj.minjerk_coefficients(np.array(path))
        move_time = problem.execution_time
        num_intervals = move_time * 1000 / len(path)
        traj = ref_mj.minjerk_trajectory(m_coeff, num_intervals=int(num_intervals))
        q = [list(x[0]) for x in traj]
        qd = [list(x[1]) for x in traj]
        qdd = [list(x[2]) for x in traj]
        psg = [move_time * n / len(traj) for n in range(0, len(traj))]
        return q, psg, qd, qdd
    return dynam_fn


# ---- fixtures -----------------------------------------------------------------------------
def gen_rne(path):
    rng = np.random.default_rng(20261015)
    N = 192
    out = {}
    for m in (0.0, 2.0, 5.0):
        q = LO + (HI - LO) * rng.random((N, 7))
        qd = rng.uniform(-2.5, 2.5, (N, 7))
        qdd = rng.uniform(-8.0, 8.0, (N, 7))
        ts, td = [], []
        for i in range(N):
            if m > 0:
                ref_rne.add_payload([0, 0, 0.03], m)
            ts.append(ref_rne.rne(list(q[i]), [0.0] * 7, [0.0] * 7))
            td.append(ref_rne.rne(list(q[i]), list(qd[i]), list(qdd[i])))
            ref_rne.remove_payload()
        tag = "m%d" % int(m)
        out["q_" + tag] = q
        out["qd_" + tag] = qd
        out["qdd_" + tag] = qdd
        out["tau_static_" + tag] = np.array(ts)
        out["tau_dyn_" + tag] = np.array(td)
    np.savez_compressed(path, masses=np.array([0.0, 2.0, 5.0]), **out)


def gen_minjerk(path):
    rng = np.random.default_rng(7)
    out = {}
    cases = [(2, 5), (3, 1), (4, 9), (7, 13), (12, 6)]
    for ci, (n, ni) in enumerate(cases):
        P = LO + (HI - LO) * rng.random((n, 7))
        if ci == 3:  # waypoints with sign changes and zero-velocity joints
            P[2] = P[1]
        c = ref_mj.minjerk_coefficients(P)
        traj = ref_mj.minjerk_trajectory(c, ni)
        out["P%d" % ci] = P
        out["ni%d" % ci] = np.array(ni)
        out["coef%d" % ci] = c
        out["x%d" % ci] = np.array([t[0] for t in traj])
        out["v%d" % ci] = np.array([t[1] for t in traj])
        out["a%d" % ci] = np.array([t[2] for t in traj])
    out["ncases"] = np.array(len(cases))
    np.savez_compressed(path, **out)


def gen_fk(path):
    rng = np.random.default_rng(77)
    q = rng.uniform(LO, HI, size=(400, 7))
    # a few structured rows: zeros, the holding pose, joint-limit corners
    q[0] = 0.0
    q[1] = TOP_HOLDING_LEFT_ARM
    q[2] = LO
    q[3] = HI
    # get_parent_to_child_transform returns inv(T_0^8) (rne.py:63); keep it raw and its inverse
    X = np.stack([ref_rne.get_parent_to_child_transform(list(r), 0, 8) for r in q])
    T = np.stack([np.linalg.inv(x) for x in X])
    np.savez_compressed(path, q=q, X=X, T=T)


def boxes_scene(rng, n, avoid):
    """SURVEY 8d synthetic boxes: centres U([0.2,0.8]x[-0.6,0.6]x[0,0.8]), half U[0.03,0.12],
    axis aligned, rejected if any configuration in `avoid` collides."""
    boxes = []
    while len(boxes) < n:
        c = rng.uniform([0.2, -0.6, 0.0], [0.8, 0.6, 0.8])
        h = rng.uniform(0.03, 0.12, 3)
        b = np.concatenate([c, np.eye(3).reshape(-1), h])
        if any(oracle.collision(q, b[None, :]) for q in avoid):
            continue
        boxes.append(b)
    return np.array(boxes).reshape(-1, 15)


class _NodeLog:
    """Records the reference's OptimalNode graph (rrt_star.py:18-63) while a run builds it:
    every node in creation order (= the order of `nodes`, rrt_star.py:185) and every
    OptimalNode.rewire call (rrt_star.py:47-58), through a subclass swapped in for the
    module attribute rrt_star_force_aware instantiates."""

    def __init__(self):
        self.nodes = []
        self.rewires = 0
        log = self

        class Node(ref_rrt.OptimalNode):
            def __init__(self, *a, **kw):
                super().__init__(*a, **kw)
                log.nodes.append(self)

            def rewire(self, *a, **kw):
                log.rewires += 1
                return super().rewire(*a, **kw)
        self.cls = Node

    def arrays(self):
        ix = {id(n): i for i, n in enumerate(self.nodes)}
        cfg = np.array([np.asarray(n.config, dtype=np.float64) for n in self.nodes])
        cost = np.array([float(n.cost) for n in self.nodes])
        par = np.array([-1 if n.parent is None else ix[id(n.parent)] for n in self.nodes],
                       dtype=np.int32)
        return cfg, cost, par


def run_reference(name, start, goal, obs, mode, mass, exec_time, iters, seed, stride=1,
                  want_found=None, informed=False, radius=0.01):
    problem = Problem(mass, exec_time, mode)
    torque_fn = TESTS[mode](problem)
    collision_fn = make_collision_fn(obs)
    sample = SampleRecorder()
    rnd = RandomRecorder()
    wp_rec = []
    dynam_fn = make_dynam_fn(problem, wp_rec)
    random.seed(seed)
    np.random.seed(seed)
    saved = ref_rrt.random, ref_rrt.OptimalNode
    log = _NodeLog()
    ref_rrt.random = rnd
    ref_rrt.OptimalNode = log.cls
    t0 = time.time()
    try:
        # the planner passes a one-element list (panda_primitives.py:346)
        path, vels, accels, psg = ref_rrt.rrt_star_force_aware(
            tuple(start), tuple(goal), distance_fn, sample, extend_fn, collision_fn, torque_fn,
            dynam_fn, radius=[radius], max_time=50, max_iterations=iters, informed=informed)
    finally:
        ref_rrt.random, ref_rrt.OptimalNode = saved
    dt = time.time() - t0
    if want_found is not None and (path is not None) != want_found:
        return False
    res = dict(start=np.array(start, dtype=np.float64), goal=np.array(goal, dtype=np.float64),
               obs=oracle.obstacles_array(obs), mode=np.array(MODE_ID[mode]),
               mass=np.array(float(mass)), exec_time=np.array(float(exec_time)),
               iters=np.array(iters), seed=np.array(seed),
               replay_random=np.array(rnd.vals, dtype=np.float64),
               replay_uniform=np.array(sample.u, dtype=np.float64).reshape(-1, 7),
               found=np.array(path is not None), stride=np.array(stride),
               informed=np.array(bool(informed)), radius=np.array(float(radius)),
               n_rewires=np.array(log.rewires))
    cfg, cost, par = log.arrays()
    res["tree_cfg"], res["tree_cost"], res["tree_parent"] = cfg, cost, par
    if wp_rec:
        res["waypoints"] = wp_rec[-1]
    if path is not None:
        q = np.array(path); qd = np.array(vels); qdd = np.array(accels); p = np.array(psg)
        res["n_traj"] = np.array(len(q))
        idx = np.unique(np.concatenate([np.arange(0, len(q), stride), [len(q) - 1]]))
        res["traj_idx"] = idx
        res["q"] = q[idx]; res["qd"] = qd[idx]; res["qdd"] = qdd[idx]; res["psg"] = p[idx]
        res["sum_q"] = q.sum(0); res["sum_qd"] = qd.sum(0); res["sum_qdd"] = qdd.sum(0)
    np.savez_compressed(os.path.join(HERE, "rrt_%s.npz" % name), **res)
    print("%-22s found=%s waypoints=%s traj=%s random=%d uniform=%d nodes=%d rewires=%d  %.1fs" % (
        name, path is not None, len(wp_rec[-1]) if wp_rec else None,
        len(path) if path is not None else None, len(rnd.vals), len(sample.u), len(cfg),
        log.rewires, dt))
    return True


def pick_query(rng, obs_n, mode, mass, need_block=True, tries=20000, near=None, iters=150,
               random_start=False):
    """Random goal (collision free, torque feasible) whose straight edge from the start is
    blocked, so the tree has to grow.  Pre-screened with the oracle RRT (Philox stream)."""
    start = np.array(TOP_HOLDING_LEFT_ARM)
    for _ in range(tries):
        if random_start:
            start = LO + (HI - LO) * rng.random(7)
        if near is None:
            goal = LO + (HI - LO) * rng.random(7)
        else:
            goal = np.clip(start + rng.normal(0, near, 7), LO, HI)
        obs = boxes_scene(rng, obs_n, [start, goal]) if obs_n else np.zeros((0, 15))
        if oracle.collision(goal, obs) or not oracle.torque_ok(goal, MODE_ID[mode], mass):
            continue
        if not oracle.torque_ok(start, MODE_ID[mode], mass):
            continue
        safe, ns, _ = oracle.check_edge(start, goal, obs, MODE_ID[mode], mass)
        if need_block and safe == ns:
            continue
        if not need_block and safe != ns:
            continue
        ok = sum(oracle.rrt_run(start, goal, iters, obs, MODE_ID[mode], mass, 1.0, seed=sd,
                                validate=False)["status"] == 0 for sd in range(3))
        if need_block and ok < 2:
            continue
        return start, goal, obs
    raise RuntimeError("no query found")


def search(name, rng, n_obs, mode, mass, exec_time, iters, seed, want_found=True, block=True,
           near=None, random_start=False):
    for attempt in range(60):
        s, g, o = pick_query(rng, n_obs, mode, mass, need_block=block, near=near,
                             iters=iters if want_found else 150, random_start=random_start)
        if run_reference(name, s, g, o, mode, mass, exec_time, iters, seed + 100 * attempt,
                         want_found=want_found):
            return
    raise RuntimeError("no golden query for " + name)


def gen_c1k():
    """C1 at BASELINE configs[0]'s own size: empty scene, 0 kg, base, 1000 RRT* iterations,
    T_exec 5 (the goal is reached at it=1 and the loop runs on to 1000)."""
    run_reference("c1_1k_base", TOP_HOLDING_LEFT_ARM, (0.5, 0.2, 0.1, -1.5, 0.3, 1.8, 0.2),
                  [], "base", 0.0, 5.0, 1000, 0, stride=37)


def gen_informed():
    """informed=True (rrt_star.py:163-165; the reference planner never sets it): the empty-scene
    rne query of rrt_empty_rne5.npz, run on past the goal so that draws that cannot beat the
    goal's cost are rejected (they consume the sample stream but not the iteration budget)."""
    z = np.load(os.path.join(HERE, "rrt_empty_rne5.npz"))
    run_reference("empty_rne5_informed", z["start"], z["goal"], [], "rne", 5.0, 1.0,
                  2 * int(z["iters"]), int(z["seed"]), stride=7, want_found=True, informed=True)


def gen_rewire():
    """Reference runs at the large rewire radii where OptimalNode.rewire actually fires
    (rrt_star.py:183-192; the planner's radius=[0.01] never rewires: every other golden has
    n_rewires = 0).  Each fixture stores the reference's final tree (configs, costs, parents
    in node order) and its rewire count, and must have rewired at least `min_rw` times."""
    rng = np.random.default_rng(4321)
    cases = [  # name, obstacles, mode, mass, exec_time, iterations, seed, radius, min_rw
        ("rewire_empty_rne5_r4", 0, "rne", 5.0, 1.0, 400, 11, 4.0, 1),
        ("rewire_box4_nov2_r8", 4, "nov", 2.0, 1.0, 300, 12, 8.0, 50),
        ("rewire_box16_rne5_r6", 16, "rne", 5.0, 1.0, 500, 13, 6.0, 20),
        ("rewire_box8_base_r8", 8, "base", 0.0, 0.5, 250, 14, 8.0, 50),
    ]
    for name, n_obs, mode, mass, et, iters, seed, radius, min_rw in cases:
        for attempt in range(60):
            s, g, o = pick_query(rng, n_obs, mode, mass, need_block=True, iters=iters,
                                 random_start=n_obs == 0)
            if not run_reference(name, s, g, o, mode, mass, et, iters, seed + 100 * attempt,
                                 want_found=True, radius=radius):
                continue
            z = np.load(os.path.join(HERE, "rrt_%s.npz" % name))
            if int(z["n_rewires"]) >= min_rw:
                break
        else:
            raise RuntimeError("no rewiring golden query for " + name)


def main():
    if "--only-rewire" in sys.argv:
        gen_rewire()
        return
    if "--only-informed" in sys.argv:
        gen_informed()
        return
    if "--only-fk" in sys.argv:
        gen_fk(os.path.join(HERE, "fk_golden.npz"))
        return
    if "--only-c1k" in sys.argv:
        gen_c1k()
        return
    gen_fk(os.path.join(HERE, "fk_golden.npz"))
    gen_rne(os.path.join(HERE, "rne_golden.npz"))
    gen_minjerk(os.path.join(HERE, "minjerk_golden.npz"))
    rng = np.random.default_rng(1234)
    # C1-like: empty scene, base, straight edge succeeds (SURVEY App. C goal), T_exec 5
    run_reference("c1_base_direct", TOP_HOLDING_LEFT_ARM, (0.5, 0.2, 0.1, -1.5, 0.3, 1.8, 0.2),
                  [], "base", 0.0, 5.0, 60, 0, stride=37)
    gen_c1k()
    # empty scene, torque-blocked straight edge -> tree growth
    search("empty_rne5", rng, 0, "rne", 5.0, 1.0, 300, 1, random_start=True)
    search("empty_nov5", rng, 0, "nov", 5.0, 1.0, 300, 2, random_start=True)
    # boxes (oracle collision semantics)
    search("box4_nov2", rng, 4, "nov", 2.0, 1.0, 150, 3)
    search("box16_rne5", rng, 16, "rne", 5.0, 1.0, 150, 4)
    search("box8_base", rng, 8, "base", 0.0, 0.5, 300, 5)
    # the goal is never reached within the budget
    search("box16_rne5_short", rng, 16, "rne", 5.0, 1.0, 4, 6, want_found=False)
    gen_informed()


if __name__ == "__main__":
    main()
