"""rrt_star.py drop-in: force-aware RRT* with the reference's callback API.

Reference: src/rrt_star.py:151-211 (rrt_star_force_aware).  Three ways through it, picked by
which callbacks this package built (utils.get_*_fn, panda_primitives torque tests / dynamics
fn -- recognised by type):

* engine loop -- distance, extend, collision and torque are the package's own: the tree lives
  on the GPU.  The host keeps the reference's RNG consumption (Python `random()` for the goal
  bias, then the sample callback, which may be foreign) and hands each iteration's draw to
  tcmp_plan_round (nearest / extend / collision / torque / insert / rewire on the device);
  tcmp_plan_finish does retrace + min-jerk + the final dynamic torque validation.  A foreign
  dynam_fn is applied on the host to the engine's retraced waypoints.
* host loop -- distance or extend is foreign: the tree is kept as arrays
  on the host (_Tree).  Each foreign callback is called exactly where the reference calls it;
  the package's own collision / torque tests are evaluated by the engine in one batched
  launch per extend sequence (tcmp_check_configs / tcmp_torque_ok, or tcmp_check_edges for
  the whole edge when extend is native too), and a native distance is a vectorised argmin.
* rrt_star_batched -- the engine-native frontier: B device-sampled candidates per round.
"""
from __future__ import print_function

from random import random
from time import time

import numpy as np

from . import _lib

INF = float('inf')


def elapsed_time(start_time):
    return time() - start_time


# ---- which callbacks are the package's own ---------------------------------------------------
def _kinds(distance, sample, extend, collision, torque_fn, dynam_fn):
    from .panda_primitives import DynamFn, TorqueTest
    from .utils import CollisionFn, DistanceFn, ExtendFn
    return dict(distance=isinstance(distance, DistanceFn), extend=isinstance(extend, ExtendFn),
                collision=isinstance(collision, CollisionFn),
                torque=isinstance(torque_fn, TorqueTest), dynam=isinstance(dynam_fn, DynamFn))


def _radius_value(radius):
    r = np.asarray(radius, dtype=np.float64).reshape(-1)
    if r.size != 1:
        raise ValueError("radius must be a scalar or a 1-element list (reference: [0.01])")
    return float(r[0])


def rrt_star_force_aware(start, goal, distance, sample, extend, collision, torque_fn, dynam_fn,
                         radius, max_time=INF, max_iterations=INF, goal_probability=.2,
                         informed=False):
    """rrt_star.py:151-211 -> (path, vels, accels, psg) or (None, None, None, None)."""
    k = _kinds(distance, sample, extend, collision, torque_fn, dynam_fn)
    if k["distance"] and k["extend"] and k["collision"] and k["torque"]:
        res, _, _ = _rrt_engine(start, goal, distance, sample, extend, collision, torque_fn,
                                dynam_fn, radius, max_iterations, goal_probability, k["dynam"],
                                informed)
        return res
    return _rrt_host(start, goal, distance, sample, extend, collision, torque_fn, dynam_fn,
                     radius, max_time, max_iterations, goal_probability, informed, k)


# ---- shared tail: dynam_fn + final validation (rrt_star.py:202-211) --------------------------
def _validate_and_return(rrt_path, dynam_fn, torque_fn, native_torque):
    path, psg, vels, accels = dynam_fn(rrt_path, len(rrt_path))
    vels = vels[:len(path)]
    accels = accels[:len(path)]
    if path is None:
        return None, None, None, None
    if native_torque and len(path):
        q = np.asarray(path, dtype=np.float64)[:, :7]
        first_fail, _ = _lib.engine().validate(q, np.asarray(vels, dtype=np.float64)[:, :7],
                                               np.asarray(accels, dtype=np.float64)[:, :7],
                                               torque_fn.mode, torque_fn.payload_mass,
                                               want_tau=False)
        if first_fail >= 0:
            return None, None, None, None
    else:
        for i in range(len(path)):
            if not torque_fn(path[i], velocities=vels[i], accelerations=accels[i]):
                return None, None, None, None
    return path, vels, accels, psg


def _finish(eng, dynam_fn=None, torque_fn=None):
    """tcmp_plan_finish -> the reference's return tuple.  dynam_fn: a foreign dynamics fn,
    applied on the host to the engine's retraced waypoints (tcmp_plan_retrace: no device
    min-jerk or validation runs for it); else the engine's min-jerk and validation stand."""
    r = eng.plan_retrace() if dynam_fn is not None else eng.plan_finish()
    if r.status == _lib.PLAN_NO_GOAL:
        print("failed to find goal")
        return (None, None, None, None), r, None
    if dynam_fn is not None:
        out = eng.plan_fetch(r)
        rrt_path = [tuple(x) for x in out["waypoints"]]
        return _validate_and_return(rrt_path, dynam_fn, torque_fn, True), r, out
    print("run min jerk")
    if r.status == _lib.PLAN_MINJERK_ASSERT:
        raise AssertionError("Invalid number of intervals chosen (must be greater than 0)")
    out = eng.plan_fetch(r)
    if r.status == _lib.PLAN_VALIDATION_FAILED:
        return (None, None, None, None), r, out
    path = [list(x) for x in out["q"]]
    vels = [list(x) for x in out["qd"]]
    accels = [list(x) for x in out["qdd"]]
    psg = [float(x) for x in out["psg"]]
    return (path, vels, accels, psg), r, out


# ---- engine loop ---------------------------------------------------------------------------
def _rrt_engine(start, goal, distance, sample, extend, collision, torque_fn, dynam_fn, radius,
                max_iterations, goal_probability, native_dynam=True, informed=False):
    if max_iterations == INF:
        raise ValueError("max_iterations must be finite (the reference's time guard never "
                         "fires, rrt_star.py:159, so INF iterations never return)")
    max_iterations = int(max_iterations)
    eng = collision.engine
    start = tuple(float(x) for x in start)
    goal = tuple(float(x) for x in goal)
    st = eng.plan_begin(start, goal, torque_fn.mode, torque_fn.payload_mass,
                        dynam_fn.execution_time if native_dynam else 0.0,
                        max_nodes=max_iterations + 1, max_batch=1,
                        weights=distance.weights, resolutions=extend.resolutions,
                        radius=_radius_value(radius), goal_probability=goal_probability)
    if st == _lib.PLAN_START_GOAL_COLLISION:
        print("start config in collision")
        return (None, None, None, None), None, None
    goal_found = False
    goal_cost = INF
    it = 0
    while it < max_iterations:
        # rrt_star.py:160-161: random() only while the goal is open and it > 0
        do_goal = (not goal_found) and (it == 0 or random() < goal_probability)
        s = goal if do_goal else sample()
        # informed RRT* (rrt_star.py:163-165): goal_n.cost is fixed once its insertion round
        # (rewiring included) is over -- only the newest node is ever rewired
        if informed and goal_found and distance(start, s) + distance(s, goal) >= goal_cost:
            print("greater than cost")
            continue
        it += 1
        found = eng.plan_round(np.asarray([s], dtype=np.float64)[:, :7], [do_goal])
        if found and not goal_found and informed:
            goal_cost = eng.plan_goal()[1]
        goal_found = found
    return _finish(eng, None if native_dynam else dynam_fn, torque_fn)


def rrt_star_batched(start, goal, obstacles, torque_mode, payload_mass, execution_time,
                     n_samples, batch=65536, seed=0, weights=None, resolutions=None,
                     radius=0.01, goal_probability=0.2, device=0, engine=None,
                     self_collisions=False):
    """Engine-native batched frontier: n_samples Philox-drawn candidates, `batch` per round
    (self_collisions: the arm's self-collision pairs too, utils.py:3138-3149).

    Returns ((path, vels, accels, psg) | (None,)*4, PlanResult, raw arrays)."""
    from .scene import mesh_pack, obstacle_array
    eng = engine if engine is not None else _lib.engine(device)
    eng.set_scene(obstacle_array(obstacles), mesh_pack(obstacles))
    eng.set_self_collision(self_collisions)
    st = eng.plan_begin(start, goal, torque_mode, payload_mass, execution_time,
                        max_nodes=int(n_samples) + 1, max_batch=int(batch), seed=seed,
                        weights=weights, resolutions=resolutions, radius=radius,
                        goal_probability=goal_probability)
    if st == _lib.PLAN_START_GOAL_COLLISION:
        return (None, None, None, None), None, None
    eng.plan_run(int(n_samples), int(batch))
    return _finish(eng)


# ---- host loop -------------------------------------------------------------------------------
class _Tree:
    """The reference's OptimalNode graph (rrt_star.py:18-63) as arrays.

    Node i: the configuration object the callbacks produced, a row of `q` (float copy for the
    vectorised nearest), the parent index (-1 for the root), the cost (parent cost + edge
    length), and its edge's intermediate points (retrace output, rrt_star.py:42-45) -- either
    a list, or (from, to, n_safe) when the engine checked the edge, regenerated through the
    package's extend fn at retrace.  Children sets, set_solution and the recursive update()
    are not kept: the force-aware loop only rewires the node it has just inserted, which has
    no children yet (rrt_star.py:183-192; its second rewire loop never runs because the
    `filter` iterator is already exhausted, rrt_star.py:193)."""

    def __init__(self, root):
        self.configs = [root]
        self.q = np.zeros((1024, 7))
        self.q[0] = np.asarray(root, dtype=np.float64)[:7]
        self.parent = [-1]
        self.cost = [0.0]
        self.edge = [[]]

    def __len__(self):
        return len(self.configs)

    def add(self, config, parent, d, edge):
        n = len(self.configs)
        if n == len(self.q):
            self.q = np.concatenate([self.q, np.zeros_like(self.q)])
        self.q[n] = np.asarray(config, dtype=np.float64)[:7]
        self.configs.append(config)
        self.parent.append(parent)
        self.cost.append(self.cost[parent] + d)
        self.edge.append(edge)
        return n

    def reparent(self, i, parent, d, edge):
        self.parent[i] = parent
        self.cost[i] = self.cost[parent] + d
        self.edge[i] = edge

    def retrace(self, i, extend):
        chain = []
        while i >= 0:
            chain.append(i)
            i = self.parent[i]
        out = []
        for n in reversed(chain):
            e = self.edge[n]
            if isinstance(e, tuple):  # engine-checked edge: regenerate its points
                a, b, n_safe = e
                pts = []
                for k, q in enumerate(extend(a, b)):
                    if k >= n_safe - 1:
                        break
                    pts.append(q)
                e = pts
            out.extend(e)
            out.append(self.configs[n])
        return out


def _rrt_host(start, goal, distance, sample, extend, collision, torque_fn, dynam_fn, radius,
              max_time=INF, max_iterations=INF, goal_probability=.2, informed=False, kinds=None,
              stats=None):
    """rrt_star.py:151-211 with the tree on the host, for foreign distance / extend callbacks.
    Callback call order is the reference's, except that the package's
    own collision and torque tests are evaluated for a whole extend sequence at once (they
    are pure functions, so that is unobservable).  stats (a dict, optional) receives the final
    tree ("tree": _Tree) and the rewire count ("n_rewires")."""
    k = kinds if kinds is not None else _kinds(distance, sample, extend, collision, torque_fn,
                                               dynam_fn)
    eng = collision.engine if k["collision"] else None
    if collision(start) or collision(goal):
        print("start config in collision")
        return (None, None, None, None)
    w = np.asarray(distance.weights, dtype=np.float64) if k["distance"] else None

    def nearest(tree, s):
        if w is not None:  # argmin (rrt_star.py:9-14): first index wins ties
            d = tree.q[:len(tree)] - np.asarray(s, dtype=np.float64)[:7]
            return int(np.argmin(np.sqrt((d * d) @ w)))
        best, bi = INF, 0
        for i, c in enumerate(tree.configs):
            v = distance(c, s)
            if v < best:
                best, bi = v, i
        return bi

    def safe_prefix(a, b):
        """safe_path_force_aware(extend(a, b), collision, torque) (rrt_star.py:90-98):
        (last safe configuration or None, that edge's intermediate points)."""
        if k["extend"] and k["collision"] and k["torque"]:
            ns, _, last = eng.check_edges([a], [b], torque_fn.mode, torque_fn.payload_mass,
                                          resolutions=extend.resolutions)
            if ns[0] == 0:
                return None, None
            return tuple(last[0]), (a, b, int(ns[0]))
        pts = list(extend(a, b))
        coll = collision.batch(pts) if (k["collision"] and pts) else None
        tq = (_lib.engine().torque_ok(np.asarray(pts, dtype=np.float64)[:, :7], torque_fn.mode,
                                      torque_fn.payload_mass)
              if (k["torque"] and pts) else None)
        n = 0
        for i, q in enumerate(pts):
            if (coll[i] if coll is not None else collision(q)):
                break
            if not (tq[i] if tq is not None else torque_fn(q)):
                break
            n += 1
        if n == 0:
            return None, None
        return pts[n - 1], pts[:n - 1]

    tree = _Tree(start)
    goal_n = None
    n_rewires = 0
    t0 = time()
    it = 0
    while (t0 - time()) < max_time and it < max_iterations:  # (sic) rrt_star.py:159
        do_goal = goal_n is None and (it == 0 or random() < goal_probability)
        s = goal if do_goal else sample()
        if informed and goal_n is not None and \
                distance(start, s) + distance(s, goal) >= tree.cost[goal_n]:
            print("greater than cost")
            continue
        it += 1
        near = nearest(tree, s)
        last, edge = safe_prefix(tree.configs[near], s)
        if last is None:
            continue
        new = tree.add(last, near, distance(tree.configs[near], last), edge)
        if do_goal and distance(last, goal) < 1e-2:
            goal_n = new
        # neighbours within `radius` among all nodes, `new` included (the lazy filter is
        # consumed after nodes.append(new), rrt_star.py:183-186), in index order
        for n in range(len(tree)):
            if not distance(tree.configs[n], last) < radius:
                continue
            d = distance(tree.configs[n], last)
            if tree.cost[n] + d < tree.cost[new]:
                end, pts = safe_prefix(tree.configs[n], last)
                if end is not None and distance(last, end) < 1e-6:
                    tree.reparent(new, n, d, pts)
                    n_rewires += 1
    if stats is not None:
        stats.update(tree=tree, n_rewires=n_rewires)
    if goal_n is None:
        print("failed to find goal")
        return None, None, None, None
    return _validate_and_return(tree.retrace(goal_n, extend), dynam_fn, torque_fn, k["torque"])
