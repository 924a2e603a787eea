"""rrt_star.py drop-in: force-aware RRT* with the reference's callback API.

Reference: src/rrt_star.py:151-211.  When every callback was built by this package
(utils.get_*_fn, panda_primitives torque tests / dynamics fn), the loop runs on the GPU
engine: the host keeps the reference's RNG consumption (Python `random()` for the goal
bias, np.random.uniform through the sample fn) and hands each iteration's draw to
tcmp_plan_round (nearest / extend / collision / torque / insert / rewire on the device),
then tcmp_plan_finish does retrace + min-jerk + the final dynamic torque validation.
Foreign callbacks run the same algorithm on the host, calling them one at a time.

rrt_star_batched() is the engine-native frontier: B device-sampled candidates per round.
"""
from __future__ import print_function

from random import random
from time import time

import numpy as np

from . import _lib

INF = float('inf')


def elapsed_time(start_time):
    return time() - start_time


def argmin(function, sequence):  # rrt_star.py:9-14
    values = list(sequence)
    scores = [function(x) for x in values]
    return values[scores.index(min(scores))]


class OptimalNode(object):  # rrt_star.py:18-63
    def __init__(self, config, parent=None, d=0, path=[], iteration=None):
        self.config = config
        self.parent = parent
        self.children = set()
        self.d = d
        self.path = path
        if parent is not None:
            self.cost = parent.cost + d
            self.parent.children.add(self)
        else:
            self.cost = d
        self.solution = False
        self.creation = iteration
        self.last_rewire = iteration

    def set_solution(self, solution):
        if self.solution is solution:
            return
        self.solution = solution
        if self.parent is not None:
            self.parent.set_solution(solution)

    def retrace(self):
        if self.parent is None:
            return self.path + [self.config]
        return self.parent.retrace() + self.path + [self.config]

    def rewire(self, parent, d, path, iteration=None):
        if self.solution:
            self.parent.set_solution(False)
        self.parent.children.remove(self)
        self.parent = parent
        self.parent.children.add(self)
        if self.solution:
            self.parent.set_solution(True)
        self.d = d
        self.path = path
        self.update()
        self.last_rewire = iteration

    def update(self):
        self.cost = self.parent.cost + self.d
        for n in self.children:
            n.update()


def safe_path(sequence, collision):  # rrt_star.py:82-88
    path = []
    for q in sequence:
        if collision(q):
            break
        path.append(q)
    return path


def safe_path_force_aware(sequence, collision, torque):  # rrt_star.py:90-98
    path = []
    for q in sequence:
        if collision(q):
            break
        if not torque(q):
            break
        path.append(q)
    return path


def _native(distance, sample, extend, collision, torque_fn, dynam_fn):
    from .panda_primitives import DynamFn, TorqueTest
    from .utils import CollisionFn, DistanceFn, ExtendFn, SampleFn
    return (isinstance(distance, DistanceFn) and isinstance(sample, SampleFn)
            and isinstance(extend, ExtendFn) and isinstance(collision, CollisionFn)
            and isinstance(torque_fn, TorqueTest) and isinstance(dynam_fn, DynamFn)
            and np.allclose(sample.lower, _lib_limits()[0]) and np.allclose(sample.upper, _lib_limits()[1]))


def _lib_limits():
    from .scene import JOINT_LOWER, JOINT_UPPER
    return JOINT_LOWER, JOINT_UPPER


def _radius_value(radius):
    r = np.asarray(radius, dtype=np.float64).reshape(-1)
    if r.size != 1:
        raise ValueError("radius must be a scalar or a 1-element list (reference: [0.01])")
    return float(r[0])


def _finish(eng, start_hint=None):
    r = eng.plan_finish()
    if r.status == _lib.PLAN_NO_GOAL:
        print("failed to find goal")
        return (None, None, None, None), r, None
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


def rrt_star_force_aware(start, goal, distance, sample, extend, collision, torque_fn, dynam_fn,
                         radius, max_time=INF, max_iterations=INF, goal_probability=.2,
                         informed=False):
    """rrt_star.py:151-211 -> (path, vels, accels, psg) or (None, None, None, None)."""
    if not informed and _native(distance, sample, extend, collision, torque_fn, dynam_fn):
        res, _, _ = _rrt_native(start, goal, distance, sample, extend, collision, torque_fn,
                                dynam_fn, radius, max_iterations, goal_probability)
        return res
    return _rrt_host(start, goal, distance, sample, extend, collision, torque_fn, dynam_fn,
                     radius, max_time, max_iterations, goal_probability, informed)


def _rrt_native(start, goal, distance, sample, extend, collision, torque_fn, dynam_fn, radius,
                max_iterations, goal_probability):
    if max_iterations == INF:
        raise ValueError("max_iterations must be finite (the reference's time guard never "
                         "fires, rrt_star.py:159, so INF iterations never return)")
    max_iterations = int(max_iterations)
    eng = collision.engine
    start = tuple(float(x) for x in start)
    goal = tuple(float(x) for x in goal)
    st = eng.plan_begin(start, goal, torque_fn.mode, torque_fn.payload_mass,
                        dynam_fn.execution_time, max_nodes=max_iterations + 1, max_batch=1,
                        weights=distance.weights, resolutions=extend.resolutions,
                        radius=_radius_value(radius), goal_probability=goal_probability)
    if st == _lib.PLAN_START_GOAL_COLLISION:
        print("start config in collision")
        return (None, None, None, None), None, None
    goal_found = False
    it = 0
    while it < max_iterations:
        do_goal = (not goal_found) and (it == 0 or random() < goal_probability)
        s = goal if do_goal else sample()
        it += 1
        goal_found = eng.plan_round(np.asarray([s], dtype=np.float64), [do_goal])
    return _finish(eng)


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


def _rrt_host(start, goal, distance, sample, extend, collision, torque_fn, dynam_fn, radius,
              max_time=INF, max_iterations=INF, goal_probability=.2, informed=False):
    """The reference loop verbatim (rrt_star.py:151-211) for foreign callbacks."""
    if collision(start) or collision(goal):
        print("start config in collision")
        return (None, None, None, None)
    nodes = [OptimalNode(start)]
    goal_n = None
    t0 = time()
    it = 0
    while (t0 - time()) < max_time and it < max_iterations:
        do_goal = goal_n is None and (it == 0 or random() < goal_probability)
        s = goal if do_goal else sample()
        if informed and goal_n is not None and distance(start, s) + distance(s, goal) >= goal_n.cost:
            print("greater than cost")
            continue
        it += 1
        nearest = argmin(lambda n: distance(n.config, s), nodes)
        path = safe_path_force_aware(extend(nearest.config, s), collision, torque_fn)
        if len(path) == 0:
            continue
        new = OptimalNode(path[-1], parent=nearest, d=distance(nearest.config, path[-1]),
                          path=path[:-1], iteration=it)
        if do_goal and distance(new.config, goal) < 1e-2:
            goal_n = new
            goal_n.set_solution(True)
        neighbors = filter(lambda n: distance(n.config, new.config) < radius, nodes)
        nodes.append(new)
        for n in neighbors:
            d = distance(n.config, new.config)
            if n.cost + d < new.cost:
                path = safe_path_force_aware(extend(n.config, new.config), collision, torque_fn)
                if len(path) != 0 and distance(new.config, path[-1]) < 1e-6:
                    new.rewire(n, d, path[:-1], iteration=it)
        # the reference's second rewire loop never runs: `neighbors` is an exhausted
        # iterator by then (rrt_star.py:193)
    if goal_n is None:
        print("failed to find goal")
        return None, None, None, None
    rrtPath = goal_n.retrace()
    path, psg, vels, accels = dynam_fn(rrtPath, len(rrtPath))
    vels = vels[:len(path)]
    accels = accels[:len(path)]
    if path is None:
        return None, None, None, None
    for i in range(len(path)):
        if not torque_fn(path[i], velocities=vels[i], accelerations=accels[i]):
            return None, None, None, None
    return path, vels, accels, psg
