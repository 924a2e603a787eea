"""panda_primitives.py drop-in: torque tests, min-jerk dynamics fn, force-aware planning.

Reference: src/panda_primitives.py.  Factories return callable objects with the reference
closures' signatures; rrt_star_force_aware recognises them and runs on the GPU engine.
"""
import datetime

import numpy as np

from . import _lib
from . import rne as rne_mod
from .rrt_star import rrt_star_force_aware
from .scene import get_mass
from .utils import (PI, SELF_COLLISIONS, MAX_DISTANCE, TOP_HOLDING_LEFT_ARM,
                    check_initial_end_force_aware, create_trajectory, get_arm_joints,
                    get_collision_fn, get_distance_fn, get_extend_fn, get_max_force,
                    get_max_velocities, get_sample_fn)

METHOD = "arne"   # panda_primitives.py:8
MASS = 5          # panda_primitives.py:9
MAX_GRASP_WIDTH = 0.07
GRASP_LENGTH = 0.15


def arm_conf(_, __):
    return [0, -PI / 4, 0.0, -6 * PI / 8, 0, PI / 2, PI / 4]


class TorqueTest:
    """Torque-limit test closure (panda_primitives.py:13-193).

    mode: _lib.TORQUE_BASE / TORQUE_NOV / TORQUE_RNE / TORQUE_DYN.  Joint 7 is never checked
    and a torque equal to its limit fails (`range(len(max_limits)-1)`, `>=`).  For nov/rne the
    payload is added iff the resolved mass exceeds 0.01 kg; dyn applies m*9.81 at the grasp
    target through the Jacobian, with no threshold."""

    def __init__(self, problem, mode, default_mass=None):
        self.problem = problem
        self.mode = mode
        self.default_mass = default_mass
        self.max_limits = [get_max_force(problem.robot, j) for j in get_arm_joints(problem.robot)]

    def resolved_mass(self, ptotalMass=None):
        p = self.problem
        if self.mode == _lib.TORQUE_BASE:
            return 0.0
        if self.mode in (_lib.TORQUE_NOV, _lib.TORQUE_DYN):     # :131-135 / :71-75
            m = p.payload_mass
            if m is None and p.payload is not None:
                m = get_mass(p.payload)
            elif p.payload is None:
                m = 0
            return float(m)
        m = self.default_mass if ptotalMass is None else ptotalMass   # :171-174
        if m is None and p.payload is not None:
            m = get_mass(p.payload)
        return float(m)

    def __call__(self, poses=None, ptotalMass=None, velocities=None, accelerations=None):
        if self.mode == _lib.TORQUE_BASE:
            return True
        m = self.resolved_mass(ptotalMass)
        if (self.mode in (_lib.TORQUE_RNE, _lib.TORQUE_DYN) and velocities is not None
                and accelerations is not None):
            return bool(_lib.engine().torque_ok([poses], self.mode, m, qd=[velocities[:7]],
                                                 qdd=[accelerations[:7]])[0])
        return bool(_lib.engine().torque_ok([poses], self.mode, m)[0])

    @property
    def payload_mass(self):
        return self.resolved_mass(None)


def get_torque_limits_not_exceded_test_base(problem, mass=None):
    return TorqueTest(problem, _lib.TORQUE_BASE)


def get_torque_limits_not_exceded_test_v3_nov(problem, mass=None):
    return TorqueTest(problem, _lib.TORQUE_NOV)


def get_torque_limits_not_exceded_test_v4(problem, mass=None):
    # ptotalMass default = problem.payload_mass bound at creation (:171)
    return TorqueTest(problem, _lib.TORQUE_RNE, default_mass=problem.payload_mass)


def get_torque_limits_not_exceded_test_v2(problem, mass=None):
    """`dyn` mode (panda_primitives.py:60-116): tau = M qdd + C qd + g + J^T [0,0,m g,0,0,0]
    with J the grasp-target Jacobian.  M, C, g come from panda_dynamics_model in the reference,
    a module it does not ship (panda_primitives.py:6); here they are rne.py's model without the
    payload, so the absolute numbers are parity unpinned against pdm.  Mass as
    :71-75 (problem.payload_mass, else the payload body's mass, 0 without a payload;
    ptotalMass is ignored there, and here)."""
    return TorqueTest(problem, _lib.TORQUE_DYN)


class DynamFn:
    """get_dynamics_fn_v5 (panda_primitives.py:295-318): min-jerk through the RRT path with
    unit segment durations, int(execution_time*1000/len(path)) samples per segment."""

    def __init__(self, problem, resolutions):
        self.problem = problem
        self.resolutions = resolutions

    @property
    def execution_time(self):
        return self.problem.execution_time

    def __call__(self, path, dur=None, vel0=None, acc0=None):
        print("run min jerk")
        move_time = self.problem.execution_time
        num_intervals = move_time * 1000 / len(path)
        q, qd, qdd = _lib.engine().minjerk(np.asarray(path, dtype=np.float64), int(num_intervals))
        q = [list(x) for x in q]
        qd = [list(x) for x in qd]
        qdd = [list(x) for x in qdd]
        psg = [move_time * n / len(q) for n in range(0, len(q))]
        return q, psg, qd, qdd


def get_dynamics_fn_v5(problem, resolutions):
    return DynamFn(problem, resolutions)


def open_arm(robot, arm):
    """Fingers at their upper limit (0.04): the engine's collision model is built open."""
    return None


def plan_joint_motion_force_aware(body, joints, end_conf, torque_fn, dynam_fn, obstacles=[],
                                  attachments=[], self_collisions=True, disabled_collisions=set(),
                                  weights=None, radius=None, max_distance=MAX_DISTANCE,
                                  use_aabb=False, cache=True, custom_limits={}, start_conf=None,
                                  **kwargs):
    """panda_primitives.py:327-346."""
    assert len(joints) == len(end_conf)
    if (weights is None) and (radius is not None):
        weights = np.reciprocal(radius)
    sample_fn = get_sample_fn(body, joints, custom_limits=custom_limits)
    distance_fn = get_distance_fn(body, joints, weights=weights)
    extend_fn = get_extend_fn(body, joints, resolutions=radius)
    collision_fn = get_collision_fn(body, joints, obstacles, attachments, self_collisions,
                                    disabled_collisions, custom_limits=custom_limits,
                                    max_distance=max_distance, use_aabb=use_aabb, cache=cache)
    if start_conf is None:
        start_conf = getattr(body, "conf", None)
    if not check_initial_end_force_aware(start_conf, end_conf, collision_fn, torque_fn):
        return None, None, None  # (sic) the reference returns a 3-tuple here (:345)
    return rrt_star_force_aware(start_conf, end_conf, distance_fn, sample_fn, extend_fn,
                                collision_fn, torque_fn, dynam_fn, radius=[0.01], **kwargs)


def select_torque_test(problem):
    """panda_primitives.py:228-236."""
    method = problem.torque_test
    if method == "rne":
        return get_torque_limits_not_exceded_test_v4(problem)
    elif method == "dyn":
        return get_torque_limits_not_exceded_test_v2(problem)
    elif method == "base":
        return get_torque_limits_not_exceded_test_base(problem)
    elif method == "nov":
        return get_torque_limits_not_exceded_test_v3_nov(problem)
    # the reference falls through and raises UnboundLocalError at :242
    raise UnboundLocalError("local variable 'torque_test_right' referenced before assignment")


def planner_fn_force_aware(start_conf, pose, problem):
    """panda_primitives.py:223-282: grasp pose -> goal IK -> force-aware RRT* -> Trajectory."""
    from .ik import grasp_conf_for_pose
    robot = problem.robot
    obstacles = problem.fixed
    torque_test = select_torque_test(problem)
    resolutions = 0.2 ** np.ones(7)
    dynam_fn = get_dynamics_fn_v5(problem, resolutions)
    timestamp = str(datetime.datetime.now())
    from ._lib import engine as get_engine
    from .ik import body_collision
    from .scene import mesh_pack, obstacle_array
    eng = get_engine()
    grasp_conf = grasp_conf_for_pose(problem, start_conf, pose, engine=eng)
    # any(pairwise_collision(robot, b) for b in obstacles) (:260): body level, link0 included
    eng.set_scene(obstacle_array(obstacles), mesh_pack(obstacles))
    if grasp_conf is None or body_collision(eng, grasp_conf):
        print('Grasp IK failure', grasp_conf)
        return None
    if not torque_test(grasp_conf):
        print('grasp conf torques exceded')
        return None
    print("found grasp")
    arm_joints = get_arm_joints(robot)
    res = plan_joint_motion_force_aware(
        robot, arm_joints, grasp_conf, torque_test, dynam_fn, attachments=[],
        obstacles=obstacles, self_collisions=SELF_COLLISIONS, max_time=50, custom_limits={},
        radius=resolutions / 2, max_iterations=50, start_conf=start_conf)
    approach_path, approach_vels, approach_accels, approach_dts = res  # 3-tuple -> ValueError (sic)
    if approach_path is None:
        print('Approach path failure')
        return None
    return create_trajectory(robot, arm_joints, approach_path, bodies=[problem.payload],
                             velocities=approach_vels, accelerations=approach_accels,
                             dts=approach_dts, ts=timestamp, dynam_fn=rne_mod.rne)
