"""Drop-in subset of the reference utils.py used by the force-aware planner.

Reference: src/utils.py (pybullet helpers).  The closures the planner builds are returned
here as callable objects so rrt_star_force_aware can recognise them and run the whole loop
on the GPU engine; called directly they behave like the reference closures (one
configuration per call, computed by libtcmp).
"""
import numpy as np

from . import _lib
from .scene import (ARM_JOINT_NAMES, JOINT_EFFORT, JOINT_LOWER, JOINT_UPPER, JOINT_VELOCITY,
                    Box, ConvexMesh, Payload, PandaRobot, get_mass, mesh_pack,
                    obstacle_array)

PI = np.pi
INF = float("inf")
TOP_HOLDING_LEFT_ARM = [0, -PI / 4, 0.0, -6 * PI / 8, 0, PI / 2, PI / 4]  # utils.py:45
PANDA_GRIPPER_ROOT = 'panda_hand'          # utils.py:38
PANDA_TOOL_FRAME = 'panda_grasptarget'     # utils.py:39
GRIPPER_JOINT_NAMES = ['panda_hand_joint', 'panda_finger_joint1', 'panda_finger_joint2',
                       'panda_grasptarget_hand']
SELF_COLLISIONS = False                    # utils.py:56
MAX_DISTANCE = 0.04                        # utils.py:2781
DEFAULT_RESOLUTION = np.radians(3)         # utils.py:3052

__all__ = [
    "Problem", "TOP_HOLDING_LEFT_ARM", "get_sample_fn", "get_distance_fn", "get_difference_fn",
    "get_extend_fn", "get_refine_fn", "get_limits_fn", "get_collision_fn", "all_between",
    "convex_combination", "check_initial_end_force_aware", "create_trajectory", "Conf",
    "Trajectory", "get_arm_joints", "get_custom_limits", "get_max_force", "get_max_velocities",
    "PandaRobot", "Box", "Payload", "get_mass",
]


class Problem:
    """utils.py:86-93, verbatim fields.  robot: PandaRobot; fixed: [Box]; payload: Payload."""

    def __init__(self, robot, fixed, payload, payload_mass, execution_time, torque_test="arne"):
        self.robot = robot
        self.fixed = fixed
        self.payload = payload
        self.payload_mass = payload_mass
        self.execution_time = execution_time
        self.torque_test = torque_test


def get_arm_joints(robot, arm=None):
    return list(range(7))


def get_max_force(robot, joint):
    return float(JOINT_EFFORT[joint])


def get_max_velocities(robot, joints):
    return tuple(float(JOINT_VELOCITY[j]) for j in joints)


def get_custom_limits(body, joints, custom_limits={}, circular_limits=None):
    """utils.py:1593-1602 (the Panda has no circular joints)."""
    lo, hi = [], []
    for j in joints:
        if j in custom_limits:
            a, b = custom_limits[j]
        else:
            a, b = JOINT_LOWER[j], JOINT_UPPER[j]
        lo.append(a)
        hi.append(b)
    return tuple(lo), tuple(hi)


def all_between(lower_limits, values, upper_limits):  # utils.py:1150-1154
    assert len(lower_limits) == len(values)
    assert len(values) == len(upper_limits)
    return np.less_equal(lower_limits, values).all() and np.less_equal(values, upper_limits).all()


def convex_combination(x, y, w=0.5):  # utils.py:1156-1157
    return (1 - w) * np.array(x) + w * np.array(y)


def get_difference_fn(body, joints):  # utils.py:2995-3001
    def fn(q2, q1):
        return tuple(v2 - v1 for v2, v1 in zip(q2, q1))
    return fn


class SampleFn:
    """get_sample_fn (utils.py:2985-2990): uniform in the joint limits via
    np.random.uniform(size=7) (utils.py:2943) and convex_combination."""

    def __init__(self, lower, upper):
        self.lower = np.asarray(lower, dtype=np.float64)
        self.upper = np.asarray(upper, dtype=np.float64)

    def __call__(self):
        w = np.random.uniform(size=len(self.lower))
        return tuple((1 - w) * self.lower + w * self.upper)


def get_sample_fn(body, joints, custom_limits={}, **kwargs):
    lo, hi = get_custom_limits(body, joints, custom_limits)
    return SampleFn(lo, hi)


class DistanceFn:
    """get_distance_fn (utils.py:3010-3017): sqrt(dot(weights, diff*diff))."""

    def __init__(self, weights):
        self.weights = np.asarray(weights, dtype=np.float64)

    def __call__(self, q1, q2):
        diff = np.array(tuple(v2 - v1 for v2, v1 in zip(q2, q1)))
        return np.sqrt(np.dot(self.weights, diff * diff))


def get_distance_fn(body, joints, weights=None):
    if weights is None:
        weights = np.ones(len(joints))
    return DistanceFn(weights)


def get_refine_fn(body, joints, num_steps=0):  # utils.py:3031-3041
    num_steps = num_steps + 1

    def fn(q1, q2):
        q = q1
        for i in range(num_steps):
            positions = (1. / (num_steps - i)) * np.array(tuple(a - b for a, b in zip(q2, q))) + q
            q = tuple(positions)
            yield q
    return fn


class ExtendFn:
    """get_extend_fn (utils.py:3068-3077): int(norm(diff/res)) + 1 incremental steps."""

    def __init__(self, resolutions):
        self.resolutions = np.asarray(resolutions, dtype=np.float64)

    def __call__(self, q1, q2):
        steps = int(np.linalg.norm(np.divide(tuple(a - b for a, b in zip(q2, q1)),
                                             self.resolutions), ord=2))
        return get_refine_fn(None, None, num_steps=steps)(q1, q2)


def get_extend_fn(body, joints, resolutions=None, norm=2):
    if resolutions is None:
        resolutions = DEFAULT_RESOLUTION * np.ones(len(joints))
    return ExtendFn(resolutions)


def get_limits_fn(body, joints, custom_limits={}, verbose=False):  # utils.py:3154-3163
    lo, hi = get_custom_limits(body, joints, custom_limits)

    def limits_fn(q):
        return not all_between(lo, q, hi)
    return limits_fn


class CollisionFn:
    """get_collision_fn (utils.py:3165-3218): joint limits, the self-collision link pairs when
    self_collisions (get_self_link_pairs, utils.py:3138-3149), then every moving link hull vs
    every fixed obstacle with the -MAX_DISTANCE closest-point threshold.  Evaluated by the
    engine (tcmp_check_configs) on a handle of its own, created on first use with the scene
    uploaded once; rrt_star_force_aware plans on that same handle."""

    def __init__(self, body, obstacles, device=0, self_collisions=False):
        self.body = body
        self.obstacles = obstacle_array(obstacles)
        self.meshes = mesh_pack(obstacles)
        self.device = device
        self.self_collisions = bool(self_collisions)
        self._engine = None

    @property
    def engine(self):
        if self._engine is None:
            e = _lib.Engine(self.device)
            e.set_scene(self.obstacles, self.meshes)
            e.set_self_collision(self.self_collisions)
            self._engine = e
        return self._engine

    def __call__(self, q, verbose=False):
        return bool(self.engine.collides([np.asarray(q, dtype=np.float64)[:7]])[0])

    def batch(self, qs):
        return self.engine.collides(np.asarray(qs, dtype=np.float64)[:, :7])


def get_collision_fn(body, joints, obstacles=[], attachments=[], self_collisions=True,
                     disabled_collisions=set(), custom_limits={}, use_aabb=False, cache=False,
                     max_distance=MAX_DISTANCE, **kwargs):
    if disabled_collisions:
        raise NotImplementedError("disabled_collisions are not in the engine (the reference "
                                  "passes set(), panda_primitives.py:270)")
    if list(attachments):
        raise NotImplementedError("attachments are not in the engine (the reference planner "
                                  "passes none, panda_primitives.py:270)")
    if custom_limits:
        raise NotImplementedError("custom joint limits are not in the engine")
    if max_distance != MAX_DISTANCE:
        raise NotImplementedError("the engine's collision threshold is MAX_DISTANCE=0.04")
    return CollisionFn(body, obstacles, self_collisions=self_collisions)


def check_initial_end_force_aware(start_conf, end_conf, collision_fn, torque_fn, verbose=True):
    """utils.py:3323-3338."""
    if collision_fn(start_conf, verbose=verbose):
        print('Warning: initial configuration is in collision')
        return False
    if collision_fn(end_conf, verbose=verbose):
        print('Warning: end configuration is in collision')
        return False
    if not torque_fn(start_conf):
        print('Warning: initial configuration excedes torque limits')
        print(start_conf)
        return False
    if not torque_fn(end_conf):
        print('Warning: end configuration excedes torque limits')
        return False
    return True


class Conf(object):
    """utils.py:3360-3387."""

    def __init__(self, body, joints, values=None, init=False, velocities=None,
                 accelerations=None, movables=None, dt=None, dynam_fn=None, torques=None):
        self.body = body
        self.joints = joints
        if values is None:
            values = getattr(body, "conf", None)
        self.values = tuple(values)
        self.init = init
        if torques is None and dynam_fn is not None:
            torques = dynam_fn(values, velocities, accelerations)
        self.torques = torques
        self.velocities = velocities[:len(joints)] if velocities is not None else velocities
        self.accelerations = accelerations[:len(joints)] if accelerations is not None else accelerations
        self.dt = dt

    def iterate(self):
        yield self

    def __repr__(self):
        return 'q{}'.format(id(self) % 1000)


class Trajectory(object):
    """utils.py:3389-3405 (path of Conf)."""

    def __init__(self, path, bodies, ts=None, reverse_traj=False):
        path = list(path)
        if reverse_traj:
            dts = [c.dt for c in path]
            for i, c in enumerate(path):
                c.velocities = (np.multiply(c.velocities, -1)).tolist()
                c.accelerations = (np.multiply(c.accelerations, -1)).tolist()
                c.dt = dts[(len(path) - 1) - i]
        self.path = tuple(path)
        self.bodies = bodies
        self.ts = ts

    def __len__(self):
        return len(self.path)

    def __repr__(self):
        return 't({})'.format(len(self.path))


def create_trajectory(robot, joints, path, bodies, velocities=None, accelerations=None,
                      movables=None, dts=None, ts=None, dynam_fn=None):
    """utils.py:3340-3347.  With dynam_fn=rne (panda_primitives.py:281) the per-sample
    torques are computed in one batched engine call instead of one call per Conf."""
    from . import rne as rne_mod
    confs = []
    index = 0
    if velocities is not None:
        n = len(velocities)
        torques = None
        if dynam_fn is rne_mod.rne and n:
            torques = rne_mod.rne_batch(np.asarray(path[:n]), np.asarray(velocities[:n]),
                                        np.asarray(accelerations[:n]))
        for i in range(n):
            if torques is not None:
                confs.append(Conf(robot, joints, path[i], velocities=velocities[i],
                                  movables=bodies, accelerations=accelerations[i], dt=dts[i],
                                  torques=torques[i]))
            else:
                confs.append(Conf(robot, joints, path[i], velocities=velocities[i],
                                  movables=bodies, accelerations=accelerations[i], dt=dts[i],
                                  dynam_fn=dynam_fn))
            index += 1
    for i in range(index, len(path)):
        confs.append(Conf(robot, joints, path[i], velocities=None))
    return Trajectory(confs, bodies=bodies, ts=ts)
