"""Goal IK for planner_fn_force_aware.

The reference turns an object pose into the RRT* goal configuration with
  panda_primitives.py:240-265  top grasp, gripper pose, 25 x bi_panda_inverse_kinematics
  franka_ik_fast.py:46-79      sample_tool_ik / bi_panda_inverse_kinematics
  ikfast.py:67-71, 136-169     frame change to panda_link8, free-joint stream, limit filter
  ikfast_panda_arm.cpp:12839   the analytic solver (get_ik)
The solver runs on the GPU (libtcmp.so tcmp_ik, csrc/tcmp_ik.h): ONE launch solves every
free-joint draw of a sample_tool_ik call (the current joint 7, then up to 24 uniform draws),
and the host replays the reference's generator over the results.  The pose algebra here is
pybullet's (position + quaternion xyzw, getQuaternionFromEuler = Rz(yaw) Ry(pitch) Rx(roll),
multiplyTransforms / invertTransform), done in numpy.

Consumption of np.random matches the reference (one uniform per free draw actually reached:
the state is restored and replayed after the batched solve).  The order ikfast lists
solutions in is not reproduced; the reference shuffles it (randomize, ikfast.py:163) so the
chosen solution is random in both.
"""
import random
from collections import namedtuple

import numpy as np

from .scene import JOINT_LOWER, JOINT_UPPER

# ---- pybullet pose algebra ------------------------------------------------------------------


def quat_from_euler(euler):
    """p.getQuaternionFromEuler (roll, pitch, yaw) -> xyzw."""
    r, p, y = [0.5 * float(v) for v in euler]
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    return np.array([sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
                     cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy])


def matrix_from_quat(q):
    x, y, z, w = [float(v) for v in q]
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def quat_from_matrix(R):
    R = np.asarray(R, dtype=np.float64)
    t = np.trace(R)
    if t > 0:
        s = 2.0 * np.sqrt(t + 1.0)
        q = [(R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s, 0.25 * s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = 2.0 * np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2])
        q = [0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s, (R[2, 1] - R[1, 2]) / s]
    elif R[1, 1] > R[2, 2]:
        s = 2.0 * np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2])
        q = [(R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s, (R[0, 2] - R[2, 0]) / s]
    else:
        s = 2.0 * np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1])
        q = [(R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s, (R[1, 0] - R[0, 1]) / s]
    return np.array(q)


def Pose(point=None, euler=None):
    """utils.py:245-248."""
    point = np.zeros(3) if point is None else np.asarray(point, dtype=np.float64)
    euler = np.zeros(3) if euler is None else euler
    return point, quat_from_euler(euler)


def unit_pose():
    return np.zeros(3), np.array([0.0, 0.0, 0.0, 1.0])


def to_matrix(pose):
    """(point, quat) or 4x4 -> 4x4."""
    if isinstance(pose, np.ndarray) and pose.shape == (4, 4):
        return pose.astype(np.float64)
    point, quat = pose
    T = np.eye(4)
    T[:3, :3] = matrix_from_quat(quat)
    T[:3, 3] = np.asarray(point, dtype=np.float64)
    return T


def from_matrix(T):
    return np.array(T[:3, 3]), quat_from_matrix(T[:3, :3])


def multiply(*poses):
    """utils.py:113-117 (p.multiplyTransforms chain)."""
    T = to_matrix(poses[0])
    for nxt in poses[1:]:
        T = T @ to_matrix(nxt)
    return from_matrix(T)


def invert(pose):
    """utils.py:109-111 (p.invertTransform)."""
    T = to_matrix(pose)
    Ti = np.eye(4)
    Ti[:3, :3] = T[:3, :3].T
    Ti[:3, 3] = -T[:3, :3].T @ T[:3, 3]
    return from_matrix(Ti)


def point_from_pose(pose):
    return np.asarray(pose[0], dtype=np.float64)


# ---- robot frames (panda_mod.urdf) ------------------------------------------------------------
# panda_hand_joint rpy (0 0 -0.785398163397) (:7-11) then panda_grasptarget_hand xyz 0.105
# (:87-91): world_from_target = world_from_link8 * EE_TO_TOOL.
_HAND_YAW = -0.785398163397
EE_TO_TOOL = np.eye(4)
EE_TO_TOOL[:3, :3] = np.array([[np.cos(_HAND_YAW), -np.sin(_HAND_YAW), 0.0],
                               [np.sin(_HAND_YAW), np.cos(_HAND_YAW), 0.0], [0.0, 0.0, 1.0]])
EE_TO_TOOL[:3, 3] = EE_TO_TOOL[:3, :3] @ np.array([0.0, 0.0, 0.105])
TOOL_FROM_EE = np.linalg.inv(EE_TO_TOOL)  # get_relative_pose(ee_link, tool_link), ikfast.py:69

TOOL_POSE = Pose(point=(0.0, 0.0, 0.1))   # utils.py:250
MAX_GRASP_WIDTH = 0.07                    # panda_primitives.py:194
GRASP_LENGTH = 0.15                       # panda_primitives.py:195
TOP_HOLDING_LEFT_ARM = [0, -np.pi / 4, 0.0, -6 * np.pi / 8, 0, np.pi / 2, np.pi / 4]  # utils.py:45

Grasp = namedtuple("Grasp", ["grasp_type", "body", "value", "approach", "carry"])


def approximate_as_prism(body, body_pose=None):
    """utils.py:2762-2766 for a Payload record: AABB centre and extents (w, l, h)."""
    T = to_matrix(unit_pose() if body_pose is None else body_pose)
    half = 0.5 * body.size
    corners = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])
    pts = (corners * half + body.center) @ T[:3, :3].T + T[:3, 3]
    lo, hi = pts.min(0), pts.max(0)
    return (lo + hi) / 2.0, hi - lo


def get_top_grasps(body, under=False, tool_pose=TOOL_POSE, body_pose=None,
                   max_width=MAX_GRASP_WIDTH, grasp_length=GRASP_LENGTH):
    """panda_primitives.py:197-215."""
    body_pose = unit_pose() if body_pose is None else body_pose
    center, (w, l, h) = approximate_as_prism(body, body_pose=body_pose)
    reflect_z = Pose(euler=[0, np.pi, 0])
    translate_z = Pose(point=[0, 0, h - grasp_length])
    translate_center = Pose(point=point_from_pose(body_pose) - center)
    grasps = []
    if w <= max_width:
        for i in range(1 + under):
            rotate_z = Pose(euler=[0, 0, np.pi / 2 + i * np.pi])
            grasps += [multiply(tool_pose, translate_z, rotate_z, reflect_z, translate_center,
                                body_pose)]
    if l <= max_width:
        for i in range(1 + under):
            rotate_z = Pose(euler=[0, 0, i * np.pi])
            grasps += [multiply(tool_pose, translate_z, rotate_z, reflect_z, translate_center,
                                body_pose)]
    return grasps


def get_top_grasp(body):
    """panda_primitives.py:217-221."""
    approach_vector = np.array([1.0, 0.0, 0.0])
    grasp = get_top_grasps(body)[0]
    return Grasp("top", body, grasp, multiply((approach_vector, np.array([0, 0, 0, 1.0])), grasp),
                 TOP_HOLDING_LEFT_ARM)


# ---- ikfast_inverse_kinematics / sample_tool_ik / bi_panda_inverse_kinematics ------------------


def get_base_from_ee(world_from_target, world_from_base=None):
    """ikfast.py:67-71: base_from_ee = inv(world_from_base) world_from_target tool_from_ee."""
    Wb = np.eye(4) if world_from_base is None else to_matrix(world_from_base)
    return np.linalg.inv(Wb) @ to_matrix(world_from_target) @ TOOL_FROM_EE


def _violates_limits(q):
    """utils.py:1574-1581."""
    return bool(np.any(q < JOINT_LOWER) or np.any(JOINT_UPPER < q))


def ik_candidates(engine, world_from_target, current_conf, max_attempts=25, rng=None,
                  shuffle=None):
    """ikfast_inverse_kinematics (ikfast.py:136-169) as a list: one GPU launch for every
    free value, then the reference's generator replayed in order.  Yields nothing to the
    RNGs beyond what the lazy reference generator would have drawn."""
    rng = np.random if rng is None else rng
    shuffle = random.shuffle if shuffle is None else shuffle
    base_from_ee = get_base_from_ee(world_from_target)
    lo7, hi7 = JOINT_LOWER[6], JOINT_UPPER[6]
    current = np.asarray(current_conf, dtype=np.float64)
    # free stream: current joint 7, then interval_generator draws (utils.py:2941-2983)
    state = rng.get_state() if hasattr(rng, "get_state") else None
    draws = [rng.uniform(size=1)[0] for _ in range(max_attempts - 1)]
    free = np.array([current[6]] + [(1 - w) * lo7 + w * hi7 for w in draws])
    sols, cnt = engine.ik(np.repeat(base_from_ee[None], len(free), axis=0), free)
    out = []
    used = len(free)
    for k in range(len(free)):
        cands = [sols[k, i].copy() for i in range(cnt[k])]
        shuffle(cands)  # randomize (ikfast.py:163, utils.py:3662)
        hits = [c for c in cands if not _violates_limits(c)]
        if hits:
            out.append(hits)
            used = k + 1
            break
    if state is not None:
        rng.set_state(state)
        for _ in range(max(0, used - 1)):
            rng.uniform(size=1)
    return out[0] if out else []


def sample_tool_ik(engine, tool_pose, current_conf, max_attempts=25, rng=None, shuffle=None):
    """franka_ik_fast.py:46-62: the first limit-valid solution of the free-joint stream."""
    hits = ik_candidates(engine, tool_pose, current_conf, max_attempts=max_attempts, rng=rng,
                         shuffle=shuffle)
    return None if not hits else hits[0]


def body_collision(engine, conf):
    """any(pairwise_collision(robot, b) for b in obstacles) with the robot at `conf`
    (franka_ik_fast.py:78, panda_primitives.py:260): body_collision -> get_closest_points at
    the default max_distance = -MAX_DISTANCE (utils.py:2781,2833,2866-2880) over EVERY link of
    the robot -- the moving links and the static base panda_link0 -- with no joint-limit test.
    The scene is the one last given to `engine.set_scene`."""
    hit = bool(engine.collides_body([conf])[0])
    if hit:
        print('body collision')  # utils.py:2877-2878
    return hit


def bi_panda_inverse_kinematics(engine, gripper_pose, current_conf, collision_fn=None,
                                max_attempts=25, rng=None, shuffle=None):
    """franka_ik_fast.py:64-79.  Returns (conf or None, robot conf afterwards): the reference
    sets the joints to the IK solution before the collision check (:73), so a rejected
    solution becomes the next attempt's current configuration.  collision_fn defaults to the
    reference's body-level check (:78, `body_collision` above)."""
    if collision_fn is None:
        collision_fn = lambda q: body_collision(engine, q)  # noqa: E731
    conf = sample_tool_ik(engine, gripper_pose, current_conf, max_attempts=max_attempts, rng=rng,
                          shuffle=shuffle)
    if conf is None:
        return None, current_conf
    if collision_fn(conf):
        return None, conf
    return conf, conf


def grasp_conf_for_pose(problem, start_conf, pose, engine=None, rng=None, shuffle=None,
                        retries=25):
    """panda_primitives.py:240-258: top grasp of problem.payload at `pose` (world_from_object,
    (point, quat) or 4x4), gripper pose, up to 25 IK attempts with the body collision check."""
    from ._lib import engine as get_engine
    from .scene import mesh_pack, obstacle_array

    eng = get_engine() if engine is None else engine
    eng.set_scene(obstacle_array(problem.fixed), mesh_pack(problem.fixed))
    grasp = get_top_grasp(problem.payload)
    gripper_pose = multiply(from_matrix(to_matrix(pose)), invert(grasp.value))
    collision_fn = lambda q: body_collision(eng, q)  # noqa: E731  (franka_ik_fast.py:78)
    current = np.asarray(start_conf, dtype=np.float64)
    for _ in range(retries):
        conf, current = bi_panda_inverse_kinematics(eng, gripper_pose, current, collision_fn,
                                                    rng=rng, shuffle=shuffle)
        if conf is not None:
            return tuple(float(v) for v in conf)
    return None
