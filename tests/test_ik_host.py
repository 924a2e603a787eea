"""CPU: goal-IK pieces.

ikfast itself cannot be built here (ikfast.h:41 needs python2.7/Python.h), so the IK oracle
(oracle/tcmp_oracle_ik.c) is pinned through the reference's own forward kinematics:
fk_golden.npz holds rne.get_parent_to_child_transform(q, 0, 8) outputs (rne.py:46-63), and
every IK solution has to map back to the requested pose through that FK.  The host glue
(ik.py) is checked against a lazy restatement of the reference generator
(ikfast.py:136-169, franka_ik_fast.py:46-62) driven by the oracle solver.
"""
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN

import oracle as O

from torque_constrained_motion_planning_amd import ik as IK
from torque_constrained_motion_planning_amd import scene as SC

LO = SC.JOINT_LOWER
HI = SC.JOINT_UPPER


def _fk():
    return np.load(os.path.join(GOLDEN, "fk_golden.npz"))


def test_fk_matches_reference_dh():
    z = _fk()
    for q, T in zip(z["q"], z["T"]):
        assert np.abs(O.fk8(q) - T).max() < 1e-12


def _wrapped(a):
    return (a + np.pi) % (2 * np.pi) - np.pi


def test_ik_round_trip_and_completeness():
    z = _fk()
    found = 0
    for i, (q, T) in enumerate(zip(z["q"], z["T"])):
        sols, br = O.ik8(T, q[6])
        assert len(sols) in (0, 4, 8)
        for s in sols:
            # every solution reproduces the pose through the reference FK
            assert np.abs(O.fk8(s) - T).max() < 1e-9
            assert np.all(np.abs(s) <= np.pi + 1e-12)  # ikfast's (-pi, pi] range
            assert s[6] == q[6]
        if len(sols) and np.abs(_wrapped(sols - q)).max(1).min() < 1e-8:
            found += 1
        elif i != 0:  # row 0 is q = 0: wrist and elbow both singular
            raise AssertionError("row %d: the generating configuration is not a branch" % i)
    assert found >= len(z["q"]) - 1


def test_ik_unreachable_pose_has_no_solution():
    T = np.eye(4)
    T[:3, 3] = [2.0, 0.0, 0.5]
    sols, _ = O.ik8(T, 0.3)
    assert len(sols) == 0


def test_pose_algebra_matches_pybullet_conventions():
    e = (0.3, -0.7, 1.1)
    R = IK.matrix_from_quat(IK.quat_from_euler(e))
    assert np.abs(R - SC.rotation_rpy(*e)).max() < 1e-12
    q = IK.quat_from_matrix(R)
    assert np.abs(IK.matrix_from_quat(q) - R).max() < 1e-12
    a = IK.Pose(point=(0.1, 0.2, 0.3), euler=e)
    b = IK.Pose(point=(-0.4, 0.0, 0.9), euler=(1.0, 0.2, -0.5))
    ab = IK.to_matrix(IK.multiply(a, b))
    assert np.abs(ab - IK.to_matrix(a) @ IK.to_matrix(b)).max() < 1e-12
    assert np.abs(IK.to_matrix(IK.multiply(a, IK.invert(a))) - np.eye(4)).max() < 1e-12


def test_top_grasp_of_the_coke_payload():
    body = SC.Payload.coke(5.0)
    center, ext = IK.approximate_as_prism(body)
    assert np.allclose(center, [0, 0, 0.023]) and np.allclose(ext, [0.03, 0.03, 0.05])
    grasps = IK.get_top_grasps(body)
    assert len(grasps) == 2  # w and l both below MAX_GRASP_WIDTH
    G = IK.to_matrix(grasps[0])
    # tool_pose * translate_z * rotate_z(pi/2) * reflect_z * translate_center
    expect = (IK.to_matrix(IK.TOOL_POSE) @ IK.to_matrix(IK.Pose(point=[0, 0, 0.05 - 0.15]))
              @ IK.to_matrix(IK.Pose(euler=[0, 0, np.pi / 2]))
              @ IK.to_matrix(IK.Pose(euler=[0, np.pi, 0]))
              @ IK.to_matrix(IK.Pose(point=[0, 0, -0.023])))
    assert np.abs(G - expect).max() < 1e-12
    # gripper z axis points down onto the object
    assert np.allclose(G[:3, 2], [0, 0, -1])


def test_base_from_ee_inverts_the_tool_offset():
    z = _fk()
    for q, T in zip(z["q"][:20], z["T"][:20]):
        world_from_tool = T @ IK.EE_TO_TOOL
        assert np.abs(IK.get_base_from_ee(world_from_tool) - T).max() < 1e-12


class OracleEngine:
    """Engine.ik stand-in on CPU (test only): the oracle solver in branch order."""

    def ik(self, poses, free):
        poses = np.asarray(poses).reshape(-1, 4, 4)
        sols = np.zeros((len(poses), 8, 7))
        cnt = np.zeros(len(poses), dtype=np.int32)
        for i, (T, f) in enumerate(zip(poses, free)):
            s, _ = O.ik8(T, f)
            sols[i, :len(s)] = s
            cnt[i] = len(s)
        return sols, cnt


def _reference_generator(world_from_tool, current, max_attempts=25):
    """ikfast_inverse_kinematics + sample_tool_ik restated lazily (ikfast.py:136-169,
    franka_ik_fast.py:46-62, utils.py:2941-2983/3662) with the oracle as get_ik."""
    base_from_ee = IK.get_base_from_ee(world_from_tool)

    def frees():
        yield current[6]
        while True:
            w = np.random.uniform(size=1)
            yield ((1 - w) * LO[6] + w * HI[6])[0]

    def gen():
        for k, f in enumerate(frees()):
            if k >= max_attempts:
                return
            s, _ = O.ik8(base_from_ee, f)
            cands = [r.copy() for r in s]
            random.shuffle(cands)
            for c in cands:
                if not (np.any(c < LO) or np.any(HI < c)):
                    yield c

    g = gen()
    for _ in range(max_attempts):
        try:
            return next(g)
        except StopIteration:
            break
    return None


@pytest.mark.parametrize("seed", range(6))
def test_sample_tool_ik_replays_reference_generator(seed):
    z = _fk()
    rs = np.random.RandomState(seed)
    q = z["q"][10 + seed]
    world_from_tool = z["T"][10 + seed] @ IK.EE_TO_TOOL
    current = np.clip(q + rs.normal(0, 0.3, 7), LO, HI)
    np.random.seed(100 + seed)
    random.seed(200 + seed)
    ref = _reference_generator(world_from_tool, current)
    after_np, after_py = np.random.uniform(), random.random()
    np.random.seed(100 + seed)
    random.seed(200 + seed)
    got = IK.sample_tool_ik(OracleEngine(), world_from_tool, current)
    assert (ref is None) == (got is None)
    if ref is not None:
        assert np.array_equal(ref, got)
    # both RNG streams are left exactly where the lazy reference leaves them
    assert np.random.uniform() == after_np and random.random() == after_py


def test_unreachable_target_consumes_all_draws():
    T = np.eye(4)
    T[:3, 3] = [3.0, 0.0, 0.0]
    np.random.seed(5)
    assert IK.sample_tool_ik(OracleEngine(), T, np.zeros(7)) is None
    x = np.random.uniform()
    np.random.seed(5)
    np.random.uniform(size=24)
    assert np.random.uniform() == x
