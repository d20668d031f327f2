"""xArm6 kinematics + Pose3d (reference utils/xarm_sim_robot.py, utils/pose3d.py, constants.py).

Parity pin: the reference's INITIAL_JOINT_POSITIONS (constants.py:62-65) are documented as the effector pose
translation (0.3, -0.2, 0.145), rotation rotvec (0, pi, 0); our FK must reproduce that from the joints alone."""
import numpy as np
from scipy.spatial import transform

from pytorch_rt1_for_distributed_training_amd.sim import REWARDS, LanguageTable, board, kinematics as K


def test_fk_of_reference_initial_joints_matches_documented_pose():
    pose = K.forward_kinematics(K.INITIAL_JOINT_POSITIONS)
    assert np.allclose(pose.translation, [0.3, -0.2, 0.145], atol=1e-3)
    err = (pose.rotation * K.EFFECTOR_DOWN_ROTATION.inv()).magnitude()
    assert err < 0.01


def test_fk_zero_configuration():
    pose = K.forward_kinematics(np.zeros(6))           # xArm6 zero pose: flange at (207, 0, 112) mm, pointing down
    assert np.allclose(pose.translation, [0.207, 0.0, 0.112], atol=1e-3)
    assert np.allclose(pose.rotation.as_matrix()[:, 2], [0, 0, -1], atol=1e-6)


def test_jacobian_matches_finite_differences():
    q = K.INITIAL_JOINT_POSITIONS + 0.1
    J = K.jacobian(q)
    eps = 1e-6
    for i in range(6):
        dq = np.zeros(6)
        dq[i] = eps
        Tp, Tm = K._link_transforms(q + dq)[6], K._link_transforms(q - dq)[6]
        assert np.allclose((Tp[:3, 3] - Tm[:3, 3]) / (2 * eps), J[:3, i], atol=1e-5)
        w = transform.Rotation.from_matrix(Tp[:3, :3] @ Tm[:3, :3].T).as_rotvec() / (2 * eps)
        assert np.allclose(w, J[3:, i], atol=1e-5)


def test_ik_round_trip_over_the_workspace():
    rng = np.random.default_rng(0)
    q = K.INITIAL_JOINT_POSITIONS.copy()
    for _ in range(25):
        xy = rng.uniform(board.WORKSPACE_BOUNDS[0], board.WORKSPACE_BOUNDS[1])
        target = K.effector_pose(xy)
        q, ok = K.inverse_kinematics(target, q)
        assert ok
        pose = K.forward_kinematics(q)
        assert np.allclose(pose.translation, target.translation, atol=1e-4)
        assert (pose.rotation * target.rotation.inv()).magnitude() < 1e-3
        assert np.all(q >= K.JOINT_LOWER) and np.all(q <= K.JOINT_UPPER)


def test_pose3d_serialisation_and_vec7():
    p = K.Pose3d(transform.Rotation.from_rotvec([0.1, -0.2, 0.3]), np.array([0.1, 0.2, 0.3]))
    q = K.Pose3d.deserialize(p.serialize())
    assert np.allclose(q.vec7, p.vec7) and q.vec7.shape == (7,)
    assert np.allclose(K.Pose3d.from_matrix(p.matrix).vec7, p.vec7)


def test_env_arm_tracks_effector_and_restores_state():
    env = LanguageTable(reward_factory=REWARDS["block2block"], seed=3)
    env.reset()
    rng = np.random.default_rng(1)
    for _ in range(15):
        env.step(rng.uniform(-0.03, 0.03, 2))
        pose = env.robot.forward_kinematics()
        assert env.robot.last_ik_converged
        assert np.allclose(pose.translation[:2], env.world.effector_target, atol=1e-4)
        assert abs(pose.translation[2] - board.EFFECTOR_HEIGHT) < 1e-4
    s = env.get_state()
    q = env.robot.get_joint_positions()
    env.step([0.05, 0.05])
    env.set_state(s)
    assert np.allclose(env.robot.get_joint_positions(), q)
