"""xArm6 kinematics and the 6-DoF pose container -- no pybullet.

Behavioural spec: ``language_table/environments/utils/xarm_sim_robot.py:40-220`` (an xArm6 whose link 6 carries
the end effector; ``forward_kinematics`` returns link 6's world pose, ``inverse_kinematics`` solves joint targets
for a world pose, ``set_target_effector_pose`` drives the joints there) and ``utils/pose3d.py:40-67``
(``Pose3d``: rotation + translation, ``vec7``, (de)serialisation).  The env keeps the effector at
``EFFECTOR_HEIGHT`` pointing straight down (``constants.py:25-26``) and moves it in x/y only
(``language_table.py:599-616``).

The reference gets FK/IK from pybullet's URDF model.  Here the arm is the xArm6 modified-DH chain (UFACTORY's
published parameters); its link-6 frame reproduces the reference: FK of the reference's
``INITIAL_JOINT_POSITIONS`` (``constants.py:62-65``) lands on the documented start pose (0.3, -0.2, 0.145), effector
down, to 0.6 mm (``tests/test_kinematics.py``).  IK is damped least squares on the 6-D pose error with joint
limits, warm-started from the current joints, so successive targets along a push stay on one IK branch.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Optional

import numpy as np
from scipy.spatial import transform

from . import board

# modified DH (Craig): T_i = RotX(alpha_{i-1}) TransX(a_{i-1}) RotZ(theta_i + offset_i) TransZ(d_i)
DH_ALPHA = np.array([0.0, -np.pi / 2, 0.0, -np.pi / 2, np.pi / 2, -np.pi / 2])
DH_A = np.array([0.0, 0.0, 0.28948866, 0.0775, 0.0, 0.076])
DH_D = np.array([0.267, 0.0, 0.0, 0.3425, 0.0, 0.097])
DH_OFFSET = np.array([0.0, -1.3849179, 1.3849179, 0.0, 0.0, 0.0])
JOINT_LOWER = np.array([-2 * np.pi, -2.059, -3.927, -2 * np.pi, -1.69297, -2 * np.pi])
JOINT_UPPER = np.array([2 * np.pi, 2.0944, 0.19198, 2 * np.pi, np.pi, 2 * np.pi])

HOME_JOINT_POSITIONS = np.deg2rad([0, -20, -80, 0, 100, -30])
# the reference env's start configuration (constants.py:62-65): effector at (0.3, -0.2, 0.145), pointing down
INITIAL_JOINT_POSITIONS = np.array([-0.5875016909413221, 0.15985553866983415, -0.4992862770497537,
                                    0.0017427885915130214, 0.33927183830553914, -3.7249551487437524])
EFFECTOR_DOWN_ROTATION = transform.Rotation.from_rotvec([0.0, np.pi, 0.0])


@dataclasses.dataclass
class Pose3d:
    """Rotation + translation (the reference's ``Pose3d``)."""
    rotation: transform.Rotation
    translation: np.ndarray

    @property
    def vec7(self) -> np.ndarray:
        return np.concatenate([self.translation, self.rotation.as_quat()])

    @property
    def matrix(self) -> np.ndarray:
        T = np.eye(4)
        T[:3, :3] = self.rotation.as_matrix()
        T[:3, 3] = self.translation
        return T

    @staticmethod
    def from_matrix(T: np.ndarray) -> "Pose3d":
        return Pose3d(transform.Rotation.from_matrix(T[:3, :3]), np.asarray(T[:3, 3], np.float64).copy())

    def asdict(self) -> Dict:
        return {"rotation": self.rotation, "translation": self.translation}

    def serialize(self) -> Dict:
        return {"rotation": self.rotation.as_quat().tolist(), "translation": np.asarray(self.translation).tolist()}

    @staticmethod
    def deserialize(data: Dict) -> "Pose3d":
        return Pose3d(transform.Rotation.from_quat(data["rotation"]), np.array(data["translation"], np.float64))

    def __eq__(self, other) -> bool:
        return (np.array_equal(self.rotation.as_quat(), other.rotation.as_quat()) and
                np.array_equal(self.translation, other.translation))


def _link_transforms(q: np.ndarray) -> np.ndarray:
    """[7, 4, 4]: base (identity) and the world pose of links 1..6."""
    out = np.empty((7, 4, 4))
    out[0] = np.eye(4)
    ca, sa = np.cos(DH_ALPHA), np.sin(DH_ALPHA)
    th = np.asarray(q, np.float64) + DH_OFFSET
    ct, st = np.cos(th), np.sin(th)
    for i in range(6):
        Ti = np.array([[ct[i], -st[i], 0.0, DH_A[i]],
                       [st[i] * ca[i], ct[i] * ca[i], -sa[i], -sa[i] * DH_D[i]],
                       [st[i] * sa[i], ct[i] * sa[i], ca[i], ca[i] * DH_D[i]],
                       [0.0, 0.0, 0.0, 1.0]])
        out[i + 1] = out[i] @ Ti
    return out


def forward_kinematics(q: np.ndarray) -> Pose3d:
    return Pose3d.from_matrix(_link_transforms(q)[6])


def jacobian(q: np.ndarray) -> np.ndarray:
    """Geometric Jacobian [6, 6] (linear; angular) of link 6 in the world frame (all joints revolute about
    their local z)."""
    Ts = _link_transforms(q)
    p_e = Ts[6][:3, 3]
    J = np.empty((6, 6))
    for i in range(6):
        z = Ts[i + 1][:3, 2]
        p = Ts[i + 1][:3, 3]
        J[:3, i] = np.cross(z, p_e - p)
        J[3:, i] = z
    return J


def inverse_kinematics(target: Pose3d, q0: Optional[np.ndarray] = None, max_iters: int = 200,
                       tol_pos: float = 1e-5, tol_rot: float = 1e-4, damping: float = 1e-3):
    """(joints, converged): damped least squares on [position error; rotation-vector error]."""
    q = np.array(INITIAL_JOINT_POSITIONS if q0 is None else q0, np.float64)
    R_t = target.rotation.as_matrix()
    p_t = np.asarray(target.translation, np.float64)
    lam2 = damping ** 2
    for _ in range(max_iters):
        T = _link_transforms(q)[6]
        e_p = p_t - T[:3, 3]
        e_r = transform.Rotation.from_matrix(R_t @ T[:3, :3].T).as_rotvec()
        if np.linalg.norm(e_p) < tol_pos and np.linalg.norm(e_r) < tol_rot:
            return q, True
        J = jacobian(q)
        err = np.concatenate([e_p, 0.5 * e_r])
        Jw = J.copy()
        Jw[3:] *= 0.5                                  # weight rotation (rad) against position (m)
        dq = Jw.T @ np.linalg.solve(Jw @ Jw.T + lam2 * np.eye(6), err)
        m = np.abs(dq).max()
        if m > 0.2:                                    # trust region: no wrap-around jumps of the 2-pi joints
            dq *= 0.2 / m
        q = np.clip(q + dq, JOINT_LOWER, JOINT_UPPER)
    T = _link_transforms(q)[6]
    e_p = np.linalg.norm(p_t - T[:3, 3])
    e_r = np.linalg.norm(transform.Rotation.from_matrix(R_t @ T[:3, :3].T).as_rotvec())
    return q, bool(e_p < 1e-3 and e_r < 1e-2)


class XArmSimRobot:
    """Joint-space xArm6 (the reference's ``XArmSimRobot`` role): IK-driven position targets; the joints reach
    their target each control step (the reference's stiff position control does so within the 1/10 s step)."""

    def __init__(self, initial_joint_positions: np.ndarray = INITIAL_JOINT_POSITIONS):
        self.initial_joint_positions = np.array(initial_joint_positions, np.float64)
        self._q = self.initial_joint_positions.copy()
        self._q_target = self._q.copy()
        self.last_ik_converged = True

    @property
    def num_joints(self) -> int:
        return 6

    def reset_joints(self, q):
        self._q = np.array(q, np.float64)
        self._q_target = self._q.copy()

    def get_joint_positions(self) -> np.ndarray:
        return self._q.copy()

    def forward_kinematics(self) -> Pose3d:
        return forward_kinematics(self._q)

    def inverse_kinematics(self, world_effector_pose: Pose3d, max_iterations: int = 200) -> np.ndarray:
        q, ok = inverse_kinematics(world_effector_pose, self._q, max_iters=max_iterations)
        self.last_ik_converged = ok
        return q

    def set_target_joint_positions(self, q):
        self._q_target = np.clip(np.array(q, np.float64), JOINT_LOWER, JOINT_UPPER)

    def set_target_effector_pose(self, world_effector_pose: Pose3d):
        self.set_target_joint_positions(self.inverse_kinematics(world_effector_pose))

    def step(self):
        self._q = self._q_target.copy()

    def get_state(self) -> Dict[str, np.ndarray]:
        return {"q": self._q.copy(), "q_target": self._q_target.copy()}

    def set_state(self, s: Dict[str, np.ndarray]):
        self._q, self._q_target = np.array(s["q"]), np.array(s["q_target"])


def effector_pose(xy) -> Pose3d:
    """The env's effector pose for a table point: ``EFFECTOR_HEIGHT``, pointing down."""
    return Pose3d(EFFECTOR_DOWN_ROTATION, np.array([xy[0], xy[1], board.EFFECTOR_HEIGHT], np.float64))
