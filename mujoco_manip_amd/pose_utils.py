"""Host-side SE(3) codecs (mirror of mujoco_manip/pose_utils.py:15-209) for the façade.

The device kernels apply the same conventions: quaternions (qx, qy, qz, qw), 6D rotation =
first two rows of R, 8-DoF = [x, y, z, qx, qy, qz, qw, g], 10-DoF = [x, y, z, r11..r23, g].
"""
from __future__ import annotations

import numpy as np


def pos_rotmat_to_se3(pos, rotmat):
    T = np.eye(4)
    T[:3, :3] = rotmat
    T[:3, 3] = pos
    return T


def rotmat_to_quat_xyzw(R):
    """Branch-exact with pose_utils.py:57-82 (the quaternion sign is observable)."""
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        s = 2.0 * np.sqrt(tr + 1.0)
        return np.array([(R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s, 0.25 * s])
    if R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = 2.0 * np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2])
        return np.array([0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s, (R[2, 1] - R[1, 2]) / s])
    if R[1, 1] > R[2, 2]:
        s = 2.0 * np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2])
        return np.array([(R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s, (R[0, 2] - R[2, 0]) / s])
    s = 2.0 * np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1])
    return np.array([(R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s, (R[1, 0] - R[0, 1]) / s])


def quat_xyzw_to_rotmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def rotmat_to_6d(R):
    return R[:2, :].flatten().astype(np.float32)


def rotmat_from_6d(d6):
    a1, a2 = np.asarray(d6[:3], float), np.asarray(d6[3:6], float)
    b1 = a1 / max(np.linalg.norm(a1), 1e-12)
    b2 = a2 - np.dot(b1, a2) * b1
    b2 = b2 / max(np.linalg.norm(b2), 1e-12)
    return np.stack([b1, b2, np.cross(b1, b2)], axis=0)


def se3_to_pos_quat_g(T, gripper):
    return np.array([*T[:3, 3], *rotmat_to_quat_xyzw(T[:3, :3]), gripper], dtype=np.float32)


def se3_to_pos_rot6d_g(T, gripper):
    return np.array([*T[:3, 3], *rotmat_to_6d(T[:3, :3]), gripper], dtype=np.float32)


def se3_from_pos_quat_g(dof8):
    return pos_rotmat_to_se3(dof8[:3], quat_xyzw_to_rotmat(dof8[3:7]))


def se3_from_pos_rot6d_g(dof10):
    return pos_rotmat_to_se3(dof10[:3], rotmat_from_6d(dof10[3:9]))
