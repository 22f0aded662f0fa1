"""Pose math of the fusion host.

Restates, in NumPy float64:
  * `parse_extrinsic`  — src/SfM_CUDA/utils.cu:8-24 (quaternion -> Rodrigues -> C2W, f32, inverted)
  * `parse_pos`        — src/TSDF_Python/tsdf_utils.py:64-77 (same, float64)
  * `transform44`      — src/TSDF_Python/tsdf_utils.py:32-61 (TUM reference formula, inverted)
  * `slerp`            — src/TSDF_Python/tsdf_utils.py:80-100
  * `relative_pose`    — E = W2C_k * (W2C_0)^-1 (tsdf.cu:217, tsdf.py:63-64)
TUM trajectory lines are `ts tx ty tz qx qy qz qw` with the camera-to-world pose.
"""
from __future__ import annotations

import math

import numpy as np


def rodrigues(rvec) -> np.ndarray:
    """Rotation matrix of an axis-angle vector (cv::Rodrigues semantics)."""
    r = np.asarray(rvec, dtype=np.float64).reshape(3)
    theta = float(np.linalg.norm(r))
    if theta < 1e-300:
        return np.eye(3)
    k = r / theta
    c, s = math.cos(theta), math.sin(theta)
    kx = np.array([[0.0, -k[2], k[1]], [k[2], 0.0, -k[0]], [-k[1], k[0], 0.0]])
    return c * np.eye(3) + (1.0 - c) * np.outer(k, k) + s * kx


def _c2w_from_pos(pos) -> np.ndarray:
    pos = np.asarray(pos, dtype=np.float64).reshape(7)
    axis = pos[3:6]
    n = float(np.linalg.norm(axis))
    theta = 2.0 * math.atan2(n, pos[6])
    rot = rodrigues(theta * (axis / n)) if n > 0 else np.eye(3)  # normalised first (tsdf_utils.py:68-70)
    m = np.eye(4)
    m[:3, :3] = rot
    m[:3, 3] = pos[:3]
    return m


def parse_pos(pos) -> np.ndarray:
    """tsdf_utils.py:64-77: [tx ty tz qx qy qz qw] -> W2C (float64 4x4)."""
    return np.linalg.inv(_c2w_from_pos(pos))


def parse_extrinsic(pos) -> np.ndarray:
    """utils.cu:8-24: as parse_pos, but the C2W matrix is rounded to float32 before the
    inversion and the result is float32 (the inverse is taken in float64 of the f32
    matrix and rounded once)."""
    c2w = _c2w_from_pos(pos).astype(np.float32)
    return np.linalg.inv(c2w.astype(np.float64)).astype(np.float32)


def transform44(l) -> np.ndarray:
    """tsdf_utils.py:32-61 (TUM benchmark formula), returning the inverse (W2C) -- except
    for a near-zero quaternion, where the reference returns the translation matrix itself,
    un-inverted (tsdf_utils.py:46-52), and so does this."""
    l = np.asarray(l, dtype=np.float64)
    t = l[:3]
    q = np.array(l[3:7], dtype=np.float64, copy=True)
    nq = float(np.dot(q, q))
    if nq < 1e-7:
        m = np.eye(4)
        m[:3, 3] = t
        return m
    q *= math.sqrt(2.0 / nq)
    q = np.outer(q, q)
    m = np.array(
        (
            (1.0 - q[1, 1] - q[2, 2], q[0, 1] - q[2, 3], q[0, 2] + q[1, 3], t[0]),
            (q[0, 1] + q[2, 3], 1.0 - q[0, 0] - q[2, 2], q[1, 2] - q[0, 3], t[1]),
            (q[0, 2] - q[1, 3], q[1, 2] + q[0, 3], 1.0 - q[0, 0] - q[1, 1], t[2]),
            (0.0, 0.0, 0.0, 1.0),
        ),
        dtype=np.float64,
    )
    return np.linalg.inv(m)


def slerp(q1, q2, t: float) -> np.ndarray:
    """tsdf_utils.py:80-100 (linear fallback above dot 0.9995, shortest arc)."""
    q1 = np.asarray(q1, dtype=np.float64)
    q2 = np.asarray(q2, dtype=np.float64)
    q1 = q1 / np.linalg.norm(q1)
    q2 = q2 / np.linalg.norm(q2)
    dot = float(np.dot(q1, q2))
    if dot < 0:
        q1 = -q1
        dot = -dot
    if dot > 0.9995:
        return q1 + t * (q2 - q1)
    dot = max(min(dot, 1.0), -1.0)
    theta_0 = math.acos(dot)
    theta = theta_0 * t
    s1 = math.cos(theta) - dot * math.sin(theta) / math.sin(theta_0)
    s2 = math.sin(theta) / math.sin(theta_0)
    return s1 * q1 + s2 * q2


def interpolate_pose(traj: np.ndarray, ts: float) -> np.ndarray:
    """TSDF_Python/main.py:127-140: lerp translation + slerp rotation between the bracketing
    trajectory rows (first row with time >= ts and its predecessor).  As in the reference,
    a first row at or after ts pairs with row -1 (Python's last row), which passes the
    main.py:134 assertion only when ts equals the first time stamp."""
    for k in range(traj.shape[0]):
        if traj[k, 0] < ts:
            continue
        t = (ts - traj[k - 1, 0]) / (traj[k, 0] - traj[k - 1, 0])
        assert 0 <= t <= 1  # main.py:134
        return np.concatenate(
            [(traj[k, 1:4] - traj[k - 1, 1:4]) * t + traj[k - 1, 1:4], slerp(traj[k - 1, -4:], traj[k, -4:], t)]
        )
    raise ValueError(f"timestamp {ts} is after the trajectory")


def relative_pose(extrinsic, init_extrinsic_inv) -> np.ndarray:
    """E = extrinsic * init_extrinsic_inv (tsdf.cu:217 / tsdf.py:63-64), rounded to f32."""
    return (np.asarray(extrinsic, np.float64) @ np.asarray(init_extrinsic_inv, np.float64)).astype(np.float32)


def c2w_to_tum(ts: float, c2w: np.ndarray) -> str:
    """Format a camera-to-world pose as one TUM groundtruth line."""
    R = np.asarray(c2w, np.float64)[:3, :3]
    t = np.asarray(c2w, np.float64)[:3, 3]
    # rotation matrix -> quaternion (x, y, z, w)
    tr = np.trace(R)
    if tr > 0:
        s = math.sqrt(tr + 1.0) * 2
        qw, qx, qy, qz = 0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        qw, qx, qy, qz = (R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        qw, qx, qy, qz = (R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        qw, qx, qy, qz = (R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s
    return f"{ts:.4f} {t[0]:.9f} {t[1]:.9f} {t[2]:.9f} {qx:.9f} {qy:.9f} {qz:.9f} {qw:.9f}"
