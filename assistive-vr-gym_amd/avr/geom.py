"""Small rigid-transform helpers (numpy, float64) shared by the model compiler and the
host-side reset path.  Conventions follow PyBullet: quaternions are (x, y, z, w) and
Euler angles are URDF/PyBullet fixed-axis roll-pitch-yaw, R = Rz(yaw) Ry(pitch) Rx(roll)
(`p.getQuaternionFromEuler`, used e.g. at feeding.py:182,185,277 of the reference).
"""
import numpy as np


def quat_from_euler(rpy):
    r, p, y = [0.5 * float(a) for a in rpy]
    cr, sr = np.cos(r), np.sin(r)
    cp, sp = np.cos(p), np.sin(p)
    cy, sy = np.cos(y), np.sin(y)
    return np.array([
        sr * cp * cy - cr * sp * sy,
        cr * sp * cy + sr * cp * sy,
        cr * cp * sy - sr * sp * cy,
        cr * cp * cy + sr * sp * sy,
    ])


def quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([
        aw * bx + ax * bw + ay * bz - az * by,
        aw * by - ax * bz + ay * bw + az * bx,
        aw * bz + ax * by - ay * bx + az * bw,
        aw * bw - ax * bx - ay * by - az * bz,
    ])


def quat_conj(q):
    return np.array([-q[0], -q[1], -q[2], q[3]])


def quat_to_mat(q):
    x, y, z, w = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def quat_axis_angle(axis, ang):
    axis = np.asarray(axis, float)
    n = np.linalg.norm(axis)
    if n < 1e-12:
        return np.array([0.0, 0.0, 0.0, 1.0])
    s = np.sin(0.5 * ang) / n
    return np.array([axis[0] * s, axis[1] * s, axis[2] * s, np.cos(0.5 * ang)])


def quat_rotate(q, v):
    return quat_to_mat(q) @ np.asarray(v, float)


def tf_mul(pa, qa, pb, qb):
    """(pa,qa) * (pb,qb) -- p.multiplyTransforms."""
    return np.asarray(pa, float) + quat_rotate(qa, pb), quat_mul(qa, qb)


def tf_inv(p, q):
    qi = quat_conj(q)
    return -quat_rotate(qi, p), qi


def quat_normalize(q):
    q = np.asarray(q, float)
    return q / np.linalg.norm(q)
