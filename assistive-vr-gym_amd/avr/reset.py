"""Host-side reset path for FeedingJaco-v0 (FeedingEnv.reset, feeding.py:144-331).

It produces the initial per-env state block that the device step consumes:
  * human pose: setup_human_joints + enforce_joint_limits (world_creation.py:135-179,110-133)
    with the Feeding joint targets (feeding.py:242-245) -> per-env world poses of the human's
    collision links (the human is fully static unless the impairment is 'tremor', whose head/neck
    chain, joints 24..27, is simulated on the device: _tremor_state);
  * bowl position jitter (feeding.py:184), IK of the Jaco tool link to the spoon-above-bowl
    target (feeding.py:276-278; util.py:34-105 -- restated as damped least squares with random
    restarts, because p.calculateInverseKinematics is a Bullet internal);
  * gripper (feeding.py:279, world_creation.py:309-328), spoon on the tool frame
    (world_creation.py:330-365), 8 food spheres above the spoon (feeding.py:291-308).
The 100 settling stepSimulation calls (feeding.py:319-320) run on the device (avr_settle).

Per-env randomness: numpy Generator seeded with (seed, env_id), so resets do not depend on
how envs are sharded over GPUs.  (The reference draws from one np_random stream per env
object; those draws cannot be reproduced bit-for-bit and are not part of the step path.)
"""
import numpy as np

from . import _abi as ABI
from . import geom as G

HUMAN_SCALED = set(range(7, 14)) | set(range(17, 24)) | set(range(24, 28))   # limit_scale joints
HEAD_CHAIN = (24, 25, 26, 27)          # controllable joints under 'tremor' (feeding.py:219)


# ----------------------------------------------------------------------------- Jaco FK / IK
def robot_fk(A, q):
    """Link frames and COM frames of the robot for DoF vector q (same recursion as the kernel)."""
    nl = int(A['n_links'])
    base_p, base_q = A['robot_base'][:3], A['robot_base'][3:]
    LP = np.zeros((nl, 3)); LQ = np.zeros((nl, 4))
    CP = np.zeros((nl, 3)); CQ = np.zeros((nl, 4))
    AX = np.zeros((nl, 3)); OR = np.zeros((nl, 3))
    for i in range(nl):
        p = A['rl_parent'][i]
        pp, pq = (base_p, base_q) if p < 0 else (LP[p], LQ[p])
        tp, tq = G.tf_mul(pp, pq, A['rl_jpos'][i], A['rl_jquat'][i])
        OR[i] = tp
        AX[i] = G.quat_rotate(tq, A['rl_axis'][i])
        dof = A['rl_dof'][i]
        if A['rl_jtype'][i] == 1:
            tq = G.quat_mul(tq, G.quat_axis_angle(A['rl_axis'][i], q[dof]))
        elif A['rl_jtype'][i] == 2:
            tp = tp + AX[i] * q[dof]
        LP[i], LQ[i] = tp, tq
        CP[i], CQ[i] = G.tf_mul(tp, tq, A['rl_com_pos'][i], A['rl_com_quat'][i])
    return LP, LQ, CP, CQ, AX, OR


def _chain(A, link):
    out = []
    k = link
    while k >= 0:
        out.append(k)
        k = A['rl_parent'][k]
    return out


def _rot_err(q_tgt, q_cur):
    dq = G.quat_mul(q_tgt, G.quat_conj(q_cur))
    if dq[3] < 0:
        dq = -dq
    s = np.linalg.norm(dq[:3])
    if s < 1e-12:
        return np.zeros(3)
    ang = 2.0 * np.arctan2(s, dq[3])
    return dq[:3] / s * ang


def table_clear(A, q, margin=0.05):
    """True if no robot hull vertex lies inside the (inflated) table box.  Stands in for the
    reference's collision screening of IK restarts (util.py:41-46) so that reset states do not
    start with the arm buried in the table."""
    _, _, CP, CQ, _, _ = robot_fk(A, q)
    tb = int(A['task_table_body'])
    s0 = A['body_shape_start'][tb]
    tpose = A['st_pose'][A['body_index'][tb]]
    sp = A['shape_pose'][s0]
    c = tpose[:3] + sp[:3]
    he = A['shape_param'][s0][:3] + margin
    for b in range(len(A['body_kind'])):
        if A['body_kind'][b] != 0:
            continue
        l = A['body_index'][b]
        for s in range(A['body_shape_start'][b], A['body_shape_start'][b] + A['body_shape_count'][b]):
            if A['shape_kind'][s] != 3:
                continue
            v0, nv = A['shape_hull'][s][:2]
            V = A['hull_verts'][v0:v0 + nv]
            p, qq = G.tf_mul(CP[l], CQ[l], A['shape_pose'][s][:3], A['shape_pose'][s][3:])
            W = V @ G.quat_to_mat(qq).T + p
            inside = np.all(np.abs(W - c) <= he, axis=1)   # box inflated by `margin` on all sides
            if inside.any():
                return False
    return True


def ik(A, link, target_pos, target_quat, arm_dofs, lower, upper, rng, q0=None,
       iters=300, restarts=40, tol=0.01):
    """Damped-least-squares IK for the COM frame of `link` (util.py:34-57 semantics: random
    rest pose per restart, accept at < tol position and quaternion error)."""
    nd = int(A['n_dof'])
    best, best_err = None, np.inf
    chain = _chain(A, link)
    for r in range(restarts):
        q = np.zeros(nd) if q0 is None else q0.copy()
        q[arm_dofs] = rng.uniform(lower, upper)
        for it in range(iters):
            _, _, CP, CQ, AX, OR = robot_fk(A, q)
            ep = target_pos - CP[link]
            er = _rot_err(target_quat, CQ[link])
            err = np.concatenate([ep, er])
            if np.linalg.norm(ep) < 1e-5 and np.linalg.norm(er) < 1e-4:
                break
            J = np.zeros((6, len(arm_dofs)))
            for c, dof in enumerate(arm_dofs):
                l = [k for k in chain if A['rl_dof'][k] == dof]
                if not l:
                    continue
                l = l[0]
                J[:3, c] = np.cross(AX[l], CP[link] - OR[l])
                J[3:, c] = AX[l]
            lam = 1e-2
            dq = J.T @ np.linalg.solve(J @ J.T + lam * lam * np.eye(6), err)
            q[arm_dofs] = np.clip(q[arm_dofs] + dq, lower, upper)
        _, _, CP, CQ, _, _ = robot_fk(A, q)
        pe = np.linalg.norm(target_pos - CP[link])
        qe = min(np.linalg.norm(target_quat - CQ[link]), np.linalg.norm(target_quat + CQ[link]))
        if pe < tol and qe < tol and table_clear(A, q):
            return q, True
        if pe < best_err:
            best, best_err = q.copy(), pe
    return best, False


# ----------------------------------------------------------------------------- human
_HJ = {}


def _human_limits(A, gender):
    """Per-gender joint-limit tables of human_joint_angles (cached): lower, upper, the
    limit_scale joint mask and the mask of clamped joints (revolute with a limit)."""
    if gender not in _HJ:
        lo = A['human_%s_lower' % gender].astype(float)
        hi = A['human_%s_upper' % gender].astype(float)
        n = len(lo)
        scaled = np.zeros(n, bool)
        scaled[[j for j in HUMAN_SCALED if j < n]] = True
        clamp = (A['human_%s_jtype' % gender] == 1)
        _HJ[gender] = (lo, hi, scaled, clamp)
    return _HJ[gender]


def human_joint_angles(A, gender, rng, limit_scale=1.0):
    """Feeding (non-VR, non-new) human joint setup: fixed arm/leg poses + random head
    (feeding.py:242-245), clamped by enforce_joint_limits (world_creation.py:110-133)."""
    lo0, hi0, scaled, clamp = _human_limits(A, gender)
    q = np.zeros(len(lo0))
    for j, ang in [(10, -90), (20, -90), (28, -90), (31, 80), (35, -90), (38, 80)]:
        q[j] = np.deg2rad(ang)
    for j in (25, 26, 27):
        q[j] = rng.uniform(np.deg2rad(-30), np.deg2rad(30))
    lo = np.where(scaled, lo0 * limit_scale, lo0)
    hi = np.where(scaled, hi0 * limit_scale, hi0)
    c = clamp & ~((lo == 0) & (hi == -1))
    q[c] = np.minimum(np.maximum(q[c], lo[c]), hi[c])
    return q


def human_link_poses(A, gender, q):
    """World poses (link == COM frames) of the 42 human links; base pose from feeding.py:245."""
    base_p = np.array([0, 0.03, 0.89 - 0.23725 if gender == 'male' else 0.86 - 0.225])
    base_q = np.array([0, 0, 0, 1.0])
    par = A['human_%s_parent' % gender]
    jt = A['human_%s_jtype' % gender]
    ax = A['human_%s_axis' % gender]
    pos = A['human_%s_pos' % gender]
    n = len(par)
    P = np.zeros((n, 3)); Q = np.zeros((n, 4))
    for i in range(n):
        pp, pq = (base_p, base_q) if par[i] < 0 else (P[par[i]], Q[par[i]])
        p, qq = G.tf_mul(pp, pq, pos[i], [0, 0, 0, 1])
        if jt[i] == 1:
            qq = G.quat_mul(qq, G.quat_axis_angle(ax[i], q[i]))
        P[i], Q[i] = p, qq
    return base_p, base_q, P, Q


def human_slot_poses(A, gender, q):
    base_p, base_q, P, Q = human_link_poses(A, gender, q)
    out = np.zeros((ABI.MAX_HUMAN, 7))
    for s, l in enumerate(A['human_slot_link']):
        if l < 0:
            out[s] = np.concatenate([base_p, base_q])
        else:
            out[s] = np.concatenate([P[l], Q[l]])
    return out


# ----------------------------------------------------------------------------- full reset
def feeding_reset_state(A, md, seed, env_id, gender=None, impairment='none'):
    """One env's initial state block (float64[STATE_WORDS]) before the settle frames."""
    rng = _rng(seed, env_id)
    if gender is None:
        gender = 'male' if rng.integers(2) == 0 else 'female'     # feeding.py:169
    impairment = _impairment(rng, impairment)
    limit_scale = rng.uniform(0.5, 1.0) if impairment == 'limits' else 1.0   # world_creation.py:71
    st = np.zeros(ABI.STATE_WORDS)
    qh = human_joint_angles(A, gender, rng, limit_scale)
    st[ABI.S_HUMAN:ABI.S_HUMAN + ABI.MAX_HUMAN * 7] = human_slot_poses(A, gender, qh).ravel()
    if impairment == 'tremor':
        _tremor_state(st, md, qh, rng)
    bowl_pos = np.array([-0.15, -0.55, 0.75]) + np.array([rng.uniform(-0.05, 0.05), rng.uniform(-0.05, 0.05), 0])
    target_pos = bowl_pos + np.array([0, -0.1, 0.4]) + rng.uniform(-0.05, 0.05, size=3)
    target_quat = G.quat_from_euler([np.pi / 2.0, 0, np.pi / 2.0])
    arm = md.arm_dofs
    lower = np.array([md.desc.arm_lower[i] if md.desc.arm_lower[i] > -1e9 else -2 * np.pi for i in range(len(arm))])
    upper = np.array([md.desc.arm_upper[i] if md.desc.arm_upper[i] < 1e9 else 2 * np.pi for i in range(len(arm))])
    tool = int(A['task_tool_link'])
    q0 = np.zeros(int(A['n_dof']))
    for d in md.finger_dofs:
        q0[d] = md.params['finger_target']
    q, ok = ik(A, tool, target_pos, target_quat, arm, lower, upper, rng, q0=q0)
    st[ABI.S_Q:ABI.S_Q + len(q)] = q
    # motors: arm keeps PyBullet's default velocity motors until the first take_step;
    # gripper position motors (world_creation.py:328)
    for d in arm:
        st[ABI.S_KP + d] = 0.0
        st[ABI.S_QTGT + d] = 0.0
        st[ABI.S_MAXIMP + d] = md.params['default_motor_impulse']
    for d in md.finger_dofs:
        st[ABI.S_KP + d] = md.params['finger_gain']
        st[ABI.S_QTGT + d] = md.params['finger_target']
        st[ABI.S_MAXIMP + d] = md.params['finger_force'] * md.params['time_step']
    # spoon at tool frame (x) offset (world_creation.py:332-343)
    _, _, CP, CQ, _, _ = robot_fk(A, q)
    off = A['task_tool_offset']
    sp, sq = G.tf_mul(CP[tool], CQ[tool], off[:3], off[3:])
    fb = ABI.S_FREE
    st[fb:fb + 3] = sp
    st[fb + 3:fb + 7] = sq
    bq = G.quat_from_euler([np.pi / 2.0, 0, 0])
    b = ABI.S_FREE + ABI.FB_WORDS
    st[b:b + 3] = bowl_pos
    st[b + 3:b + 7] = bq
    r = 0.005
    k = 0
    for i in range(2):
        for j in range(2):
            for kk in range(2):
                f = ABI.S_FREE + ABI.FB_WORDS * (2 + k)
                st[f:f + 3] = np.array([i * 2 * r - 0.005, j * 2 * r, kk * 2 * r + 0.02]) + sp
                st[f + 3:f + 7] = [0, 0, 0, 1]
                k += 1
    t = ABI.S_TASK
    gi = 0 if gender == 'male' else 1
    head = st[ABI.S_HUMAN + 7 * int(A['task_head_slot']):][:7]
    mouth = A['task_mouth_male'] if gi == 0 else A['task_mouth_female']
    st[t + ABI.T_TARGET:t + ABI.T_TARGET + 3] = G.tf_mul(head[:3], head[3:], mouth, [0, 0, 0, 1])[0]
    st[t + ABI.T_ALIVE] = (1 << 8) - 1
    st[t + ABI.T_GENDER] = gi
    return st, dict(gender=gender, impairment=impairment, ik_ok=ok, bowl_pos=bowl_pos, target_pos=target_pos)


def batch_reset_states(A, md, seed, env_ids, genders=None, impairment='none'):
    S = np.zeros((len(env_ids), ABI.STATE_WORDS))
    meta = []
    for k, e in enumerate(env_ids):
        g = None if genders is None else genders[k]
        S[k], m = feeding_reset_state(A, md, seed, e, gender=g, impairment=impairment)
        meta.append(m)
    return S, meta


# ----------------------------------------------------------------------------- batched reset
def _qmul(a, b):
    a, b = np.asarray(a), np.asarray(b)
    ax, ay, az, aw = a[..., 0], a[..., 1], a[..., 2], a[..., 3]
    bx, by, bz, bw = b[..., 0], b[..., 1], b[..., 2], b[..., 3]
    out = np.empty(np.broadcast_shapes(a.shape, b.shape))
    out[..., 0] = aw * bx + ax * bw + ay * bz - az * by
    out[..., 1] = aw * by - ax * bz + ay * bw + az * bx
    out[..., 2] = aw * bz + ax * by - ay * bx + az * bw
    out[..., 3] = aw * bw - ax * bx - ay * by - az * bz
    return out


def _cross(a, b):
    a, b = np.asarray(a), np.asarray(b)
    out = np.empty(np.broadcast_shapes(a.shape, b.shape))
    out[..., 0] = a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1]
    out[..., 1] = a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2]
    out[..., 2] = a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]
    return out


def _qrot(q, v):
    u = q[..., :3]
    t = 2.0 * _cross(u, v)
    return v + q[..., 3:4] * t + _cross(u, t)


def _qaxis(axis, ang):
    s = np.sin(0.5 * ang)[..., None]
    return np.concatenate([axis * s, np.cos(0.5 * ang)[..., None]], -1)


def robot_fk_batch(A, Q):
    """Vectorised robot_fk over envs: Q (N, ndof) -> COM pos/quat, joint axes/origins (N, nl, .)."""
    N = Q.shape[0]
    nl = int(A['n_links'])
    bp = np.broadcast_to(A['robot_base'][:3], (N, 3))
    bq = np.broadcast_to(A['robot_base'][3:], (N, 4))
    LP = np.zeros((N, nl, 3)); LQ = np.zeros((N, nl, 4))
    CP = np.zeros((N, nl, 3)); CQ = np.zeros((N, nl, 4))
    AX = np.zeros((N, nl, 3)); OR = np.zeros((N, nl, 3))
    for i in range(nl):
        p = A['rl_parent'][i]
        pp, pq = (bp, bq) if p < 0 else (LP[:, p], LQ[:, p])
        tp = pp + _qrot(pq, np.broadcast_to(A['rl_jpos'][i], (N, 3)))
        tq = _qmul(pq, np.broadcast_to(A['rl_jquat'][i], (N, 4)))
        OR[:, i] = tp
        AX[:, i] = _qrot(tq, np.broadcast_to(A['rl_axis'][i], (N, 3)))
        dof = A['rl_dof'][i]
        if A['rl_jtype'][i] == 1:
            tq = _qmul(tq, _qaxis(np.broadcast_to(A['rl_axis'][i], (N, 3)), Q[:, dof]))
        LP[:, i], LQ[:, i] = tp, tq
        CP[:, i] = tp + _qrot(tq, np.broadcast_to(A['rl_com_pos'][i], (N, 3)))
        CQ[:, i] = _qmul(tq, np.broadcast_to(A['rl_com_quat'][i], (N, 4)))
    return CP, CQ, AX, OR


def ik_accept(pe, qe, tol):
    """ik_random_restarts' acceptance (util.py:49): position error below tol, and the quaternion
    distance below tol or np.isclose to 2 (the other cover of the rotation, atol tol)."""
    return (pe < tol) & ((qe < tol) | (np.abs(qe - 2.0) <= tol + 2e-5))


def ik_alt_orients(seed, env_ids, episodes, restarts, stream='numpy'):
    """The target orientations ik_random_restarts switches to after a self-contact
    (util.py:44-46: the original's Euler angles + uniform(-45, 45) degrees each, then
    getQuaternionFromEuler), one per restart, drawn up front from a sub-stream of each env's reset
    stream: (N, restarts, 4).  FeedingJaco's target orientation is Euler (pi/2, 0, pi/2)
    (feeding.py:277), which getEulerFromQuaternion returns unchanged."""
    env_ids = list(env_ids)
    eps = [0] * len(env_ids) if episodes is None else list(episodes)
    if stream == 'philox':
        U = philox_uniforms(int(seed) ^ _ALT_TAG, env_ids, eps, 3 * restarts).reshape(len(env_ids), restarts, 3)
        D = -45.0 + 90.0 * U
    else:
        D = np.stack([np.random.default_rng([int(seed), int(e), int(ep), _ALT_TAG]).uniform(-45, 45, size=(restarts, 3))
                      for e, ep in zip(env_ids, eps)]) if env_ids else np.zeros((0, restarts, 3))
    E = np.array([np.pi / 2.0, 0.0, np.pi / 2.0]) + np.deg2rad(D)
    return quat_from_euler_batch(E)


def quat_from_euler_batch(E):
    """p.getQuaternionFromEuler over (..., 3) roll, pitch, yaw: q = qz(yaw) qy(pitch) qx(roll)."""
    r, p, y = 0.5 * E[..., 0], 0.5 * E[..., 1], 0.5 * E[..., 2]
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    return np.stack([sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
                     cr * cp * cy + sr * sp * sy], -1)


_ALT_TAG = 0xA1745


def ik_batch(A, link, tpos, tquat, arm_dofs, lower, upper, init, q0, iters=80, tol=0.01, alt=None, self_contact=None):
    """Vectorised DLS IK (ik_random_restarts, util.py:34-57), one random restart per round for
    every env that has not converged yet.  init (N, restarts, n_arm): the restarts' starting
    joints, drawn up front from each env's reset stream (reset_inputs).  Every env runs on its
    own: it stops updating at the first 10th iteration at which it has converged, so its result
    does not depend on the other envs of the batch (or on how envs are sharded over GPUs).
    step_sim's self-contact screening (util.py:41-46): with self_contact (a function of joint
    rows -> touching robot shape pairs: the device's avr_robot_self_contact, or the oracle's) and
    alt (N, restarts, 4: ik_alt_orients), a restart whose solution touches itself switches the
    env's target orientation to alt[restart] for its own check and the later restarts.  Accepted:
    ik_accept and table_clear; else the restart closest to the target position (util.py:51-54).
    Restated on the device by avr_reset_ik (csrc/avr_reset_ik.hip), which runs the same rules one
    env at a time."""
    N = tpos.shape[0]
    restarts = init.shape[1]
    chain = _chain(A, link)
    cols = []
    for dof in arm_dofs:
        l = [k for k in chain if A['rl_dof'][k] == dof]
        cols.append(l[0] if l else -1)
    done = np.zeros(N, bool)
    Qout = np.repeat(q0[None], N, 0)
    best = np.full(N, np.inf)
    tquat = np.array(tquat, float, copy=True)
    for r in range(restarts):
        idx = np.nonzero(~done)[0]
        if len(idx) == 0:
            break
        Q = np.repeat(q0[None], len(idx), 0)
        Q[:, arm_dofs] = init[idx, r]
        tp, tq = tpos[idx], tquat[idx]
        live = np.ones(len(idx), bool)     # per env: stops at the first 10th iteration that has converged
        for it in range(iters):
            CP, CQ, AX, OR = robot_fk_batch(A, Q)
            ep = tp - CP[:, link]
            dq = _qmul(tq, CQ[:, link] * np.array([-1, -1, -1, 1.0]))
            dq = np.where(dq[:, 3:4] < 0, -dq, dq)
            s = np.linalg.norm(dq[:, :3], axis=1)
            ang = 2.0 * np.arctan2(s, dq[:, 3])
            er = np.where(s[:, None] > 1e-12, dq[:, :3] / np.maximum(s, 1e-12)[:, None] * ang[:, None], 0.0)
            err = np.concatenate([ep, er], 1)
            if it % 10 == 9:
                live &= ~((np.linalg.norm(ep, axis=1) < 1e-5) & (np.linalg.norm(er, axis=1) < 1e-4))
                if not live.any():
                    break
            J = np.zeros((len(idx), 6, len(arm_dofs)))
            for c, l in enumerate(cols):
                if l < 0:
                    continue
                J[:, :3, c] = _cross(AX[:, l], CP[:, link] - OR[:, l])
                J[:, 3:, c] = AX[:, l]
            JJ = J @ np.transpose(J, (0, 2, 1)) + 1e-4 * np.eye(6)[None]
            step = np.transpose(J, (0, 2, 1)) @ np.linalg.solve(JJ, err[..., None])
            rows = np.nonzero(live)[0]
            Q[np.ix_(rows, arm_dofs)] = np.clip(Q[:, arm_dofs] + step[..., 0], lower, upper)[rows]
        CP, CQ, _, _ = robot_fk_batch(A, Q)
        if alt is not None and self_contact is not None:
            sc = np.asarray(self_contact(Q)) > 0
            tquat[idx[sc]] = alt[idx[sc], r]
            tq = tquat[idx]
        pe = np.linalg.norm(tp - CP[:, link], axis=1)
        qe = np.linalg.norm(tq - CQ[:, link], axis=1)
        acc = ik_accept(pe, qe, tol)
        for k, e in enumerate(idx):
            if pe[k] < best[e]:
                best[e] = pe[k]
                Qout[e] = Q[k]
            if acc[k] and table_clear(A, Q[k]):
                Qout[e] = Q[k]
                done[e] = True
    return Qout, done


IMPAIRMENTS = ('none', 'limits', 'weakness', 'tremor')   # world_creation.py:65-72


def _impairment(rng, impairment):
    """Resolve the impairment of one env (world_creation.py:66-69; FeedingJaco-v0 itself asks
    for 'random', feeding.py:175).  The human is static for none / limits / weakness
    (feeding.py:244 passes no controllable joints, world_creation.py:157-159 zeroes the masses);
    'tremor' keeps the head/neck chain's masses and drives it with motors (env.py:327-337)."""
    if impairment == 'random':
        return IMPAIRMENTS[int(rng.integers(4))]
    if impairment == 'no_tremor':
        return IMPAIRMENTS[int(rng.integers(3))]
    if impairment in IMPAIRMENTS:
        return impairment
    raise ValueError('unknown impairment %r' % impairment)


def _tremor_state(st, md, qh, rng):
    """Head-chain state of a 'tremor' env: human_tremors ~ U(+-20 deg) for the 4 controllable
    joints (world_creation.py:136-139), target_human_joint_positions = the chain's angles after
    setup (feeding.py:246-248), chain DoFs after the robot's, at rest.  Its motors stay off
    (VELOCITY_CONTROL, force 0: world_creation.py:162-168) until the first take_step."""
    nd = md.n_dof
    for k, j in enumerate(HEAD_CHAIN):
        st[ABI.S_Q + nd + k] = qh[j]
        st[ABI.S_HCH + k] = qh[j]
    st[ABI.S_HCH + ABI.HC_N:ABI.S_HCH + 2 * ABI.HC_N] = rng.uniform(np.deg2rad(-20), np.deg2rad(20), size=ABI.HC_N)
    st[ABI.S_TASK + ABI.T_HDYN] = 1.0


def _rng(seed, env_id, episode=0):
    """Per-env, per-episode reset stream: independent of batch composition and GPU count."""
    key = [int(seed), int(env_id)] if not episode else [int(seed), int(env_id), int(episode)]
    return np.random.default_rng(key)


def arm_limits(md):
    """IK joint bounds of the arm: the URDF limits, +-2 pi for continuous joints."""
    arm = md.arm_dofs
    lower = np.array([md.desc.arm_lower[i] if md.desc.arm_lower[i] > -1e9 else -2 * np.pi for i in range(len(arm))])
    upper = np.array([md.desc.arm_upper[i] if md.desc.arm_upper[i] < 1e9 else 2 * np.pi for i in range(len(arm))])
    return lower, upper


def keepout_box(A, margin=0.05):
    """The table box inflated by `margin` (table_clear's screening box) as {center, pad, half
    extents, pad} -- avr_reset_ik's keepout8."""
    tb = int(A['task_table_body'])
    s0 = A['body_shape_start'][tb]
    c = A['st_pose'][A['body_index'][tb]][:3] + A['shape_pose'][s0][:3]
    he = A['shape_param'][s0][:3] + margin
    return np.array([c[0], c[1], c[2], 0.0, he[0], he[1], he[2], 0.0])


def human_slot_poses_batch(A, genders, QH):
    """human_slot_poses for many envs at once: genders (N,) str, QH (N, n_joints) -> (N, MAX_HUMAN, 7)."""
    N = len(genders)
    out = np.zeros((N, ABI.MAX_HUMAN, 7))
    for g in ('male', 'female'):
        idx = np.array([k for k in range(N) if genders[k] == g], int)
        if not len(idx):
            continue
        Qg = QH[idx]
        n = len(idx)
        base_p = np.array([0, 0.03, 0.89 - 0.23725 if g == 'male' else 0.86 - 0.225])
        par = A['human_%s_parent' % g]
        jt = A['human_%s_jtype' % g]
        ax = A['human_%s_axis' % g]
        pos = A['human_%s_pos' % g]
        nl = len(par)
        P = np.zeros((n, nl, 3)); Qq = np.zeros((n, nl, 4))
        bp = np.broadcast_to(base_p, (n, 3)); bq = np.broadcast_to(np.array([0, 0, 0, 1.0]), (n, 4))
        for i in range(nl):
            pp, pq = (bp, bq) if par[i] < 0 else (P[:, par[i]], Qq[:, par[i]])
            P[:, i] = pp + _qrot(pq, np.broadcast_to(pos[i], (n, 3)))
            q = pq
            if jt[i] == 1:
                q = _qmul(pq, _qaxis(np.broadcast_to(ax[i], (n, 3)), Qg[:, i]))
            Qq[:, i] = q
        for s_, l in enumerate(A['human_slot_link']):
            if l < 0:
                out[idx, s_, :3] = base_p
                out[idx, s_, 3:] = [0, 0, 0, 1.0]
            else:
                out[idx, s_, :3] = P[:, l]
                out[idx, s_, 3:] = Qq[:, l]
    return out


# ----------------------------------------------------------------------------- counter-based stream
# The 'philox' reset stream: draw j of env e's episode ep is uniform (0, 1) from Philox4x32-10
# (the action generator's family) with key (seed, seed >> 32 ^ 'RSET') and counter
# (e, ep, j // 4, 0x5EED) -- a pure function of (seed, env, episode, j), so every draw of a batch
# of resets comes out of a few vectorised numpy passes (no per-env Python, GIL-light), and the
# same numbers can be generated anywhere.  Fixed draw slots:
PH_GENDER, PH_IMPAIR, PH_LIMIT, PH_HEAD, PH_TREMOR, PH_BOWL, PH_TARGET, PH_INIT = 0, 1, 2, 3, 6, 14, 16, 24
_PH_TAG = 0x52534554


def philox_uniforms(seed, env_ids, episodes, n):
    """(N, n) float64 uniforms in (0, 1) of the 'philox' reset stream."""
    from ._lib import philox4x32_10
    e = np.asarray(env_ids, np.uint64)
    ep = np.asarray(episodes, np.uint64)
    seed = int(seed)
    out = np.zeros((len(e), 4 * ((n + 3) // 4)))
    for b in range((n + 3) // 4):
        c = [e, ep, np.full_like(e, b), np.full_like(e, 0x5EED)]
        r = philox4x32_10(c, seed & 0xFFFFFFFF, ((seed >> 32) ^ _PH_TAG) & 0xFFFFFFFF)
        for k in range(4):
            out[:, 4 * b + k] = (r[k].astype(np.float64) + 0.5) * (1.0 / 4294967296.0)
    return out[:, :n]


def human_joint_angles_batch(A, gender, head, limit_scale):
    """human_joint_angles for many envs of one gender: head (N, 3) angles, limit_scale (N,)."""
    lo0, hi0, scaled, clamp = _human_limits(A, gender)
    N = len(head)
    q = np.zeros((N, len(lo0)))
    for j, ang in [(10, -90), (20, -90), (28, -90), (31, 80), (35, -90), (38, 80)]:
        q[:, j] = np.deg2rad(ang)
    q[:, 25:28] = head
    ls = np.asarray(limit_scale, float)[:, None]
    lo = np.where(scaled[None], lo0[None] * ls, lo0[None])
    hi = np.where(scaled[None], hi0[None] * ls, hi0[None])
    c = clamp[None] & ~((lo == 0) & (hi == -1))
    return np.where(c, np.minimum(np.maximum(q, lo), hi), q)


def _draws_philox(A, md, seed, env_ids, genders, impairment, episodes, restarts):
    """The reset draws of the 'philox' stream, vectorised over envs."""
    N = len(env_ids)
    lower, upper = arm_limits(md)
    na = len(md.arm_dofs)
    U = philox_uniforms(seed, env_ids, episodes, PH_INIT + restarts * na)
    gl = list(genders) if genders is not None else ['male' if u < 0.5 else 'female' for u in U[:, PH_GENDER]]
    if impairment == 'random':
        il = [IMPAIRMENTS[min(3, int(4 * u))] for u in U[:, PH_IMPAIR]]
    elif impairment == 'no_tremor':
        il = [IMPAIRMENTS[min(2, int(3 * u))] for u in U[:, PH_IMPAIR]]
    elif impairment in IMPAIRMENTS:
        il = [impairment] * N
    else:
        raise ValueError('unknown impairment %r' % impairment)
    lim = np.array([x == 'limits' for x in il])
    ls = np.where(lim, 0.5 + 0.5 * U[:, PH_LIMIT], 1.0)
    head = np.deg2rad(-30) + np.deg2rad(60) * U[:, PH_HEAD:PH_HEAD + 3]
    n_j = max(len(A['human_male_parent']), len(A['human_female_parent']))
    QH = np.zeros((N, n_j))
    for g in ('male', 'female'):
        idx = np.array([k for k in range(N) if gl[k] == g], int)
        if len(idx):
            q = human_joint_angles_batch(A, g, head[idx], ls[idx])
            QH[idx, :q.shape[1]] = q
    trem = np.deg2rad(-20) + np.deg2rad(40) * U[:, PH_TREMOR:PH_TREMOR + ABI.HC_N]
    bowl = np.array([-0.15, -0.55, 0.75]) + np.concatenate([-0.05 + 0.1 * U[:, PH_BOWL:PH_BOWL + 2], np.zeros((N, 1))], 1)
    tpos = bowl + np.array([0, -0.1, 0.4]) + (-0.05 + 0.1 * U[:, PH_TARGET:PH_TARGET + 3])
    init = lower + (upper - lower) * U[:, PH_INIT:PH_INIT + restarts * na].reshape(N, restarts, na)
    return gl, il, ls, QH, trem, bowl, tpos, init


def reset_inputs(A, md, seed, env_ids, genders=None, impairment='none', episodes=None, restarts=40, vector_fk=True, stream='numpy'):
    """Everything FeedingEnv.reset draws, for many envs (feeding.py:144-331 minus the IK): state
    rows without the arm's joints, spoon and food (S, float64), the tool link's IK target
    (target7: position + quaternion), the restarts' starting joints (init, (N, restarts, n_arm))
    and per-env meta.  stream 'numpy' (the host reset's per-env Generator; its order: gender,
    impairment, limit scale, head angles, tremor draws, bowl jitter, target jitter, then the IK
    restarts) or 'philox' (counter-based, vectorised: philox_uniforms).
    vector_fk: human link poses by the batched FK (else the per-env one)."""
    if stream == 'philox':
        return _inputs_from_draws(A, md, *_draws_philox(A, md, seed, list(env_ids), genders, impairment,
                                                        [0] * len(env_ids) if episodes is None else list(episodes), restarts))
    if stream != 'numpy':
        raise ValueError('unknown reset stream %r' % stream)
    env_ids = list(env_ids)
    N = len(env_ids)
    eps = [0] * N if episodes is None else list(episodes)
    rngs = [_rng(seed, e, ep) for e, ep in zip(env_ids, eps)]
    S = np.zeros((N, ABI.STATE_WORDS))
    lower, upper = arm_limits(md)
    arm = md.arm_dofs
    gl, il, QH = [], [], []
    tpos, bowl = np.zeros((N, 3)), np.zeros((N, 3))
    init = np.zeros((N, restarts, len(arm)))
    for k in range(N):
        rng = rngs[k]
        g = genders[k] if genders is not None else ('male' if rng.integers(2) == 0 else 'female')
        gl.append(g)
        imp = _impairment(rng, impairment)
        il.append(imp)
        ls = rng.uniform(0.5, 1.0) if imp == 'limits' else 1.0
        qh = human_joint_angles(A, g, rng, ls)
        QH.append(qh)
        if not vector_fk:
            S[k, ABI.S_HUMAN:ABI.S_HUMAN + ABI.MAX_HUMAN * 7] = human_slot_poses(A, g, qh).ravel()
        if imp == 'tremor':
            _tremor_state(S[k], md, qh, rng)
        bowl[k] = np.array([-0.15, -0.55, 0.75]) + np.array([rng.uniform(-0.05, 0.05), rng.uniform(-0.05, 0.05), 0])
        tpos[k] = bowl[k] + np.array([0, -0.1, 0.4]) + rng.uniform(-0.05, 0.05, size=3)
        init[k] = rng.uniform(lower, upper, size=(restarts, len(arm)))
    if vector_fk:
        nj = max(len(q) for q in QH)
        QHa = np.zeros((N, nj))
        for k, q in enumerate(QH):
            QHa[k, :len(q)] = q
        S[:, ABI.S_HUMAN:ABI.S_HUMAN + ABI.MAX_HUMAN * 7] = human_slot_poses_batch(A, gl, QHa).reshape(N, -1)
    tq = np.repeat(G.quat_from_euler([np.pi / 2.0, 0, np.pi / 2.0])[None], N, 0)
    q0 = np.zeros(int(A['n_dof']))
    for d in md.finger_dofs:
        q0[d] = md.params['finger_target']
    S[:, ABI.S_Q:ABI.S_Q + len(q0)] = q0
    for d in arm:
        S[:, ABI.S_KP + d] = 0.0
        S[:, ABI.S_QTGT + d] = 0.0
        S[:, ABI.S_MAXIMP + d] = md.params['default_motor_impulse']
    for d in md.finger_dofs:
        S[:, ABI.S_KP + d] = md.params['finger_gain']
        S[:, ABI.S_QTGT + d] = md.params['finger_target']
        S[:, ABI.S_MAXIMP + d] = md.params['finger_force'] * md.params['time_step']
    b = ABI.S_FREE + ABI.FB_WORDS
    S[:, b:b + 3] = bowl
    S[:, b + 3:b + 7] = G.quat_from_euler([np.pi / 2.0, 0, 0])
    t = ABI.S_TASK
    gi = np.array([0 if g == 'male' else 1 for g in gl])
    hs = ABI.S_HUMAN + 7 * int(A['task_head_slot'])
    for k in range(N):
        head = S[k, hs:hs + 7]
        mouth = A['task_mouth_male'] if gi[k] == 0 else A['task_mouth_female']
        S[k, t + ABI.T_TARGET:t + ABI.T_TARGET + 3] = G.tf_mul(head[:3], head[3:], mouth, [0, 0, 0, 1])[0]
    S[:, t + ABI.T_ALIVE] = (1 << 8) - 1
    S[:, t + ABI.T_GENDER] = gi
    target7 = np.concatenate([tpos, tq], 1)
    meta = [dict(gender=gl[k], impairment=il[k], bowl_pos=bowl[k], target_pos=tpos[k]) for k in range(N)]
    return S, target7, init, q0, meta


def _inputs_from_draws(A, md, gl, il, ls, QH, trem, bowl, tpos, init):
    """reset_inputs' state rows from already-drawn values (the 'philox' stream), vectorised."""
    N = len(gl)
    S = np.zeros((N, ABI.STATE_WORDS))
    S[:, ABI.S_HUMAN:ABI.S_HUMAN + ABI.MAX_HUMAN * 7] = human_slot_poses_batch(A, gl, QH).reshape(N, -1)
    tr = np.array([x == 'tremor' for x in il])
    if tr.any():
        nd = md.n_dof
        for k, j in enumerate(HEAD_CHAIN):
            S[tr, ABI.S_Q + nd + k] = QH[tr, j]
            S[tr, ABI.S_HCH + k] = QH[tr, j]
        S[tr, ABI.S_HCH + ABI.HC_N:ABI.S_HCH + 2 * ABI.HC_N] = trem[tr]
        S[tr, ABI.S_TASK + ABI.T_HDYN] = 1.0
    q0 = np.zeros(int(A['n_dof']))
    for d in md.finger_dofs:
        q0[d] = md.params['finger_target']
    _fill_common(A, md, S, q0, gl, bowl)
    tq = np.repeat(G.quat_from_euler([np.pi / 2.0, 0, np.pi / 2.0])[None], N, 0)
    target7 = np.concatenate([tpos, tq], 1)
    meta = [dict(gender=gl[k], impairment=il[k], limit_scale=float(ls[k]), bowl_pos=bowl[k], target_pos=tpos[k]) for k in range(N)]
    return S, target7, init, q0, meta


def _fill_common(A, md, S, q0, gl, bowl):
    """Motors, bowl, mouth target, alive mask and gender words of reset state rows."""
    N = len(S)
    arm = md.arm_dofs
    S[:, ABI.S_Q:ABI.S_Q + len(q0)] = q0
    for d in arm:
        S[:, ABI.S_KP + d] = 0.0
        S[:, ABI.S_QTGT + d] = 0.0
        S[:, ABI.S_MAXIMP + d] = md.params['default_motor_impulse']
    for d in md.finger_dofs:
        S[:, ABI.S_KP + d] = md.params['finger_gain']
        S[:, ABI.S_QTGT + d] = md.params['finger_target']
        S[:, ABI.S_MAXIMP + d] = md.params['finger_force'] * md.params['time_step']
    b = ABI.S_FREE + ABI.FB_WORDS
    S[:, b:b + 3] = bowl
    S[:, b + 3:b + 7] = G.quat_from_euler([np.pi / 2.0, 0, 0])
    t = ABI.S_TASK
    gi = np.array([0 if g == 'male' else 1 for g in gl])
    hs = ABI.S_HUMAN + 7 * int(A['task_head_slot'])
    mouth = np.where(gi[:, None] == 0, A['task_mouth_male'][None], A['task_mouth_female'][None])
    S[:, t + ABI.T_TARGET:t + ABI.T_TARGET + 3] = S[:, hs:hs + 3] + _qrot(S[:, hs + 3:hs + 7], mouth)
    S[:, t + ABI.T_ALIVE] = (1 << 8) - 1
    S[:, t + ABI.T_GENDER] = gi


def place_tool_bodies(A, S, Q):
    """Arm joints Q into S, the spoon on the tool frame (world_creation.py:332-343) and the food
    spheres above it (feeding.py:291-308) -- what avr_reset_ik does on the device after its IK."""
    tool = int(A['task_tool_link'])
    CP, CQ, _, _ = robot_fk_batch(A, Q)
    off = A['task_tool_offset']
    for k in range(len(S)):
        st = S[k]
        st[ABI.S_Q:ABI.S_Q + Q.shape[1]] = Q[k]
        sp, sq = G.tf_mul(CP[k, tool], CQ[k, tool], off[:3], off[3:])
        st[ABI.S_FREE:ABI.S_FREE + 3] = sp
        st[ABI.S_FREE + 3:ABI.S_FREE + 7] = sq
        r = 0.005
        n = 0
        for i in range(2):
            for j in range(2):
                for kk in range(2):
                    f = ABI.S_FREE + ABI.FB_WORDS * (2 + n)
                    st[f:f + 3] = np.array([i * 2 * r - 0.005, j * 2 * r, kk * 2 * r + 0.02]) + sp
                    st[f + 3:f + 7] = [0, 0, 0, 1]
                    n += 1
    return S


def batch_reset_states_fast(A, md, seed, env_ids, genders=None, impairment='none', episodes=None, stream='numpy', self_contact=None):
    """Vectorised equivalent of batch_reset_states (same per-env draws and acceptance rules,
    IK batched across envs).  episodes[k] selects the k-th env's episode stream (default 0);
    stream: reset_inputs' draw stream; self_contact: ik_batch's self-contact screening."""
    S, target7, init, q0, meta = reset_inputs(A, md, seed, env_ids, genders, impairment, episodes, vector_fk=False, stream=stream)
    lower, upper = arm_limits(md)
    alt = ik_alt_orients(seed, env_ids, episodes, init.shape[1], stream) if self_contact is not None else None
    Q, ok = ik_batch(A, int(A['task_tool_link']), target7[:, :3], target7[:, 3:], md.arm_dofs, lower, upper, init, q0,
                     alt=alt, self_contact=self_contact)
    place_tool_bodies(A, S, Q)
    for k, m in enumerate(meta):
        m['ik_ok'] = bool(ok[k])
    return S, meta
