"""Host reset path of DressingJaco-v0 (BASELINE configs[4]; a build-defined task, see
include/avr_dressing.h and DESIGN.md section 10).

Per env (numpy Generator keyed by (seed, env id, episode), like the other tasks' resets):
  * gender, and the seated human of FeedingJaco's scene (human_joint_angles: feeding.py:242-245
    arm and leg targets, random head) -> the left arm's collision geometry in the world: the
    upper-arm and forearm capsules and the hand sphere (links 19, 21, 23 of human_creation.py's
    left arm) and the cloth spheres at the shoulder, elbow and wrist (human_creation.py:90-95,
    136-141: links 18, 20, 22);
  * the sleeve's start: its held cuff (ring 0) just beyond the hand along the forearm axis
    (jittered), the tool frame's z axis pointing back along the forearm towards the elbow; the
    Jaco's arm joints by damped least squares to that tool pose (random restarts, as the other
    resets' IK, util.py:34-105 semantics) -- the robot is kinematic in this task, so no collision
    screening applies.  prepare_reset draws everything on the host; the IK then runs on the device
    (avr_reset_ik, the facade's default) or on the host (finish_reset, the checker);
  * the sleeve in its rest shape: ring k centred k * spacing beyond the cuff, away from the arm.
"""
import numpy as np

from . import _abi as ABI
from . import geom as G
from . import reset as RS

DR = ABI.DR
# the Jaco's base for dressing the left arm (build-defined: the FeedingJaco base mirrored to the
# person's left side and moved forward so that the hand, the elbow and the shoulder are in reach)
DR_BASE = np.array([0.65, -0.3, 0.36, 0.0, 0.0, 0.0, 1.0])
CLOTH_SPHERE_R = {'male': (0.043, 0.043, 0.033), 'female': (0.0355, 0.0355, 0.027)}   # human_creation.py:93-95, 139-141
SH_LINK, EL_LINK, WR_LINK = 18, 20, 22          # cloth-sphere links of the left arm (DFS order)
UA_LINK, FA_LINK, HAND_LINK = 19, 21, 23


def dressing_scene():
    """FeedingJaco's compiled scene with the dressing task's robot base."""
    A = dict(ABI.load_scene(ABI.TASK_FEEDING))
    A['robot_base'] = DR_BASE.copy()
    A['task_dressing'] = np.int32(1)
    return A


def _slot_shape(A, link, gender):
    """(shape index) of the compiled human shape on `link` for `gender`."""
    sl = list(A['human_slot_link'])
    slot = sl.index(link)
    g = 0 if gender == 'male' else 1
    for b in range(len(A['body_kind'])):
        if A['body_kind'][b] == ABI.BODY_HUMAN and A['body_index'][b] == slot:
            for s in range(A['body_shape_start'][b], A['body_shape_start'][b] + A['body_shape_count'][b]):
                if A['shape_gender'][s] in (-1, g):
                    return s
    raise KeyError(link)


def arm_geometry(A, gender, qh):
    """The left arm's world geometry: the GEO words of the state block (avr_dressing.h)."""
    _, _, P, Q = RS.human_link_poses(A, gender, qh)
    geo = np.zeros(32)
    geo[0:3], geo[3:6], geo[6:9] = P[SH_LINK], P[EL_LINK], P[WR_LINK]
    s = _slot_shape(A, HAND_LINK, gender)
    geo[9:12] = G.tf_mul(P[HAND_LINK], Q[HAND_LINK], A['shape_pose'][s][:3], A['shape_pose'][s][3:])[0]
    for off, link in ((12, UA_LINK), (19, FA_LINK)):
        s = _slot_shape(A, link, gender)
        c, q = G.tf_mul(P[link], Q[link], A['shape_pose'][s][:3], A['shape_pose'][s][3:])
        ax = G.quat_rotate(q, [0, 0, 1.0]) * A['shape_param'][s][1]          # GEOM_CAPSULE: z-aligned, half height
        geo[off:off + 3], geo[off + 3:off + 6], geo[off + 6] = c + ax, c - ax, A['shape_param'][s][0]
    geo[26] = A['shape_param'][_slot_shape(A, HAND_LINK, gender)][0]
    geo[27:30] = CLOTH_SPHERE_R[gender]
    return geo


def _frame_z(z, x_hint):
    """Quaternions (N, 4) of the frames whose z axes are z (N, 3), x axes the projection of x_hint."""
    from scipy.spatial.transform import Rotation
    z = z / np.linalg.norm(z, axis=-1, keepdims=True)
    x = x_hint - np.sum(x_hint * z, -1, keepdims=True) * z
    x /= np.linalg.norm(x, axis=-1, keepdims=True)
    return Rotation.from_matrix(np.stack([x, np.cross(z, x), z], -1)).as_quat()


def arm_geometry_batch(A, gender, QH):
    """arm_geometry for many envs of one gender: QH (N, n_joints) -> (N, 32)."""
    from .reset_scratch import human_link_poses_batch
    _, _, P, Q = human_link_poses_batch(A, gender, QH)
    N = len(QH)
    geo = np.zeros((N, 32))
    geo[:, 0:3], geo[:, 3:6], geo[:, 6:9] = P[:, SH_LINK], P[:, EL_LINK], P[:, WR_LINK]
    s = _slot_shape(A, HAND_LINK, gender)
    geo[:, 9:12] = P[:, HAND_LINK] + RS._qrot(Q[:, HAND_LINK], np.broadcast_to(A['shape_pose'][s][:3], (N, 3)))
    for off, link in ((12, UA_LINK), (19, FA_LINK)):
        s = _slot_shape(A, link, gender)
        sp = A['shape_pose'][s]
        c = P[:, link] + RS._qrot(Q[:, link], np.broadcast_to(sp[:3], (N, 3)))
        q = RS._qmul(Q[:, link], np.broadcast_to(sp[3:], (N, 4)))
        ax = RS._qrot(q, np.broadcast_to([0, 0, 1.0], (N, 3))) * A['shape_param'][s][1]    # GEOM_CAPSULE: z-aligned
        geo[:, off:off + 3], geo[:, off + 3:off + 6], geo[:, off + 6] = c + ax, c - ax, A['shape_param'][s][0]
    geo[:, 26] = A['shape_param'][_slot_shape(A, HAND_LINK, gender)][0]
    geo[:, 27:30] = CLOTH_SPHERE_R[gender]
    return geo


def arm_limits(md):
    arm = md.arm_dofs
    lo = np.array([md.desc.arm_lower[i] if md.desc.arm_lower[i] > -1e9 else -2 * np.pi for i in range(len(arm))])
    hi = np.array([md.desc.arm_upper[i] if md.desc.arm_upper[i] < 1e9 else 2 * np.pi for i in range(len(arm))])
    return arm, lo, hi


def _fk_chain(A, Q, link):
    """RS.robot_fk_batch restricted to the chain root .. `link` (the same operations in the same
    order for those links; other links are left zero): (CP, CQ, AX, OR) (N, n_links, .)."""
    N = Q.shape[0]
    nl = int(A['n_links'])
    chain = sorted(int(k) for k in RS._chain(A, link))
    bp = np.broadcast_to(A['robot_base'][:3], (N, 3))
    bq = np.broadcast_to(A['robot_base'][3:], (N, 4))
    LP = np.zeros((N, nl, 3)); LQ = np.zeros((N, nl, 4))
    CP = np.zeros((N, nl, 3)); CQ = np.zeros((N, nl, 4))
    AX = np.zeros((N, nl, 3)); OR = np.zeros((N, nl, 3))
    for i in chain:
        p = A['rl_parent'][i]
        pp, pq = (bp, bq) if p < 0 else (LP[:, p], LQ[:, p])
        tp = pp + RS._qrot(pq, np.broadcast_to(A['rl_jpos'][i], (N, 3)))
        tq = RS._qmul(pq, np.broadcast_to(A['rl_jquat'][i], (N, 4)))
        OR[:, i] = tp
        AX[:, i] = RS._qrot(tq, np.broadcast_to(A['rl_axis'][i], (N, 3)))
        if A['rl_jtype'][i] == 1:
            tq = RS._qmul(tq, RS._qaxis(np.broadcast_to(A['rl_axis'][i], (N, 3)), Q[:, A['rl_dof'][i]]))
        LP[:, i], LQ[:, i] = tp, tq
    CP[:, link] = LP[:, link] + RS._qrot(LQ[:, link], np.broadcast_to(A['rl_com_pos'][link], (N, 3)))
    CQ[:, link] = RS._qmul(LQ[:, link], np.broadcast_to(A['rl_com_quat'][link], (N, 4)))
    return CP, CQ, AX, OR


def _dls(A, link, cols, arm, lo, hi, Qr, tpos, tquat, iters, res):
    """Damped-least-squares iterations on the rows of Qr (in place) towards the tool poses
    (tpos, tquat); a row stops once its position error and rotation angle are below res."""
    conj = np.array([-1, -1, -1, 1.0])
    act = np.arange(len(Qr))                       # rows still iterating
    for it in range(iters + 1):
        Q = Qr[act]
        CP, CQ, AX, OR = _fk_chain(A, Q, link)
        tp, tq = tpos[act], tquat[act]
        ep = tp - CP[:, link]
        dq = RS._qmul(tq, CQ[:, link] * conj)
        dq = np.where(dq[:, 3:4] < 0, -dq, dq)
        s = np.linalg.norm(dq[:, :3], axis=1)
        ang = 2.0 * np.arctan2(s, dq[:, 3])
        live = (np.linalg.norm(ep, axis=1) >= res) | (ang >= res)
        if it == iters or not live.any():
            break
        act, Q, ep, dq, s, ang = act[live], Q[live], ep[live], dq[live], s[live], ang[live]
        CP, AX, OR = CP[live], AX[live], OR[live]
        er = np.where(s[:, None] > 1e-12, dq[:, :3] / np.maximum(s, 1e-12)[:, None] * ang[:, None], 0.0)
        J = np.zeros((len(act), 6, len(arm)))
        for c, l in enumerate(cols):
            J[:, :3, c] = RS._cross(AX[:, l], CP[:, link] - OR[:, l])
            J[:, 3:, c] = AX[:, l]
        JJ = J @ np.transpose(J, (0, 2, 1)) + 1e-4 * np.eye(6)[None]
        step = np.transpose(J, (0, 2, 1)) @ np.linalg.solve(JJ, np.concatenate([ep, er], 1)[..., None])
        Qr[act[:, None], arm] = np.clip(Q[:, arm] + step[..., 0], lo, hi)
    CP, CQ, _, _ = _fk_chain(A, Qr, link)
    return CP[:, link], CQ[:, link]


def ik_accept(P, Qq, tp, tq, tol):
    """util.py:49's acceptance of a restart: position error below tol and the orientation's
    quaternion distance below tol or np.isclose to 2 (the other cover of the rotation, atol tol)."""
    pe = np.linalg.norm(tp - P, axis=1)
    qd = np.linalg.norm(tq - Qq, axis=1)
    return (pe < tol) & ((qd < tol) | np.isclose(qd, 2.0, atol=tol)), pe


def ik_batch(A, link, tpos, tquat, arm, lo, hi, init, iters=150, tol=0.01, res=1e-6, split=2):
    """Vectorised damped-least-squares IK of the tool link's COM frame (RS.ik_batch's update rule)
    with per-env restarts init (N, R, 7); no collision screening (the robot is kinematic here).
    A row stops iterating once its position error and rotation angle are below `res`
    (calculateInverseKinematics' residualThreshold role; at 1e-6 the joint angles stay within
    ~4e-6 rad of running all 150 iterations); the first restart that meets util.py:49's rule
    (ik_accept) is kept, else the restart closest to the target position (util.py:51-54).  The
    first `split` restarts run in turn over the envs still unsolved; the rest run side by side for
    the few envs left (rows are independent, so the result is the same as running them in turn,
    with far fewer passes).  The device restatement is avr_reset_ik (csrc/avr_dressing.hip).
    Returns (Q (N, ndof), ok (N,))."""
    N, R, _ = init.shape
    nd = int(A['n_dof'])
    chain = RS._chain(A, link)
    cols = [[k for k in chain if A['rl_dof'][k] == d][0] for d in arm]
    Qout = np.zeros((N, nd))
    done = np.zeros(N, bool)
    best = np.full(N, np.inf)                     # closest restart so far (util.py:51-54)
    for r in range(R):
        idx = np.nonzero(~done)[0]
        if not len(idx):
            break
        rs = [r] if r < split else list(range(r, R))
        n = len(idx)
        Qr = np.zeros((n * len(rs), nd))            # restart-major rows
        Qr[:, arm] = np.concatenate([init[idx, q] for q in rs])
        tp, tq = np.tile(tpos[idx], (len(rs), 1)), np.tile(tquat[idx], (len(rs), 1))
        P, Qq = _dls(A, link, cols, arm, lo, hi, Qr, tp, tq, iters, res)
        good, pe = ik_accept(P, Qq, tp, tq, tol)
        good, pe = good.reshape(len(rs), n), pe.reshape(len(rs), n)
        Qr = Qr.reshape(len(rs), n, nd)
        for k in range(len(rs)):                    # restarts in order: first accepted, else the closest
            take = ~done[idx] & (good[k] | (pe[k] < best[idx]))
            Qout[idx[take]] = Qr[k, take]
            best[idx[take]] = np.where(good[k, take], -1.0, pe[k, take])
            done[idx[good[k]]] = True
        if len(rs) > 1:
            break
    return Qout, done


def cloth_rest(p_tool, q_tool):
    """Particle positions [NP][3] of the sleeve at rest: ring k centred k * spacing along -z of
    the tool frame, particle j at angle 2 pi j / segs in the frame's x-y plane."""
    R = G.quat_to_mat(q_tool)
    th = 2 * np.pi * np.arange(DR.SEGS) / DR.SEGS
    ring = np.stack([DR.RADIUS * np.cos(th), DR.RADIUS * np.sin(th), np.zeros(DR.SEGS)], 1)
    X = np.zeros((DR.RINGS, DR.SEGS, 3))
    for k in range(DR.RINGS):
        X[k] = p_tool + (ring - np.array([0, 0, k * DR.SPACING])) @ R.T
    return X.reshape(-1, 3)


def cloth_rest_batch(P, Qt):
    """cloth_rest for many tool frames: P (N, 3), Qt (N, 4) -> (N, NP, 3)."""
    N = len(P)
    th = 2 * np.pi * np.arange(DR.SEGS) / DR.SEGS
    ring = np.stack([DR.RADIUS * np.cos(th), DR.RADIUS * np.sin(th), np.zeros(DR.SEGS)], 1)
    loc = (ring[None] - np.arange(DR.RINGS)[:, None, None] * np.array([0, 0, DR.SPACING])).reshape(-1, 3)
    Rm = np.stack([G.quat_to_mat(q) for q in Qt])
    return P[:, None] + np.einsum('nij,pj->npi', Rm, loc)


def prepare_reset(A, md, seed, env_ids, genders=None, episodes=None, restarts=8):
    """The host part of a reset: per-env draws (gender, the seated human's joints, the start-pose
    jitter, the IK restarts) and the arm geometry.  Returns (S (N, STATE_WORDS) with the geometry and
    gender words set and no arm / sleeve yet, tpos (N, 3), tquat (N, 4), init (N, restarts, 7),
    genders); finish_reset (host IK) or avr_reset_ik (device) completes it."""
    n = len(env_ids)
    episodes = [0] * n if episodes is None else list(episodes)
    arm, lo, hi = arm_limits(md)
    S = np.zeros((n, DR.STATE_WORDS))
    init = np.zeros((n, restarts, len(arm)))
    jit = np.zeros((n, 3))
    gl, QH = [], []
    for k, e in enumerate(env_ids):              # the per-env draws, in the stream's order
        rng = RS._rng(seed, e, episodes[k])
        g = genders[k] if genders is not None else ('male' if rng.integers(2) == 0 else 'female')
        QH.append(RS.human_joint_angles(A, g, rng))
        jit[k] = rng.uniform(-0.02, 0.02, 3)
        init[k] = rng.uniform(lo, hi, size=(restarts, len(arm)))
        gl.append(g)
    gl = np.array(gl)
    geo = np.zeros((n, 32))
    for g in ('male', 'female'):
        sel = np.nonzero(gl == g)[0]
        if len(sel):
            geo[sel] = arm_geometry_batch(A, g, np.array([QH[k] for k in sel]))
    el, wr = geo[:, 3:6], geo[:, 6:9]
    u = (wr - el) / np.linalg.norm(wr - el, axis=1, keepdims=True)
    hand_end = wr + u * geo[:, 26:27] * 2                  # util.py:191
    tpos = hand_end + u * 0.06 + jit
    tquat = _frame_z(-u, np.array([0, 0, 1.0]))
    S[:, DR.S_GEO:DR.S_GEO + 32] = geo
    S[:, DR.S_TASK + DR.T_GENDER] = (gl == 'female').astype(float)
    return S, tpos, tquat, init, gl


def finish_reset(A, md, P):
    """The host IK (ik_batch) and the sleeve in its rest shape on the tool frame: (S, meta)."""
    S, tpos, tquat, init, gl = P
    S = S.copy()
    n = len(S)
    arm, lo, hi = arm_limits(md)
    tool = int(A['task_tool_link'])
    Q, ok = ik_batch(A, tool, tpos, tquat, arm, lo, hi, init)
    CP, CQ, _, _ = RS.robot_fk_batch(A, Q)
    S[:, DR.S_Q:DR.S_Q + 7] = Q[:, arm]
    S[:, DR.S_QT:DR.S_QT + 7] = Q[:, arm]
    S[:, DR.S_TOOL:DR.S_TOOL + 3] = CP[:, tool]
    S[:, DR.S_TOOL + 3:DR.S_TOOL + 7] = CQ[:, tool]
    S[:, DR.S_X:DR.S_X + 4 * DR.NP].reshape(n, DR.NP, 4)[:, :, :3] = cloth_rest_batch(CP[:, tool], CQ[:, tool])
    meta = [dict(gender=str(gl[k]), impairment='none', ik_ok=bool(ok[k])) for k in range(n)]
    return S, meta


def batch_reset_states(A, md, seed, env_ids, genders=None, episodes=None, restarts=8):
    """(S (N, STATE_WORDS) float64, meta) for the global env ids: prepare_reset + the host IK."""
    return finish_reset(A, md, prepare_reset(A, md, seed, env_ids, genders, episodes, restarts))
