"""Host-side reset path for ScratchItchPR2-v0 (ScratchItchEnv.reset, scratch_itch.py:130-273).

It produces the initial per-env state block (ScratchItch layout, `_abi.SI`) the device step
consumes:
  * gender, impairment (world_creation.py:66-72: limit_scale, human_strength, human_tremors);
  * the human pose: setup_human_joints with the ScratchItch joint targets (scratch_itch.py:257-259;
    world_creation.py:135-179) clamped by the (scaled) joint limits; the right arm (controllable
    joints 4..13; its revolute joints 7..13 are the articulated chain) keeps its masses and gets
    reactive position motors (gain 0.01, force human_strength) or, under 'tremor', the take_step
    tremor motors;
  * the PR2: reset_robot_joints (env.py:450-464), then position_robot_toc (env.py:489-585): random
    base poses, IK of the left gripper tool frame (link 76) to the start goal and to the human's
    shoulder / elbow / wrist, best base by goals reached then joint-limit-weighted manipulability
    (JLWKI, env.py:466-477,536-553).  p.calculateInverseKinematics is a Bullet internal: it is
    restated as damped least squares with a random rest pose per attempt (util.py:76-105);
  * the gripper open at 0.25 (world_creation.py:309-328), the scratcher on link 76's COM frame
    (world_creation.py:330-365), and the target (generate_target, scratch_itch.py:275-287;
    util.point_on_capsule, util.py:112-132).
ScratchItch's reset runs no settling frames after the tool is attached.

Per-env randomness: numpy Generator keyed by (seed, env_id[, episode]) as in reset.py; the
reference's single np_random stream cannot be reproduced draw for draw.
"""
import numpy as np

from . import _abi as ABI
from . import geom as G
from .reset import _cross, _impairment, _qaxis, _qmul, _qrot, _rng, arm_limits, human_link_poses

SI = ABI.SI
HUMAN_SCALED = set(range(7, 14)) | set(range(17, 24)) | set(range(24, 28))   # limit_scale joints (human_creation.py)
ARM_CHAIN = (7, 8, 9, 10, 11, 12, 13)
CONTROLLABLE = tuple(range(4, 14))            # scratch_itch.py:191
JOINT_TARGETS = [(7, 30), (10, -90), (20, -90), (28, -90), (31, 80), (35, -90), (38, 80)]   # scratch_itch.py:257
LEFT_ARM_RESET = (1.75, 1.25, 1.5, -0.5, 1, 0, 1)     # env.py:456-457


# ----------------------------------------------------------------------------- human
def human_joint_angles(A, gender, limit_scale=1.0):
    """(q[42], scaled lower, scaled upper): setup_human_joints + enforce_joint_limits."""
    n = len(A['human_%s_parent' % gender])
    q = np.zeros(n)
    for j, ang in JOINT_TARGETS:
        q[j] = np.deg2rad(ang)
    lo = A['human_%s_lower' % gender].copy()
    hi = A['human_%s_upper' % gender].copy()
    for j in HUMAN_SCALED:
        lo[j] *= limit_scale
        hi[j] *= limit_scale
    jt = A['human_%s_jtype' % gender]
    for j in range(n):
        if jt[j] == 1 and not (lo[j] == 0 and hi[j] == -1):
            q[j] = min(max(q[j], lo[j]), hi[j])
    return q, lo, hi


def point_on_capsule(rng, length, radius):
    """util.point_on_capsule(p1=0, p2=[0, 0, -length], radius, theta in [0, 2 pi))."""
    axis = np.array([0.0, 0.0, -1.0])
    L = rng.uniform(radius, length)
    m = int(np.argmax(np.abs(axis)))
    y = np.zeros(3)
    y[(m + 1) % 3] = 1
    ortho = np.cross(axis, y)
    ortho /= np.linalg.norm(ortho)
    normal = np.cross(axis, ortho)
    th = rng.uniform(0, 2 * np.pi)
    return L * axis + radius * np.cos(th) * ortho + radius * np.sin(th) * normal


# ----------------------------------------------------------------------------- PR2 arm FK / IK
def arm_fk(A, Q, bp, bq, links=None):
    """Batched FK of the compiled robot (the PR2 left-arm subtree) on per-row bases (N, 3/4):
    COM positions/quaternions and joint axes/origins, (N, nl, .).  `links` (ascending, closed
    under parents) restricts the work to those links; the others stay zero."""
    N = Q.shape[0]
    nl = int(A['n_links'])
    LP = np.zeros((N, nl, 3)); LQ = np.zeros((N, nl, 4))
    CP = np.zeros((N, nl, 3)); CQ = np.zeros((N, nl, 4))
    AX = np.zeros((N, nl, 3)); OR = np.zeros((N, nl, 3))
    for i in (range(nl) if links is None else links):
        p = A['rl_parent'][i]
        pp, pq = (bp, bq) if p < 0 else (LP[:, p], LQ[:, p])
        tp = pp + _qrot(pq, np.broadcast_to(A['rl_jpos'][i], (N, 3)))
        tq = _qmul(pq, np.broadcast_to(A['rl_jquat'][i], (N, 4)))
        OR[:, i] = tp
        AX[:, i] = _qrot(tq, np.broadcast_to(A['rl_axis'][i], (N, 3)))
        dof = A['rl_dof'][i]
        if A['rl_jtype'][i] == 1:
            tq = _qmul(tq, _qaxis(np.broadcast_to(A['rl_axis'][i], (N, 3)), Q[:, dof]))
        elif A['rl_jtype'][i] == 2:
            tp = tp + AX[:, i] * Q[:, dof][:, None]
        LP[:, i], LQ[:, i] = tp, tq
        CP[:, i] = tp + _qrot(tq, np.broadcast_to(A['rl_com_pos'][i], (N, 3)))
        CQ[:, i] = _qmul(tq, np.broadcast_to(A['rl_com_quat'][i], (N, 4)))
    return CP, CQ, AX, OR


def _chain(A, link):
    out = []
    k = link
    while k >= 0:
        out.append(k)
        k = A['rl_parent'][k]
    return sorted(out)


def _chain_cols(A, link, dofs):
    chain = _chain(A, link)
    cols = []
    for d in dofs:
        l = [k for k in chain if A['rl_dof'][k] == d]
        cols.append(l[0] if l else -1)
    return cols


def arm_jacobian(A, link, cols, CP, AX, OR):
    N = CP.shape[0]
    J = np.zeros((N, 6, len(cols)))
    for c, l in enumerate(cols):
        if l < 0:
            continue
        J[:, :3, c] = _cross(AX[:, l], CP[:, link] - OR[:, l])
        J[:, 3:, c] = AX[:, l]
    return J


def ik_dls(A, link, Q0, bp, bq, tp, tq, dofs, lower, upper, iters):
    """Damped least squares on the rows of Q0 (N, nd) towards positions tp (N, 3) and, when tq is
    not None, orientations tq (N, 4) of link's COM frame (FK of link's chain only).  A row stops
    at an iteration it % 10 == 9 where every component of its error is below 1e-6 (the rule of
    the device search, avr_base_search); the loop ends once every row has."""
    Q = Q0.copy()
    chain = _chain(A, link)
    cols = _chain_cols(A, link, dofs)
    live = np.ones(len(Q), bool)
    for it in range(iters):
        CP, CQ, AX, OR = arm_fk(A, Q, bp, bq, chain)
        ep = tp - CP[:, link]
        J = arm_jacobian(A, link, cols, CP, AX, OR)
        if tq is not None:
            dq = _qmul(tq, CQ[:, link] * np.array([-1, -1, -1, 1.0]))
            dq = np.where(dq[:, 3:4] < 0, -dq, dq)
            s = np.linalg.norm(dq[:, :3], axis=1)
            ang = 2.0 * np.arctan2(s, dq[:, 3])
            er = np.where(s[:, None] > 1e-12, dq[:, :3] / np.maximum(s, 1e-12)[:, None] * ang[:, None], 0.0)
            err = np.concatenate([ep, er], 1)
            Jr = J
        else:
            err = ep
            Jr = J[:, :3]
        if it % 10 == 9:
            live &= ~np.all(np.abs(err) < 1e-6, axis=1)
            if not live.any():
                break
        k = Jr.shape[1]
        JJ = Jr @ np.transpose(Jr, (0, 2, 1)) + 1e-4 * np.eye(k)[None]
        step = np.transpose(Jr, (0, 2, 1)) @ np.linalg.solve(JJ, err[..., None])
        Qn = np.clip(Q[:, dofs] + step[..., 0], lower, upper)
        Q[:, dofs] = np.where(live[:, None], Qn, Q[:, dofs])
    CP, CQ, AX, OR = arm_fk(A, Q, bp, bq, chain)
    return Q, CP, CQ, AX, OR


def jlwki(J, q, lower, upper):
    """Joint-limit-weighted kinematic isotropy (env.py:466-477, 548-553), rows of J (N, 6, 7)."""
    phi, lam = 0.5, 0.05
    qr = 0.5 * (upper - lower)
    w = 1.0 - np.power(phi, (qr - np.abs(qr - q + lower)) / (lam * qr) + 1)
    w = np.maximum(w, 0.001)
    M = J @ (w[:, :, None] * np.transpose(J, (0, 2, 1)))
    det = np.maximum(np.linalg.det(M), 0.0)
    return np.power(det, 1.0 / 6.0) / (np.trace(M, axis1=1, axis2=2) / 6.0)


def base_search_draws(rngs, attempts, lo, hi, pos_offset=(0.1, 0, 0), tstart=None):
    """Per-env draws of position_robot_toc: the start goal (ScratchItch: jittered, drawn first;
    tstart given: none), then one block of `attempts` rows (base x, base y, yaw, rest pose) per
    env (env.py:509-511, util.py:99).  Returns tstart (N, 3), base7 (N, attempts, 7), rest
    (N, attempts, n_arm)."""
    N, na = len(rngs), len(lo)
    if tstart is None:
        tstart = np.stack([np.array([-0.55, 0, 0.8]) + r.uniform(-0.05, 0.05, size=3) for r in rngs])
    U = np.stack([r.random((attempts, 3 + na)) for r in rngs]) if N else np.zeros((0, attempts, 3 + na))
    base = np.zeros((N, attempts, 7))
    base[..., :3] = np.array([-0.85, -0.4, 0]) + np.asarray(pos_offset, float)
    base[..., 0] += -0.5 + 0.5 * U[..., 0]                     # uniform(-0.5, 0) (right side)
    base[..., 1] += -0.5 + U[..., 1]                           # uniform(-0.5, 0.5)
    yaw = np.deg2rad(-30 + 60 * U[..., 2])                     # uniform(-30, 30) degrees
    base[..., 5] = np.sin(0.5 * yaw)
    base[..., 6] = np.cos(0.5 * yaw)
    rest = lo + (hi - lo) * U[..., 3:]
    return np.asarray(tstart, float), base, rest


def position_robot_toc(A, md, rngs, human_goals, attempts=100, iters=200, tstart=None, pos_offset=(0.1, 0, 0), sim=None):
    """Batched position_robot_toc for the PR2 (env.py:489-585; scratch_itch.py:189-190,
    bed_bathing.py:317): per env, `attempts` random base poses; at each the start goal (link 76
    to the start target with identity orientation, base offset pos_offset) must be reached (0.03
    on position and quaternion), then the shoulder / elbow / wrist positions count as further
    goals; the best base maximises goals reached, then summed manipulability.  tstart: the start
    targets (N, 3), or None for ScratchItch's jittered target (drawn first from each stream).
    sim: a _lib.Sim of the task -- the search runs on the device (avr_base_search, fp32), else
    here in fp64 (the device search's checker).
    Returns (base_pos, base_quat, arm q, start target, ok) per env."""
    lo, hi = arm_limits(md)
    tstart, base, rest = base_search_draws(rngs, attempts, lo, hi, pos_offset, tstart)
    return base_search(A, md, tstart, base, rest, human_goals, iters, sim)


RETRY_BLOCKS = 10      # position_robot_toc keeps drawing until a start goal is reached (env.py:509); capped here
_RETRY_TAG = 0x7E7


def _retry_draws(retry, env_rows, k, attempts, lo, hi, tstart):
    """Block k of further attempts for the given rows of a batch: drawn from a sub-stream of each
    env's reset stream (seed, env id, episode, tag + k)."""
    rngs = [np.random.default_rng([int(retry['seed']), int(retry['env_ids'][r]), int(retry['episodes'][r]), _RETRY_TAG + k]) for r in env_rows]
    _, base, rest = base_search_draws(rngs, attempts, lo, hi, retry['pos_offset'], tstart[env_rows])
    return base, rest


def base_search(A, md, tstart, base, rest, human_goals, iters=200, sim=None, retry=None):
    """The search of position_robot_toc on drawn attempts (base_search_draws): on the device when
    sim is given, else here in fp64.  retry (dict: seed, env_ids, episodes, pos_offset): an env
    none of whose attempts reaches the start goal draws further blocks of attempts and takes the
    first that does, as the reference's `while iteration < attempts or best_position is None`
    (env.py:509) -- up to RETRY_BLOCKS blocks, then the closest attempt of the first block.
    Returns (base_pos, base_quat, arm q, start target, ok)."""
    N, attempts = base.shape[:2]
    nd = int(A['n_dof'])
    arm = np.array(md.arm_dofs)
    if sim is not None:
        best, ok, qa = sim.base_search(base, rest, tstart, human_goals, iters=iters, tol=0.03)
        bsel = base[np.arange(N), best].copy()
        if retry is not None:
            lo, hi = arm_limits(md)
            for k in range(RETRY_BLOCKS):
                rows = np.nonzero(~ok)[0]
                if not len(rows):
                    break
                b2, r2 = _retry_draws(retry, rows, k, attempts, lo, hi, tstart)
                _, _, _, res = sim.base_search(b2, r2, tstart[rows], human_goals[rows], iters=iters, tol=0.03, per_attempt=True)
                hit = res[..., 0] > 0
                for j, e in enumerate(rows):
                    if not hit[j].any():
                        continue
                    a = int(np.argmax(hit[j]))              # the first attempt that reaches the start goal
                    _, ok1, q1 = sim.base_search(b2[j:j + 1, a:a + 1], r2[j:j + 1, a:a + 1], tstart[e:e + 1], human_goals[e:e + 1],
                                                 iters=iters, tol=0.03)
                    bsel[e], qa[e], ok[e] = b2[j, a], q1[0], bool(ok1[0])
        out_q = np.zeros((N, nd))
        for d in md.finger_dofs:
            out_q[:, d] = md.params['finger_target']
        out_q[:, arm] = qa
        return bsel[:, :3].copy(), bsel[:, 3:].copy(), out_q, tstart, ok
    res = base_search_host(A, md, base, rest, tstart, human_goals, iters)
    goals, manip, pe, Qs = res
    out_bp, out_bq, out_q, ok = np.zeros((N, 3)), np.zeros((N, 4)), np.zeros((N, nd)), np.zeros(N, bool)
    for e in range(N):
        best = None
        for a in range(attempts):
            g, mm = goals[e, a], manip[e, a]
            if g > 0 and (best is None or g > goals[e, best] or (g == goals[e, best] and mm > manip[e, best])):
                best = a
        if best is None:                                  # no start goal reached: the closest attempt
            best = int(np.argmin(pe[e]))
        else:
            ok[e] = True
        out_bp[e], out_bq[e], out_q[e] = base[e, best, :3], base[e, best, 3:], Qs[e, best]
    if retry is not None:
        lo, hi = arm_limits(md)
        for k in range(RETRY_BLOCKS):
            rows = np.nonzero(~ok)[0]
            if not len(rows):
                break
            b2, r2 = _retry_draws(retry, rows, k, attempts, lo, hi, tstart)
            g2, _, _, Q2 = base_search_host(A, md, b2, r2, tstart[rows], human_goals[rows], iters)
            for j, e in enumerate(rows):
                hit = g2[j] > 0
                if hit.any():
                    a = int(np.argmax(hit))
                    out_bp[e], out_bq[e], out_q[e], ok[e] = b2[j, a, :3], b2[j, a, 3:], Q2[j, a], True
    return out_bp, out_bq, out_q, tstart, ok


def base_search_host(A, md, base, rest, tstart, human_goals, iters):
    """Every attempt of the search in fp64: (goals reached or -1 (N, attempts), manipulability,
    start-goal position error, start-goal joints (N, attempts, nd))."""
    N, attempts = base.shape[:2]
    M = N * attempts
    nd = int(A['n_dof'])
    arm = np.array(md.arm_dofs)
    link = int(A['task_tool_link'])
    lo, hi = arm_limits(md)
    bp = base[..., :3].reshape(M, 3)
    bq = base[..., 3:].reshape(M, 4)
    Q0 = np.zeros((M, nd))
    Q0[:, arm] = rest.reshape(M, len(arm))
    for d in md.finger_dofs:
        Q0[:, d] = md.params['finger_target']
    tp = np.repeat(tstart, attempts, 0)
    tq = np.tile(np.array([0, 0, 0, 1.0]), (M, 1))
    Qs, CP, CQ, AX, OR = ik_dls(A, link, Q0, bp, bq, tp, tq, arm, lo, hi, iters)
    pe = np.linalg.norm(tp - CP[:, link], axis=1)
    qe = np.linalg.norm(tq - CQ[:, link], axis=1)
    ok0 = (pe < 0.03) & ((qe < 0.03) | (np.abs(qe - 2) < 0.03))
    cols = _chain_cols(A, link, arm)
    manip = np.where(ok0, jlwki(arm_jacobian(A, link, cols, CP, AX, OR), Qs[:, arm], lo, hi), 0.0)
    goals = ok0.astype(int)
    for g in range(3):                                   # shoulder, elbow, wrist (position only)
        hp = np.repeat(human_goals[:, g], attempts, 0)
        Qg, CPg, _, AXg, ORg = ik_dls(A, link, Q0, bp, bq, hp, None, arm, lo, hi, iters)
        okg = ok0 & (np.linalg.norm(hp - CPg[:, link], axis=1) < 0.03)
        manip = manip + np.where(okg, jlwki(arm_jacobian(A, link, cols, CPg, AXg, ORg), Qg[:, arm], lo, hi), 0.0)
        goals = goals + okg.astype(int)
    goals = np.where(ok0, goals, -1).reshape(N, attempts)
    return goals, manip.reshape(N, attempts), pe.reshape(N, attempts), Qs.reshape(N, attempts, nd)


# ----------------------------------------------------------------------------- full reset
def human_joint_angles_batch(A, gender, limit_scale):
    """human_joint_angles for many envs of one gender: limit_scale (N,) -> q (N, n), lo, hi (N, n)."""
    n = len(A['human_%s_parent' % gender])
    lo0 = A['human_%s_lower' % gender].astype(float)
    hi0 = A['human_%s_upper' % gender].astype(float)
    sc = np.zeros(n, bool)
    sc[[j for j in HUMAN_SCALED if j < n]] = True
    ls = np.asarray(limit_scale, float)[:, None]
    lo = np.where(sc[None], lo0[None] * ls, lo0[None])
    hi = np.where(sc[None], hi0[None] * ls, hi0[None])
    q = np.zeros(n)
    for j, ang in JOINT_TARGETS:
        q[j] = np.deg2rad(ang)
    q = np.broadcast_to(q, lo.shape)
    c = (A['human_%s_jtype' % gender] == 1)[None] & ~((lo == 0) & (hi == -1))
    return np.where(c, np.minimum(np.maximum(q, lo), hi), q), lo, hi


def human_link_poses_batch(A, gender, QH):
    """reset.human_link_poses for many envs of one gender: QH (N, n) -> base_p (3,), base_q (4,),
    P (N, n, 3), Q (N, n, 4)."""
    base_p = np.array([0, 0.03, 0.89 - 0.23725 if gender == 'male' else 0.86 - 0.225])
    base_q = np.array([0, 0, 0, 1.0])
    par, jt, ax, pos = (A['human_%s_%s' % (gender, k)] for k in ('parent', 'jtype', 'axis', 'pos'))
    N, n = QH.shape
    P = np.zeros((N, n, 3)); Q = np.zeros((N, n, 4))
    bp, bq = np.broadcast_to(base_p, (N, 3)), np.broadcast_to(base_q, (N, 4))
    for i in range(n):
        pp, pq = (bp, bq) if par[i] < 0 else (P[:, par[i]], Q[:, par[i]])
        P[:, i] = pp + _qrot(pq, np.broadcast_to(pos[i], (N, 3)))
        Q[:, i] = _qmul(pq, _qaxis(np.broadcast_to(ax[i], (N, 3)), QH[:, i])) if jt[i] == 1 else pq
    return base_p, base_q, P, Q


def batch_reset_states(A, md, seed, env_ids, genders=None, impairment='random', episodes=None, attempts=100, iters=200, sim=None):
    """Initial ScratchItch state blocks (float64 (N, SI.STATE_WORDS)) and per-env metadata.
    sim: run the base-pose search on the device (position_robot_toc)."""
    return finish_reset(A, md, prepare_reset(A, md, seed, env_ids, genders, impairment, episodes, attempts), iters, sim)


def prepare_reset(A, md, seed, env_ids, genders=None, impairment='random', episodes=None, attempts=100):
    """Everything of the reset that needs no search result -- every draw, in each env's stream
    order (human, base search, target), the human pose, motors and target -- vectorised over envs
    (AVRVecEnv prepares the next episode's resets on a background thread)."""
    env_ids = list(env_ids)
    N = len(env_ids)
    eps = [0] * N if episodes is None else list(episodes)
    rngs = [_rng(seed, e, ep) for e, ep in zip(env_ids, eps)]
    S = np.zeros((N, SI.STATE_WORDS))
    nd = int(A['n_dof'])
    nc = len(ARM_CHAIN)
    slot_link = np.asarray(A['human_slot_link'])
    gl, il, ls, strength = [], [], np.ones(N), np.ones(N)
    tremors = np.zeros((N, len(CONTROLLABLE)))
    for k in range(N):                      # the human's draws (scratch_itch.py:163, world_creation.py:66-72)
        rng = rngs[k]
        gl.append(genders[k] if genders is not None else ('male' if rng.integers(2) == 0 else 'female'))
        imp = _impairment(rng, impairment)
        il.append(imp)
        if imp == 'limits':
            ls[k] = rng.uniform(0.5, 1.0)
        if imp == 'weakness':
            strength[k] = rng.uniform(0.25, 1.0)
        if imp == 'tremor':
            tremors[k] = rng.uniform(np.deg2rad(-10), np.deg2rad(10), size=len(CONTROLLABLE))
    nj = len(A['human_male_parent'])
    QH, LO, HI = np.zeros((N, nj)), np.zeros((N, nj)), np.zeros((N, nj))
    P = np.zeros((N, nj, 3)); Q = np.zeros((N, nj, 4))
    BP, BQ = np.zeros((N, 3)), np.zeros((N, 4))
    for g in ('male', 'female'):
        idx = np.array([k for k in range(N) if gl[k] == g], int)
        if not len(idx):
            continue
        qh, lo, hi = human_joint_angles_batch(A, g, ls[idx])
        bp, bq, Pg, Qg = human_link_poses_batch(A, g, qh)
        QH[idx], LO[idx], HI[idx], P[idx], Q[idx], BP[idx], BQ[idx] = qh, lo, hi, Pg, Qg, bp, bq
    for s_, l in enumerate(slot_link):
        o = SI.S_HUMAN + 7 * s_
        S[:, o:o + 3] = BP if l < 0 else P[:, l]
        S[:, o + 3:o + 7] = BQ if l < 0 else Q[:, l]
    goals = P[:, [9, 11, 13]]                                   # shoulder, elbow, wrist (scratch_itch.py:187-190)
    chain = list(ARM_CHAIN)
    S[:, SI.S_Q + nd:SI.S_Q + nd + nc] = QH[:, chain]
    S[:, SI.S_HCH:SI.S_HCH + nc] = QH[:, chain]                 # target_human_joint_positions
    S[:, SI.S_HCH + SI.HC_N:SI.S_HCH + SI.HC_N + nc] = tremors[:, [CONTROLLABLE.index(j) for j in chain]]
    S[:, SI.S_HCH + 2 * SI.HC_N:SI.S_HCH + 2 * SI.HC_N + nc] = LO[:, chain]
    S[:, SI.S_HCH + 3 * SI.HC_N:SI.S_HCH + 3 * SI.HC_N + nc] = HI[:, chain]
    # reactive motors (world_creation.py:171-179), replaced by take_step's under 'tremor'
    S[:, SI.S_QTGT + nd:SI.S_QTGT + nd + nc] = QH[:, chain]
    S[:, SI.S_KP + nd:SI.S_KP + nd + nc] = md.params['reactive_gain']
    S[:, SI.S_MAXIMP + nd:SI.S_MAXIMP + nd + nc] = md.params['reactive_force'] * strength[:, None] * md.params['time_step']
    t = SI.S_TASK
    S[:, t + SI.T_GENDER] = [0 if g == 'male' else 1 for g in gl]
    S[:, t + SI.T_HDYN] = 1.0
    S[:, t + SI.T_TREMOR] = [1.0 if i == 'tremor' else 0.0 for i in il]
    S[:, t + SI.T_STRENGTH] = strength
    meta = [dict(gender=gl[k], impairment=il[k], limit_scale=float(ls[k]), strength=float(strength[k])) for k in range(N)]
    lo_a, hi_a = arm_limits(md)
    tstart, base, rest = base_search_draws(rngs, attempts, lo_a, hi_a)
    # generate_target (scratch_itch.py:275-287): each env's limb and point, drawn after the search's
    gidx = {'male': 0, 'female': 1}
    limbs = np.zeros(N, int)
    on_arm = np.zeros((N, 3))
    for k in range(N):
        li, ln, rad = A['task_limbs'][gidx[gl[k]]][int(rngs[k].integers(2))]
        limbs[k] = int(li)
        on_arm[k] = point_on_capsule(rngs[k], ln, rad)
    si = np.array([list(slot_link).index(l) for l in limbs])
    lp = S[np.arange(N)[:, None], SI.S_HUMAN + 7 * si[:, None] + np.arange(7)[None]]
    S[:, t + SI.T_LIMB] = [chain.index(l) for l in limbs]
    S[:, t + SI.T_ONARM:t + SI.T_ONARM + 3] = on_arm
    S[:, t + SI.T_TARGET:t + SI.T_TARGET + 3] = lp[:, :3] + _qrot(lp[:, 3:], on_arm)
    for k in range(N):
        meta[k].update(limb=int(limbs[k]), start_goal=tstart[k])
    retry = dict(seed=seed, env_ids=env_ids, episodes=eps, pos_offset=(0.1, 0, 0))
    return dict(S=S, meta=meta, goals=goals, tstart=tstart, base=base, rest=rest, retry=retry)


def finish_reset(A, md, P, iters=200, sim=None):
    """The base-pose search (on the device when sim is given) and the robot and tool placement
    it decides, on a prepare_reset result.  Returns (S, meta)."""
    S, meta = P['S'].copy(), [dict(m) for m in P['meta']]
    N = len(S)
    nd = int(A['n_dof'])
    bp, bq, Qa, tstart, ok = base_search(A, md, P['tstart'], P['base'], P['rest'], P['goals'], iters, sim, P.get('retry'))
    CP, CQ, _, _ = arm_fk(A, Qa, bp, bq)
    link = int(A['task_tool_link'])
    S[:, SI.S_RBASE:SI.S_RBASE + 3] = bp
    S[:, SI.S_RBASE + 3:SI.S_RBASE + 7] = bq
    S[:, SI.S_Q:SI.S_Q + nd] = Qa
    S[:, SI.S_KP:SI.S_KP + nd] = 0.0                 # default velocity motors (PyBullet createJointMotors)
    S[:, SI.S_QTGT:SI.S_QTGT + nd] = 0.0
    S[:, SI.S_MAXIMP:SI.S_MAXIMP + nd] = md.params['default_motor_impulse']
    for d in md.finger_dofs:                         # set_gripper_open_position(0.25) (world_creation.py:323-328)
        S[:, SI.S_KP + d] = md.params['finger_gain']
        S[:, SI.S_QTGT + d] = md.params['finger_target']
        S[:, SI.S_MAXIMP + d] = md.params['finger_force'] * md.params['time_step']
    # scratcher: its base (handle) COM on link 76's COM frame; the body frame is the composite COM
    hq = CQ[:, link]
    S[:, SI.S_FREE:SI.S_FREE + 3] = CP[:, link] - _qrot(hq, np.broadcast_to(A['task_tool_pivot'], (N, 3)))
    S[:, SI.S_FREE + 3:SI.S_FREE + 7] = hq
    for k in range(N):
        meta[k].update(base_ok=bool(ok[k]))
    return S, meta
