"""Host-side reset path for BedBathingPR2-v0 (BedBathingEnv.reset, bed_bathing.py:155-357).

The initial per-env state block (the PR2 layout, `_abi.BB`) comes out of three phases:
  1. the human lying on the bed: gender (:182), impairment 'none' (:188), joint targets
     (7: 50 deg, 8: -50 deg, 17: -30 deg, 28/35: -60 deg, :283) clamped by the joint limits, base at
     [0, 0, 0.7] pitched -30 deg (:194); the right arm (joints 4..13 non-static: the revolute
     7..13 are the articulated chain) falls onto the mattress for 100 frames under gravity -1
     with the human's 0.1 N velocity motors (:284-289, world_creation.py:162-166), then the human
     becomes static (:292-300).  The settle has no random input, so its result depends on the
     gender only: it runs once per gender on the device (settled_arms) and is reused;
  2. position_robot_toc (:317; env.py:489-585): random PR2 base poses, IK of link 76 to the start
     goal [-0.5, -0.1, 1] (identity orientation) and to the settled shoulder / elbow / wrist,
     best base by goals reached then manipulability (reset_scratch.position_robot_toc);
  3. the gripper open at 0.2 (:319), the wiper on link 76's COM frame (:320), every wipe target
     alive (generate_targets, :359-380; their positions are compiled into the scene).

Per-env randomness: numpy Generator keyed by (seed, env_id[, episode]) as in reset.py.
"""
import numpy as np

from . import _abi as ABI
from . import geom as G
from .reset import _qaxis, _qmul, _qrot, _rng
from .reset_scratch import ARM_CHAIN, LEFT_ARM_RESET, position_robot_toc

BB = ABI.BB
JOINT_TARGETS = ((7, 50), (8, -50), (17, -30), (28, -60), (35, -60))    # bed_bathing.py:283
START_GOAL = np.array([-0.5, -0.1, 1.0])                                 # bed_bathing.py:314
PR2_INIT_BASE = np.array([-2.0, -2.0, 0.0])                              # world_creation.py:195

_SETTLED = {}


def human_joint_angles(A, gender):
    """(q, lower, upper): setup_human_joints with the bed-bathing targets, enforce_joint_limits
    (world_creation.py:110-133; impairment 'none': limit_scale 1)."""
    n = len(A['human_%s_parent' % gender])
    q = np.zeros(n)
    for j, ang in JOINT_TARGETS:
        q[j] = np.deg2rad(ang)
    lo = A['human_%s_lower' % gender].astype(float)
    hi = A['human_%s_upper' % gender].astype(float)
    jt = A['human_%s_jtype' % gender]
    for j in range(n):
        if jt[j] == 1 and not (lo[j] == 0 and hi[j] == -1):
            q[j] = min(max(q[j], lo[j]), hi[j])
    return q, lo, hi


def human_link_poses(A, gender, q, base=None):
    """World poses (link == COM frames) of the human links on the bed (base: bed_bathing.py:194)."""
    base = A['bb_human_base'] if base is None else base
    bp, bq = np.asarray(base[:3], float), np.asarray(base[3:], float)
    par, jt, ax, pos = (A['human_%s_%s' % (gender, k)] for k in ('parent', 'jtype', 'axis', 'pos'))
    n = len(par)
    P = np.zeros((n, 3)); Q = np.zeros((n, 4))
    for i in range(n):
        pp, pq = (bp, bq) if par[i] < 0 else (P[par[i]], Q[par[i]])
        P[i] = pp + _qrot(pq, pos[i])
        qq = pq
        if jt[i] == 1:
            qq = _qmul(pq, _qaxis(np.asarray(ax[i], float), np.float64(q[i])))
        Q[i] = qq
    return bp, bq, P, Q


def slot_poses(A, gender, q):
    bp, bq, P, Q = human_link_poses(A, gender, q)
    out = np.zeros((BB.MAX_HUMAN, 7))
    for s, l in enumerate(A['human_slot_link']):
        out[s] = np.concatenate([bp, bq]) if l < 0 else np.concatenate([P[l], Q[l]])
    return out


def _tool_pose(A, CPl, CQl):
    """The wiper's body frame (composite COM) with its base (handle) COM on link 76's COM frame."""
    return CPl - G.quat_rotate(CQl, A['task_tool_pivot']), CQl


def settle_states(A, md, genders):
    """Phase-1 state rows (one per gender given): human on the bed with the right arm articulated
    and at its joint targets, chain motors = the 0.1 N velocity motors, PR2 at its load pose."""
    from .reset_scratch import arm_fk
    nd = int(A['n_dof'])
    S = np.zeros((len(genders), BB.STATE_WORDS))
    arm = np.array(md.arm_dofs)
    Q0 = np.zeros((1, nd))
    Q0[0, arm] = LEFT_ARM_RESET
    for d in md.finger_dofs:
        Q0[0, d] = md.params['finger_target']
    bq = np.array([[0, 0, 0, 1.0]])
    CP, CQ, _, _ = arm_fk(A, Q0, PR2_INIT_BASE[None], bq)
    link = int(A['task_tool_link'])
    tp, tq = _tool_pose(A, CP[0, link], CQ[0, link])
    dt = md.params['time_step']
    for k, g in enumerate(genders):
        st = S[k]
        qh, lo, hi = human_joint_angles(A, g)
        st[BB.S_HUMAN:BB.S_HUMAN + 7 * BB.MAX_HUMAN] = slot_poses(A, g, qh).ravel()
        st[BB.S_RBASE:BB.S_RBASE + 3] = PR2_INIT_BASE
        st[BB.S_RBASE + 6] = 1.0
        st[BB.S_Q:BB.S_Q + nd] = Q0[0]
        for d in range(nd):
            st[BB.S_MAXIMP + d] = md.params['default_motor_impulse']
        st[BB.S_FREE:BB.S_FREE + 3] = tp
        st[BB.S_FREE + 3:BB.S_FREE + 7] = tq
        for c, j in enumerate(ARM_CHAIN):
            st[BB.S_Q + nd + c] = qh[j]
            st[BB.S_HCH + c] = qh[j]
            st[BB.S_HCH + 2 * BB.HC_N + c] = lo[j]
            st[BB.S_HCH + 3 * BB.HC_N + c] = hi[j]
            st[BB.S_KP + nd + c] = 0.0                    # VELOCITY_CONTROL, target velocity 0
            st[BB.S_MAXIMP + nd + c] = md.params['settle_motor_force'] * dt
        st[BB.S_TASK + BB.T_GENDER] = 0 if g == 'male' else 1
        st[BB.S_TASK + BB.T_HDYN] = 1.0
    return S


def settled_arms(A, md, device=0, frames=None, runner=None):
    """{gender: (chain q (7,), slot poses (MAX_HUMAN, 7))} after the reset's settle, run once per
    process on the device (runner: a function (S, frames) -> settled S, e.g. the oracle's, for
    tests).  The settle has no random input: its result depends on the gender alone."""
    frames = md.params['settle_frames'] if frames is None else frames
    # cached per scene object (held in the entry, so its id cannot be reused by another scene)
    # and device; a runner's result is not cached
    key = (id(A), frames, device)
    if runner is None and key in _SETTLED and _SETTLED[key][0] is A:
        return _SETTLED[key][1]
    S = settle_states(A, md, ('male', 'female'))
    if runner is None:
        from . import _lib
        sim = _lib.Sim(md, 2, device=device)
        try:
            sim.set_state(S.astype(np.float32))
            sim.settle(frames)
            St = sim.get_state().astype(np.float64)
        finally:
            sim.close()
    else:
        St = runner(S, frames)
    nd = int(A['n_dof'])
    out = {}
    for k, g in enumerate(('male', 'female')):
        out[g] = (St[k, BB.S_Q + nd:BB.S_Q + nd + len(ARM_CHAIN)].copy(),
                  St[k, BB.S_HUMAN:BB.S_HUMAN + 7 * BB.MAX_HUMAN].reshape(BB.MAX_HUMAN, 7).copy())
    if runner is None:
        _SETTLED[key] = (A, out)
    return out


def batch_reset_states(A, md, seed, env_ids, genders=None, episodes=None, attempts=100, iters=200, settled=None, device=0, sim=None):
    """Initial BedBathing state blocks (float64 (N, BB.STATE_WORDS)) and per-env metadata.
    settled: settled_arms() output (computed on the device when None).  sim: run the base-pose
    search on the device (reset_scratch.position_robot_toc)."""
    P = prepare_reset(A, md, seed, env_ids, genders, episodes, attempts, settled, device)
    return finish_reset(A, md, P, iters, sim)


def prepare_reset(A, md, seed, env_ids, genders=None, episodes=None, attempts=100, settled=None, device=0):
    """The reset's draws (gender, the base search's attempts) and the settled human, vectorised
    over envs; no search result is needed (AVRVecEnv prepares the next episode's resets on a
    background thread)."""
    from .reset_scratch import base_search_draws
    from .reset import arm_limits
    env_ids = list(env_ids)
    N = len(env_ids)
    eps = [0] * N if episodes is None else list(episodes)
    rngs = [_rng(seed, e, ep) for e, ep in zip(env_ids, eps)]
    settled = settled_arms(A, md, device) if settled is None else settled
    nd = int(A['n_dof'])
    S = np.zeros((N, BB.STATE_WORDS))
    gl = [genders[k] if genders is not None else ('male' if rngs[k].integers(2) == 0 else 'female') for k in range(N)]   # bed_bathing.py:182
    js = A['bb_joint_slots']
    goals = np.zeros((N, 3, 3))
    for g in ('male', 'female'):
        idx = np.array([k for k in range(N) if gl[k] == g], int)
        if not len(idx):
            continue
        qc, slots = settled[g]
        S[idx, BB.S_HUMAN:BB.S_HUMAN + 7 * BB.MAX_HUMAN] = slots.ravel()
        goals[idx] = slots[js, :3]                                     # shoulder, elbow, wrist (:305-307)
        S[idx, BB.S_Q + nd:BB.S_Q + nd + len(qc)] = qc
    lo, hi = arm_limits(md)
    tstart, base, rest = base_search_draws(rngs, attempts, lo, hi, (0, 0, 0), np.repeat(START_GOAL[None], N, 0))
    retry = dict(seed=seed, env_ids=env_ids, episodes=eps, pos_offset=(0, 0, 0))
    return dict(S=S, genders=gl, goals=goals, tstart=tstart, base=base, rest=rest, retry=retry)


def finish_reset(A, md, P, iters=200, sim=None):
    """The base-pose search (on the device when sim is given) and the robot, gripper, wiper and
    wipe targets it places, on a prepare_reset result.  Returns (S, meta)."""
    from .reset_scratch import arm_fk, base_search
    S = P['S'].copy()
    gl = P['genders']
    N = len(S)
    nd = int(A['n_dof'])
    bp, bq, Qa, _, ok = base_search(A, md, P['tstart'], P['base'], P['rest'], P['goals'], iters, sim, P.get('retry'))
    for d in md.finger_dofs:                                           # set_gripper_open_position(0.2, set_instantly)
        Qa[:, d] = md.params['finger_target']
    CP, CQ, _, _ = arm_fk(A, Qa, bp, bq)
    link = int(A['task_tool_link'])
    S[:, BB.S_RBASE:BB.S_RBASE + 3] = bp
    S[:, BB.S_RBASE + 3:BB.S_RBASE + 7] = bq
    S[:, BB.S_Q:BB.S_Q + nd] = Qa
    S[:, BB.S_MAXIMP:BB.S_MAXIMP + nd] = md.params['default_motor_impulse']   # default velocity motors (createJointMotors)
    for d in md.finger_dofs:                                           # gripper position motors (world_creation.py:323-328)
        S[:, BB.S_KP + d] = md.params['finger_gain']
        S[:, BB.S_QTGT + d] = md.params['finger_target']
        S[:, BB.S_MAXIMP + d] = md.params['finger_force'] * md.params['time_step']
    cq = CQ[:, link]                                                   # the wiper: base COM on link 76's COM frame
    S[:, BB.S_FREE:BB.S_FREE + 3] = CP[:, link] - _qrot(cq, np.broadcast_to(A['task_tool_pivot'], (N, 3)))
    S[:, BB.S_FREE + 3:BB.S_FREE + 7] = cq
    t = BB.S_TASK
    gi = np.array([0 if g == 'male' else 1 for g in gl])
    S[:, t + BB.T_GENDER] = gi
    S[:, t + BB.T_HDYN] = 0.0                                          # the human is static from here on (:292-300)
    nt = A['bb_ntgt'].sum(1)[gi].astype(int)
    for w in range(6):                                                 # every target alive
        nb = np.clip(nt - 24 * w, 0, 24)
        S[:, t + BB.T_WIPE + w] = (1 << nb) - 1
    S[:, t + BB.T_NTGT] = nt
    meta = [dict(gender=gl[k], impairment='none', base_ok=bool(ok[k]), n_targets=int(nt[k])) for k in range(N)]   # (bed_bathing.py:188)
    return S, meta
