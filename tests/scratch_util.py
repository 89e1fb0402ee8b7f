"""ScratchItchPR2 test helpers: reset states (host reset path, few IK attempts for speed) and
contact states -- the human's right arm posed (7 chain angles, least squares) so that the
scratch target on the limb lies on the scratcher's tip sphere, pressed in by `depth`."""
import numpy as np

from avr import _abi as ABI
from avr import geom as G
from avr import reset_scratch as RSS

SI = ABI.SI


def scene():
    A = ABI.load_scene(ABI.TASK_SCRATCH)
    return A, ABI.ModelDesc(A)


def reset_states(A, md, ids, impairment='random', attempts=12, iters=80):
    S, meta = RSS.batch_reset_states(A, md, 1001, list(ids), impairment=impairment, attempts=attempts, iters=iters)
    return S, meta


def _arm_fk(A, gender, qh, q7):
    q = qh.copy()
    q[list(RSS.ARM_CHAIN)] = q7
    return RSS.human_link_poses(A, gender, q)


def contact_states(A, md, S, meta, depth=0.002):
    """Copy of S with each env's human arm chain re-posed so that target_on_arm meets the tool
    tip sphere (radius 0.01) at `depth` penetration; chain motors target the new pose."""
    from scipy.optimize import least_squares
    S = S.copy()
    nd = md.n_dof
    slot_link = list(A['human_slot_link'])
    for k in range(len(S)):
        st = S[k]
        g = meta[k]['gender']
        ls = meta[k]['limit_scale']
        qh, lo, hi = RSS.human_joint_angles(A, g, ls)
        tb = st[SI.S_FREE:SI.S_FREE + 7]
        tip = G.tf_mul(tb[:3], tb[3:], A['task_tool_tip'], [0, 0, 0, 1])[0]
        li = int(RSS.ARM_CHAIN[int(st[SI.S_TASK + SI.T_LIMB])])
        on = st[SI.S_TASK + SI.T_ONARM:SI.S_TASK + SI.T_ONARM + 3]
        n_loc = np.array([on[0], on[1], 0.0])
        n_loc /= np.linalg.norm(n_loc)

        def resid(x):
            _, _, P, Q = _arm_fk(A, g, qh, x)
            R = G.quat_to_mat(Q[li])
            c = P[li] + R @ on + R @ n_loc * (0.01 - depth)
            return np.concatenate([c - tip, 0.05 * (x - qh[list(RSS.ARM_CHAIN)])])

        x0 = qh[list(RSS.ARM_CHAIN)]
        lb = np.array([lo[j] for j in RSS.ARM_CHAIN]) + 1e-6
        ub = np.array([hi[j] for j in RSS.ARM_CHAIN]) - 1e-6
        x = least_squares(resid, np.clip(x0, lb, ub), bounds=(lb, ub)).x
        base_p, base_q, P, Q = _arm_fk(A, g, qh, x)
        for s, l in enumerate(slot_link):
            if l >= 0:
                st[SI.S_HUMAN + 7 * s:SI.S_HUMAN + 7 * s + 7] = np.concatenate([P[l], Q[l]])
        for c in range(len(RSS.ARM_CHAIN)):
            st[SI.S_Q + nd + c] = x[c]
            st[SI.S_HCH + c] = x[c]
            st[SI.S_QTGT + nd + c] = x[c]
        lp = np.concatenate([P[li], Q[li]])
        st[SI.S_TASK + SI.T_TARGET:SI.S_TASK + SI.T_TARGET + 3] = G.tf_mul(lp[:3], lp[3:], on, [0, 0, 0, 1])[0]
    return S
