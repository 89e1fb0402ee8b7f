"""DressingJaco test helpers: reset states and a scripted dressing controller -- actions that move
the held cuff along the forearm past the elbow and up the upper arm (a damped-least-squares step
of the tool frame towards a waypoint each env step), so that the sleeve is pulled onto the arm and
the contact / sleeve-on-arm terms are exercised."""
import numpy as np

from avr import _abi as ABI
from avr import reset as RS
from avr import reset_dressing as RD

DR = ABI.DR


def scene():
    A = RD.dressing_scene()
    return A, ABI.ModelDesc(A)


def reset_states(A, md, ids, genders=None):
    S, meta = RD.batch_reset_states(A, md, 1001, list(ids), genders=genders)
    return S, meta


def waypoint(S, t, T=120):
    """The cuff's goal at env step t: from its start over the hand to the elbow (first half), then
    up the upper arm towards the shoulder."""
    geo = S[:, DR.S_GEO:DR.S_GEO + 32]
    sh, el, wr = geo[:, 0:3], geo[:, 3:6], geo[:, 6:9]
    u = (wr - el) / np.linalg.norm(wr - el, axis=1, keepdims=True)
    start = wr + u * 0.15
    if t < T / 2:
        return start + (el - start) * (t / (T / 2))
    return el + (sh - el) * 0.8 * min((t - T / 2) / (T / 2), 1.0)


def controller(A, md, St, t, gain=1.0):
    """Actions (N, 7) moving the tool COM towards waypoint(t) with its z axis along the arm segment
    being covered (DLS on the Jaco's tool-link Jacobian), as caller actions of take_step."""
    arm, lo, hi = RD.arm_limits(md)
    tool = int(A['task_tool_link'])
    N = len(St)
    nd = int(A['n_dof'])
    Q = np.zeros((N, nd))
    Q[:, arm] = St[:, DR.S_Q:DR.S_Q + 7]
    CP, CQ, AX, OR = RS.robot_fk_batch(A, Q)
    goal = waypoint(St, t)
    ep = goal - CP[:, tool]
    ep = ep / np.maximum(1.0, np.linalg.norm(ep, axis=1, keepdims=True) / 0.05)     # at most 5 cm per step
    chain = RS._chain(A, tool)
    cols = [[k for k in chain if A['rl_dof'][k] == d][0] for d in arm]
    J = np.zeros((N, 3, 7))
    for c, l in enumerate(cols):
        J[:, :, c] = RS._cross(AX[:, l], CP[:, tool] - OR[:, l])
    JJ = J @ np.transpose(J, (0, 2, 1)) + 1e-3 * np.eye(3)[None]
    dq = (np.transpose(J, (0, 2, 1)) @ np.linalg.solve(JJ, ep[..., None]))[..., 0]
    # take_step: the target moves 5 x clip(a) x 0.05 per env step
    return np.clip(gain * dq / 0.25, -1, 1).astype(np.float32)
