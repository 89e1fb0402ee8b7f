"""BedBathingPR2 test helpers: wiping contact states -- the PR2's arm solved by IK (the reset's DLS
restatement) so that the cloth (tool link 1) lies on an upward-facing upper-arm target, pressed in
by `depth`, its face along the arm's surface normal there."""
import numpy as np

from avr import _abi as ABI
from avr import geom as G
from avr import reset_bedbath as RBB
from avr import reset_scratch as RSS

BB = ABI.BB


def _frame_z(n, x_hint):
    """Rotation (quaternion) whose z axis is n, x axis the projection of x_hint."""
    z = n / np.linalg.norm(n)
    x = x_hint - np.dot(x_hint, z) * z
    if np.linalg.norm(x) < 1e-6:
        x = np.cross(z, [1.0, 0, 0]) if abs(z[0]) < 0.9 else np.cross(z, [0, 1.0, 0])
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    from scipy.spatial.transform import Rotation
    return Rotation.from_matrix(np.stack([x, y, z], 1)).as_quat()


def wipe_states(A, md, S, depth=0.002, tries=12, strict=True):
    """Copy of S with every env's left arm re-solved so the cloth presses on an upper-arm target;
    returns (states, target index per env).  strict=False drops the envs whose base pose reaches
    none of the `tries` upward-facing targets (strict: an assertion)."""
    S = S.copy()
    nd = int(A['n_dof'])
    arm = np.array(md.arm_dofs)
    lo = np.array([md.desc.arm_lower[i] if md.desc.arm_lower[i] > -1e9 else -2 * np.pi for i in range(len(arm))])
    hi = np.array([md.desc.arm_upper[i] if md.desc.arm_upper[i] < 1e9 else 2 * np.pi for i in range(len(arm))])
    link = int(A['task_tool_link'])
    tip, piv = A['task_tool_tip'], A['task_tool_pivot']
    ks, keep = [], []
    for e in range(len(S)):
        st = S[e]
        g = int(st[BB.S_TASK + BB.T_GENDER])
        ls = int(A['bb_limb_slots'][0])
        lp = st[BB.S_HUMAN + 7 * ls:BB.S_HUMAN + 7 * ls + 7]
        R = G.quat_to_mat(lp[3:])
        nu = int(A['bb_ntgt'][g][0])
        T = A['bb_targets'][g][:nu, :3]
        nrm = (R @ np.concatenate([T[:, :2], np.zeros((nu, 1))], 1).T).T
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        order = np.argsort(-nrm[:, 2])            # facing up first
        bp, bq = st[BB.S_RBASE:BB.S_RBASE + 3][None], st[BB.S_RBASE + 3:BB.S_RBASE + 7][None]
        tb = st[BB.S_FREE:BB.S_FREE + 7]
        xh = G.quat_rotate(tb[3:], [1.0, 0, 0])
        best = None
        for k in order[:tries]:
            tw = lp[:3] + R @ T[k]
            n = nrm[k]
            cq = _frame_z(n, xh)
            cc = tw + n * (0.0025 - depth)
            body_p = cc - G.quat_rotate(cq, tip)
            tp = body_p + G.quat_rotate(cq, piv)
            Q0 = st[BB.S_Q:BB.S_Q + nd][None].copy()
            Q, CP, CQ, _, _ = RSS.ik_dls(A, link, Q0, bp, bq, tp[None], cq[None], arm, lo, hi, 400)
            pe = np.linalg.norm(CP[0, link] - tp)
            qe = min(np.linalg.norm(CQ[0, link] - cq), np.linalg.norm(CQ[0, link] + cq))
            if pe < 1e-3 and qe < 1e-2:
                best = (k, Q[0], CP[0, link], CQ[0, link])
                break
        if best is None and not strict:
            continue
        assert best is not None, 'env %d: no upper-arm target reachable' % e
        keep.append(e)
        k, q, cp, cq = best
        st[BB.S_Q:BB.S_Q + nd] = q
        st[BB.S_QD:BB.S_QD + nd] = 0
        for d in arm:
            st[BB.S_QTGT + d] = q[d]
        p, qq = RBB._tool_pose(A, cp, cq)
        st[BB.S_FREE:BB.S_FREE + 3] = p
        st[BB.S_FREE + 3:BB.S_FREE + 7] = qq
        st[BB.S_FREE + 7:BB.S_FREE + 13] = 0
        ks.append(int(k))
    return S[keep], ks
