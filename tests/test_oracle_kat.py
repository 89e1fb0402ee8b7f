"""Known-answer tests pinning the CPU oracle (oracle/avr_oracle.c, TEST INFRASTRUCTURE).

PyBullet is absent from this image, so the oracle cannot be checked against the
reference's own outputs: these tests pin it against closed forms and against independent
brute-force computations of the Bullet semantics it restates.
"""
import numpy as np
import pytest
from scipy.spatial import ConvexHull

from avr import _abi as ABI
from avr import geom as G
from avr import reset as RS

IDENT = np.array([0, 0, 0, 0, 0, 0, 1.0])


@pytest.fixture(scope='module')
def orc(scene, oracle_built):
    from oracle.oracle import Oracle
    A, md = scene
    o = Oracle(md, 1)
    return o


def shape_of(A, body, kind):
    s0, c = A['body_shape_start'][body], A['body_shape_count'][body]
    for s in range(s0, s0 + c):
        if A['shape_kind'][s] == kind:
            return s
    raise LookupError


def hull_world(A, s):
    vs, vc = A['shape_hull'][s][:2]
    V = A['hull_verts'][vs:vs + vc]
    p, q = A['shape_pose'][s][:3], A['shape_pose'][s][3:7]
    R = G.quat_to_mat(q)
    return V @ R.T + p


def point_triangle_dist(P, T):
    """distance from point P to each triangle T[k] (3x3), Ericson-style region tests."""
    a, b, c = T[:, 0], T[:, 1], T[:, 2]
    ab, ac, ap = b - a, c - a, P - a
    d1, d2 = (ab * ap).sum(1), (ac * ap).sum(1)
    bp = P - b
    d3, d4 = (ab * bp).sum(1), (ac * bp).sum(1)
    cp = P - c
    d5, d6 = (ab * cp).sum(1), (ac * cp).sum(1)
    va = d3 * d6 - d5 * d4
    vb = d5 * d2 - d1 * d6
    vc = d1 * d4 - d3 * d2
    out = np.empty(len(T))
    for k in range(len(T)):
        if d1[k] <= 0 and d2[k] <= 0:
            q = a[k]
        elif d3[k] >= 0 and d4[k] <= d3[k]:
            q = b[k]
        elif vc[k] <= 0 and d1[k] >= 0 and d3[k] <= 0:
            q = a[k] + d1[k] / (d1[k] - d3[k]) * ab[k]
        elif d6[k] >= 0 and d5[k] <= d6[k]:
            q = c[k]
        elif vb[k] <= 0 and d2[k] >= 0 and d6[k] <= 0:
            q = a[k] + d2[k] / (d2[k] - d6[k]) * ac[k]
        elif va[k] <= 0 and (d4[k] - d3[k]) >= 0 and (d5[k] - d6[k]) >= 0:
            w = (d4[k] - d3[k]) / ((d4[k] - d3[k]) + (d5[k] - d6[k]))
            q = b[k] + w * (c[k] - b[k])
        else:
            den = 1.0 / (va[k] + vb[k] + vc[k])
            q = a[k] + ab[k] * vb[k] * den + ac[k] * vc[k] * den
        out[k] = np.linalg.norm(P - q)
    return out


def signed_dist_to_hull(P, V):
    h = ConvexHull(V)
    inside = np.all(h.equations[:, :3] @ P + h.equations[:, 3] <= 0)
    if inside:
        return -np.min(-(h.equations[:, :3] @ P + h.equations[:, 3]))
    return point_triangle_dist(P, V[h.simplices]).min()


# ----------------------------------------------------------------------------- narrowphase
def test_sphere_sphere_closed_form(scene, orc):
    A, _ = scene
    s = shape_of(A, int(A['task_food_body0']), 0)
    r = A['shape_param'][s][0]
    pa = IDENT.copy(); pb = IDENT.copy()
    pb[:3] = [0.003, 0.004, 2 * r + 0.001 - 0.005]      # |d| = 0.001 + 2r - 0.005 + ...
    hit, out = orc.narrowphase(s, pa, s, pb, 0.02)
    l = np.linalg.norm(pb[:3])
    assert hit
    assert out[6] == pytest.approx(l - 2 * r, abs=1e-12)
    assert np.allclose(out[:3], (pa[:3] - pb[:3]) / l, atol=1e-12)                  # normal on B, B -> A
    assert np.allclose(out[3:6], pb[:3] + out[:3] * r, atol=1e-12)                  # point on B
    pb[:3] = [0, 0, 2 * r + 0.05]
    hit, _ = orc.narrowphase(s, pa, s, pb, 0.02)
    assert not hit


def test_sphere_box_face_region(scene, orc):
    A, _ = scene
    sf = shape_of(A, int(A['task_food_body0']), 0)
    sb = shape_of(A, int(A['task_table_body']), 2)
    r = A['shape_param'][sf][0]
    top = A['shape_pose'][sb][2] + A['shape_param'][sb][2]
    for gap in (0.003, -0.002):
        pa = IDENT.copy(); pa[:3] = [0.1, -0.05, top + r + gap]
        hit, out = orc.narrowphase(sf, pa, sb, IDENT, 0.02)
        assert hit
        assert out[6] == pytest.approx(gap, abs=1e-12)
        assert np.allclose(out[:3], [0, 0, 1], atol=1e-12)
        assert out[5] == pytest.approx(top, abs=1e-12)


def test_sphere_capsule_closed_form(scene, orc):
    A, _ = scene
    sf = shape_of(A, int(A['task_food_body0']), 0)
    sc = int(np.nonzero(A['shape_kind'] == 1)[0][0])
    rs = A['shape_param'][sf][0]
    rc, hh = A['shape_param'][sc][:2]
    pc = IDENT.copy()
    q = G.quat_from_euler([0.3, -0.2, 0.5]); pc[3:] = q
    pose_c = G.tf_mul(pc[:3], pc[3:], A['shape_pose'][sc][:3], A['shape_pose'][sc][3:7])
    axis = G.quat_to_mat(pose_c[1])[:, 2]
    # point beside the segment (side region) and beyond the end cap
    for t, side, gap in ((0.3, np.array([1.0, 0.2, 0.0]), 0.004), (1.6, np.array([0.0, 0.0, 1.0]), 0.006)):
        side = side - axis * (side @ axis)
        side = side / np.linalg.norm(side) if np.linalg.norm(side) > 0 else axis
        seg_pt = pose_c[0] + axis * hh * min(t, 1.0)
        d_dir = side if t <= 1 else axis
        P = seg_pt + d_dir * (rc + rs + gap)
        pa = IDENT.copy(); pa[:3] = P
        # reference: distance from P to the segment minus radii
        a0, a1 = pose_c[0] - axis * hh, pose_c[0] + axis * hh
        u = np.clip((P - a0) @ (a1 - a0) / ((a1 - a0) @ (a1 - a0)), 0, 1)
        want = np.linalg.norm(P - (a0 + u * (a1 - a0))) - rc - rs
        hit, out = orc.narrowphase(sf, pa, sc, pc, 0.05)
        assert hit
        assert out[6] == pytest.approx(want, abs=1e-10)


@pytest.mark.parametrize('offset', [0.004, 0.012, -0.0015, -0.0075])
def test_hull_sphere_gjk_epa_vs_bruteforce(scene, orc, offset):
    """GJK (separated) and EPA (penetrating) against an exact point-to-polytope distance."""
    A, _ = scene
    sf = shape_of(A, int(A['task_food_body0']), 0)
    r = A['shape_param'][sf][0]
    rng = np.random.default_rng(3)
    spoon = int(A['task_spoon_body'])
    s0, c = A['body_shape_start'][spoon], A['body_shape_count'][spoon]
    checked = 0
    for s in rng.choice(np.arange(s0, s0 + c), 6, replace=False):
        V = hull_world(A, s)
        if len(V) < 4:
            continue
        mh = A['shape_margin'][s]
        h = ConvexHull(V)
        # a point at a known offset outside (or inside) the hull along a facet normal
        k = rng.integers(len(h.simplices))
        n = h.equations[k, :3]
        ctr = V[h.simplices[k]].mean(0)
        P = ctr + n * (offset + mh + r)
        want = signed_dist_to_hull(P, V) - mh - r
        pa = IDENT.copy(); pa[:3] = P
        hit, out = orc.narrowphase(sf, pa, s, IDENT, 0.05)
        assert hit
        assert out[6] == pytest.approx(want, abs=2e-5), (s, offset)
        checked += 1
    assert checked >= 3


# ----------------------------------------------------------------------------- kinematics
def test_fk_matches_independent_numpy_fk(scene, orc):
    A, md = scene
    S, _ = RS.batch_reset_states_fast(A, md, 1001, [5])
    orc.set_state(S)
    out = orc.robot_fk(0)
    _, _, CP, CQ, _, _ = RS.robot_fk(A, S[0, ABI.S_Q:ABI.S_Q + int(A['n_dof'])])
    assert np.allclose(out[:, :3], CP, atol=1e-12)
    dots = np.abs((out[:, 3:] * CQ).sum(1))
    assert np.allclose(dots, 1.0, atol=1e-12)


# ----------------------------------------------------------------------------- dynamics
def _one_env_state(scene):
    A, md = scene
    S, _ = RS.batch_reset_states_fast(A, md, 1001, [0])
    return A, md, S


def test_free_fall_matches_damped_recurrence(scene, oracle_built):
    """A contact-free food particle follows v' = v + dt (g - v (k + k|v|)), p' = p + dt v'
    (Bullet's default multibody damping k = 0.04, Appendix A.5; semi-implicit Euler A.1)."""
    from oracle.oracle import Oracle
    A, md, S = _one_env_state(scene)
    f = ABI.S_FREE + ABI.FB_WORDS * 2                   # food 0
    S[0, f:f + 3] = [0.0, 5.0, 50.0]
    S[0, f + 3:f + 7] = [0, 0, 0, 1]
    S[0, f + 7:f + 13] = 0
    o = Oracle(md, 1)
    o.set_state(S)
    dt, k, g = 0.01, ABI.FEEDING_PARAMS['linear_damping'], np.array([0, 0, -9.81])
    p, v = S[0, f:f + 3].copy(), np.zeros(3)
    for _ in range(60):
        o.substep(dt)
        v = v + dt * (g - v * (k + k * np.linalg.norm(v)))
        p = p + dt * v
    St = o.get_state()[0]
    assert np.allclose(St[f + 7:f + 10], v, atol=1e-12)
    assert np.allclose(St[f:f + 3], p, atol=1e-12)


def test_particle_comes_to_rest_on_table(scene, oracle_built):
    from oracle.oracle import Oracle
    A, md, S = _one_env_state(scene)
    sb = shape_of(A, int(A['task_table_body']), 2)
    top = A['st_pose'][2][2] + A['shape_pose'][sb][2] + A['shape_param'][sb][2]
    r = 0.005
    f = ABI.S_FREE + ABI.FB_WORDS * 3                   # food 1, placed on the table's far side
    S[0, f:f + 3] = [0.35 + 0.6, -0.9 - 0.4, top + r + 0.002]
    S[0, f + 3:f + 7] = [0, 0, 0, 1]
    S[0, f + 7:f + 13] = 0
    o = Oracle(md, 1)
    o.set_state(S)
    for _ in range(300):
        o.substep(0.01)
    St = o.get_state()[0]
    z = St[f + 2]
    assert top + r - 2e-3 < z < top + r + 1e-4
    assert np.linalg.norm(St[f + 7:f + 10]) < 1e-3
    assert abs(St[f] - (0.35 + 0.6)) < 1e-3 and abs(St[f + 1] - (-0.9 - 0.4)) < 1e-3


def test_oracle_is_deterministic_and_thread_invariant(scene, oracle_built):
    from oracle.oracle import Oracle
    from avr import _lib
    A, md = scene
    S, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(4)))
    outs = []
    for th in (1, 4):
        o = Oracle(md, 4)
        o.set_threads(th)
        o.set_state(S)
        o.settle(5)
        for t in range(2):
            o.step(_lib.random_actions(1001, np.arange(4), t))
        outs.append(o.get_state())
    assert np.array_equal(outs[0], outs[1])


# ----------------------------------------------------------------------------- tremor head chain
def test_tremor_head_chain_fk_matches_host_fk(scene, oracle_built):
    """The oracle's head chain (4 links appended to the robot, root on the chest slot) publishes
    the neck / head poses of the host's full 42-joint human FK (reset.human_slot_poses)."""
    from oracle.oracle import Oracle
    A, md = scene
    env = 9
    S, meta = RS.batch_reset_states_fast(A, md, 1001, [env], impairment='tremor')
    g = meta[0]['gender']
    rng = RS._rng(1001, env)
    rng.integers(2)                                     # the gender draw
    qh = RS.human_joint_angles(A, g, rng, 1.0)
    assert np.allclose(S[0, md.n_dof:md.n_dof + 4], qh[24:28])
    dq = np.array([0.05, -0.2, 0.15, 0.3])
    qh[24:28] += dq
    S[0, md.n_dof:md.n_dof + 4] += dq
    o = Oracle(md, 1)
    o.set_state(S)
    o.robot_fk(0)
    St = o.get_state()[0]
    want = RS.human_slot_poses(A, g, qh)
    checked = 0
    for slot in A['hc_slot']:
        if slot < 0:
            continue
        got = St[ABI.S_HUMAN + 7 * slot:ABI.S_HUMAN + 7 * slot + 7]
        assert np.allclose(got[:3], want[slot][:3], atol=1e-12)
        assert abs(abs(np.dot(got[3:], want[slot][3:])) - 1) < 1e-12
        checked += 1
    assert checked == 2                                 # neck capsule, head mesh


def test_tremor_targets_alternate_and_hard_limits_hold(scene, oracle_built):
    """take_step tremor targets (env.py:330-331) and enforce_hard_human_joint_limits
    (env.py:389-410): a neck pushed 0.05 rad past its upper limit is back within limits after
    the first frame and stays there."""
    from oracle.oracle import Oracle
    from avr import _lib
    A, md = scene
    nd = md.n_dof
    S, _ = RS.batch_reset_states_fast(A, md, 1001, [11, 12], impairment='tremor')
    S[:, nd] = A['hc_upper'][0] + 0.05
    o = Oracle(md, 2)
    o.set_state(S)
    moved = 0.0
    for t in range(3):
        o.step(_lib.random_actions(1001, np.arange(2), t))
        St = o.get_state()
        sg = 1.0 if t % 2 == 0 else -1.0
        want = S[:, ABI.S_HCH:ABI.S_HCH + 4] + sg * S[:, ABI.S_HCH + 4:ABI.S_HCH + 8]
        assert np.allclose(St[:, ABI.S_QTGT + nd:ABI.S_QTGT + nd + 4], want, atol=1e-12)
        assert np.all(St[:, ABI.S_KP + nd:ABI.S_KP + nd + 4] == ABI.FEEDING_PARAMS['human_gain'])
        q = St[:, nd:nd + 4]
        assert np.all(q <= A['hc_upper'] + 1e-12) and np.all(q >= A['hc_lower'] - 1e-12)
        moved = max(moved, np.abs(q[:, 1:] - S[:, nd + 1:nd + 4]).max())
    assert moved > 1e-3                                 # the motors do shake the head


def test_static_human_views_ignore_the_chain(scene, oracle_built):
    """Without 'tremor' the chain DoFs, targets and head pose are untouched by a step."""
    from oracle.oracle import Oracle
    from avr import _lib
    A, md = scene
    nd = md.n_dof
    S, _ = RS.batch_reset_states_fast(A, md, 1001, [0, 1], impairment='weakness')
    o = Oracle(md, 2)
    o.set_state(S)
    o.step(_lib.random_actions(1001, np.arange(2), 0))
    St = o.get_state()
    assert np.all(St[:, nd:nd + 4] == 0) and np.all(St[:, ABI.S_HCH:ABI.S_CP] == 0)
    h = slice(ABI.S_HUMAN, ABI.S_HCH)
    assert np.array_equal(St[:, h], S[:, h])


# ----------------------------------------------------------------------------- dynamics KATs
# (SURVEY 7 "KATs that need no PyBullet"; synthetic chains from tests/kat_scene.py)
def _run(md, S, n, dt):
    from oracle.oracle import Oracle
    o = Oracle(md, 1)
    o.set_state(S)
    out = []
    for _ in range(n):
        o.substep(dt)
        out.append(o.get_state()[0].copy())
    return np.array(out)


def test_motor_row_closed_form(oracle_built):
    """POSITION_CONTROL motor (btMultiBodyJointMotor): the row's target velocity is
    kp (q* - q) / dt and, unsaturated and alone, the solve meets it exactly, so
    q_{n+1} - q* = (1 - kp) (q_n - q*): geometric convergence at rate kp per sub-step."""
    import kat_scene as K
    A = K.chain_scene([dict(parent=-1, axis=[0, 0, 1], jpos=[0, 0, 0], com_pos=[0.3, 0, 0], mass=2.0, inertia=[0.01, 0.02, 0.03])])
    md = K.desc(A)
    kp, q0, qs, dt = 0.1, 0.2, 1.0, 0.01
    St = _run(md, K.state(md, [q0], kp=[kp], target=[qs], maximp=[1e6]), 40, dt)
    q = St[:, ABI.S_Q]
    want = qs + (q0 - qs) * (1 - kp) ** np.arange(1, 41)
    assert np.allclose(q, want, rtol=0, atol=1e-12)
    assert np.allclose(St[:, ABI.S_QD], kp * (np.concatenate([[q0], want[:-1]]) - qs) * -1 / dt, atol=1e-9)


def test_motor_impulse_cap(oracle_built):
    """A saturated motor applies at most its max impulse per sub-step: the joint's velocity grows by
    maximp / I_axis (I_axis = m r^2 + I_zz about the joint) per sub-step while far from target."""
    import kat_scene as K
    m, r, izz = 2.0, 0.3, 0.03
    A = K.chain_scene([dict(parent=-1, axis=[0, 0, 1], jpos=[0, 0, 0], com_pos=[r, 0, 0], mass=m, inertia=[0.01, 0.02, izz])])
    md = K.desc(A)
    imp, dt = 1e-3, 0.01
    St = _run(md, K.state(md, [0.0], kp=[0.1], target=[100.0], maximp=[imp]), 10, dt)
    Ia = m * r * r + izz
    assert np.allclose(St[:, ABI.S_QD], imp / Ia * np.arange(1, 11), rtol=1e-9)


def test_pendulum_small_angle_period(oracle_built):
    """Compound pendulum (point-like bob, no damping, motors off) released at 0.02 rad: its period
    is 2 pi sqrt(I / (m g r)) to within the time step (semi-implicit Euler)."""
    import kat_scene as K
    m, r = 1.0, 0.5
    A = K.chain_scene([dict(parent=-1, axis=[1, 0, 0], jpos=[0, 0, 1], com_pos=[0, 0, -r], mass=m, inertia=[1e-6, 1e-6, 1e-6])])
    md = K.desc(A, robot_gravity=(0.0, 0.0, -9.81))
    dt = 1e-3
    St = _run(md, K.state(md, [0.02]), 4000, dt)
    q = St[:, ABI.S_Q]
    up = np.nonzero((q[:-1] < 0) & (q[1:] >= 0))[0]          # upward zero crossings
    T = np.diff(up).mean() * dt
    want = 2 * np.pi * np.sqrt((m * r * r + 1e-6) / (m * 9.81 * r))
    assert abs(T - want) < 2 * dt, (T, want)
    assert np.abs(q).max() < 0.0201                           # amplitude kept (no damping)


def test_double_pendulum_energy_drift(oracle_built):
    """Frictionless double pendulum from 1 rad / 0.5 rad over 2 s: the total energy -- kinetic
    and potential from an independent planar model of the same chain -- deviates by O(dt) only
    (semi-implicit Euler; measured 0.66 % at dt 1e-3), halving with dt.  A mass-matrix or bias-force
    error would leave a deviation that does not vanish with dt."""
    import kat_scene as K
    m1, m2, l1, l2 = 1.0, 0.7, 0.4, 0.3
    links = [dict(parent=-1, axis=[1, 0, 0], jpos=[0, 0, 1], com_pos=[0, 0, -l1], mass=m1, inertia=[1e-3, 1e-3, 1e-3]),
             dict(parent=0, axis=[1, 0, 0], jpos=[0, 0, -l1], com_pos=[0, 0, -l2], mass=m2, inertia=[1e-3, 1e-3, 1e-3])]
    A = K.chain_scene(links)
    md = K.desc(A, robot_gravity=(0.0, 0.0, -9.81))

    def energy(q, qd):
        # planar in y-z; link 1's COM is also joint 2 (jpos l1); R_x(a) (0, 0, -l) = (0, l sin a, -l cos a)
        a1, a2 = q[0], q[0] + q[1]
        c1 = np.array([np.sin(a1) * l1, -np.cos(a1) * l1])
        c2 = c1 + np.array([np.sin(a2) * l2, -np.cos(a2) * l2])
        w1, w2 = qd[0], qd[0] + qd[1]
        v1 = w1 * np.array([np.cos(a1), np.sin(a1)]) * l1
        v2 = v1 + w2 * np.array([np.cos(a2), np.sin(a2)]) * l2
        T = 0.5 * m1 * v1 @ v1 + 0.5 * m2 * v2 @ v2 + 0.5 * 1e-3 * (w1 * w1 + w2 * w2)
        return T + 9.81 * (m1 * c1[1] + m2 * c2[1])

    E0 = energy(np.array([1.0, 0.5]), np.zeros(2))
    errs = []
    for dt in (1e-3, 5e-4):
        St = _run(md, K.state(md, [1.0, 0.5]), int(round(2.0 / dt)), dt)
        errs.append(max(abs(energy(s[ABI.S_Q:ABI.S_Q + 2], s[ABI.S_QD:ABI.S_QD + 2]) - E0) for s in St))
    assert errs[0] < 1e-2 * abs(E0), errs
    assert 0.45 < errs[1] / errs[0] < 0.55, errs


def test_torque_free_body_keeps_angular_momentum(oracle_built):
    """A free body with distinct principal inertias spinning about a near-principal axis, no
    gravity, no damping: its world angular momentum R I R^T w is conserved to 1e-3 over 1 s at
    dt 1e-3 (explicit gyroscopic term)."""
    import kat_scene as K
    I = np.array([0.01, 0.02, 0.03])
    A = K.chain_scene([dict(parent=-1, axis=[0, 0, 1], jpos=[0, 0, 0], com_pos=[0, 0, 0], mass=1.0, inertia=[1e-3, 1e-3, 1e-3])],
                      free_inertia=I, free_mass=1.0)
    md = K.desc(A)
    S = K.state(md, [0.0])
    f = ABI.S_FREE
    S[0, f + 10:f + 13] = [3.0, 0.2, 0.1]
    St = _run(md, S, 1000, 1e-3)

    def L(s):
        Rm = G.quat_to_mat(s[f + 3:f + 7])
        return Rm @ (I * (Rm.T @ s[f + 10:f + 13]))

    L0 = I * np.array([3.0, 0.2, 0.1])
    drift = max(np.linalg.norm(L(s) - L0) for s in St)
    assert drift < 1e-3 * np.linalg.norm(L0), drift
    assert np.allclose(St[-1, f:f + 3], [100, 100, 100], atol=1e-12)     # no linear motion


def test_resting_sphere_normal_force_is_weight(scene, oracle_built):
    """A food sphere at rest on the table (SURVEY 7 'normal force = mg'): the normal impulses of
    its contact points sum to m g dt per sub-step (getContactPoints normalForce = impulse / dt)."""
    from oracle.oracle import Oracle
    A, md, S = _one_env_state(scene)
    sb = shape_of(A, int(A['task_table_body']), 2)
    top = A['st_pose'][2][2] + A['shape_pose'][sb][2] + A['shape_param'][sb][2]
    f = ABI.S_FREE + ABI.FB_WORDS * 3
    S[0, f:f + 3] = [0.35 + 0.6, -0.9 - 0.4, top + 0.005 + 0.001]
    S[0, f + 3:f + 7] = [0, 0, 0, 1]
    S[0, f + 7:f + 13] = 0
    o = Oracle(md, 1)
    o.set_state(S)
    dt = 0.01
    for _ in range(300):
        o.substep(dt)
    St = o.get_state()[0]
    food_body = int(A['task_food_body0']) + 1
    imp = 0.0
    for k in range(int(St[ABI.S_TASK + ABI.T_NCP])):
        c = St[ABI.S_CP + ABI.CP_WORDS * k:][:ABI.CP_WORDS]
        if food_body in (A['shape_body'][int(c[ABI.CP_SA])], A['shape_body'][int(c[ABI.CP_SB])]):
            imp += c[ABI.CP_IMP]
    assert imp / dt == pytest.approx(0.001 * 9.81, rel=2e-2)


# ----------------------------------------------------------------------------- torsional friction KATs
def _rolling_scene(scene, rolling=0.0, spinning=0.0):
    """FeedingJaco's scene with rolling / spinning friction on the table (the combined coefficient
    of a food sphere on it is table_coeff x food friction 0.5 + food_coeff 0 x table friction,
    btManifoldResult [ext]); no damping, 50 solver iterations (a converged solve of the
    one-point contact)."""
    A, md = scene
    A = dict(A)
    tb = int(A['task_table_body'])
    A['body_rolling'] = np.zeros(len(A['body_kind'])); A['body_rolling'][tb] = rolling
    A['body_spinning'] = np.zeros(len(A['body_kind'])); A['body_spinning'][tb] = spinning
    return A, ABI.ModelDesc(A, dict(linear_damping=0.0, angular_damping=0.0, solver_iterations=50))


def _sphere_on_table(scene, A, md, v, w):
    """Food sphere 1 resting on the table's far side (settled for 100 sub-steps), then given
    linear velocity v and angular velocity w."""
    from oracle.oracle import Oracle
    _, _, S = _one_env_state(scene)
    sb = shape_of(A, int(A['task_table_body']), 2)
    top = A['st_pose'][2][2] + A['shape_pose'][sb][2] + A['shape_param'][sb][2]
    f = ABI.S_FREE + ABI.FB_WORDS * 3
    S[0, f:f + 3] = [0.35 + 0.5, -0.9 - 0.4, top + 0.005 + 0.001]
    S[0, f + 3:f + 7] = [0, 0, 0, 1]
    S[0, f + 7:f + 13] = 0
    o = Oracle(md, 1)
    o.set_state(S)
    for _ in range(100):
        o.substep(0.01)
    S = o.get_state()
    S[0, f + 7:f + 10] = v
    S[0, f + 10:f + 13] = w
    o.set_state(S)
    return o, f


def test_rolling_friction_decelerates_a_rolling_sphere(scene, oracle_built):
    """A sphere rolling without slipping on a plane with rolling friction mu_r (btMultiBody torsional
    rows about the contact's tangent axes, limit mu_r x normal impulse [ext]): the rolling
    resistance torque mu_r m g against no-slip gives a = -mu_r g / (r (1 + I / (m r^2))) =
    -mu_r g / (1.4 r).  Without rolling friction the sphere keeps rolling (no damping here)."""
    r, g, dt = 0.005, 9.81, 0.01
    mu_r = 1e-4                                  # table 2e-4 x food friction 0.5
    v0 = 0.2
    for rolling, want in ((0.0, 0.0), (2e-4, -mu_r * g / (1.4 * r))):
        A, md = _rolling_scene(scene, rolling=rolling)
        o, f = _sphere_on_table(scene, A, md, [v0, 0, 0], [0, v0 / r, 0])
        vs = []
        for _ in range(40):
            o.substep(dt)
            vs.append(o.get_state()[0, f + 7])
        vs = np.array(vs)
        a = np.polyfit(np.arange(1, 41) * dt, vs, 1)[0]
        assert a == pytest.approx(want, abs=0.02 * abs(-mu_r * g / (1.4 * r))), (rolling, a, want)
        St = o.get_state()[0]
        assert abs(St[f + 7] - St[f + 11] * r) < 1e-3 * v0         # still rolling without slipping


def test_spinning_friction_torque_is_bounded_by_mu_n(scene, oracle_built):
    """A sphere spinning about the contact normal with spinning friction mu_s: the torsional row
    about the normal saturates at mu_s x the normal impulse, so the spin decays linearly at
    mu_s m g / I_zz (torque bounded by mu_spin N); without spinning friction it keeps spinning."""
    m, r, g, dt = 0.001, 0.005, 9.81, 0.01
    I = 0.4 * m * r * r
    mu_s = 1e-5                                   # table 2e-5 x food friction 0.5
    w0 = 5.0
    for spinning, want in ((0.0, 0.0), (2e-5, -mu_s * m * g / I)):
        A, md = _rolling_scene(scene, spinning=spinning)
        o, f = _sphere_on_table(scene, A, md, [0, 0, 0], [0, 0, w0])
        ws = []
        for _ in range(20):
            o.substep(dt)
            ws.append(o.get_state()[0, f + 12])
        alpha = np.polyfit(np.arange(1, 21) * dt, np.array(ws), 1)[0]
        assert alpha == pytest.approx(want, abs=0.02 * mu_s * m * g / I), (spinning, alpha, want)
        assert np.all(np.array(ws) > 0)


# ----------------------------------------------------------------------------- solver residual threshold
def test_pgs_stops_at_the_residual_threshold(oracle_built):
    """PyBullet's solverResidualThreshold (1e-7 on the largest squared row residual of a PGS
    iteration, [ext]): one unsaturated motor row alone (the chain scene's weld rows have max force 0)
    is met exactly by the first iteration, so the second changes nothing and the solve stops there:
    2 iterations of the 10 allowed, every sub-step, and the motor's closed form still holds."""
    import kat_scene as K
    from oracle.oracle import Oracle
    A = K.chain_scene([dict(parent=-1, axis=[0, 0, 1], jpos=[0, 0, 0], com_pos=[0.3, 0, 0], mass=2.0, inertia=[0.01, 0.02, 0.03])])
    md = K.desc(A)
    kp, q0, qs, dt = 0.1, 0.2, 1.0, 0.01
    o = Oracle(md, 1)
    o.set_state(K.state(md, [q0], kp=[kp], target=[qs], maximp=[1e6]))
    for _ in range(20):
        o.substep(dt)
    st = o.stats()
    assert st[4] == 20 and st[3] == 2 * 20, st
    assert o.get_state()[0, ABI.S_Q] == pytest.approx(qs + (q0 - qs) * (1 - kp) ** 20, abs=1e-12)


def test_pgs_iterations_used_per_task(scene, oracle_built):
    """How many of their PGS iterations the tasks' solves use under the residual threshold: the
    PR2 tasks' reset states (arm in free space, 50 allowed) stop well before 50; FeedingJaco's food
    pile in the spoon never converges to 1e-7 within its 10 (measured: every solve runs all 10)."""
    from oracle.oracle import Oracle
    from avr import _lib
    import scratch_util as U
    A, md = U.scene()
    S, _ = U.reset_states(A, md, range(4))
    o = Oracle(md, 4)
    o.set_state(S.astype(np.float64))
    for t in range(5):
        o.step(_lib.random_actions(1001, np.arange(4), t))
    st = o.stats()
    print('ScratchItchPR2: %.1f iterations per solve of 50' % (st[3] / st[4]))
    assert st[4] == 4 * 5 * 5 and st[3] / st[4] < 25
    A, md, S = _one_env_state(scene)
    o = Oracle(md, 1)
    o.set_state(S)
    o.settle(20)
    s0 = o.stats()
    o.step(_lib.random_actions(1001, np.arange(1), 0))
    st = o.stats() - s0
    print('FeedingJaco: %.1f iterations per solve of 10' % (st[3] / st[4]))
    assert st[4] == 10 and st[3] <= 10 * 10


def _pr2_contact_pool(task):
    """Reset and contact states of a PR2 task on the CPU (BedBathing's arm settle on the oracle)."""
    from oracle.oracle import Oracle
    if task == ABI.TASK_SCRATCH:
        import scratch_util as U
        A, md = U.scene()
        S, meta = U.reset_states(A, md, range(16))
        C = U.contact_states(A, md, S, meta)
    else:
        import bedbath_util as U
        from avr import reset_bedbath as RBB
        A = ABI.load_scene(ABI.TASK_BEDBATH)
        md = ABI.ModelDesc(A)

        def run(S, frames):
            o = Oracle(md, len(S))
            o.set_state(S)
            o.settle(frames)
            return o.get_state()
        settled = RBB.settled_arms(A, md, runner=run)
        S, _ = RBB.batch_reset_states(A, md, 1001, list(range(8)), attempts=6, iters=60, settled=settled)
        C, _ = U.wipe_states(A, md, S, strict=False)
    return A, md, np.concatenate([S, C]).astype(np.float64)


@pytest.mark.parametrize('task', [ABI.TASK_SCRATCH, ABI.TASK_BEDBATH], ids=['ScratchItchPR2', 'BedBathingPR2'])
def test_pgs_exit_per_env_vs_per_island(task, oracle_built):
    """The build leaves the PGS when the whole env has converged (one solve group per env, DESIGN
    section 8); Bullet checks the residual per solve group, and splits islands into groups of at least
    minimumSolverBatchSize rows ([ext], not pinned by the reference).  The oracle's island variant
    (avr_oracle_set_island_exit: each island -- robot, human chain, each free body and what rows
    connect them -- leaves on its own residual) bounds what the assumption moves: reset and contact
    states, 5 gym steps of small random actions, both variants from the same states.  Measured
    (ScratchItch): joint angles within 8e-5 rad, velocities 7e-4 rad/s, rewards 4e-5 -- an order of
    magnitude inside the 1e-3 rad parity tolerance; BedBathing: identical (its wiping states form
    one island: the wiper welded to the gripper, pressed on the arm)."""
    from oracle.oracle import Oracle
    from avr import _lib
    A, md, P = _pr2_contact_pool(task)
    L = ABI.LAYOUTS[task]
    n = len(P)
    nd = md.n_dof + int(A['hc_n'])
    runs = []
    for island in (False, True):
        o = Oracle(md, n)
        o.set_threads(8)
        o.set_state(P)
        o.set_island_exit(island)
        traj = []
        for t in range(5):
            _, r, _, _ = o.step(_lib.random_actions(1001, np.arange(n), t) * 0.2)
            traj.append((o.get_state(), r))
        runs.append((traj, o.stats()))
    dq = max(float(np.abs(a[0][:, :nd] - b[0][:, :nd]).max()) for a, b in zip(runs[0][0], runs[1][0]))
    dqd = max(float(np.abs(a[0][:, L.S_QD:L.S_QD + nd] - b[0][:, L.S_QD:L.S_QD + nd]).max()) for a, b in zip(runs[0][0], runs[1][0]))
    drew = max(float(np.abs(a[1] - b[1]).max()) for a, b in zip(runs[0][0], runs[1][0]))
    print('PGS exit per env vs per island over 5 steps: |dq| %.3g rad, |dqd| %.3g rad/s, |dreward| %.3g; iterations per solve %.1f / %.1f'
          % (dq, dqd, drew, runs[0][1][3] / runs[0][1][4], runs[1][1][3] / runs[1][1][4]))
    assert dq < 2e-4 and dqd < 5e-3 and drew < 1e-3, (dq, dqd, drew)
