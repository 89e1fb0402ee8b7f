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
