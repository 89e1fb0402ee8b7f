"""Device reset IK (include/avr.h avr_reset_ik, csrc/avr_reset_ik.hip) against the host reset path
(avr/reset.py ik_batch + place_tool_bodies, the restatement of feeding.py:276-308 /
util.py:34-105 this build already checks against the oracle).

CPU: the reset inputs (draw order, batched human FK) reproduce the host reset bit for bit.
GPU: on the same inputs, the device accepts the same envs, lands the tool within tolerance,
finds the host's joint solution, places spoon and food like the host, and a device-reset episode
matches the oracle run from the device's own reset state."""
import numpy as np
import pytest

from avr import _abi as ABI
from avr import reset as RS

A = ABI.load_scene()
MD = ABI.ModelDesc(A)


def _host_ik_per_env(S, t7, init, q0):
    """ik_batch one env at a time (ik_batch's per-env early exit makes this equal to one batched
    call; test_ik_batch_is_batch_independent)."""
    lower, upper = RS.arm_limits(MD)
    tool = int(A['task_tool_link'])
    Q, ok = [], []
    for k in range(len(S)):
        q, o = RS.ik_batch(A, tool, t7[k:k + 1, :3], t7[k:k + 1, 3:], MD.arm_dofs, lower, upper, init[k:k + 1], q0)
        Q.append(q[0]); ok.append(bool(o[0]))
    return np.array(Q), np.array(ok)


def test_reset_inputs_reproduce_host_reset():
    ids = list(range(20, 32))
    S, meta = RS.batch_reset_states_fast(A, MD, 1001, ids, impairment='random')
    Si, t7, init, q0, mi = RS.reset_inputs(A, MD, 1001, ids, impairment='random')
    lower, upper = RS.arm_limits(MD)
    Q, ok = RS.ik_batch(A, int(A['task_tool_link']), t7[:, :3], t7[:, 3:], MD.arm_dofs, lower, upper, init, q0)
    RS.place_tool_bodies(A, Si, Q)
    # batched human FK vs the per-env one: same products, different association -> ulp-level
    np.testing.assert_allclose(Si, S, rtol=0, atol=1e-12)
    assert [m['gender'] for m in mi] == [m['gender'] for m in meta]
    assert [m['impairment'] for m in mi] == [m['impairment'] for m in meta]


def test_ik_batch_is_batch_independent():
    """An env's reset state does not depend on the other envs of the batch (per-env early exit),
    so sharded resets equal single-process ones (multi-GPU)."""
    S1, _ = RS.batch_reset_states_fast(A, MD, 1001, list(range(6)), impairment='random')
    S2, _ = RS.batch_reset_states_fast(A, MD, 1001, [3, 4, 5], impairment='random')
    np.testing.assert_array_equal(S1[3:], S2)


def test_restart_draws_follow_the_env_stream():
    """init[k, r] is what the r-th rng.uniform(lower, upper) of the host reset returned."""
    _, _, init, _, _ = RS.reset_inputs(A, MD, 1001, [5], impairment='none')
    rng = RS._rng(1001, 5)
    g = 'male' if rng.integers(2) == 0 else 'female'
    RS.human_joint_angles(A, g, rng, 1.0)
    rng.uniform(-0.05, 0.05); rng.uniform(-0.05, 0.05); rng.uniform(-0.05, 0.05, size=3)
    lower, upper = RS.arm_limits(MD)
    for r in range(3):
        np.testing.assert_array_equal(init[0, r], rng.uniform(lower, upper))


def test_keepout_box_is_table_clear_box():
    box = RS.keepout_box(A)
    tb = int(A['task_table_body'])
    s0 = A['body_shape_start'][tb]
    he = A['shape_param'][s0][:3]
    np.testing.assert_allclose(box[4:7], he + 0.05)
    assert box[3] == 0 and box[7] == 0


def test_host_ik_is_chaotic_from_far_starts():
    """The host IK itself: fp32-rounded restart draws (a 1e-8 perturbation) give a different
    valid solution for some envs and the identical one for most."""
    N = 8
    S, t7, init, q0, meta = RS.reset_inputs(A, MD, 1001, list(range(N)), impairment='random')
    Q1, o1 = _host_ik_per_env(S, t7, init, q0)
    Q2, o2 = _host_ik_per_env(S, t7, init.astype(np.float32).astype(np.float64), q0)
    d = np.abs(Q1 - Q2).max(1)
    assert np.all(o1) and np.all(o2)
    assert np.mean(d < 1e-3) >= 0.5 and d.max() > 1.0, d


@pytest.mark.gpu
def test_device_ik_matches_host_ik():
    from avr import _lib
    N = 48
    S, t7, init, q0, meta = RS.reset_inputs(A, MD, 1001, list(range(N)), impairment='random')
    Qh, okh = _host_ik_per_env(S, t7, init, q0)
    sim = _lib.Sim(MD, N)
    try:
        sim.set_state(np.zeros((N, ABI.STATE_WORDS), np.float32))
        _, okd = sim.reset_ik(None, S, t7, init, iters=80, tol=0.01, keepout8=RS.keepout_box(A), frames=0)
        G = sim.get_state().astype(np.float64)
    finally:
        sim.close()
    nd = int(A['n_dof'])
    Qd = G[:, ABI.S_Q:ABI.S_Q + nd]
    agree = okd == okh
    assert agree.mean() >= 0.95, (okd, okh)
    # every device-accepted solution satisfies the acceptance rule when re-checked in fp64
    tool = int(A['task_tool_link'])
    CP, CQ, _, _ = RS.robot_fk_batch(A, Qd)
    pe = np.linalg.norm(t7[:, :3] - CP[:, tool], axis=1)
    qe = np.linalg.norm(t7[:, 3:] - CQ[:, tool], axis=1)
    acc = RS.ik_accept(pe, qe, 0.0101)          # (util.py:49's rule, fp32 slack)
    for k in np.nonzero(okd)[0]:
        assert acc[k], (k, pe[k], qe[k])
        assert RS.table_clear(A, Qd[k])
    # same restart sequence and rules: where the DLS path from the restart's start is well
    # conditioned, the same joint solution.  From far-off starts the undamped steps of the 7-DoF arm
    # (1-D null space, continuous joints clipped at +-2 pi) amplify fp32-vs-fp64 rounding into a
    # different, equally valid solution: rounding only the restart draws to fp32 moves the host's
    # own fp64 solution by radians for 4 of envs 0..15 (test_host_ik_is_chaotic_from_far_starts);
    # on MI355X 24 of 44 envs agree within 1e-3 rad.  The bar: a large identical share plus the
    # validity checks above.
    both = okd & okh
    dq = np.abs(Qd - Qh).max(1)[both]
    assert np.mean(dq < 1e-3) >= 0.4, np.sort(dq)
    # non-arm joints, human, bowl, task words untouched; spoon + food placed from the device joints
    arm = set(MD.arm_dofs)
    other = [d for d in range(nd) if d not in arm]
    np.testing.assert_allclose(Qd[:, other], S[:, ABI.S_Q + np.array(other)], atol=1e-6)
    H = slice(ABI.S_HUMAN, ABI.S_HUMAN + 7 * ABI.MAX_HUMAN)
    np.testing.assert_allclose(G[:, H], S[:, H], atol=1e-6)
    P = RS.place_tool_bodies(A, S.copy(), Qd)
    F = slice(ABI.S_FREE, ABI.S_FREE + ABI.FB_WORDS * (2 + 8))
    np.testing.assert_allclose(G[:, F], P[:, F], atol=2e-5)


@pytest.mark.gpu
def test_device_reset_episode_matches_oracle():
    """A device-reset env (IK + 100 settle frames) then 20 random steps: the oracle started from
    the device's post-IK state follows the same trajectory (free-space tolerance; bowl/food contact
    is present, so 20 steps)."""
    from avr import _lib
    from oracle.oracle import Oracle
    N = 8
    S, t7, init, q0, meta = RS.reset_inputs(A, MD, 1001, list(range(100, 100 + N)), impairment='no_tremor')
    sim = _lib.Sim(MD, N)
    try:
        sim.set_state(np.zeros((N, ABI.STATE_WORDS), np.float32))
        _, ok = sim.reset_ik(None, S, t7, init, keepout8=RS.keepout_box(A), frames=0)
        S0 = sim.get_state()
        obs_g = sim.settle(100)
        o = Oracle(MD, N, 'f32')
        o.set_state(S0.astype(np.float64))
        obs_c = o.settle(100)
        np.testing.assert_allclose(obs_g, obs_c, atol=3e-3)
        for t in range(20):
            a = _lib.random_actions(1001, np.arange(N), t)
            x = sim.step(a)
            y = o.step(a)
        G, C = sim.get_state(), o.get_state()
        d = np.abs(G[:, :7] - C[:, :7]).max(1)
        assert np.median(d) < 1e-3 and d.max() < 5e-2, d
    finally:
        sim.close()


# ---------------------------------------------------------------- the counter-based reset stream
def test_philox_stream_is_independent_of_batch_composition():
    a = RS.philox_uniforms(1001, [3, 7, 9], [0, 2, 1], 40)
    b = RS.philox_uniforms(1001, [7], [2], 40)
    np.testing.assert_array_equal(a[1], b[0])
    assert np.all((a > 0) & (a < 1))
    assert not np.array_equal(RS.philox_uniforms(1001, [7], [3], 40), b)     # episodes differ
    assert not np.array_equal(RS.philox_uniforms(1002, [7], [2], 40), b)     # seeds differ


def test_philox_inputs_match_the_per_env_restatement():
    """The vectorised build from philox draws equals the per-env functions (human_slot_poses,
    the mouth target) fed the same draws."""
    from avr import geom as G

    ids = list(range(40, 56))
    S, t7, init, q0, meta = RS.reset_inputs(A, MD, 1001, ids, impairment='random', stream='philox')
    gl, il, ls, QH, trem, bowl, tpos, init2 = RS._draws_philox(A, MD, 1001, ids, None, 'random', [0] * len(ids), 40)
    np.testing.assert_array_equal(init, init2)
    lower, upper = RS.arm_limits(MD)
    assert np.all(init >= lower) and np.all(init <= upper)
    hs = ABI.S_HUMAN + 7 * int(A['task_head_slot'])
    for k in range(len(ids)):
        n = len(A['human_%s_parent' % gl[k]])
        ref = RS.human_slot_poses(A, gl[k], QH[k, :n]).ravel()
        np.testing.assert_allclose(S[k, ABI.S_HUMAN:ABI.S_HUMAN + ABI.MAX_HUMAN * 7], ref, rtol=0, atol=1e-12)
        head = S[k, hs:hs + 7]
        mouth = A['task_mouth_male'] if gl[k] == 'male' else A['task_mouth_female']
        np.testing.assert_allclose(S[k, ABI.S_TASK:ABI.S_TASK + 3], G.tf_mul(head[:3], head[3:], mouth, [0, 0, 0, 1])[0], atol=1e-12)
        assert (S[k, ABI.S_TASK + ABI.T_HDYN] == 1.0) == (il[k] == 'tremor')


def test_philox_human_angles_equal_per_env_clamps():
    """human_joint_angles_batch == human_joint_angles on the same head draws and limit scales."""
    class Fixed:
        def __init__(self, vals):
            self.v = list(vals)

        def uniform(self, lo, hi):
            return self.v.pop(0)

    rng = np.random.default_rng(0)
    for g in ('male', 'female'):
        head = rng.uniform(np.deg2rad(-30), np.deg2rad(30), size=(12, 3))
        ls = np.where(rng.uniform(size=12) < 0.5, rng.uniform(0.5, 1.0, size=12), 1.0)
        B = RS.human_joint_angles_batch(A, g, head, ls)
        for k in range(12):
            np.testing.assert_array_equal(B[k], RS.human_joint_angles(A, g, Fixed(head[k]), ls[k]))


# ---------------------------------------------------------------- step_sim self-contact screening
def _touching_config(o, n=400):
    """A few arm configurations whose links touch (oracle), and the finger-open rest pose."""
    _, _, _, q0, _ = RS.reset_inputs(A, MD, 1001, [0], impairment='none')
    lower, upper = RS.arm_limits(MD)
    rng = np.random.default_rng(7)
    Q = np.repeat(q0[None], n, 0)
    Q[:, MD.arm_dofs] = rng.uniform(lower, upper, size=(n, len(lower)))
    sc = o.robot_self_contact(Q)
    return Q, sc, q0


def test_quat_from_euler_batch_matches_geom():
    from avr import geom as G
    rng = np.random.default_rng(3)
    E = rng.uniform(-3, 3, size=(20, 3))
    B = RS.quat_from_euler_batch(E)
    for k in range(20):
        np.testing.assert_allclose(B[k], G.quat_from_euler(E[k]), atol=1e-12)


@pytest.mark.parametrize('stream', ['numpy', 'philox'])
def test_alt_orients_are_the_target_rotated_within_45_degrees(stream):
    """util.py:44-46: getQuaternionFromEuler(getEulerFromQuaternion(orient) + U(-45, 45) deg)."""
    from avr import geom as G
    al = RS.ik_alt_orients(1001, [4, 9, 11], [0, 1, 0], 40, stream)
    assert al.shape == (3, 40, 4)
    np.testing.assert_allclose(np.linalg.norm(al, axis=-1), 1.0, atol=1e-12)
    q0 = G.quat_from_euler([np.pi / 2.0, 0, np.pi / 2.0])
    ang = 2 * np.arccos(np.clip(np.abs(al @ q0), 0, 1))
    assert ang.max() < np.deg2rad(45) * np.sqrt(3) + 1e-9 and ang.min() > 0
    # per env and episode, independent of the batch
    np.testing.assert_array_equal(RS.ik_alt_orients(1001, [9], [1], 40, stream)[0], al[1])


def test_oracle_self_contact_flags_folded_arms_only():
    from oracle.oracle import Oracle
    S, t7, init, q0, _ = RS.reset_inputs(A, MD, 1001, [0], impairment='none')
    o = Oracle(MD, 1, 'f64')
    o.set_state(S)
    Q, sc, q0 = _touching_config(o)
    assert 0 < (sc > 0).sum() < len(sc) // 4        # the Jaco's joint limits keep folding rare
    # the reset's IK solutions (48 envs) are all free of self-contact
    lower, upper = RS.arm_limits(MD)
    S, t7, init, q0, _ = RS.reset_inputs(A, MD, 1001, list(range(24)), impairment='none')
    Qs, ok = RS.ik_batch(A, int(A['task_tool_link']), t7[:, :3], t7[:, 3:], MD.arm_dofs, lower, upper, init, q0)
    assert np.all(o.robot_self_contact(Qs[ok]) == 0)


def test_ik_screening_switches_the_target_orientation():
    """A restart that touches itself is checked against (and later restarts aim at) its re-drawn
    orientation: with every solution touching, acceptance needs a solution to hit the re-drawn
    orientation it was not aiming at -- none does -- and the closest restart is kept; with none
    touching the screening changes nothing."""
    N = 4
    S, t7, init, q0, _ = RS.reset_inputs(A, MD, 1001, list(range(N)), impairment='none')
    lower, upper = RS.arm_limits(MD)
    tool = int(A['task_tool_link'])
    alt = RS.ik_alt_orients(1001, range(N), None, init.shape[1])
    init = init[:, :3]
    alt = alt[:, :3]
    Q0, ok0 = RS.ik_batch(A, tool, t7[:, :3], t7[:, 3:], MD.arm_dofs, lower, upper, init, q0)
    Qn, okn = RS.ik_batch(A, tool, t7[:, :3], t7[:, 3:], MD.arm_dofs, lower, upper, init, q0, alt=alt,
                          self_contact=lambda Q: np.zeros(len(Q), int))
    np.testing.assert_array_equal(Qn, Q0)
    np.testing.assert_array_equal(okn, ok0)
    Qa, oka = RS.ik_batch(A, tool, t7[:, :3], t7[:, 3:], MD.arm_dofs, lower, upper, init, q0, alt=alt,
                          self_contact=lambda Q: np.ones(len(Q), int))
    assert not oka.any()
    CP, _, _, _ = RS.robot_fk_batch(A, Qa)
    assert np.all(np.linalg.norm(CP[:, tool] - t7[:, :3], axis=1) < 0.01)   # the closest restart reached the position


@pytest.mark.gpu
def test_device_self_contact_matches_oracle():
    """avr_robot_self_contact (the device pipeline on the robot-robot candidate pairs) counts the
    same touching shape pairs as the oracle, on random arm configurations (fp32 vs fp64: a pair
    within rounding of its contact threshold may differ)."""
    from avr import _lib
    from oracle.oracle import Oracle
    S, _, _, _, _ = RS.reset_inputs(A, MD, 1001, [0], impairment='none')
    o = Oracle(MD, 1, 'f64')
    o.set_state(S)
    Q, sc, q0 = _touching_config(o, 1024)
    sim = _lib.Sim(MD, 1)
    try:
        sim.set_state(S.astype(np.float32))
        sd = sim.robot_self_contact(Q)
    finally:
        sim.close()
    assert (sc > 0).sum() >= 3
    assert np.mean((sd > 0) == (sc > 0)) >= 0.995, (np.nonzero(sd != sc), sd[sd != sc], sc[sd != sc])
    assert np.mean(sd == sc) >= 0.99


@pytest.mark.gpu
def test_device_ik_screening_matches_host_and_leaves_no_self_contact():
    """The device IK with the self-contact screening (alt orientations) accepts the envs the host
    IK with the same screening accepts, and over 4096 device resets no accepted reset state starts
    with the robot touching itself."""
    from avr import _lib
    N = 48
    ids = list(range(N))
    S, t7, init, q0, _ = RS.reset_inputs(A, MD, 1001, ids, impairment='random')
    alt = RS.ik_alt_orients(1001, ids, None, init.shape[1])
    lower, upper = RS.arm_limits(MD)
    sim = _lib.Sim(MD, N)
    try:
        sim.set_state(np.zeros((N, ABI.STATE_WORDS), np.float32))
        Qh, okh = RS.ik_batch(A, int(A['task_tool_link']), t7[:, :3], t7[:, 3:], MD.arm_dofs, lower, upper, init, q0,
                              alt=alt, self_contact=sim.robot_self_contact)
        _, okd = sim.reset_ik(None, S, t7, init, keepout8=RS.keepout_box(A), frames=0, alt=alt)
    finally:
        sim.close()
    assert np.mean(okd == okh) >= 0.95, (okd, okh)
    E = 4096
    ids = list(range(E))
    S, t7, init, q0, _ = RS.reset_inputs(A, MD, 77, ids, impairment='random', stream='philox')
    alt = RS.ik_alt_orients(77, ids, None, init.shape[1], 'philox')
    sim = _lib.Sim(MD, E)
    try:
        sim.set_state(np.zeros((E, ABI.STATE_WORDS), np.float32))
        _, ok = sim.reset_ik(None, S, t7, init, keepout8=RS.keepout_box(A), frames=0, alt=alt)
        q, _ = sim.get_q()
        sc = sim.robot_self_contact(q)
    finally:
        sim.close()
    assert ok.mean() >= 0.9
    assert np.all(sc[ok] == 0), np.nonzero(sc[ok])
