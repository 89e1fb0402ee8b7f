"""BedBathingPR2-v0 (BASELINE configs[3], its PR2 variant: BedBathingSawyer-v0 does not exist in
the reference): compiled scene facts, the reset's arm settle, the wipe-target and
closest-distance glue on the CPU oracle; the gfx950 kernels through the C-ABI against the oracle
on the GPU.

Pins beyond self-consistency:
  * the wipe-target counts follow util.capsule_points' closed form (sections x points per ring);
  * the male arm settle lands within 0.02 rad of the right-arm pose the reference itself
    hard-codes for its VR/replay bed bathing (bed_bathing.py:232, joint_angles; the VR env's
    default participant is male, bed_bathing.py:12) -- the one PyBullet-produced number the
    reference holds for this path.  With the bed's rolling / spinning friction 5 (bed_bathing.py:282,
    torsional rows, btMultiBodyConstraintSolver [ext]) the male settle is 0.012 rad from it;
    without it 0.046 rad.  The female body's proportions differ (human_creation.py:116-161), so
    its settle is held to 0.1 rad only.
Tolerances (fp32 kernel vs fp64 oracle) as in test_scratch.py: one sub-step 1e-5 rad; 200
contact-free steps 1e-3 rad; wipe bookkeeping bit-identical; rewards 2e-3.
"""
import os

import numpy as np
import pytest

from avr import _abi as ABI

BB = ABI.BB
REF = '/root/reference/assistive_gym/envs/assets'
# bed_bathing.py:232: joint_angles of the VR/replay bed bathing.  The reference applies them to
# joints range(7) (:233), but the seven values are the right arm's settled pose (joints 7..13):
# the non-VR settle below reproduces them within 0.012 rad, which no other joint set comes near
VR_ARM = np.array([0.39717707, 0.27890519, -0.00883447, -0.67345593, -0.00568484, 0.05987911, 0.00957937])


@pytest.fixture(scope='module')
def bb():
    A = ABI.load_scene(ABI.TASK_BEDBATH)
    return A, ABI.ModelDesc(A)


def oracle(md, n, precision='f64'):
    from oracle.oracle import Oracle
    o = Oracle(md, n, precision)
    o.set_threads(4)
    return o


def _oracle_runner(md, precision='f64'):
    def run(S, frames):
        o = oracle(md, len(S), precision)
        o.set_state(S)
        o.settle(frames)
        return o.get_state()
    return run


@pytest.fixture(scope='module')
def settled(bb):
    from avr import reset_bedbath as RBB
    A, md = bb
    return RBB.settled_arms(A, md, runner=_oracle_runner(md))


@pytest.fixture(scope='module')
def states(bb, settled):
    from avr import reset_bedbath as RBB
    A, md = bb
    return RBB.batch_reset_states(A, md, 1001, list(range(8)), attempts=12, iters=80, settled=settled)


# ------------------------------------------------------------------ scene
def test_wipe_targets_follow_capsule_points(bb):
    A, md = bb
    # util.capsule_points: int(L / 0.03) sections, int(2 pi r / 0.03) points per ring (bed_bathing.py:362-370)
    for g, ((Lu, ru), (Lf, rf)) in enumerate((((0.279, 0.043), (0.257, 0.033)), ((0.264, 0.0355), (0.234, 0.027)))):
        nu = int(Lu / 0.03) * int(2 * np.pi * ru / 0.03)
        nf = int(Lf / 0.03) * int(2 * np.pi * rf / 0.03)
        assert tuple(A['bb_ntgt'][g]) == (nu, nf)
        T = A['bb_targets'][g]
        r = np.linalg.norm(T[:nu, :2], axis=1)
        np.testing.assert_allclose(r, ru, atol=1e-12)                       # on the capsule's surface
        assert np.all(T[:nu, 2] < 0) and np.all(T[:nu, 2] > -Lu)
        assert np.all(T[nu:nu + nf, 3] == 1) and np.all(T[:nu, 3] == 0)
    assert tuple(A['bb_ntgt'].sum(1)) == (129, 91)


def test_bed_and_wiper(bb):
    A, md = bb
    k = A['body_kind']
    static = np.nonzero(k == ABI.BODY_STATIC)[0]
    assert len(static) == 4                                                  # plane, 2 mattress boxes, frame
    fr = A['body_friction'][static]
    assert np.allclose(fr[1:], 5.0)                                          # bed_bathing.py:282
    assert A['body_shape_count'][static[3]] == 44                            # hospital_bed_frame_vhacd: 44 hulls
    np.testing.assert_allclose(A['st_pose'][1], [0, -0.53, 0.4, 0, 0, 0, 1])
    assert np.isclose(A['fb_mass'][0], 3.0)                                  # wiper: 3 links of 1 kg
    assert int(A['task_tool_handle_shapes']) == 2                            # handle + 'tool' boxes precede the cloth
    # cloth COM (tool link 1): handle origin - 0.035 - 0.0075 in z
    np.testing.assert_allclose(A['task_tool_tip'] - A['task_tool_pivot'], [0, 0, -0.0425], atol=1e-12)
    np.testing.assert_allclose(A['bb_human_base'][:3], [0, 0, 0.7])


@pytest.mark.skipif(not os.path.isdir(REF), reason='reference assets not mounted (GPU box)')
def test_committed_bedbath_scene_matches_compiler(tmp_path):
    from avr import model_compiler as MC
    _, A = MC.compile_bedbath(str(tmp_path))
    B = ABI.load_scene(ABI.TASK_BEDBATH)
    assert set(A) == set(B)
    for k in A:
        np.testing.assert_array_equal(np.asarray(A[k]), B[k], err_msg=k)


# ------------------------------------------------------------------ reset
# The vector pins the MALE settle: our male settle lands within 0.012 rad of it, the female's
# elbow 0.088 rad away (a shorter, lighter forearm rests at -0.585 rad, not -0.674): the reference
# recorded it on the male model, and holds no female value.  The male bound (0.02) is tight
# against how strongly the settle responds to the Bullet defaults the restatement assumes
# (tools/bb_settle_sensitivity.py, profiles/r05_bb_settle_sensitivity.txt): erp 0.1 / 0.8 move
# the male arm 0.072 / 0.20 rad from the vector, no damping or 0.1 damping 0.040 / 0.061, 10
# solver iterations 0.061, warm start 0.1 0.017; the assumed set (erp 0.2, damping 0.04, 50
# iterations, warm start 0.85) is the nearest.  The female bound is a plausibility check only.
VR_TOL = {'male': 0.02, 'female': 0.1}


def test_arm_settle_matches_reference_vr_pose(bb, settled):
    """The 100-frame drop of the right arm onto the mattress (bed_bathing.py:283-289), fp64 oracle,
    against the arm pose the reference hard-codes for its VR/replay bed bathing (male: 0.012 rad
    with the bed's rolling / spinning friction, 0.046 without; the female has no reference value,
    see VR_TOL)."""
    for g in ('male', 'female'):
        q, slots = settled[g]
        assert np.abs(q - VR_ARM).max() < VR_TOL[g], (g, q)
    A, md = bb
    js = A['bb_joint_slots']
    q, slots = settled['male']
    assert slots[js[2], 2] < 0.7       # the wrist came down onto the mattress (top at z ~0.55)


def test_reset_states(bb, states):
    A, md = bb
    S, meta = states
    assert all(m['base_ok'] for m in meta)
    for k, m in enumerate(meta):
        st = S[k]
        assert st[BB.S_TASK + BB.T_HDYN] == 0 and st[BB.S_TASK + BB.T_TREMOR] == 0
        nt = int(st[BB.S_TASK + BB.T_NTGT])
        assert nt == m['n_targets'] == (129 if m['gender'] == 'male' else 91)
        bits = sum(bin(int(st[BB.S_TASK + BB.T_WIPE + w])).count('1') for w in range(6))
        assert bits == nt
        fin = [st[BB.S_Q + d] for d in md.finger_dofs]
        assert np.allclose(fin, 0.2)


def test_oracle_episode_without_contact(bb, states):
    from avr import _lib
    A, md = bb
    S, meta = states
    o = oracle(md, len(S))
    o.set_state(S)
    obs = o.settle(0)
    assert obs.shape == (len(S), 24) and np.all(obs[:, 23] == 0)
    for t in range(5):
        a = _lib.random_actions(1001, np.arange(len(S)), t)
        ob, r, d, info = o.step(a)
        # no contact: reward = -closest distance - 0.01 sum a^2 - 0.25 |v_cloth|
        assert np.all(info[:, 0] == 0)
        dist = np.array([o.bb_closest(e) for e in range(len(S))])
        assert np.all(dist > 0) and np.all(-r >= dist + 0.01 * (a.astype(np.float64) ** 2).sum(1) - 1e-5)


def wipe_states(A, md, S):
    import bedbath_util as U
    return U.wipe_states(A, md, S)


def test_oracle_wiping(bb, states):
    """Pressing the cloth onto a target wipes it (and the neighbours within 2.5 cm of the contact
    points): task_success counts them, the reward carries 5 x the count, the bits clear.  (The
    arm's motors are weak -- 1 N, config.ini:13 -- so in some envs the contact pushes the cloth off
    before the step's last sub-step, whose contacts are the ones get_total_force sees.)"""
    A, md = bb
    S, meta = states
    W, ks = wipe_states(A, md, S)
    o = oracle(md, len(W))
    o.set_state(W)
    zero = np.zeros((len(W), 7), np.float32)
    ob, r, d, info = o.step(zero)
    St = o.get_state()
    n_wiping = 0
    for e in range(len(W)):
        nt = int(St[e, BB.S_TASK + BB.T_NTGT])
        alive = sum(bin(int(St[e, BB.S_TASK + BB.T_WIPE + w])).count('1') for w in range(6))
        wiped = nt - alive
        assert wiped == St[e, BB.S_TASK + BB.T_SUCCESS]
        if wiped == 0:
            continue
        n_wiping += 1
        k = ks[e]
        assert not (int(St[e, BB.S_TASK + BB.T_WIPE + k // 24]) >> (k % 24)) & 1      # the pressed target is gone
        assert r[e] > 5.0 * wiped - 2.0                                           # wiping_reward_weight 5
        assert ob[e, 23] > 0                                                       # tool force in the obs
    assert n_wiping >= len(W) // 2, n_wiping


# ------------------------------------------------------------------ GPU
def _sim(md, n, **kw):
    from avr import _lib
    return _lib.Sim(md, n, **kw)


@pytest.mark.gpu
def test_bedbath_device_settle_matches_oracle(bb):
    from avr import reset_bedbath as RBB
    A, md = bb
    g = RBB.settled_arms(A, md)
    c = RBB.settled_arms(A, md, runner=_oracle_runner(md, 'f32'))
    for gender in ('male', 'female'):
        assert np.abs(g[gender][0] - c[gender][0]).max() < 2e-3, (g[gender][0], c[gender][0])
        assert np.abs(g[gender][0] - VR_ARM).max() < VR_TOL[gender]


@pytest.mark.gpu
def test_bedbath_one_substep_matches_oracle(bb, states):
    A, md = bb
    S, meta = states
    S32 = S.astype(np.float32)
    n, nd = len(S), md.n_dof
    sim, o = _sim(md, n), oracle(md, n)
    sim.set_state(S32); o.set_state(S32.astype(np.float64))
    sim.substep(0.02); o.substep(0.02)
    G, C = sim.get_state(), o.get_state()
    assert np.abs(G[:, :nd] - C[:, :nd]).max() < 1e-5
    assert np.abs(G[:, BB.S_FREE:BB.S_FREE + 13] - C[:, BB.S_FREE:BB.S_FREE + 13]).max() < 1e-4
    sim.close()


@pytest.mark.gpu
def test_bedbath_200_steps_within_1e3(bb, states):
    """200 gym steps of full-scale random actions: every env the fp64 oracle itself holds to
    1e-3 under a 1e-6 perturbation of its actions stays within 1e-3 rad of it, and its obs and
    reward within 2e-3 or three times the perturbed oracle's own obs / reward spread (the PGS's
    residual-threshold exit is a discrete decision: an iteration more or less moves a contact's
    impulse at the 3e-4 velocity level, and the cloth's speed term of the reward follows); an env
    the perturbation moves further has met a contact bifurcation (the arm or the cloth striking
    the bed, whose rolling / spinning friction 5 locks the contact either way) -- there the GPU
    stays within 20x that spread.  At most 2 of the 8 envs may be such."""
    from avr import _lib
    A, md = bb
    S, meta = states
    S32 = S.astype(np.float32)
    n, nd = len(S), md.n_dof
    sim, o, op = _sim(md, n), oracle(md, n), oracle(md, n)
    sim.set_state(S32); o.set_state(S32.astype(np.float64)); op.set_state(S32.astype(np.float64))
    assert np.abs(sim.settle(0) - o.settle(0)).max() < 1e-5
    rng = np.random.default_rng(5)
    w, spread, wobs, wrew = np.zeros(n), np.zeros(n), np.zeros(n), np.zeros(n)
    sobs, srew = np.zeros(n), np.zeros(n)
    for t in range(200):
        a = _lib.random_actions(1001, np.arange(n), t)
        g = sim.step(a)
        c = o.step(a)
        cp = op.step((a + 1e-6 * rng.standard_normal(a.shape)).astype(np.float32))
        wobs = np.maximum(wobs, np.abs(g[0][:, :23] - c[0][:, :23]).max(1))
        wrew = np.maximum(wrew, np.abs(g[1] - c[1]))
        sobs = np.maximum(sobs, np.abs(cp[0][:, :23] - c[0][:, :23]).max(1))
        srew = np.maximum(srew, np.abs(cp[1] - c[1]))
        assert np.array_equal(g[2], c[2])
        if t % 20 == 19:
            G, C, Cp = sim.get_state()[:, :nd], o.get_state()[:, :nd], op.get_state()[:, :nd]
            w = np.maximum(w, np.abs(G - C).max(1))
            spread = np.maximum(spread, np.abs(Cp - C).max(1))
    sim.close()
    print('bedbath 200 steps: GPU vs fp64 oracle dq %s obs %s reward %s; oracle spread under 1e-6 action noise dq %s obs %s reward %s' % (
        w, wobs, wrew, spread, sobs, srew))
    calm = spread < 1e-3
    assert calm.sum() >= n - 2, spread
    assert np.all(w[calm] < 1e-3), w
    assert np.all(wobs[calm] < np.maximum(2e-3, 3 * sobs[calm])) and np.all(wrew[calm] < np.maximum(2e-3, 3 * srew[calm])), (wobs, sobs, wrew, srew)
    assert np.all(w[~calm] <= 20 * spread[~calm]), (w, spread)


@pytest.mark.gpu
def test_bedbath_wiping_matches_oracle(bb, states):
    """The constructed wiping contact: same targets wiped (bit-identical words), same success
    count, reward within 2e-3 (the closest distance is a penetration depth here: EPA on both)."""
    A, md = bb
    S, meta = states
    W, ks = wipe_states(A, md, S)
    W32 = W.astype(np.float32)
    n = len(W)
    sim, o = _sim(md, n), oracle(md, n, 'f32')
    sim.set_state(W32); o.set_state(W32.astype(np.float64))
    zero = np.zeros((n, 7), np.float32)
    g = sim.step(zero)
    c = o.step(zero)
    G, C = sim.get_state(), o.get_state()
    words = slice(BB.S_TASK + BB.T_WIPE, BB.S_TASK + BB.T_WIPE + 6)
    assert np.array_equal(G[:, words], C[:, words].astype(np.float32))
    assert np.array_equal(G[:, BB.S_TASK + BB.T_SUCCESS], C[:, BB.S_TASK + BB.T_SUCCESS].astype(np.float32))
    assert np.count_nonzero(G[:, BB.S_TASK + BB.T_SUCCESS] >= 1) >= n // 2
    np.testing.assert_allclose(g[1], c[1], atol=2e-3)
    np.testing.assert_allclose(g[0][:, :23], c[0][:, :23], atol=2e-3)
    sim.close()
