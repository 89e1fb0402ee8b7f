"""Human proportions (hipbone_to_mouth_height): create_human scales the human by
hmhs = height / 0.6 (male) or / 0.54 (female) -- capsule lengths, capsule offsets and joint
offsets along the body (human_creation.py:60-63,75-115,121-161); BedBathing's wipe targets move
with it (position_scale, bed_bathing.py:359-370).  The reference takes the height from setup()
(feeding.py:20-28) or a recording's setup.pkl (feeding.py:153-156).

The model compiler rebuilds a scene at any per-gender height from its asset cache (no reference
assets needed, as on the GPU box); at the default heights the rebuild is the committed npz bit
for bit.  The GPU tests hold the kernels at non-default heights to the same one-sub-step
tolerances as at the defaults, against the fp64 oracle on the same rebuilt scene.
"""
import numpy as np
import pytest

from avr import _abi as ABI
from avr import model_compiler as MC

H_ODD = {'male': 0.66, 'female': 0.50}


@pytest.fixture
def no_reference(monkeypatch):
    """The GPU box's situation: the reference's assets are absent."""
    monkeypatch.setattr(MC, 'REF_ASSETS', '/nonexistent/reference/assets')


@pytest.mark.parametrize('task', [ABI.TASK_FEEDING, ABI.TASK_SCRATCH, ABI.TASK_BEDBATH])
def test_default_heights_rebuild_is_the_committed_scene(task, no_reference):
    A = ABI.load_scene(task)
    B = MC.scene_arrays(ABI.SCENES[task])
    assert set(B) - set(A) == {'human_heights'}
    for k in A:
        assert A[k].dtype == B[k].dtype and np.array_equal(A[k], B[k]), k


def _human_capsules(A, gender):
    gi = 0 if gender == 'male' else 1
    m = (A['shape_gender'] == gi) & (A['shape_kind'] == MC.CAPSULE)
    return A['shape_param'][m], A['shape_pose'][m]


@pytest.mark.parametrize('gender', ['male', 'female'])
def test_capsules_scale_with_height(gender, no_reference):
    """Limb capsules (upper arm, forearm, thigh, shin, foot, neck) have length x hmhs; the torso
    capsules (chest, shoulders, waist, hips) keep theirs; radii never change (rs = 1).  The other
    gender's human is untouched."""
    A = ABI.load_scene(ABI.TASK_FEEDING)
    h = H_ODD[gender]
    s = h / MC.DEFAULT_HEIGHT[gender]
    B = MC.scene_arrays('feeding_jaco', {gender: h})
    (pa, _), (pb, _) = _human_capsules(A, gender), _human_capsules(B, gender)
    np.testing.assert_array_equal(pa[:, 0], pb[:, 0])                   # radii
    ratio = pb[:, 1] / pa[:, 1]
    scaled = np.isclose(ratio, s, rtol=1e-12)
    kept = np.isclose(ratio, 1.0, rtol=1e-12)
    assert np.all(scaled | kept)
    assert scaled.sum() == 11 and kept.sum() == 5, (scaled.sum(), kept.sum())   # neck, 2 x (arm 2, leg 3); chest, 2 shoulders, waist, hips
    other = 'female' if gender == 'male' else 'male'
    np.testing.assert_array_equal(_human_capsules(A, other)[0], _human_capsules(B, other)[0])
    np.testing.assert_array_equal(A['human_%s_pos' % other], B['human_%s_pos' % other])
    # joint offsets: the lateral ones (shoulder / hip widths) do not change; the ones along the
    # body are affine in hs (e.g. hand_p = -(0.033 rs + 0.257 hs), foot_p = -0.403 hs - 0.025)
    pa, pb = A['human_%s_pos' % gender], B['human_%s_pos' % gender]
    np.testing.assert_array_equal(pa[:, 0], pb[:, 0])
    h2 = MC.DEFAULT_HEIGHT[gender] + 2 * (h - MC.DEFAULT_HEIGHT[gender])
    pc = MC.scene_arrays('feeding_jaco', {gender: h2})['human_%s_pos' % gender]
    np.testing.assert_allclose(pc - pa, 2 * (pb - pa), rtol=1e-9, atol=1e-12)
    assert np.abs(pb - pa).max() > 0.01


def test_bed_targets_follow_the_arm(no_reference):
    """generate_targets: the same rings (count from the unscaled capsule), axial positions x hmhs."""
    A = ABI.load_scene(ABI.TASK_BEDBATH)
    s = 0.5 / 0.54
    B = MC.scene_arrays('bed_bathing_pr2', {'female': 0.5})
    np.testing.assert_array_equal(A['bb_ntgt'], B['bb_ntgt'])
    n = int(A['bb_ntgt'][1].sum())
    ta, tb = A['bb_targets'][1, :n], B['bb_targets'][1, :n]
    np.testing.assert_array_equal(ta[:, :2], tb[:, :2])                 # ring radius, angle
    np.testing.assert_allclose(tb[:, 2], ta[:, 2] * s, rtol=1e-12, atol=1e-15)
    np.testing.assert_array_equal(A['bb_targets'][0], B['bb_targets'][0])


def test_height_bounds_and_names():
    with pytest.raises(ValueError):
        MC.human_heights({'male': 2.0})
    with pytest.raises(ValueError):
        MC.human_heights({'child': 0.5})
    assert MC.human_heights({'female': None}) == MC.DEFAULT_HEIGHT


def test_feeding_reset_reaches_the_moved_mouth(no_reference):
    """The host reset at a non-default height: the mouth target (head link + mouth offset,
    feeding.py:253) rises with the human, and the IK puts the spoon near it as at the default."""
    from avr import reset as RS
    out = {}
    for tag, H in (('default', None), ('tall', {'male': 0.7})):
        A = ABI.load_scene(ABI.TASK_FEEDING) if H is None else MC.scene_arrays('feeding_jaco', H)
        md = ABI.ModelDesc(A)
        S, meta = RS.batch_reset_states_fast(A, md, 1001, list(range(4)), genders=['male'] * 4, impairment='none')
        out[tag] = S
    L = ABI.LAYOUTS[ABI.TASK_FEEDING]
    tgt = lambda S: S[:, L.S_TASK + L.T_TARGET:L.S_TASK + L.T_TARGET + 3]
    dz = tgt(out['tall'])[:, 2] - tgt(out['default'])[:, 2]
    assert np.all(dz > 0.02), dz


@pytest.mark.gpu
@pytest.mark.parametrize('task', [ABI.TASK_FEEDING, ABI.TASK_SCRATCH, ABI.TASK_BEDBATH])
def test_one_substep_at_odd_heights_matches_oracle(task):
    """One sub-step of the kernels on a scene rebuilt at male 0.66 / female 0.50 against the fp64
    oracle on the same scene: the default-height tolerances (|dq| <= 1e-5 rad, human chain 1e-5,
    free bodies 1e-4)."""
    from avr import _lib
    from oracle.oracle import Oracle
    _lib.load()
    A = MC.scene_arrays(ABI.SCENES[task], H_ODD)
    md = ABI.ModelDesc(A)
    L = md.layout
    n = 8
    genders = ['male', 'female'] * (n // 2)
    if task == ABI.TASK_FEEDING:
        from avr import reset as RS
        S, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(n)), genders=genders, impairment='tremor')
        dt = 0.01
    elif task == ABI.TASK_SCRATCH:
        from avr import reset_scratch as RSS
        S, _ = RSS.batch_reset_states(A, md, 1001, list(range(n)), genders=genders, attempts=12, iters=80)
        dt = 0.02
    else:
        from avr import reset_bedbath as RBB
        S = RBB.batch_reset_states(A, md, 1001, list(range(n)), genders=genders, attempts=12)[0]
        dt = 0.02
    S = np.asarray(S, np.float32)
    sim, o = _lib.Sim(md, n), Oracle(md, n)
    o.set_threads(8)
    sim.set_state(S); o.set_state(S.astype(np.float64))
    sim.substep(dt); o.substep(dt)
    G, C = sim.get_state(), o.get_state()
    sim.close()
    nd = min(md.n_dof + L.HC_N, L.MAX_DOF)
    assert np.abs(G[:, :nd] - C[:, :nd]).max() < 1e-5
    fb = slice(L.S_FREE, L.S_FREE + L.MAX_FREE * ABI.FB_WORDS)
    assert np.abs(G[:, fb] - C[:, fb]).max() < 1e-4


@pytest.mark.gpu
def test_vec_env_at_odd_height_tracks_oracle():
    """AVRVecEnv(human_heights=...) steps the rebuilt scene: 20 gym steps of FeedingJaco at male
    0.66 from the env's own reset, food and bowl removed (free space), within the north star's
    1e-3 rad of the fp64 oracle; the observation's mouth target differs from the default height's."""
    from avr import _lib
    from avr import env as EV
    from oracle.oracle import Oracle
    v = EV.AVRVecEnv('FeedingJaco-v0', 4, auto_reset=False, prefetch=False, human_heights={'male': 0.66})
    v.setup('male', -1, '')
    o_tall = v.reset()
    S = v.get_state().copy()
    for f in range(1, ABI.MAX_FREE):
        b = ABI.S_FREE + ABI.FB_WORDS * f
        S[:, b:b + 3] = [60.0 + 3 * f, 60.0, 500.0]
        S[:, b + 3:b + 7] = [0, 0, 0, 1]
        S[:, b + 7:b + 13] = 0
    v.set_state(S)
    o = Oracle(v.md, 4)
    o.set_threads(8)
    o.set_state(S.astype(np.float64))
    worst = 0.0
    for t in range(20):
        a = _lib.random_actions(1001, np.arange(4), t)
        v.step(a); o.step(a)
        worst = max(worst, np.abs(v.get_state()[:, :v.md.n_dof] - o.get_state()[:, :v.md.n_dof]).max())
    v.close()
    assert worst < 1e-3, worst
    d = EV.AVRVecEnv('FeedingJaco-v0', 4, auto_reset=False, prefetch=False)
    d.setup('male', -1, '')
    o_def = d.reset()
    d.close()
    assert np.abs(o_tall - o_def).max() > 1e-3
