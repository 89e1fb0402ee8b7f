"""Record / replay (the .bullet + setup.pkl + actions.pkl flow, avr/record.py) and the policy
evaluation harness (enjoy_vr.py's contract, avr/policy_eval.py)."""
import json
import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from avr import _abi as ABI
from avr import policy_eval as PE
from avr import record as R


# ------------------------------------------------------------------ CPU
class _FakeSim:
    def __init__(self, task, n):
        self.md = SimpleNamespace(task=task)
        self.n = n
        self.words = ABI.LAYOUTS[task].STATE_WORDS
        self.S = np.arange(n * self.words, dtype=np.float32).reshape(n, self.words)

    def get_state(self):
        return self.S.copy()

    def set_state(self, S):
        self.S = np.array(S, np.float32)


def test_state_snapshot_round_trip_and_layout_checks(tmp_path):
    a = _FakeSim(ABI.TASK_FEEDING, 3)
    p = str(tmp_path / 's.npz')
    R.save_state(p, a)
    b = _FakeSim(ABI.TASK_FEEDING, 3)
    b.S[:] = 0
    R.load_state(p, b)
    np.testing.assert_array_equal(a.S, b.S)
    with pytest.raises(ValueError):
        R.load_state(p, _FakeSim(ABI.TASK_SCRATCH, 3))      # other task / layout
    with pytest.raises(ValueError):
        R.load_state(p, _FakeSim(ABI.TASK_FEEDING, 4))      # other env count


def test_running_mean_std_matches_batch_statistics():
    rng = np.random.default_rng(0)
    x = rng.normal(2.0, 3.0, size=(500, 5))
    r = PE.RunningMeanStd((5,), count=0.0 + 1e-12)
    for k in range(0, 500, 37):
        r.update(x[k:k + 37])
    np.testing.assert_allclose(r.mean, x.mean(0), rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(r.var, x.var(0), rtol=1e-6)


def test_normalize_is_vecnormalize_eval():
    rms = PE.RunningMeanStd((3,), mean=[1.0, 0.0, -1.0], var=[4.0, 1e-12, 1.0])
    o = torch.tensor([[3.0, 1.0, -1.0]])
    n = PE.normalize(o, rms)
    np.testing.assert_allclose(n.numpy(), [[1.0, 10.0, 0.0]], rtol=1e-5)     # clipped at +-10


def test_policy_checkpoint_round_trip(tmp_path):
    torch.manual_seed(0)
    pol = PE.ActorCritic(25, 7)
    rms = PE.RunningMeanStd((25,), mean=np.linspace(0, 1, 25), var=np.linspace(1, 2, 25), count=7.0)
    p = str(tmp_path / 'FeedingJaco-v0.pt')
    PE.save_policy(p, pol, rms)
    pol2, rms2 = PE.load_policy(p)
    o = torch.randn(4, 25)
    h, m = torch.zeros(4, 1), torch.zeros(4, 1)
    v1, a1, _, _ = pol.act(o, h, m, deterministic=True)
    v2, a2, _, _ = pol2.act(o, h, m, deterministic=True)
    assert torch.equal(a1, a2) and torch.equal(v1, v2) and a1.shape == (4, 7) and v1.shape == (4, 1)
    np.testing.assert_array_equal(rms2.mean, rms.mean)
    assert rms2.count == 7.0


def test_setup_accepts_enjoy_vr_height_for_both_genders():
    """enjoy_vr.py:50,63 calls env.setup(gender, participant, policy_name, 0.54) for every
    participant; the reference's non-VR reset then overwrites the height with the gender's default
    (feeding.py:173-174), so setup() accepts any height, keeps it, and leaves the resets alone."""
    from avr import env as E
    for gender in ('male', 'female'):
        v = object.__new__(E.AVRVecEnv)
        v._prefetch = None
        E.AVRVecEnv.setup(v, gender, 3, 'Static', 0.54)
        assert v.genders == gender and v.participant == 3 and v.hipbone_to_mouth_height == 0.54
        assert v._genders([0, 1]) == [gender, gender]
    with pytest.raises(ValueError):
        E.AVRVecEnv.setup(v, 'other', 3, 'Static', 0.54)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_record_then_replay_is_bit_identical(tmp_path):
    from avr import env as E, _lib
    n = 4
    env = E.AVRVecEnv('FeedingJaco-v0', n, auto_reset=False, prefetch=False)
    rec = R.Recorder(env, str(tmp_path / 'rec'))
    o0 = rec.reset()
    obs, rews = [o0], []
    for t in range(15):
        o, r, d, info = rec.step(_lib.random_actions(1001, np.arange(n), t))
        obs.append(o); rews.append(r)
    rec.close()
    snap = str(tmp_path / 'frame_0.npz')
    R.save_state(snap, env)
    env.close()
    setup = json.load(open(tmp_path / 'rec' / 'setup.json'))
    assert setup['env_id'] == 'FeedingJaco-v0' and len(setup['gender']) == n
    rp = R.ReplayEnv(str(tmp_path / 'rec'))
    np.testing.assert_array_equal(rp.reset(), o0)
    for t in range(15):
        o, r, d, info = rp.step(None)
        np.testing.assert_array_equal(o, obs[t + 1])
        np.testing.assert_array_equal(r, rews[t])
        assert d.all() == (t == 14)
    assert rp.mismatch == []
    R.load_state(snap, rp.env)               # a snapshot restores into a fresh handle
    np.testing.assert_array_equal(rp.env.get_state(), np.load(tmp_path / 'rec' / 'states.npy')[-1])
    rp.close()
    res = R.savemeta(str(tmp_path / 'rec*'))
    (d, v), = res.items()
    assert v['rewards'].shape == (15, n) and v['replay_mismatch'] == []


@pytest.mark.gpu
def test_policy_evaluation_harness(tmp_path):
    torch.manual_seed(1)
    pol = PE.ActorCritic(25, 7)
    rms = PE.RunningMeanStd((25,))
    p = str(tmp_path / 'FeedingJaco-v0.pt')
    PE.save_policy(p, pol, rms)
    pol, rms = PE.load_policy(p)
    a = PE.evaluate('FeedingJaco-v0', pol, rms, n_envs=16, steps=200, setup=dict(gender='female', participant=2, policy_name='Static'))
    b = PE.evaluate('FeedingJaco-v0', pol, rms, n_envs=16, steps=200, setup=dict(gender='female', participant=2, policy_name='Static'))
    assert np.all(np.isfinite(a['returns'])) and a['done'].all()
    np.testing.assert_array_equal(a['returns'], b['returns'])          # deterministic policy, same reset streams
    assert a['task_success'].shape == (16,)


@pytest.mark.gpu
def test_enjoy_vr_setup_call_runs_for_a_male_participant():
    """enjoy_vr.py:50,63's exact setup() call -- hipbone_to_mouth_height 0.54 for every participant --
    on a male participant: the episode runs on the male default human (the reference's non-VR
    reset overwrites the height, feeding.py:173-174) and equals an episode without the height."""
    torch.manual_seed(2)
    pol = PE.ActorCritic(25, 7)
    rms = PE.RunningMeanStd((25,))
    a = PE.evaluate('FeedingJaco-v0', pol, rms, n_envs=4, steps=20, setup=dict(gender='male', participant=1, policy_name='Static',
                                                                               hipbone_to_mouth_height=0.54))
    b = PE.evaluate('FeedingJaco-v0', pol, rms, n_envs=4, steps=20, setup=dict(gender='male', participant=1, policy_name='Static'))
    assert np.all(np.isfinite(a['returns']))
    np.testing.assert_array_equal(a['returns'], b['returns'])


# ------------------------------------------------------------------ reference-format recordings
class _Evil:
    def __reduce__(self):
        return (os.system, ('echo not-run',))


@pytest.mark.parametrize('proto', [0, 2, 3, 4, 5])
def test_reference_pickle_reader_reads_setup_and_actions(tmp_path, proto):
    """setup.pkl / actions.pkl as the reference writes them (feeding.py:50-54, 328-329), every
    pickle protocol: strings, floats, numpy float scalars and float32 action arrays come back."""
    import pickle
    rng = np.random.default_rng(proto)
    acts = [rng.uniform(-1, 1, 7).astype(np.float32) for _ in range(200)]
    with open(tmp_path / 'setup.pkl', 'wb') as f:
        pickle.dump(['jaco', 'female', np.float64(0.54)], f, protocol=proto)
    with open(tmp_path / 'actions.pkl', 'wb') as f:
        pickle.dump(acts, f, protocol=proto)
    setup = R.load_reference_pickle(str(tmp_path / 'setup.pkl'))
    assert setup == ['jaco', 'female', 0.54]
    got = R.load_reference_pickle(str(tmp_path / 'actions.pkl'))
    assert len(got) == 200 and all(g.dtype == np.float32 and np.array_equal(g, a) for g, a in zip(got, acts))
    big = np.arange(12, dtype='>f8').reshape(3, 4)          # byte order and Fortran layout survive
    with open(tmp_path / 'x.pkl', 'wb') as f:
        pickle.dump({'a': (big, np.asfortranarray(big))}, f, protocol=proto)
    x = R.load_reference_pickle(str(tmp_path / 'x.pkl'))
    assert np.array_equal(x['a'][0], big) and np.array_equal(x['a'][1], big)


def test_reference_pickle_reader_refuses_code_and_object_arrays(tmp_path):
    import pickle
    for k, obj in enumerate([[_Evil()], np.array([{'a': 1}], dtype=object), {1, 2}, SimpleNamespace(a=1)]):
        p = tmp_path / ('e%d.pkl' % k)
        with open(p, 'wb') as f:
            pickle.dump(obj, f)
        with pytest.raises(pickle.UnpicklingError):
            R.load_reference_pickle(str(p))


def test_reference_pickle_reader_raises_unpicklingerror_on_malformed_input(tmp_path):
    """Truncated files and hand-built hostile states (short dtype states, negative or wrapping
    shapes, wrong data lengths) all surface as pickle.UnpicklingError, so a caller that skips bad
    recordings on that error never crashes on another exception type."""
    import pickle
    import pickletools
    good = pickle.dumps(['jaco', 'male', np.float64(0.6), np.arange(6, dtype=np.float32).reshape(2, 3)], protocol=2)
    bad = [good[:k] for k in (1, 7, len(good) // 2, len(good) - 1)]
    # a dtype whose BUILD state is a 2-tuple: ('numpy', 'dtype') ('f8', False, True) + state (3, '<')
    bad.append(b'\x80\x02cnumpy\ndtype\nX\x02\x00\x00\x00f8\x89\x88\x87R(K\x03X\x01\x00\x00\x00<tb.')
    # ndarray states with hostile shapes / lengths: _reconstruct(ndarray, (0,), b'b') + BUILD(state)
    head = b'\x80\x02cnumpy.core.multiarray\n_reconstruct\ncnumpy\nndarray\nK\x00\x85C\x01b\x87R'
    dt = b'cnumpy\ndtype\nX\x02\x00\x00\x00f4\x89\x88\x87R(K\x03X\x01\x00\x00\x00<NNNJ\xff\xff\xff\xffJ\xff\xff\xff\xffK\x00tb'
    for shape, nbytes in ((b'J\xff\xff\xff\xff\x85', 0),                               # (-1,)
                          (b'\x8a\x08\x00\x00\x00\x00\x00\x00\x00@\x8a\x08\x00\x00\x00\x00\x00\x00\x00@\x86', 0),  # (2**62, 2**62): wraps in int64
                          (b'K\x03\x85', 8)):                                          # 3 floats, 8 bytes
        bad.append(head + b'(K\x01' + shape + dt + b'\x89C' + bytes([nbytes]) + b'\x00' * nbytes + b'tb.')
    for k, blob in enumerate(bad):
        p = tmp_path / ('m%d.pkl' % k)
        p.write_bytes(blob)
        with pytest.raises(pickle.UnpicklingError):
            R.load_reference_pickle(str(p))
    pickletools.dis(good, out=open(os.devnull, 'w'))      # the well-formed blob itself is valid
    p = tmp_path / 'ok.pkl'
    p.write_bytes(good)
    assert R.load_reference_pickle(str(p))[1] == 'male'


def test_reference_env_id_from_directory_name():
    """replay_vr_savemeta.py:20's naming rule."""
    f = R.reference_env_id
    assert f('participant_3/feeding_vr_data_jaco_ppo_participant_3_2019-01-01') == 'FeedingJaco-v0'
    assert f('participant_3/scratch_itch_vr_data_pr2_x') == 'ScratchItchPR2-v0'
    assert f('participant_3/bed_bathing_vr_data_pr2_x') == 'BedBathingPR2-v0'
    assert f('participant_3/drinking_vr_data_jaco_x') == 'DrinkingJaco-v0'
    assert f('participant_3/other') is None


@pytest.mark.gpu
def test_reference_recording_replays_its_actions(tmp_path):
    """A participant directory in the reference's format (setup.pkl, actions.pkl; feeding.py:
    146-157) replayed as replay_vr_savemeta.py does: the recorded gender is set up, the 200
    recorded actions are re-simulated from this build's reset (frame_%d.bullet cannot be restored
    without Bullet's serializer), and the result equals a live episode driven by the same actions
    from the same reset."""
    from avr import env as EV
    rng = np.random.default_rng(3)
    acts = [rng.uniform(-1, 1, 7).astype(np.float32) for _ in range(200)]
    d = tmp_path / 'participant_1' / 'feeding_vr_data_jaco_ppo_participant_1'
    R.write_reference_recording(str(d), 'jaco', 'female', 0.54, acts)
    res = R.savemeta_reference(str(tmp_path), out=str(tmp_path / 'meta.npz'))
    (k, v), = res.items()
    assert v['env_id'] == 'FeedingJaco-v0' and v['observations'].shape == (200, 25) and v['proportions'] == 'recorded'
    live = EV.AVRVecEnv('FeedingJaco-v0', 1, auto_reset=False, prefetch=False)
    live.setup('female', -1, '')
    live.reset()
    assert int(live.get_state()[0, ABI.S_TASK + ABI.T_GENDER]) == 1
    rews = [float(live.step(a[None])[1][0]) for a in acts]
    live.close()
    np.testing.assert_array_equal(np.array(rews, np.float32), v['rewards'].astype(np.float32))
    z = np.load(str(tmp_path / 'meta.npz'), allow_pickle=False)
    assert z['0_actions'].shape == (200, 7)


@pytest.mark.gpu
def test_reference_recording_replays_at_its_height(tmp_path):
    """A recording whose setup.pkl holds a non-default hipbone_to_mouth_height (0.57, female)
    replays on a human built at that height (feeding.py:153-156, human_creation.py:60-63): it
    equals a live env built with human_heights={'female': 0.57} and driven by the same actions,
    and differs from the default-height replay (the mouth, hence the observation, moves)."""
    from avr import env as EV
    rng = np.random.default_rng(4)
    acts = [rng.uniform(-1, 1, 7).astype(np.float32) for _ in range(20)]
    d = tmp_path / 'participant_2' / 'feeding_vr_data_jaco_ppo_participant_2'
    R.write_reference_recording(str(d), 'jaco', 'female', 0.57, acts)
    r = R.ReferenceReplayEnv(str(d))
    assert r.proportions == 'recorded' and r.env.human_heights == {'male': 0.6, 'female': 0.57}
    o0 = r.reset()
    rep = [r.step() for _ in acts]
    r.close()
    live = EV.AVRVecEnv('FeedingJaco-v0', 1, auto_reset=False, prefetch=False, human_heights={'female': 0.57})
    live.setup('female', -1, '')
    l0 = live.reset()
    np.testing.assert_array_equal(o0, l0)
    for (o, rw, _, _), a in zip(rep, acts):
        lo, lr, _, _ = live.step(a[None])
        np.testing.assert_array_equal(o, lo)
        np.testing.assert_array_equal(rw, lr)
    live.close()
    r = R.ReferenceReplayEnv(str(d), default_proportions=True)
    assert r.proportions.startswith('default')
    od = r.reset()
    r.close()
    assert np.abs(od - o0).max() > 1e-3
