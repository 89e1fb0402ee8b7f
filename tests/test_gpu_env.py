"""Gym facade on the GPU: FeedingEnv's reset/step contract (feeding.py:56-142, env.py:274-351)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_single_env_contract():
    from avr import env as E
    e = E.make('FeedingJaco-v0')
    obs = e.reset()
    assert obs.shape == (25,) and obs.dtype == np.float64 and np.all(np.isfinite(obs))
    obs, r, done, info = e.step(e.action_space.sample(np.random.default_rng(0)))
    assert obs.shape == (25,) and isinstance(r, float) and isinstance(done, bool)
    for k in ('total_force_on_human', 'task_success', 'action_robot_len', 'action_human_len', 'obs_robot_len', 'obs_human_len'):
        assert k in info
    assert info['action_robot_len'] == 7 and info['obs_robot_len'] == 25
    e.close()


def test_vec_env_time_limit_and_auto_reset():
    from avr import env as E, _lib
    n = 8
    v = E.AVRVecEnv('FeedingJaco-v0', n)
    o = v.reset()
    assert o.shape == (n, 25)
    for t in range(E.MAX_EPISODE_STEPS):
        o, r, d, info = v.step(_lib.random_actions(1001, np.arange(n), t))
        assert np.all(np.isfinite(o)) and np.all(np.isfinite(r))
        if t < E.MAX_EPISODE_STEPS - 1:
            assert not d.any()
    assert d.all()                                       # TimeLimit(200)
    assert 'terminal_observation' in info
    assert np.all(v.episode == 1)
    St = v.get_state()
    from avr import _abi as ABI
    assert np.all(St[:, ABI.S_TASK + ABI.T_ITER] == 0)  # auto-reset restarted the episodes
    assert np.all(v.flags() & 1 == 0)
    v.close()


def test_observation_layout():
    """obs = [spoon-torso(3), spoon quat(4), spoon-target(3), arm q(7), head-torso(3), head quat(4), force(1)]."""
    from avr import env as E, _abi as ABI
    v = E.AVRVecEnv('FeedingJaco-v0', 2)
    o = v.reset()
    St = v.get_state()
    q_arm = St[:, ABI.S_Q:ABI.S_Q + 7]
    assert np.allclose(o[:, 10:17], q_arm, atol=1e-6)
    assert np.allclose(np.linalg.norm(o[:, 3:7], axis=1), 1, atol=1e-5)
    assert np.allclose(np.linalg.norm(o[:, 20:24], axis=1), 1, atol=1e-5)
    sp = St[:, ABI.S_FREE:ABI.S_FREE + 3]
    tgt = St[:, ABI.S_TASK + ABI.T_TARGET:ABI.S_TASK + ABI.T_TARGET + 3]
    assert np.allclose(o[:, 7:10], sp - tgt, atol=1e-5)
    v.close()
