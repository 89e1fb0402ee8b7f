"""The fp64 oracle reproduces the committed golden fixtures (tests/golden/make_golden.py).

This pins the restatement against itself across builds and hosts; the same fixtures are the
reference the GPU parity tests (test_gpu_parity.py) are checked against.
"""
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


@pytest.fixture(scope='module')
def golden():
    return np.load(os.path.join(HERE, 'feeding_golden.npz'))


def test_oracle_reproduces_golden(scene, oracle_built, golden):
    from oracle.oracle import Oracle
    A, md = scene
    g = golden
    n = len(g['env_ids'])
    o = Oracle(md, n)
    o.set_state(g['S0'])
    obs0 = o.settle(100)
    assert np.allclose(obs0, g['obs0'], atol=1e-5)
    assert np.allclose(o.get_state(), g['S_settled'], atol=1e-5, rtol=1e-6)
    for t in range(g['actions'].shape[0]):
        ob, r, d, i = o.step(g['actions'][t])
        assert np.allclose(ob, g['obs'][t], atol=1e-5)
        assert np.allclose(r, g['rew'][t], atol=1e-5)
        assert np.array_equal(d, g['done'][t])
        assert np.allclose(i, g['info'][t], atol=1e-5)
        assert np.allclose(o.get_state(), g['states'][t], atol=1e-5, rtol=1e-6)


def test_golden_inputs_are_the_reset_path_and_philox(scene, golden):
    from avr import reset as RS, _lib
    A, md = scene
    g = golden
    ids, trem = list(g['env_ids']), g['tremor']
    S_a, _ = RS.batch_reset_states_fast(A, md, int(g['seed']), [e for e, t in zip(ids, trem) if not t])
    S_b, _ = RS.batch_reset_states_fast(A, md, int(g['seed']), [e for e, t in zip(ids, trem) if t], impairment='tremor')
    S0 = np.concatenate([S_a, S_b])
    assert np.allclose(S0.astype(np.float32).astype(np.float64), g['S0'], atol=1e-6)
    for t in range(g['actions'].shape[0]):
        assert np.array_equal(_lib.random_actions(int(g['seed']), g['env_ids'], t), g['actions'][t])
