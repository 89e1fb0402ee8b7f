"""Host reset path (feeding.py:144-331 restated): IK, scene randomisation, determinism."""
import numpy as np

from avr import _abi as ABI
from avr import geom as G
from avr import reset as RS


def test_reset_states_are_deterministic_and_keyed_by_env_and_episode(scene):
    A, md = scene
    S1, _ = RS.batch_reset_states_fast(A, md, 1001, [3, 7])
    S2, _ = RS.batch_reset_states_fast(A, md, 1001, [7])
    assert np.array_equal(S1[1], S2[0])                 # independent of batch composition
    S3, _ = RS.batch_reset_states_fast(A, md, 1001, [7], episodes=[1])
    assert not np.array_equal(S2, S3)


def test_fast_and_reference_reset_agree_on_draws(scene):
    A, md = scene
    Sf, mf = RS.batch_reset_states_fast(A, md, 1001, [0, 1])
    Sr, mr = RS.batch_reset_states(A, md, 1001, [0, 1])
    for a, b in zip(mf, mr):
        assert a['gender'] == b['gender']
        assert np.allclose(a['bowl_pos'], b['bowl_pos']) and np.allclose(a['target_pos'], b['target_pos'])
    # the human pose and the task block follow the same draws
    h = slice(ABI.S_HUMAN, ABI.S_HUMAN + 7 * ABI.MAX_HUMAN)
    assert np.allclose(Sf[:, h], Sr[:, h])


def test_ik_reaches_target_and_spoon_rides_the_tool(scene):
    A, md = scene
    S, meta = RS.batch_reset_states_fast(A, md, 1001, list(range(6)))
    tool = int(A['task_tool_link'])
    okc = 0
    for k in range(6):
        _, _, CP, CQ, _, _ = RS.robot_fk(A, S[k, :int(A['n_dof'])])
        if meta[k]['ik_ok']:
            okc += 1
            assert np.linalg.norm(CP[tool] - meta[k]['target_pos']) < 0.02
        sp, sq = G.tf_mul(CP[tool], CQ[tool], A['task_tool_offset'][:3], A['task_tool_offset'][3:])
        assert np.allclose(S[k, ABI.S_FREE:ABI.S_FREE + 3], sp, atol=1e-9)
    assert okc >= 4


def test_reset_state_layout(scene):
    A, md = scene
    S, meta = RS.batch_reset_states_fast(A, md, 1001, [0, 1, 2, 3])
    t = ABI.S_TASK
    assert np.all(S[:, t + ABI.T_ALIVE] == 255)                    # 8 food particles alive
    assert set(S[:, t + ABI.T_GENDER]) <= {0.0, 1.0}
    assert np.all(S[:, t + ABI.T_ITER] == 0) and np.all(S[:, t + ABI.T_FLAGS] == 0)
    # food in a 2x2x2 lattice of pitch 2r above the spoon (feeding.py:299-304)
    sp = S[:, ABI.S_FREE:ABI.S_FREE + 3]
    f0 = S[:, ABI.S_FREE + ABI.FB_WORDS * 2:ABI.S_FREE + ABI.FB_WORDS * 2 + 3]
    assert np.allclose(f0 - sp, [-0.005, 0, 0.02])
    q = S[:, ABI.S_FREE + 3:ABI.S_FREE + 7]
    assert np.allclose(np.linalg.norm(q, axis=1), 1)


def test_tremor_reset_state(scene):
    """'tremor': human_tremors ~ U(+-20 deg) (world_creation.py:136-139), targets = the chain's
    starting angles (feeding.py:246-248), chain at rest with its motors off."""
    A, md = scene
    nd = md.n_dof
    S, meta = RS.batch_reset_states_fast(A, md, 1001, list(range(8)), impairment='tremor')
    assert all(m['impairment'] == 'tremor' for m in meta)
    assert np.all(S[:, ABI.S_TASK + ABI.T_HDYN] == 1)
    assert np.array_equal(S[:, ABI.S_HCH:ABI.S_HCH + 4], S[:, nd:nd + 4])
    tr = S[:, ABI.S_HCH + 4:ABI.S_HCH + 8]
    assert np.all(np.abs(tr) <= np.deg2rad(20)) and np.abs(tr).max() > np.deg2rad(5)
    assert np.all(S[:, nd] == 0)                                   # the neck starts straight
    assert np.all(np.abs(S[:, nd + 1:nd + 4]) <= np.deg2rad(30))   # head U(+-30 deg) (feeding.py:242)
    assert np.all(S[:, ABI.S_QD + nd:ABI.S_QD + nd + 4] == 0)
    assert np.all(S[:, ABI.S_MAXIMP + nd:ABI.S_MAXIMP + nd + 4] == 0)


def test_random_impairment_draws_all_four(scene):
    A, md = scene
    S, meta = RS.batch_reset_states_fast(A, md, 1001, list(range(48)), impairment='random')
    kinds = [m['impairment'] for m in meta]
    assert set(kinds) == {'none', 'limits', 'weakness', 'tremor'}
    tr = np.array([k == 'tremor' for k in kinds])
    assert np.array_equal(S[:, ABI.S_TASK + ABI.T_HDYN] == 1, tr)
