"""Compiled scene (avr/data/feeding_jaco.npz) against the reference's model facts (SURVEY
Appendix B, 8a a3.1/a10).  When the reference assets are mounted (build container only), the
committed npz is also checked to be exactly what the compiler produces from them."""
import os
import tempfile

import numpy as np
import pytest

from avr import _abi as ABI

REF = '/root/reference/assistive_gym/envs/assets'


def test_jaco_topology(scene):
    A, md = scene
    assert int(A['n_links']) == 15 and int(A['n_dof']) == 10          # 15 joints / 10 DoF
    assert list(A['task_arm_dofs']) == list(range(7))
    assert len(A['task_finger_dofs']) == 3
    par = A['rl_parent']
    assert par[0] == -1 and all(par[i] < i for i in range(1, 15))     # DFS pre-order
    lim = A['rl_has_limit'][A['rl_dof'] >= 0]
    # joints 2, 4, 6 limited; 1, 3, 5, 7 continuous (j2s7s300_gym.urdf)
    assert list(lim[:7]) == [0, 1, 0, 1, 0, 1, 0]
    lo = A['rl_lower'][np.nonzero(A['rl_has_limit'])[0]][:3]
    assert np.allclose(lo, [0.820, 0.524, 1.134], atol=2e-3)


def test_free_bodies(scene):
    A, md = scene
    m = A['fb_mass']
    assert len(m) == 10
    assert m[0] == pytest.approx(1.0) and m[1] == pytest.approx(0.1)   # spoon.urdf:10, bowl.urdf:10
    assert np.allclose(m[2:], 0.001)                                   # feeding.py:296
    g = A['fb_gravity'].reshape(-1, 3)
    assert np.allclose(g[0], 0) and np.allclose(g[1:, 2], -9.81)      # spoon gravity off (feeding.py:287)
    assert np.all(A['fb_inertia'] > 0)


def test_shapes_and_pairs(scene):
    A, md = scene
    kinds = np.bincount(A['shape_kind'], minlength=4)
    assert kinds[0] >= 8                                                # sphere shapes (food)
    spoon = int(A['task_spoon_body'])
    assert A['body_shape_count'][spoon] == 64                          # 64-piece VHACD spoon
    assert A['body_shape_count'][int(A['task_bowl_body'])] == 70
    pa, pb = A['pair_a'], A['pair_b']
    kinds_b = A['body_kind']
    # no static-static pairs; robot parent/child pairs excluded; spoon vs Jaco links 7..14 off
    for a, b in zip(pa, pb):
        assert not (kinds_b[a] == 2 and kinds_b[b] == 2)
        if kinds_b[a] == 0 and kinds_b[b] == 0:
            la, lb = A['body_index'][a], A['body_index'][b]
            assert A['rl_parent'][la] != lb and A['rl_parent'][lb] != la
        if spoon in (a, b):
            o = b if a == spoon else a
            if kinds_b[o] == 0:
                assert not (7 <= A['body_index'][o] <= 14)
    assert np.all(A['shape_margin'][A['shape_kind'] >= 2] == pytest.approx(0.001))


@pytest.mark.skipif(not os.path.isdir(REF), reason='reference assets not mounted (GPU box)')
def test_committed_scene_matches_compiler():
    from avr import model_compiler as MC
    with tempfile.TemporaryDirectory() as d:
        path, A = MC.compile_all(d)
        committed = np.load(os.path.join(MC.DATA_DIR, 'feeding_jaco.npz'))
        assert set(A) == set(committed.files)
        for k in A:
            assert np.array_equal(np.asarray(A[k]), committed[k]), k
