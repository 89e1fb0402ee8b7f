"""Host side of the gym facade (no GPU): registry mirrors the reference's ids, spaces, errors."""
import re

import numpy as np
import pytest

from avr import env as E
from avr import _abi as ABI


def test_registry_has_every_reference_id():
    # ids registered by assistive_gym/__init__.py (49 ids: 4 tasks x {PR2, Jaco} x 6 variants + HumanTesting),
    # plus BASELINE's DressingJaco-v0 (build-defined: the reference has no dressing task)
    assert len(E.REGISTRY) == 50
    assert E.REGISTRY['DressingJaco-v0'] == ('dressing', 'jaco', True)
    assert E.REGISTRY['FeedingJaco-v0'] == ('feeding', 'jaco', True)
    assert E.REGISTRY['ScratchItchPR2-v0'] == ('scratch_itch', 'pr2', True)
    assert E.REGISTRY['BedBathingPR2-v0'] == ('bed_bathing', 'pr2', True)
    assert sum(v[2] for v in E.REGISTRY.values()) == 4
    for k in E.REGISTRY:
        assert re.match(r'^[A-Za-z0-9]+-v0$', k)


def test_unbuilt_ids_raise_not_implemented():
    with pytest.raises(NotImplementedError):
        E.AVRVecEnv('BedBathingJaco-v0', 4)
    with pytest.raises(KeyError):
        E.AVRVecEnv('NoSuchEnv-v0', 4)


def test_spaces():
    b = E.Box(-1.0, 1.0, (ABI.ACT_DIM,))
    x = b.sample(np.random.default_rng(0))
    assert x.shape == (7,) and x.dtype == np.float32 and b.contains(x)
    assert not b.contains(np.full(7, 2.0, np.float32))
    assert ABI.OBS_DIM == 25 and ABI.ACT_DIM == 7 and ABI.INFO_DIM == 2


def test_constants_follow_reference():
    assert E.MAX_EPISODE_STEPS == 200      # TimeLimit in assistive_gym/__init__.py
    assert E.SETTLE_FRAMES[ABI.TASK_FEEDING] == 100    # feeding.py:318-320
    assert E.SETTLE_FRAMES[ABI.TASK_SCRATCH] == 0      # scratch_itch.py reset: no settle frames
    assert E.SETTLE_FRAMES[ABI.TASK_BEDBATH] == 0      # the arm settle precedes the robot placement
    P = ABI.FEEDING_PARAMS
    assert P['num_sub_steps'] == 2 and P['solver_iterations'] == 10    # feeding.py:289
    assert P['time_step'] == 0.02                                      # world_creation.py:75
    assert P['frame_skip'] == 5


def test_prefetch_returns_only_the_matching_key():
    calls = []
    p = E._Prefetch(lambda a, b: calls.append((a, b)) or (a, b))
    p.start(('k', 1), 3, 4)
    assert p.take(('k', 2)) is None        # a different key is never handed out
    p.start(('k', 1), 3, 4)
    assert p.take(('k', 1)) == (3, 4)
    assert p.take(('k', 1)) is None        # taken once
