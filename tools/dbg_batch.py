"""Batch-composition check at the PR2 launch shape: the sampled envs of
tests/test_pr2_launch_shape.py stepped (a) inside the 4096-env, 4-group launch, (b) alone in a
1-env handle, (c) in a 32-env handle holding their part-B block's neighbours, with the same
actions -- bitwise comparison of the state after each step, and each against the fp64 oracle.

  TASK=1 python tools/dbg_batch.py
"""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'assistive-vr-gym_amd'), ROOT, os.path.join(ROOT, 'tests')]
from avr import _abi as ABI, _lib  # noqa: E402
import test_pr2_launch_shape as T  # noqa: E402

np.set_printoptions(precision=5, suppress=True, linewidth=200)
TASK = int(os.environ.get('TASK', 1))
STEPS = int(os.environ.get('STEPS', 5))
A, md, L, P, is_c = T._pool(TASK, 16)
E = T.E_LAUNCH
PICK = T.picks(is_c)
S = np.tile(P, (E // len(P) + 1, 1))[:E].astype(np.float32)
nd = md.n_dof + (int(A['hc_n']) if TASK == ABI.TASK_SCRATCH else 0)
acts = [(_lib.random_actions(1001, np.arange(E), t) * 0.2).astype(np.float32) for t in range(STEPS)]


def run(ids, groups=None):
    if groups is not None:
        os.environ['AVR_ENV_GROUPS'] = str(groups)
    sim = _lib.Sim(md, len(ids))
    os.environ.pop('AVR_ENV_GROUPS', None)
    sim.set_state(S[ids])
    out = []
    for t in range(STEPS):
        sim.step(acts[t][ids])
        out.append(sim.get_state())
    sim.close()
    return out


full = run(np.arange(E))
o = T._oracle(md, len(PICK), 'f64')
o.set_state(S[PICK].astype(np.float64))
orc = []
for t in range(STEPS):
    o.step(acts[t][PICK])
    orc.append(o.get_state())
alone = [run(np.array([e])) for e in PICK]
for k, e in enumerate(PICK):
    blk0 = (e // 32) * 32
    blk = run(np.arange(blk0, blk0 + 32))
    j = e - blk0
    line = []
    for t in range(STEPS):
        F, Al, B, C = full[t][e], alone[k][t][0], blk[t][j], orc[t][k]
        line.append('t%d full-alone %.2e full-block %.2e alone-orc %.2e full-orc %.2e' % (
            t, np.abs(F[:nd] - Al[:nd]).max(), np.abs(F[:nd] - B[:nd]).max(), np.abs(Al[:nd] - C[:nd]).max(), np.abs(F[:nd] - C[:nd]).max()))
    bits = all(np.array_equal(full[t][e], alone[k][t][0]) for t in range(STEPS))
    print('env %4d pool %2d contact %d bit-identical full/alone %s' % (e, e % len(P), int(is_c[e % len(P)]), bits))
    if not bits:
        for s in line:
            print('   ', s)
