"""How far BedBathing's reset settle (the right arm dropped onto the mattress, bed_bathing.py:283-289)
moves under the Bullet defaults this build assumes but cannot pin: the fp64
oracle settle per gender with each assumption varied, against the reference's own settled arm pose
(bed_bathing.py:232, the VR/replay vector).  The spread is the restatement's uncertainty at that
anchor.

    python tools/bb_settle_sensitivity.py
"""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'assistive-vr-gym_amd'), ROOT, os.path.join(ROOT, 'tests')]
from avr import _abi as ABI, reset_bedbath as RBB  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
import test_bedbath as T  # noqa: E402

np.set_printoptions(precision=4, suppress=True, linewidth=160)
A = ABI.load_scene(ABI.TASK_BEDBATH)
base = ABI.ModelDesc(A)
VARIANTS = [
    ('assumed defaults', {}),
    ('erp 0.1', dict(erp=0.1)), ('erp 0.8', dict(erp=0.8)),
    ('warm start 0.1', dict(warmstart=0.1)), ('warm start 1.0', dict(warmstart=1.0)),
    ('no damping', dict(linear_damping=0.0, angular_damping=0.0)), ('damping 0.1', dict(linear_damping=0.1, angular_damping=0.1)),
    ('10 iterations', dict(solver_iterations=10)), ('200 iterations', dict(solver_iterations=200)),
]


def settle(md):
    def run(S, frames):
        o = Oracle(md, len(S))
        o.set_threads(2)
        o.set_state(S)
        o.settle(frames)
        return o.get_state()
    return RBB.settled_arms(A, md, runner=run)


rows = {}
for name, over in VARIANTS:
    md = ABI.ModelDesc(A, over) if over else base
    st = settle(md)
    rows[name] = {g: st[g][0] for g in ('male', 'female')}
    print('%-18s male %s (max dev %.4f)  female %s (max dev %.4f)' % (
        name, rows[name]['male'], np.abs(rows[name]['male'] - T.VR_ARM).max(), rows[name]['female'], np.abs(rows[name]['female'] - T.VR_ARM).max()))
print('reference (bed_bathing.py:232)', T.VR_ARM)
for g in ('male', 'female'):
    Q = np.array([rows[n][g] for n, _ in VARIANTS])
    print('%s: spread over the assumptions (max - min per joint) %s, max %.4f' % (g, Q.max(0) - Q.min(0), (Q.max(0) - Q.min(0)).max()))
