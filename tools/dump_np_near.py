"""Dump the GPU narrowphase on test_gpu_narrowphase_near_contact's queries for one task
(python tools/dump_np_near.py TASK OUT.npz): pairs, poses and the (n, 8) results, for offline
comparison with the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'assistive-vr-gym_amd'), ROOT, os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)
from avr import _abi as ABI, _lib  # noqa: E402
from test_narrowphase_pairs import _near_contact  # noqa: E402

task = int(sys.argv[1])
A = ABI.load_scene(task)
md = ABI.ModelDesc(A)
pairs, X = _near_contact(A, md, task, 3000, 22)
sim = _lib.Sim(md, 1)
try:
    g = sim.narrowphase(pairs, X)
finally:
    sim.close()
np.savez(sys.argv[2], pairs=pairs, X=X, g=g)
print('dumped', len(pairs))
